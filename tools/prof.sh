#!/bin/bash
# rocprofv3 kernel stats for one bench invocation: tools/prof.sh NAME [bench args...]
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
name=$1; shift
mkdir -p gpurun_out/prof
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o $name --output-format csv -- \
  python3 bench.py --steps 2 --warmup 1 --cpu-seconds 0 "$@" > gpurun_out/prof/$name.log 2>&1
rc=$?
echo "== $name rc=$rc"; tail -1 gpurun_out/prof/$name.log | cut -c1-260
python3 - gpurun_out/prof/${name}_kernel_stats.csv <<'PY'
import csv, sys
try:
    rows = list(csv.DictReader(open(sys.argv[1])))
except FileNotFoundError:
    sys.exit(0)
for r in rows[:10]:
    print(r['Name'][:56].ljust(56), r['Calls'].rjust(5), f"{float(r['AverageNs'])/1e3:10.1f}us", r['Percentage'][:5])
PY
exit $rc
