#!/bin/bash
# PMC counters for one bench invocation, one rocprofv3 pass per counter group:
#   tools/pmc.sh NAME KERNEL_REGEX "CTR CTR ..." ["CTR ..." ...] -- [bench args...]
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
name=$1; regex=$2; shift 2
groups=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do groups+=("$1"); shift; done
[ "$1" = "--" ] && shift
mkdir -p gpurun_out/pmc
i=0
for g in "${groups[@]}"; do
  timeout -k 10 300 rocprofv3 --pmc $g --kernel-include-regex "$regex" -d gpurun_out/pmc -o ${name}_$i \
    --output-format csv -- python3 bench.py --steps 1 --warmup 0 --cpu-seconds 0 "$@" > gpurun_out/pmc/${name}_$i.log 2>&1
  rc=$?; echo "== $name pass $i ($g) rc=$rc"; [ $rc -eq 0 ] || exit $rc
  python3 - gpurun_out/pmc/${name}_${i}_counter_collection.csv <<'PY'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
acc = collections.defaultdict(float); disp = collections.defaultdict(set)
for r in rows:
    k = (r['Kernel_Name'][:48], r['Counter_Name'])
    acc[k] += float(r['Counter_Value']); disp[k].add(r['Dispatch_Id'])
for (kn, cn), v in sorted(acc.items()):
    print(f"{kn:48s} {cn:24s} {v / len(disp[(kn, cn)]):16.1f} per dispatch")
PY
  i=$((i+1))
done
