#!/bin/bash
# Tests T (optional), then HBM-resident bench lines for the configs in CFGS
# (default C2 C5), REP times each, and a kernel timeline of one C2 run.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/qab; export TMPDIR=/tmp
if [ -n "$T" ]; then
  timeout -k 10 ${TT:-600} python -u -m pytest $T -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/qab/pt.log 2>&1
  rc=$?; tail -2 gpurun_out/qab/pt.log; [ $rc -eq 0 ] || exit $rc
fi
for cfg in ${CFGS:-C2 C5}; do for r in $(seq ${REP:-2}); do
  timeout -k 10 300 python bench.py --config $cfg --input hbm --no-per-record --no-sql-shape --cpu-seconds 0 --steps 10 $ARGS > gpurun_out/qab/$cfg.$r.log 2>&1 || exit 1
  python3 -c "import json,sys; d=json.loads([l for l in open('gpurun_out/qab/$cfg.$r.log') if l.startswith('{')][-1]); print('$cfg', round(d['value']/1e9,2), 'G', d['ms_per_step'])"
done; done
if [ -z "$NOPROF" ]; then
  bash tools/prof.sh qab_c2 --config C2 --input hbm --no-hbm --no-per-record --no-sql-shape > /dev/null && python3 tools/timeline.py gpurun_out/prof/qab_c2_kernel_trace.csv 12
fi
