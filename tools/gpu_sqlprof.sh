#!/bin/bash
# SQL op shape: its GPU tests (T overrides), then kernel statistics of the
# sql_shape bench block in each emit mode.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${T:-tests/test_gpu_sql_shape.py}
timeout -k 10 900 python -u -m pytest $T -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pt_sql.log 2>&1
rc=$?; tail -3 gpurun_out/pt_sql.log; [ $rc -eq 0 ] || exit $rc
for m in ${MODES:-per_batch per_record}; do
  bash tools/prof.sh r06_sql_$m --config C2 --input hbm --no-hbm --no-per-record --sql-emit $m --extra-steps 2 || exit $?
  grep '^{' gpurun_out/prof/r06_sql_$m.log | python3 -c "import json,sys;d=json.loads(sys.stdin.read());s=d['sql_shape'];v=s['$m'];print('$m', v['value']/1e9, v['ms_per_step'], v['lean_batches'], v['batches'], v['replays_onto_record_kernels'], v['roofline']['avg_launch_ms'])"
done
