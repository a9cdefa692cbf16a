#!/bin/bash
# Iteration session: GPU parity tests, then short benches (BENCHES="C2 C3 ...",
# AGG_NTS="1024 512"). Stops at the first failure / fault / timeout.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread ${PYTEST_ARGS} > gpurun_out/pytest_gpu.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
fi
for cfg in ${BENCHES:-C2}; do
  for nt in ${AGG_NTS:-1024}; do
    HSG_AGG_NT=$nt HSG_PHASES=${PHASES:-} timeout -k 10 300 python bench.py --config $cfg --steps ${STEPS:-3} --warmup 1 --cpu-seconds 0 ${BENCH_ARGS} > gpurun_out/bench_${cfg}_${nt}.log 2>&1
    rc=$?; echo "== $cfg nt=$nt rc=$rc"; grep '^{' gpurun_out/bench_${cfg}_${nt}.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value']/1e9, 'Grec/s', d['ms_per_step'], 'ms/step', 'frac', d['roofline']['frac'], 'touched', d['touched_per_step'])" ; [ $rc -eq 0 ] || { tail -5 gpurun_out/bench_${cfg}_${nt}.log; exit $rc; }
    [ -n "$PHASES" ] && grep phases gpurun_out/bench_${cfg}_${nt}.log | tail -2
  done
done
exit 0
