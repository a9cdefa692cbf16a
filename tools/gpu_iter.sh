#!/bin/bash
# One GPU iteration: GPU parity tests (PYTEST_K selects), then bench lines for
# the configs in CONFIGS with HSG_PHASES breakdowns. Stops at the first failure.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out; export TMPDIR=/tmp
if [ -z "$NOTEST" ]; then
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -15 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
fi
for c in ${CONFIGS-C2}; do
  HSG_PHASES=1 timeout -k 10 300 python bench.py --config $c --steps ${STEPS:-3} --warmup 1 --cpu-seconds 0 ${BENCH_ARGS} > gpurun_out/bench_$c.log 2>&1 || { tail -20 gpurun_out/bench_$c.log; exit 1; }
  grep -v phases gpurun_out/bench_$c.log | cut -c1-330; grep phases gpurun_out/bench_$c.log | tail -3
done
if [ -n "$PROF" ]; then bash tools/prof.sh $PROF --config ${PROFCFG:-C2}; fi
