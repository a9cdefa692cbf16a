cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo smoke failed; tail gpurun_out/smoke.log; exit 1; }
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -5 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
for c in C2 C5 C3; do HSG_PHASES=1 timeout -k 10 300 python bench.py --config $c --steps 2 --warmup 1 --cpu-seconds 0 > gpurun_out/bench_$c.log 2>&1 || exit 1; grep -v phases gpurun_out/bench_$c.log | cut -c1-400; grep phases gpurun_out/bench_$c.log | tail -4; done
