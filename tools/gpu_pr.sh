cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "per_record or messy or KAT or kat or configs_reduced or grace or edge" > gpurun_out/pt_pr.log 2>&1; rc=$?; tail -15 gpurun_out/pt_pr.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --cpu-seconds 0 --no-host-input > gpurun_out/bench_pr.log 2>&1; rc=$?; tail -c 1500 gpurun_out/bench_pr.log; exit $rc
