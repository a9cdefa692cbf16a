cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
timeout -k 10 400 python bench.py > gpurun_out/bench_default.log 2>&1 || { tail gpurun_out/bench_default.log; exit 1; }
tail -1 gpurun_out/bench_default.log
timeout -k 10 300 python bench.py --force-exchange --cpu-seconds 0 --steps 3 --warmup 1 > gpurun_out/bench_xchg.log 2>&1 || { tail gpurun_out/bench_xchg.log; exit 1; }
tail -1 gpurun_out/bench_xchg.log | cut -c1-300
timeout -k 10 300 python bench.py --emit per_record --records 33554432 --cpu-seconds 0 --steps 2 --warmup 1 > gpurun_out/bench_pr.log 2>&1 || { tail gpurun_out/bench_pr.log; exit 1; }
tail -1 gpurun_out/bench_pr.log | cut -c1-300
