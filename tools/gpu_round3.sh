#!/bin/bash
# Round-3 GPU pass: the new tests first (per-record, two ranks), then the bench line.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_two_ranks.py -m gpu -x -q --timeout 150 --timeout-method thread -k "${K:-per_record or two_ranks or messy or kat}" > gpurun_out/pt_r3.log 2>&1; rc=$?; tail -15 gpurun_out/pt_r3.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --cpu-seconds 0 --no-host-input > gpurun_out/bench_r3.log 2>&1; rc=$?; tail -c 1800 gpurun_out/bench_r3.log; exit $rc
