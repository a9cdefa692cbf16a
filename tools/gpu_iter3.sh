#!/bin/bash
# Round-3 iteration: session + per-record GPU parity tests, then the C2
# per-record and C4 bench lines and their kernel statistics.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/prof; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread \
  -k "${K:-session or per_record or c4 or C4 or kat or messy}" > gpurun_out/pt_iter.log 2>&1; rc=$?
tail -6 gpurun_out/pt_iter.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --emit per_record --steps 3 --warmup 1 --cpu-seconds 0 --no-host-input --no-per-record > gpurun_out/b_pr.log 2>&1 || { tail -20 gpurun_out/b_pr.log; exit 1; }
cut -c1-400 gpurun_out/b_pr.log | tail -1
timeout -k 10 300 python bench.py --config C4 --steps 2 --warmup 1 --cpu-seconds 0 --no-host-input --no-per-record > gpurun_out/b_c4.log 2>&1 || { tail -20 gpurun_out/b_c4.log; exit 1; }
cut -c1-400 gpurun_out/b_c4.log | tail -1
bash tools/prof.sh it_c2pr --emit per_record --no-host-input --no-per-record || exit $?
bash tools/prof.sh it_c4 --config C4 --no-host-input --no-per-record
