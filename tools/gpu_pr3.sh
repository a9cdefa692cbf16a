#!/bin/bash
# Per-record iteration: per-record GPU parity tests, the C2 per-record bench line and its kernel statistics.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/prof; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread \
  -k "${K:-per_record or PER_RECORD or kat or messy}" > gpurun_out/pt_pr.log 2>&1; rc=$?
tail -4 gpurun_out/pt_pr.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --emit per_record --steps 3 --warmup 1 --cpu-seconds 0 --no-host-input --no-per-record > gpurun_out/b_pr.log 2>&1 || { tail -20 gpurun_out/b_pr.log; exit 1; }
cut -c1-300 gpurun_out/b_pr.log | tail -1
bash tools/prof.sh it_c2pr --emit per_record --no-host-input --no-per-record
