#!/bin/bash
# Session iteration: session GPU parity tests, the C4 bench line and its kernel statistics.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/prof; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread \
  -k "${K:-session or c4 or C4 or kat}" > gpurun_out/pt_c4.log 2>&1; rc=$?
tail -4 gpurun_out/pt_c4.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --config C4 --steps 2 --warmup 1 --cpu-seconds 0 --no-host-input --no-per-record > gpurun_out/b_c4.log 2>&1 || { tail -20 gpurun_out/b_c4.log; exit 1; }
cut -c1-300 gpurun_out/b_c4.log | tail -1
bash tools/prof.sh it_c4 --config C4 --no-host-input --no-per-record
