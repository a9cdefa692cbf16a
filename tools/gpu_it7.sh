#!/bin/bash
# Iteration: per-record parity tests, per-record C2 bench line + kernel statistics.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/prof gpurun_out/pmc; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
  -k "${K:-per_record or PER_RECORD or segments or messy or emit_changes or changes}" > gpurun_out/pt_it7.log 2>&1; rc=$?
tail -3 gpurun_out/pt_it7.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --emit per_record --steps 3 --warmup 1 --cpu-seconds 0 --no-host-input --no-per-record > gpurun_out/b_pr.log 2>&1 || { tail -20 gpurun_out/b_pr.log; exit 1; }
tail -1 gpurun_out/b_pr.log | cut -c1-300
bash tools/prof.sh it_c2pr7 --emit per_record --no-host-input --no-per-record
