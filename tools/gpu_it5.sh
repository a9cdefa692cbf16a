#!/bin/bash
# Iteration: new GPU tests (session mirror mix, per-record segments) + per-record parity, then
# the per-record phase clocks and kernel statistics, then PMC passes on C4 / C3.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/prof; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
  -k "${K:-mirror or segments or per_record or PER_RECORD or kat or messy}" > gpurun_out/pt_it5.log 2>&1; rc=$?
tail -4 gpurun_out/pt_it5.log; [ $rc -eq 0 ] || exit $rc
HSG_PHASES=1 timeout -k 10 300 python bench.py --emit per_record --steps 2 --warmup 1 --cpu-seconds 0 --no-host-input --no-per-record > gpurun_out/b_prph.log 2>&1 || { tail -20 gpurun_out/b_prph.log; exit 1; }
grep "per-record bucket" gpurun_out/b_prph.log | tail -2; tail -1 gpurun_out/b_prph.log | cut -c1-200
bash tools/prof.sh it_c2pr --emit per_record --no-host-input --no-per-record || exit $?
bash tools/gpu_pmc4.sh
