#!/bin/bash
# Iteration: parity tests of the per-record, hopping and session paths, then the C2
# per-record, C3 and C4 bench lines with kernel statistics.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/prof; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread \
  -k "${K:-per_record or PER_RECORD or kat or messy or hopping or C3 or configs or lean or session or c4}" > gpurun_out/pt_it4.log 2>&1; rc=$?
tail -4 gpurun_out/pt_it4.log; [ $rc -eq 0 ] || exit $rc
HSG_PHASES=1 timeout -k 10 300 python bench.py --emit per_record --steps 2 --warmup 1 --cpu-seconds 0 --no-host-input --no-per-record > gpurun_out/b_prph.log 2>&1 || { tail -20 gpurun_out/b_prph.log; exit 1; }
grep "per-record bucket" gpurun_out/b_prph.log | tail -2; tail -1 gpurun_out/b_prph.log | cut -c1-200
timeout -k 10 300 python bench.py --config C3 --steps 1 --warmup 1 --cpu-seconds 0 --no-host-input --no-per-record > gpurun_out/b_c3.log 2>&1 || { tail -20 gpurun_out/b_c3.log; exit 1; }
tail -1 gpurun_out/b_c3.log | cut -c1-200
timeout -k 10 300 python bench.py --config C4 --steps 1 --warmup 1 --cpu-seconds 0 --no-host-input --no-per-record > gpurun_out/b_c4.log 2>&1 || { tail -20 gpurun_out/b_c4.log; exit 1; }
tail -1 gpurun_out/b_c4.log | cut -c1-200
bash tools/prof.sh it_c2pr --emit per_record --no-host-input --no-per-record || exit $?
bash tools/prof.sh it_c3 --config C3 --no-host-input --no-per-record || exit $?
bash tools/prof.sh it_c4 --config C4 --no-host-input --no-per-record
