#!/bin/bash
# Iteration: session + exchange parity tests, C4 bench + kernel statistics + traffic,
# force-exchange C2 line.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/prof gpurun_out/pmc; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
  -k "${K:-session or c4 or C4 or mirror or exchange or two_ranks or sharded or kat}" > gpurun_out/pt_it6.log 2>&1; rc=$?
tail -4 gpurun_out/pt_it6.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --config C4 --steps 1 --warmup 1 --cpu-seconds 0 --no-host-input --no-per-record > gpurun_out/b_c4.log 2>&1 || { tail -20 gpurun_out/b_c4.log; exit 1; }
tail -1 gpurun_out/b_c4.log | cut -c1-200
timeout -k 10 300 python bench.py --force-exchange --steps 3 --warmup 1 --cpu-seconds 0 --no-host-input --no-per-record > gpurun_out/b_fx.log 2>&1 || { tail -20 gpurun_out/b_fx.log; exit 1; }
tail -1 gpurun_out/b_fx.log | cut -c1-260
bash tools/prof.sh it_c4 --config C4 --no-host-input --no-per-record || exit $?
bash tools/traffic.sh c4 --config C4 --no-host-input --no-per-record | tail -8
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "per_record or PER_RECORD or segments or messy" > gpurun_out/pt_it6b.log 2>&1 || { tail -30 gpurun_out/pt_it6b.log; exit 1; }
tail -2 gpurun_out/pt_it6b.log
bash tools/prof.sh it_c2pr --emit per_record --no-host-input --no-per-record
