#!/bin/bash
# Round-3 full GPU pass: smoke + every -m gpu test, the default bench line, and
# kernel statistics of the per-record (EMIT CHANGES) C2 run.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
bash tools/gpu_tests.sh || exit $?
timeout -k 10 400 python bench.py > gpurun_out/bench_default.log 2>&1; rc=$?; tail -c 2500 gpurun_out/bench_default.log; [ $rc -eq 0 ] || exit $rc
bash tools/prof.sh r03_c2_pr --emit per_record --no-host-input --no-per-record
