#!/bin/bash
# Round-3 validation: smoke + every -m gpu test, then the default bench line.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
bash tools/gpu_tests.sh || exit $?
timeout -k 10 400 python bench.py > gpurun_out/bench_default.log 2>&1; rc=$?; tail -c 3000 gpurun_out/bench_default.log; exit $rc
