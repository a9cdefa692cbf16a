#!/bin/bash
# Round-4 baseline of the lines never measured before: EMIT CHANGES for C3
# (hopping) and C4 (session replay), C2f; kernel statistics of both.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/prof; export TMPDIR=/tmp
b() { name=$1; shift; timeout -k 10 400 python bench.py --cpu-seconds 0 --input hbm --no-hbm --no-per-record "$@" > gpurun_out/$name.log 2>&1; rc=$?
      echo "== $name rc=$rc"; tail -1 gpurun_out/$name.log | cut -c1-400; return $rc; }
b c3_pr --config C3 --emit per_record --records 100663296 --steps 2 --warmup 1 &&
b c4_pr --config C4 --emit per_record --records 100663296 --steps 2 --warmup 1 &&
b c2f --config C2f --steps 5 --warmup 2 &&
bash tools/prof.sh r04_c3_pr --config C3 --emit per_record --records 100663296 --input hbm --no-hbm --no-per-record &&
bash tools/prof.sh r04_c4_pr --config C4 --emit per_record --records 100663296 --input hbm --no-hbm --no-per-record
