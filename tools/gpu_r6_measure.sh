#!/bin/bash
# Round-6 bench lines (BASELINE.md formula: pinned host input in the
# decoder's transport, H2D timed; each line also carries its hbm_resident
# block) -> gpurun_out/r06/<name>.json
#   bash tools/gpu_r5_measure.sh [name ...]   (default: all)
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/r06; export TMPDIR=/tmp
b() { name=$1; shift; timeout -k 10 500 python bench.py "$@" > gpurun_out/r06/$name.log 2>&1; rc=$?
      tail -1 gpurun_out/r06/$name.log > gpurun_out/r06/$name.json
      echo "== $name rc=$rc"; cut -c1-300 gpurun_out/r06/$name.json; return $rc; }
ARGS="$*"
run() { n=$1; shift; if [ -z "$ARGS" ] || [[ " $ARGS " == *" $n "* ]]; then b $n "$@" || exit $?; fi; }
run c2_default --steps 5 --warmup 2 --cpu-seconds 10
run c2f --config C2f --steps 5 --warmup 2 --cpu-seconds 10 --no-per-record
run c5 --config C5 --steps 3 --warmup 1 --cpu-seconds 10
run c3 --config C3 --steps 2 --warmup 1 --cpu-seconds 10 --no-per-record
run c4 --config C4 --steps 2 --warmup 1 --cpu-seconds 10 --no-per-record
run c3_pr --config C3 --emit per_record --records 100663296 --steps 2 --warmup 1 --cpu-seconds 10 --no-per-record
run c4_pr --config C4 --emit per_record --records 167772160 --steps 2 --warmup 1 --cpu-seconds 10 --no-per-record
run c2_fx --force-exchange --steps 3 --warmup 1 --cpu-seconds 0 --no-per-record
run c2_fx_pr --force-exchange --emit per_record --steps 3 --warmup 1 --cpu-seconds 0 --no-per-record
# the SQL drop-in's op shape (HSG_OPF_LITERAL_FORMS + a LAST passthrough), HBM-resident, both emit modes
run c2_sql --input hbm --steps 2 --warmup 1 --cpu-seconds 0 --no-per-record --extra-steps 3
