#!/bin/bash
# Bench lines for several BASELINE configs (parity is covered by pytest).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
run() {
  local name=$1; shift
  timeout -k 10 300 python bench.py --steps 3 --warmup 1 --cpu-seconds 0 "$@" > gpurun_out/sweep_$name.log 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -1 gpurun_out/sweep_$name.log | cut -c1-600
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
}
run c2_exchange --force-exchange
run c1 --config C1
run c2f --config C2f
run c5 --config C5 --records 33554432
run c4 --config C4 --records 33554432
run c3 --config C3 --records 100000000
run c2_per_record --emit per_record --records 33554432
