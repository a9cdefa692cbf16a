#!/bin/bash
# Bench lines for the BASELINE configs (parity is covered by pytest).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
run() {
  local name=$1; shift
  timeout -k 10 300 python bench.py --steps 3 --warmup 1 --cpu-seconds 0 "$@" > gpurun_out/sweep_$name.log 2>&1
  local rc=$?
  echo "== $name rc=$rc"; grep '^{' gpurun_out/sweep_$name.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['value']/1e9,3), 'Grec/s', d['ms_per_step'], 'ms/step frac', d['roofline']['frac'])"
  [ $rc -eq 0 ] || exit $rc
}
run c2
run c2f --config C2f
run c1 --config C1
run c5 --config C5 --records 33554432
run c3 --config C3 --records 100000000
run c4 --config C4 --records 33554432
run c2_exchange --force-exchange
run c2_per_record --emit per_record --records 33554432
