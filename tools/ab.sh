#!/bin/bash
# A/B: bench the current tree and a reference worktree (.abtest/old) in one GPU session.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp; mkdir -p gpurun_out
for i in 1 2; do
  for t in . .abtest/old; do
    (cd $t && timeout -k 10 200 python bench.py --steps 3 --warmup 1 --cpu-seconds 0 ${BENCH_ARGS} > /tmp/ab.log 2>&1) || { tail -3 /tmp/ab.log; exit 1; }
    echo "== $t: $(grep '^{' /tmp/ab.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]/1e9,3), "Grec/s", d["ms_per_step"], "ms")')"
  done
done
