#!/bin/bash
# Kernel statistics and PMC traffic of every BASELINE config for one round:
#   tools/profile_round.sh ROUND [CONFIG ...]   (default C2 C3 C4 C5)
# -> gpurun_out/prof/<cfg>_kernel_stats.csv, gpurun_out/pmc/traffic_<cfg>.json
cd "${GRAFT_REPO_ROOT:-/root/repo}"
round=$1; shift
cfgs=${*:-C2 C3 C4 C5}
for c in $cfgs; do
  lc=$(echo $c | tr A-Z a-z)
  bash tools/prof.sh ${round}_$lc --config $c --input hbm --no-hbm --no-per-record || exit $?
  bash tools/traffic.sh $lc --config $c --input hbm --no-hbm --no-per-record > /dev/null || exit $?
  python3 -c "import json,sys; d=json.load(open('gpurun_out/pmc/traffic_$lc.json')); print('$c traffic/batch', d['hbm_bytes_per_batch'], 'batches', d['batches'])"
done
