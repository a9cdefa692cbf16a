#!/bin/bash
# Kernel statistics + PMC traffic of the EMIT CHANGES pipelines (C3 hopping,
# C4 sessions) at their bench sizes:
#   bash tools/gpu_evidence.sh ROUND [c3_pr] [c4_pr]
# -> gpurun_out/prof/<round>_<name>_kernel_stats.csv, gpurun_out/pmc/traffic_<name>.json
cd "${GRAFT_REPO_ROOT:-/root/repo}"
round=$1; shift
for nm in ${*:-c3_pr c4_pr}; do
  case $nm in
    c3_pr) a="--config C3 --emit per_record --records 100663296";;
    c4_pr) a="--config C4 --emit per_record --records 167772160";;
    *) echo "unknown $nm"; exit 2;;
  esac
  bash tools/prof.sh ${round}_$nm $a --input hbm --no-hbm --no-per-record || exit $?
  bash tools/traffic.sh $nm $a --input hbm --no-hbm --no-per-record > /dev/null || exit $?
  python3 -c "import json; d=json.load(open('gpurun_out/pmc/traffic_$nm.json')); print('$nm traffic/batch', d['hbm_bytes_per_batch'], 'batches', d['batches'])"
done
