#!/bin/bash
# HBM traffic of the batch pipeline from PMC counters, one rocprofv3 pass per
# counter (FETCH_SIZE and WRITE_SIZE cannot share a pass), over every hsg::
# kernel of a short bench run; summarised per batch by tools/traffic.py.
#   tools/traffic.sh NAME [bench args...]
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
name=$1; shift
mkdir -p gpurun_out/pmc
for ctr in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 300 rocprofv3 --pmc $ctr --kernel-include-regex "hsg::" -d gpurun_out/pmc -o ${name}_$ctr \
    --output-format csv -- python3 bench.py --steps 1 --warmup 1 --cpu-seconds 0 "$@" > gpurun_out/pmc/${name}_$ctr.log 2>&1
  rc=$?; echo "== $name $ctr rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
python3 tools/traffic.py gpurun_out/pmc/${name}_FETCH_SIZE_counter_collection.csv \
  gpurun_out/pmc/${name}_WRITE_SIZE_counter_collection.csv "$name" "$*" > gpurun_out/pmc/traffic_${name}.json
cat gpurun_out/pmc/traffic_${name}.json
