#!/bin/bash
# PMC passes on C4 and C3: HBM traffic per kernel (FETCH_SIZE / WRITE_SIZE) and wave stall counters.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/pmc; export TMPDIR=/tmp
bash tools/traffic.sh c4 --config C4 --no-host-input --no-per-record > /dev/null || exit $?
bash tools/traffic.sh c3 --config C3 --no-host-input --no-per-record > /dev/null || exit $?
for cfg in C4 C3; do
  lc=$(echo $cfg | tr A-Z a-z)
  timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS \
    --kernel-include-regex "hsg::" -d gpurun_out/pmc -o sq_$lc --output-format csv -- python3 bench.py --config $cfg --steps 1 --warmup 1 --cpu-seconds 0 --no-host-input --no-per-record > gpurun_out/pmc/sq_$lc.log 2>&1
  echo "== sq $cfg rc=$?"
done
python3 - <<'PY'
import csv, collections, json
for lc in ("c4", "c3"):
    print(lc, json.load(open(f"gpurun_out/pmc/traffic_{lc}.json"))["by_kernel_bytes_per_batch"])
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    try:
        rows = list(csv.DictReader(open(f"gpurun_out/pmc/sq_{lc}_counter_collection.csv")))
    except FileNotFoundError:
        continue
    for r in rows:
        agg[r["Kernel_Name"][:40]][r["Counter_Name"]] += float(r["Counter_Value"])
    for k, v in agg.items():
        if v.get("SQ_WAVES", 0) > 0:
            print(lc, k, {c: int(x) for c, x in sorted(v.items())})
PY
