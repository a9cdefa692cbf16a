"""Per-batch HBM bytes of the hsg:: kernels from two rocprofv3 --pmc CSVs.

bytes = 2 x FETCH_SIZE + WRITE_SIZE (KiB -> bytes): on gfx950 FETCH_SIZE counts
half of the bytes of wide streaming reads (MI355X_MICROARCH.md, HBM section),
WRITE_SIZE is exact for 16-byte stores. A batch = one dispatch of the first
kernel of the pipeline (k_part_hist for time windows, k_ss_phist for
sessions); the warmup step is dropped by keeping the last half of them.
"""
import collections
import csv
import json
import sys


def load(path):
    per = collections.defaultdict(float)
    names = {}
    for r in csv.DictReader(open(path)):
        d = int(r["Dispatch_Id"])
        per[d] += float(r["Counter_Value"])
        names[d] = r["Kernel_Name"]
    return per, names


fetch, names = load(sys.argv[1])
write, _ = load(sys.argv[2])
disp = sorted(names)
first = next((f for f in ("k_ss_phist", "k_ss_slot") if any(f in names[d] for d in disp)), "k_part_hist")
starts = [d for d in disp if first in names[d]]
half = starts[len(starts) // 2:]  # the timed step (warmup step first)
batches = []
for i, s in enumerate(half):
    e = half[i + 1] if i + 1 < len(half) else max(disp) + 1
    ks = [d for d in disp if s <= d < e]
    kib = sum(2 * fetch.get(d, 0.0) + write.get(d, 0.0) for d in ks)
    batches.append(kib * 1024)
by_kernel = collections.defaultdict(float)
for d in disp:
    if half and d >= half[0]:
        by_kernel[names[d].split("(")[0][:60]] += (2 * fetch.get(d, 0.0) + write.get(d, 0.0)) * 1024 / max(1, len(half))
print(json.dumps({"name": sys.argv[3], "bench_args": sys.argv[4], "batches": len(half),
                  "hbm_bytes_per_batch": int(sum(batches) / max(1, len(batches))),
                  "by_kernel_bytes_per_batch": {k: int(v) for k, v in sorted(by_kernel.items(), key=lambda x: -x[1])}},
                 indent=1))
