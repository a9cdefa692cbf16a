"""Cross-check the bench line's pipeline time against rocprofv3 --stats.

Sums the device time of the batch-pipeline kernels (every hsg:: kernel except
the state reset and the drain copy) per batch (= per k_part_hist dispatch) from
a *_kernel_stats.csv, and prints it next to roofline.avg_launch_ms of the bench
JSON line printed by the same profiled run. The HIP-event window also contains
launch gaps, so it reads a little higher.
"""
import csv
import json
import sys

stats = list(csv.DictReader(open(sys.argv[1])))
line = None
for ln in open(sys.argv[2]):
    if ln.startswith("{"):
        line = json.loads(ln)
skip = ("k_tw_reset", "k_copy_rows", "k_clear_scalars")
batches = sum(int(r["Calls"]) for r in stats if "k_part_hist" in r["Name"])
tot = sum(float(r["TotalDurationNs"]) for r in stats
          if r["Name"].startswith(("hsg::", "void hsg::")) and not any(k in r["Name"] for k in skip))
per = tot / max(1, batches) / 1e6
print(f"rocprof pipeline kernels: {per:.4f} ms per batch over {batches} batches")
if line:
    rf = line["roofline"]
    print(f"bench HIP events:         {rf['avg_launch_ms']:.4f} ms per batch; alg bytes {rf['alg_bytes_per_launch']}"
          f" -> {rf['alg_bytes_per_launch'] / per / 1e6:.1f} GB/s by rocprof time, {rf['achieved']} GB/s by events")
