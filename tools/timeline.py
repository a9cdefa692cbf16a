"""Per-batch kernel timeline from a rocprofv3 kernel_trace CSV: the last
`n` dispatches with the idle gap before each (microseconds)."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 30
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
last = rows[-n:]
t0 = int(last[0]["Start_Timestamp"])
prev = None
for r in last:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    gap = (s - prev) / 1e3 if prev else 0.0
    print(f"{(s - t0) / 1e3:9.1f} gap {gap:7.1f} dur {(e - s) / 1e3:7.1f} {r['Kernel_Name'][:72]}")
    prev = e
