"""Summarise rocprofv3 csv outputs (kernel trace stats + PMC passes) per kernel."""
import csv
import glob
import os
import sys
from collections import defaultdict

out = sys.argv[1]
pat = sys.argv[2] if len(sys.argv) > 2 else ""
for f in sorted(glob.glob(os.path.join(out, "kt", "**", "*kernel_stats.csv"), recursive=True)):
  print("== kernel stats", f)
  with open(f) as fh:
    for row in csv.DictReader(fh):
      if pat in row["Name"]:
        print("  %-60s calls %6s avg %10.1f us  total %10.1f ms  %5s%%" % (
            row["Name"][:60], row["Calls"], float(row["AverageNs"]) / 1e3,
            float(row["TotalDurationNs"]) / 1e6, row.get("Percentage", "")))
agg = defaultdict(lambda: defaultdict(float))
cnt = defaultdict(int)
for f in sorted(glob.glob(os.path.join(out, "**", "*counter_collection.csv"), recursive=True)):
  with open(f) as fh:
    for row in csv.DictReader(fh):
      name = row.get("Kernel_Name", "")
      if pat and pat not in name:
        continue
      key = name[:60]
      agg[key][row["Counter_Name"]] += float(row["Counter_Value"])
      cnt[(key, row["Counter_Name"])] += 1
for k, d in agg.items():
  print("== counters", k)
  for cn, v in sorted(d.items()):
    n = cnt[(k, cn)]
    print("  %-24s total %16.0f  per-dispatch %14.0f  (%d rows)" % (cn, v, v / max(1, n), n))
