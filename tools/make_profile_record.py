"""Copy a tools/profile_bench.sh run into profiles/<round>/ (kernel stats, PMC summary, traffic.json).

python tools/make_profile_record.py gpurun_out/prof_xxx profiles/r01 --clients 1024 --P 25000000 \
    --mode stochastic --step 0.5 --command "..."

traffic.json holds per-dispatch HBM bytes for k_encode / k_decode with the gfx950
correction of MI355X_MICROARCH.md's HBM section: FETCH_SIZE x2 for the encoder's
wide streaming reads, FETCH_SIZE as-is for the decoder's narrow 16-B reads, plus
WRITE_SIZE (both in KiB from rocprofv3).
"""
import argparse
import csv
import glob
import json
import os
import shutil
from collections import defaultdict


def main():
  ap = argparse.ArgumentParser()
  ap.add_argument("src")
  ap.add_argument("dst")
  ap.add_argument("--clients", type=int, default=1024)
  ap.add_argument("--P", type=int, default=25_000_000)
  ap.add_argument("--mode", default="stochastic")
  ap.add_argument("--step", type=float, default=0.5)
  ap.add_argument("--command", default="tools/profile_bench.sh <out> --steps 3 --warmup 1")
  a = ap.parse_args()
  os.makedirs(a.dst, exist_ok=True)
  ks = glob.glob(os.path.join(a.src, "kt", "**", "*kernel_stats.csv"), recursive=True)
  shutil.copy(ks[0], os.path.join(a.dst, "kernel_stats.csv"))
  summ = os.path.join(a.src, "summary.txt")
  if os.path.exists(summ):
    shutil.copy(summ, os.path.join(a.dst, "pmc_summary.txt"))
  per = defaultdict(lambda: defaultdict(list))
  for f in glob.glob(os.path.join(a.src, "**", "*counter_collection.csv"), recursive=True):
    with open(f) as fh:
      for row in csv.DictReader(fh):
        name = row["Kernel_Name"]
        key = "k_encode" if "k_encode<" in name else (
            "k_decode" if ("k_decode(" in name or "k_decode<" in name) else None)
        if key:
          per[key][row["Counter_Name"]].append(float(row["Counter_Value"]))
  out = {}
  for key, d in per.items():
    fetch = sum(d["FETCH_SIZE"]) / max(1, len(d["FETCH_SIZE"]))
    write = sum(d["WRITE_SIZE"]) / max(1, len(d["WRITE_SIZE"]))
    mult = 2.0 if key == "k_encode" else 1.0
    out[key] = {"FETCH_SIZE_KB": fetch, "WRITE_SIZE_KB": write,
                "hbm_bytes_corrected": (mult * fetch + write) * 1024.0,
                "correction": ("FETCH x2 (gfx950 wide streaming read, MI355X_MICROARCH.md HBM section) + WRITE"
                               if mult == 2.0 else "FETCH (narrow scattered 16-B reads: no x2) + WRITE")}
  out["config"] = {"clients": a.clients, "P": a.P, "mode": a.mode, "step": a.step, "command": a.command}
  with open(os.path.join(a.dst, "traffic.json"), "w") as fh:
    json.dump(out, fh, indent=1)
  print(json.dumps(out, indent=1))


if __name__ == "__main__":
  main()
