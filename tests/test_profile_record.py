"""CPU tests of the evidence tooling: tools/make_profile_record.py turns rocprofv3 counter
passes into the traffic files bench.py reports as roofline.traffic -- it must drop the
untimed capacity-probe dispatch and add up the kernel instances one step launches."""
import csv
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FIELDS = ["Dispatch_Id", "Kernel_Name", "Counter_Name", "Counter_Value"]


def _pass(path, rows):
  os.makedirs(os.path.dirname(path), exist_ok=True)
  with open(path, "w", newline="") as fh:
    w = csv.DictWriter(fh, fieldnames=FIELDS)
    w.writeheader()
    for r in rows:
      w.writerow(dict(zip(FIELDS, r)))


def test_probe_dropped_and_step_instances_summed(tmp_path):
  probe = "void (anonymous namespace)::k_encode2<1, false, 1, false, 2>(EncodeArgs)"
  main = "void (anonymous namespace)::k_encode2<1, false, 1, false, 4>(EncodeArgs)"
  rem = "void (anonymous namespace)::k_encode<1, false, 1, false>(EncodeArgs)"
  dec = "void (anonymous namespace)::k_decode<0, 2, false, false>(DecodeArgs)"
  for ctr, scale in (("FETCH_SIZE", 1.0), ("WRITE_SIZE", 0.25)):
    rows, did = [], 0
    # the probe round: another instance, one launch, huge counts
    did += 1
    rows.append((did, probe, ctr, 9e9 * scale))
    for step in range(4):
      did += 1
      rows.append((did, main, ctr, (1000.0 + (500.0 if step == 0 else 0.0)) * scale))  # first: warm-up, dropped
      did += 1
      rows.append((did, rem, ctr, 10.0 * scale))
      did += 1
      rows.append((did, dec, ctr, 300.0 * scale))
    _pass(str(tmp_path / "prof" / "headline" / ("fetch" if ctr == "FETCH_SIZE" else "write") /
              "run_counter_collection.csv"), rows)
  out = tmp_path / "rec"
  subprocess.check_call([sys.executable, os.path.join(ROOT, "tools", "make_profile_record.py"),
                         str(tmp_path / "prof"), str(out), "headline"], stdout=subprocess.DEVNULL)
  d = json.load(open(out / "traffic_headline.json"))
  enc = d["k_encode"]
  assert sorted(enc["kernel"]) == sorted([main, rem])  # both instances of the step, not the probe
  assert enc["FETCH_SIZE_KB"] == 1010.0 and enc["WRITE_SIZE_KB"] == 252.5
  assert enc["hbm_bytes_corrected"] == (2.0 * 1010.0 + 252.5) * 1024.0  # LDS-DMA staging: FETCH x 2
  assert probe not in enc["kernel"] and probe not in enc["other_instances"]  # its one launch was the probe
  assert d["k_decode"]["fetch_multiplier"] == 1.0 and d["k_decode"]["FETCH_SIZE_KB"] == 300.0
