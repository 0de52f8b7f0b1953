"""CPU guard (no GPU): the decoder's untracked inline-asm loads keep their destination
registers free of clobbers, copies and calls on every path until a vmcnt(0) wait
(tools/audit_async_loads.py; the fault class that took down a GPU run in round 4)."""
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))

import audit_async_loads  # noqa: E402  pylint: disable=g-import-not-at-top


def test_no_untracked_load_register_is_touched_before_its_wait(tmp_path):
  path = str(tmp_path / "fedcodec.s")
  audit_async_loads.assemble(path)
  rep = audit_async_loads.audit(path)
  assert any("k_decode" in k for k in rep), "the decoder's batch-point loads were not found"
  # every decoder instance the launcher can select (fc_decode_accumulate*: plane, quarter,
  # virtual-segment and one / two-tile spans) is in the build and audited
  with open(path) as fh:
    instances = set(re.findall(r"^\s*\.globl\s+(_ZN12_GLOBAL__N_18k_decode\S*)", fh.read(), re.M))
  assert len(instances) >= 7, sorted(instances)
  assert instances <= set(rep), sorted(instances - set(rep))
  assert not any("k_idx_" in k for k in rep), "the index rebuild must use the tracked reader"
  bad = {k: v for k, v in rep.items() if v[1]}
  assert not bad, bad
