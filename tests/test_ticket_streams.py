"""The encoders' ticket-stream mapping covers every stream with few started waves (CPU).

fedcodec.hip `ticket_stream`: wave w of workgroup b (g = b * wpg + w) counts its
start order on head h = (g + (g >> 5)) mod 32; the head's n-th started wave draws
from stream (h + n) mod 32.  A launch makes progress as long as every stream has a
started wave (DESIGN.md §2 "Ticket streams and progress").  This restates the
mapping, checks that the source still has it, and measures how many started waves
cover all 32 streams: in dispatch order, with only one XCD's workgroups running
(another kernel holding the rest), and in random start orders.
"""
import os
import random
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
K = 32  # kTicketShards = kStartHeads


def _covering(order, wpg):
  """Started waves (in `order`) until all K streams have one."""
  count, streams = {}, set()
  for i, (b, w) in enumerate(order):
    g = b * wpg + w
    h = (g + (g >> 5)) % K
    n = count.get(h, 0)
    count[h] = n + 1
    streams.add((h + n) % K)
    if len(streams) == K:
      return i + 1
  return None


def test_source_has_the_mapping():
  src = open(os.path.join(ROOT, "federated_amd", "csrc", "fedcodec.hip")).read()
  assert re.search(r"const uint32_t h = \(g \+ \(g >> 5\)\) % \(uint32_t\)kStartHeads;", src)
  assert re.search(r"return \(r \+ h\) % nshards;", src)
  assert re.search(r"constexpr int kStartHeads = 32;", src)
  assert re.search(r"constexpr int kTicketShards = 32;", src)


def test_dispatch_order_needs_32_waves():
  for wpg in (1, 8):  # k_encode (one wave per workgroup), k_encode2 (eight)
    order = [(b, w) for b in range(4096 // wpg) for w in range(wpg)]
    assert _covering(order, wpg) == K


def test_one_xcd_covers_every_stream():
  # workgroups are dealt round-robin over the 8 XCDs: XCD x runs b = x, x + 8, ... in order
  for wpg, bound in ((1, 32), (8, 104)):
    for x in range(8):
      order = [(b, w) for b in range(x, 4096 // wpg, 8) for w in range(wpg)]
      assert _covering(order, wpg) <= bound  # one XCD holds 512 encoder waves


def test_random_start_orders():
  worst = 0
  for wpg in (1, 8):
    order = [(b, w) for b in range(4096 // wpg) for w in range(wpg)]
    for seed in range(300):
      o = order[:]
      random.Random(seed).shuffle(o)
      worst = max(worst, _covering(o, wpg))
  assert worst <= 160, worst  # far below the 1024 the pigeonhole bound guarantees
