"""World-size-2 gloo test of the client-sharded round (CPU, no GPU).

Each rank encodes/decodes its contiguous block of clients (here with the CPU
oracle codec standing in for the per-rank HIP result) and the int32 partial
sums are combined with the same all-reduce federated_amd.distributed uses;
the result must equal the single-process sum bit for bit.
"""
import os
import socket

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from federated_amd import distributed


def _free_port():
  s = socket.socket()
  s.bind(("127.0.0.1", 0))
  p = s.getsockname()[1]
  s.close()
  return p


def _worker(rank, world, port, C, P, out):
  os.environ["MASTER_ADDR"] = "127.0.0.1"
  os.environ["MASTER_PORT"] = str(port)
  dist.init_process_group("gloo", rank=rank, world_size=world)
  from oracle import codec as ocodec  # pylint: disable=g-import-not-at-top
  from oracle import quantize_utils as oq  # pylint: disable=g-import-not-at-top
  rng = np.random.default_rng(42)
  xs = [(rng.standard_normal(P) * 2).astype(np.float32) for _ in range(C)]
  lo, hi = distributed.client_shard(C, world, rank)
  acc = np.zeros(P, np.int32)
  for c in range(lo, hi):
    code, _ = ocodec.run_length_gamma_encode(oq.stochastic_quantize(xs[c], 0.5, (c, c)))
    ocodec.decode_accumulate(code, acc)
  t = torch.from_numpy(acc)
  distributed.allreduce_sum_(t)
  out[rank] = t.numpy().copy()
  dist.destroy_process_group()


def test_client_shard_partitions():
  for C in [1, 7, 128, 1023]:
    for world in [1, 2, 3, 8]:
      spans = [distributed.client_shard(C, world, r) for r in range(world)]
      assert spans[0][0] == 0 and spans[-1][1] == C
      assert all(spans[i][1] == spans[i + 1][0] for i in range(world - 1))
      sizes = [h - l for l, h in spans]
      assert max(sizes) - min(sizes) <= 1


def test_two_rank_int32_allreduce_matches_single_process():
  from oracle import quantize_utils as oq  # pylint: disable=g-import-not-at-top
  C, P, world = 5, 3001, 2
  mgr = mp.Manager()
  out = mgr.dict()
  mp.spawn(_worker, args=(world, _free_port(), C, P, out), nprocs=world, join=True)
  rng = np.random.default_rng(42)
  xs = [(rng.standard_normal(P) * 2).astype(np.float32) for _ in range(C)]
  want = np.zeros(P, np.int64)
  for c in range(C):
    want += oq.stochastic_quantize(xs[c], 0.5, (c, c))
  for r in range(world):
    np.testing.assert_array_equal(out[r], want.astype(np.int32))


def test_slab_bounds_shrink_and_cover():
  for T in [1, 2, 3, 5, 10, 98, 977, 24415]:
    for n in [1, 2, 4, 8]:
      b = distributed.slab_bounds(T, n)
      assert b[0] == 0 and b[-1] == T
      assert all(b[i] < b[i + 1] for i in range(len(b) - 1))
      assert len(b) - 1 == min(n, T) or T < n * (n + 1) // 2
      sizes = [b[i + 1] - b[i] for i in range(len(b) - 1)]
      if n > 1 and T >= 10 * n * n:  # shares n : n-1 : ... : 1, the last the smallest
        assert sizes == sorted(sizes, reverse=True) and sizes[-1] < sizes[0]


def _slab_worker(rank, world, port, C, P, slabs, out):
  """aggregate_round's slab-wise asynchronous all-reduce of tile ranges."""
  os.environ["MASTER_ADDR"] = "127.0.0.1"
  os.environ["MASTER_PORT"] = str(port)
  dist.init_process_group("gloo", rank=rank, world_size=world)
  from oracle import quantize_utils as oq  # pylint: disable=g-import-not-at-top
  rng = np.random.default_rng(7)
  xs = [(rng.standard_normal(P) * 3).astype(np.float32) for _ in range(C)]
  lo, hi = distributed.client_shard(C, world, rank)
  acc = np.zeros(P, np.int64)
  for c in range(lo, hi):
    acc += oq.stochastic_quantize(xs[c], 0.5, (c, 3 * c))
  isum = torch.from_numpy(((acc + 2**31) % 2**32 - 2**31).astype(np.int32))
  bounds = distributed.slab_bounds((P + 1023) // 1024, slabs)
  works = []
  for k in range(len(bounds) - 1):
    a, b = distributed.slab_elements(bounds, k, P)
    works.append(dist.all_reduce(isum[a:b], op=dist.ReduceOp.SUM, async_op=True))
  for w in works:
    w.wait()
  out[rank] = isum.numpy().copy()
  dist.destroy_process_group()


def test_two_rank_slab_allreduce_matches_single_process():
  """P not a multiple of the 1024-element tile (partial last tile), shrinking slabs:
  the slab-wise all-reduce of int32 partial sums equals the single-process sum."""
  from oracle import quantize_utils as oq  # pylint: disable=g-import-not-at-top
  C, P, world, slabs = 6, 10_000, 2, 4
  mgr = mp.Manager()
  out = mgr.dict()
  mp.spawn(_slab_worker, args=(world, _free_port(), C, P, slabs, out), nprocs=world, join=True)
  rng = np.random.default_rng(7)
  xs = [(rng.standard_normal(P) * 3).astype(np.float32) for _ in range(C)]
  want = np.zeros(P, np.int64)
  for c in range(C):
    want += oq.stochastic_quantize(xs[c], 0.5, (c, 3 * c))
  want = ((want + 2**31) % 2**32 - 2**31).astype(np.int32)
  for r in range(world):
    np.testing.assert_array_equal(out[r], want)
