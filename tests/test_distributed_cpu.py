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


def _means_worker(rank, world, port, out):
  os.environ["MASTER_ADDR"] = "127.0.0.1"
  os.environ["MASTER_PORT"] = str(port)
  dist.init_process_group("gloo", rank=rank, world_size=world)
  # rank r holds r + 1 clients with values r + 1 (sums [n, 2n]); rank 2 none
  n = rank + 1 if rank < 2 else 0
  means, total = distributed.global_means([float(n * (rank + 1)), 2.0 * n * (rank + 1)], n,
                                          torch.device("cpu"))
  out[rank] = (means.tolist(), total)
  dist.destroy_process_group()


def test_global_means_three_ranks_one_empty():
  """elias_gamma_encode.py:100-108 / quantize_encode.py:184-185: federated_mean over
  every client of every rank, ranks may hold no clients."""
  mgr = mp.Manager()
  out = mgr.dict()
  mp.spawn(_means_worker, args=(3, _free_port(), out), nprocs=3, join=True)
  # clients: [1] from rank 0, [2, 2] from rank 1 -> mean 5/3, second sum twice that
  for r in range(3):
    means, total = out[r]
    assert total == 3
    np.testing.assert_allclose(means, [5.0 / 3.0, 10.0 / 3.0], rtol=1e-15)


def _onebit_worker(rank, world, port, C, P, out):
  """The one-bit round's reduction (distributed.onebit_round): each rank's
  client-order float32 sum of its decoded clients (oracle decode standing in for
  fc_onebit_decode_sum), then a float32 SUM all-reduce and the global distortion
  mean via global_means."""
  os.environ["MASTER_ADDR"] = "127.0.0.1"
  os.environ["MASTER_PORT"] = str(port)
  dist.init_process_group("gloo", rank=rank, world_size=world)
  from oracle import aggregators as oagg  # pylint: disable=g-import-not-at-top
  rng = np.random.default_rng(11)
  xs = [(rng.standard_normal(P) * 2 + 0.3).astype(np.float32) for _ in range(C)]
  lo, hi = distributed.client_shard(C, world, rank)
  part, meas = oagg.one_bit_sgd_next(xs[lo:hi], 0.0)
  t = torch.from_numpy(part.copy())
  distributed.allreduce_sum_(t)
  (m,), total = distributed.global_means([float(meas["avg_distortion"]) * (hi - lo)], hi - lo,
                                         torch.device("cpu"))
  out[rank] = (t.numpy().copy(), m, total)
  dist.destroy_process_group()


def test_two_rank_onebit_reduction_matches_single_process():
  """Config 5's 8-GPU split, reduction side (one_bit_sgd.py:87-112): float32 partial
  sums all-reduced equal the single-process client-order sum within the
  float-association tolerance rel 1e-6 * C."""
  from oracle import aggregators as oagg  # pylint: disable=g-import-not-at-top
  C, P, world = 7, 5003, 2
  mgr = mp.Manager()
  out = mgr.dict()
  mp.spawn(_onebit_worker, args=(world, _free_port(), C, P, out), nprocs=world, join=True)
  rng = np.random.default_rng(11)
  xs = [(rng.standard_normal(P) * 2 + 0.3).astype(np.float32) for _ in range(C)]
  want, meas = oagg.one_bit_sgd_next(xs, 0.0)
  for r in range(world):
    got, m, total = out[r]
    assert total == C
    np.testing.assert_allclose(got, want, rtol=1e-6 * C, atol=1e-6 * C * float(np.max(np.abs(want))))
    np.testing.assert_allclose(m, meas["avg_distortion"], rtol=1e-6)


def _preamble_worker(rank, world, port, counts, bad_rank, out):
  os.environ["MASTER_ADDR"] = "127.0.0.1"
  os.environ["MASTER_PORT"] = str(port)
  dist.init_process_group("gloo", rank=rank, world_size=world)
  out[rank] = distributed.round_preamble(counts[rank], rank == bad_rank, device=torch.device("cpu"))
  dist.destroy_process_group()


def test_round_preamble_global_offsets_one_clock_and_shared_errors():
  """round_preamble (the sharded factories' first collective): each rank's first
  global client index, one clock base for every rank (so clock seeds base + global
  index never repeat across ranks), and a rank-local error seen by every rank."""
  from federated_amd.aggregators import quantize_encode  # pylint: disable=g-import-not-at-top
  counts = [3, 0, 4]
  for bad_rank in (-1, 1):
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_preamble_worker, args=(3, _free_port(), counts, bad_rank, out), nprocs=3, join=True)
    res = [out[r] for r in range(3)]
    assert [r[0] for r in res] == [0, 3, 3]
    assert all(r[1] == 7 for r in res)
    assert all(r[2] == (bad_rank >= 0) for r in res)
    assert len({r[3] for r in res}) == 1 and res[0][3] > 0
    seeds = np.concatenate([quantize_encode.clock_seeds(counts[r], base=res[r][3] + res[r][0]) for r in range(3)])
    assert len(np.unique(seeds[:, 0])) == sum(counts)
