"""World-size-2 rehearsals of the client-sharded rounds on one GPU (gloo).

Two processes share cuda:0; each encodes and decodes its block of clients with
the HIP kernels.  Checked against the oracle's single-process round:
  * distributed.aggregate_round (decode in tile ranges, each range's int32 sum
    all-reduced while the next decodes): result bit for bit;
  * QuantizeEncodeFactory.next(sharded=True) (the factory surface): result bit
    for bit, measurements global (elias_gamma_encode.py:100-108,
    quantize_encode.py:184-185);
  * OneBitSGDFactory.next(sharded=True) (config 5's split, one_bit_sgd.py:87-112):
    float32 partial sums all-reduced, within rel 1e-6 * C;
  * config 4's element count (P = 11,000,000) with shrinking slabs: the int32
    sum against the oracle at sampled positions of every client, and bit for
    bit against the single-process HIP round.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from federated_amd import _lib
from federated_amd import distributed

pytestmark = pytest.mark.gpu

C, P, STEP = 6, 70_001, 0.5
F32 = np.float32


def _free_port():
  s = socket.socket()
  s.bind(("127.0.0.1", 0))
  p = s.getsockname()[1]
  s.close()
  return p


def _inputs(C=C, P=P, scale=1.5, seed=3):
  rng = np.random.default_rng(seed)
  xs = [(rng.standard_normal(P) * scale).astype(np.float32) for _ in range(C)]
  seeds = np.array([[10 + c, 20 + c] for c in range(C)], np.int64)
  return xs, seeds


def _init(rank, world, port):
  os.environ["MASTER_ADDR"] = "127.0.0.1"
  os.environ["MASTER_PORT"] = str(port)
  dist.init_process_group("gloo", rank=rank, world_size=world)
  torch.cuda.set_device(0)


def _worker(rank, world, port, path):
  _init(rank, world, port)
  xs, seeds = _inputs()
  lo, hi = distributed.client_shard(C, world, rank)
  rows = [torch.from_numpy(x).cuda() for x in xs[lo:hi]]
  rnd = distributed.aggregate_round(rows, STEP, torch.from_numpy(seeds[lo:hi]), _lib.STOCHASTIC, slabs=5)
  if rank == 0:
    np.save(path, rnd.result.cpu().numpy())
  dist.destroy_process_group()


def test_two_rank_round_matches_oracle(gpu, tmp_path):
  from oracle import quantize_utils as oq  # pylint: disable=g-import-not-at-top
  path = str(tmp_path / "round.npy")
  mp.spawn(_worker, args=(2, _free_port(), path), nprocs=2, join=True)
  xs, seeds = _inputs()
  acc = np.zeros(P, np.int64)
  for c in range(C):
    acc += oq.stochastic_quantize(xs[c], STEP, tuple(seeds[c]))
  want = acc.astype(np.int32).astype(np.float32) * np.float32(STEP)  # quantize_encode.py:189-190
  got = np.load(path)
  np.testing.assert_array_equal(got.view(np.uint32), want.view(np.uint32))


def _factory_worker(rank, world, port, Cn, rounding, path):
  _init(rank, world, port)
  from federated_amd.aggregators import quantize_encode  # pylint: disable=g-import-not-at-top
  xs, seeds = _inputs(C=Cn, seed=9)
  lo, hi = distributed.client_shard(Cn, world, rank)
  process = quantize_encode.QuantizeEncodeFactory(STEP, rounding_type=rounding).create((np.float32, (P,)))
  state = process.initialize()
  out = process.next(state, [torch.from_numpy(x).cuda() for x in xs[lo:hi]], seeds=seeds[lo:hi], sharded=True)
  m = out.measurements
  np.save(path % rank, np.concatenate([out.result.cpu().numpy().astype(np.float64),
                                       [m["avg_bitrate"], m["avg_distortion"], m["avg_sparsity"],
                                        out.state["round_num"]]]))
  dist.destroy_process_group()


@pytest.mark.parametrize("Cn,world,rounding", [(5, 2, "stochastic"), (2, 3, "uniform"), (4, 2, "dithered")],
                         ids=["5clients_2ranks", "2clients_3ranks_one_empty", "dithered_2ranks"])
def test_factory_sharded_round_matches_oracle(gpu, tmp_path, Cn, world, rounding):
  """QuantizeEncodeFactory.next(sharded=True): every rank returns the round's global
  result and measurements (a rank may hold no clients)."""
  from oracle import aggregators as oagg  # pylint: disable=g-import-not-at-top
  path = str(tmp_path / "r%d.npy")
  mp.spawn(_factory_worker, args=(world, _free_port(), Cn, rounding, path), nprocs=world, join=True)
  xs, seeds = _inputs(C=Cn, seed=9)
  want, meas, _ = oagg.quantize_encode_next(xs, STEP, rounding, seeds=seeds)
  for r in range(world):
    got = np.load(path % r)
    res = got[:P].astype(np.float32)
    if rounding == "dithered":  # float32 noise sums all-reduced: association differs
      np.testing.assert_allclose(res, want, rtol=1e-6, atol=1e-6 * Cn * STEP)
    else:
      np.testing.assert_array_equal(res.view(np.uint32), want.view(np.uint32))
    assert got[P] == meas["avg_bitrate"]  # integer bit counts: exact
    np.testing.assert_allclose(got[P + 1], meas["avg_distortion"], rtol=1e-5)
    np.testing.assert_allclose(got[P + 2], meas["avg_sparsity"], rtol=1e-6)
    assert got[P + 3] == 1.0


def _onebit_worker(rank, world, port, Cn, Pn, path):
  _init(rank, world, port)
  from federated_amd.aggregators.comparison_methods import one_bit_sgd  # pylint: disable=g-import-not-at-top
  rng = np.random.default_rng(21)
  xs = [(rng.standard_normal(Pn) * 2 + 0.25).astype(np.float32) for _ in range(Cn)]
  lo, hi = distributed.client_shard(Cn, world, rank)
  process = one_bit_sgd.OneBitSGDFactory().create((np.float32, (Pn,)))
  out = process.next((), [torch.from_numpy(x).cuda() for x in xs[lo:hi]], sharded=True, slabs=3)
  m = out.measurements
  np.save(path % rank, np.concatenate([out.result.cpu().numpy().astype(np.float64),
                                       [m["avg_bitrate"], m["avg_distortion"]]]))
  dist.destroy_process_group()


def test_onebit_sharded_round_matches_oracle(gpu, tmp_path):
  """Config 5's split: each rank's client-order float32 sum, float32 all-reduce in
  element slabs; against the single-process oracle within rel 1e-6 * C."""
  from oracle import aggregators as oagg  # pylint: disable=g-import-not-at-top
  Cn, Pn, world = 5, 100_003, 2
  path = str(tmp_path / "ob%d.npy")
  mp.spawn(_onebit_worker, args=(world, _free_port(), Cn, Pn, path), nprocs=world, join=True)
  rng = np.random.default_rng(21)
  xs = [(rng.standard_normal(Pn) * 2 + 0.25).astype(np.float32) for _ in range(Cn)]
  want, meas = oagg.one_bit_sgd_next(xs, 0.0)
  for r in range(world):
    got = np.load(path % r)
    np.testing.assert_allclose(got[:Pn], want, rtol=1e-6 * Cn, atol=1e-6 * Cn * float(np.max(np.abs(want))))
    assert np.float32(got[Pn]) == meas["avg_bitrate"]
    np.testing.assert_allclose(got[Pn + 1], meas["avg_distortion"], rtol=1e-5)


P11 = 11_000_000
C11 = 6


def _rows11(dev, lo, hi):
  g = torch.Generator(device=dev)
  rows = []
  for c in range(lo, hi):
    g.manual_seed(1100 + c)
    rows.append(torch.randn(P11, generator=g, device=dev, dtype=torch.float32))
  return rows


def _worker11(rank, world, port, path):
  _init(rank, world, port)
  lo, hi = distributed.client_shard(C11, world, rank)
  seeds = np.array([[7 + c, 5 * c] for c in range(C11)], np.int64)
  rnd = distributed.aggregate_round(_rows11(torch.device("cuda", 0), lo, hi), STEP, torch.from_numpy(seeds[lo:hi]),
                                    _lib.STOCHASTIC, slabs=4)
  if rank == 0:
    np.save(path, rnd.result.cpu().numpy())
  dist.destroy_process_group()


def test_two_rank_round_at_config4_size(gpu, tmp_path):
  """Config 4's tensor size (ResNet-18, P = 11 M: 10,743 tiles, shrinking slabs of
  4:3:2:1) over two ranks: the dequantised sum equals the single-process HIP round
  bit for bit and the oracle at 50,000 sampled positions of every client."""
  from oracle import quantize_utils as oq  # pylint: disable=g-import-not-at-top
  path = str(tmp_path / "r11.npy")
  mp.spawn(_worker11, args=(2, _free_port(), path), nprocs=2, join=True)
  got = np.load(path)
  seeds = np.array([[7 + c, 5 * c] for c in range(C11)], np.int64)
  rows = _rows11(gpu, 0, C11)
  single = distributed.aggregate_round(rows, STEP, torch.from_numpy(seeds), _lib.STOCHASTIC, multi=False)
  np.testing.assert_array_equal(got.view(np.uint32), single.result.cpu().numpy().view(np.uint32))
  idx = np.sort(np.random.default_rng(4).choice(P11, 50_000, replace=False))
  it = torch.from_numpy(idx).to(gpu)
  acc = np.zeros(idx.size, np.int64)
  for c in range(C11):
    acc += oq.stochastic_quantize_at(rows[c][it].cpu().numpy(), idx, F32(STEP), tuple(seeds[c]))
  np.testing.assert_array_equal(got[idx], oq.uniform_dequantize(acc.astype(np.int32), F32(STEP)))
  del rows, single
  torch.cuda.empty_cache()
