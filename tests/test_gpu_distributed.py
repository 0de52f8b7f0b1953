"""World-size-2 rehearsal of distributed.aggregate_round on one GPU (gloo).

Two processes share cuda:0; each encodes and decodes its block of clients with
the HIP kernels, decoding in tile ranges whose int32 sums are all-reduced
asynchronously while the next range decodes.  The round's result must equal the
oracle's single-process dequantised sum bit for bit.
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


def _free_port():
  s = socket.socket()
  s.bind(("127.0.0.1", 0))
  p = s.getsockname()[1]
  s.close()
  return p


def _inputs():
  rng = np.random.default_rng(3)
  xs = [(rng.standard_normal(P) * 1.5).astype(np.float32) for _ in range(C)]
  seeds = np.array([[10 + c, 20 + c] for c in range(C)], np.int64)
  return xs, seeds


def _worker(rank, world, port, path):
  os.environ["MASTER_ADDR"] = "127.0.0.1"
  os.environ["MASTER_PORT"] = str(port)
  dist.init_process_group("gloo", rank=rank, world_size=world)
  torch.cuda.set_device(0)
  xs, seeds = _inputs()
  lo, hi = distributed.client_shard(C, world, rank)
  rows = [torch.from_numpy(x).cuda() for x in xs[lo:hi]]
  out, _ = distributed.aggregate_round(rows, STEP, torch.from_numpy(seeds[lo:hi]), _lib.STOCHASTIC,
                                       slabs=5)
  if rank == 0:
    np.save(path, out.cpu().numpy())
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
