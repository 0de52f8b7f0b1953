"""Client-sharded multi-GPU aggregation (one process per GPU, RCCL over xGMI).

A round's clients are independent until the server sum
(``federated_aggregate`` accumulate/merge, elias_gamma_encode.py:63-88), and
the sum is an associative int32 sum.  So each rank encodes and decodes its
contiguous block of clients and the ranks' int32 partial sums are combined
with ONE all-reduce (backend "nccl" = RCCL on ROCm; "gloo" in CPU tests).
Integer addition is exact and order-independent, so the result is bit-identical
to the single-GPU sum for any world size or ring order.  The dequantise then
runs once, on every rank (each rank holds the server result).

The round's measurements are global, as the reference's ``federated_mean``s
define them (quantize_encode.py:184-185, elias_gamma_encode.py:100-108): every
rank contributes its clients' sums to one small float64 all-reduce.

Config 5's one-bit codec (one_bit_sgd.py:87-112) sums decoded float32 values:
each rank adds its clients in client order, then the float32 partial sums are
all-reduced -- a different float association than one process's client-order
sum, so that result is compared with a tolerance.
"""
import collections

import numpy as np
import torch
import torch.distributed as dist

from federated_amd import _lib
from federated_amd import codec

F32 = np.float32


def client_shard(nclients, world, rank):
  """Contiguous block [lo, hi) of clients for `rank` (sizes differ by <= 1)."""
  base, extra = divmod(int(nclients), int(world))
  lo = rank * base + min(rank, extra)
  return lo, lo + base + (1 if rank < extra else 0)


def is_multi(group=None):
  return dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1


def allreduce_sum_(t, group=None):
  """In-place SUM all-reduce of an integer (or float) tensor; no-op at world 1."""
  if is_multi(group):
    dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
  return t


def slab_bounds(T, n):
  """Tile boundaries of `n` decode slabs over T tiles, shrinking towards the end.

  Slab k gets a share proportional to n - k (e.g. 4:3:2:1 of the tiles for n = 4):
  every slab's all-reduce overlaps the decode of the next one, so only the last
  slab's all-reduce (and the dequantise) is exposed, and the last slab is the
  smallest.  Returns n + 1 increasing boundaries from 0 to T (empty slabs are
  dropped when T < n).
  """
  T, n = int(T), max(1, int(n))
  w = [n - k for k in range(n)]
  tot = sum(w)
  b = [0]
  acc = 0
  for k in range(n):
    acc += w[k]
    b.append((T * acc) // tot)
  out = [b[0]]
  for x in b[1:]:
    if x > out[-1]:
      out.append(x)
  if out[-1] != T:
    out.append(T)
  return out


def slab_elements(bounds, k, P, tile=1024):
  """Element range [lo, hi) of slab k (the last tile may be partial)."""
  return bounds[k] * tile, min(int(P), bounds[k + 1] * tile)


def global_means(local_sums, nclients_local, device, group=None):
  """Global per-client means of float64 local sums: ONE all-reduce of
  [sums..., client count] (a no-op at world 1).  Returns (means, total clients)."""
  v = torch.tensor(list(local_sums) + [float(nclients_local)], dtype=torch.float64, device=device)
  allreduce_sum_(v, group)
  v = v.cpu().numpy()
  n = v[-1]
  return (v[:-1] / n if n else np.zeros(len(v) - 1)), int(n)


def round_preamble(nclients_local, bad=False, group=None, device=None):
  """What every rank of a sharded round must agree on before its collectives: ONE
  small all-reduce of [client count per rank..., any rank's local error, rank 0's
  clock].  Returns (lo, total, any_bad, base): this rank's first global client
  index, the round's client count, whether any rank flagged an error (every rank
  then raises instead of blocking in a later collective) and one clock base for
  the whole round (rank 0's ``tf.timestamp()*1e6``, quantize_encode.py:141-144)."""
  import time  # pylint: disable=g-import-not-at-top
  world = dist.get_world_size(group)
  rank = dist.get_rank(group)
  if device is None:
    device = torch.device("cuda", torch.cuda.current_device())
  v = torch.zeros(world + 2, dtype=torch.int64, device=device)
  v[rank] = int(nclients_local)
  v[world] = 1 if bad else 0
  if rank == 0:
    v[world + 1] = int(time.time() * 1e6)
  dist.all_reduce(v, op=dist.ReduceOp.SUM, group=group)
  v = v.cpu().numpy()
  return int(v[:rank].sum()), int(v[:world].sum()), bool(v[world]), int(v[world + 1])


RoundOutput = collections.namedtuple("RoundOutput", ["result", "batch", "measurements"])


def client_measurements(batch, P):
  """Per-client float32 distortion and sparsity, float64 bitstring bits
  (quantize_encode.py:150-155, elias_gamma_encode.py:100-101) of a local batch."""
  dist_, nnz = codec.finalize(batch)
  size = F32(P)
  distortion = (dist_.cpu().numpy().astype(np.float32) / size).astype(np.float32)
  sparsity = ((size - nnz.cpu().numpy().astype(np.float32)) / size).astype(np.float32)
  bits = 8.0 * batch.nbytes().astype(np.float64)
  return distortion, sparsity, bits


def aggregate_round(local_rows, step, local_seeds, mode, group=None, prescale=None, slabs=4, norms=None,
                    caps=None, P=None, dequant_step=None, multi=None):
  """One QuantizeEncode round over this rank's clients; the server result and the
  round's measurements are global.

  Encode (fused quantise + run-length gamma) this rank's clients, decode them in
  `slabs` tile ranges (fc_decode_accumulate_tiles, shrinking ranges: slab_bounds)
  and all-reduce each range's int32 sum asynchronously (the collective's stream
  waits for that range's decode) while the next range decodes.  Integer sums
  make the result independent of the range split, the client split and the ring
  order.  A rank may hold no clients (it contributes zeros).  Dithered mode also
  all-reduces the float32 noise sum (tolerance, as TFF's federated_sum).

  ``dequant_step``: the server's step (quantize_encode.py:189-190 dequantises
  with the un-normalised state step); defaults to ``step``.  ``multi``: reduce
  over the group (default: whenever torch.distributed runs with > 1 rank).
  Returns RoundOutput(result float32 [P] on every rank, local EncodedBatch or None,
  OrderedDict(avg_bitrate f64, avg_distortion f32, avg_sparsity f32)).
  """
  rows = list(local_rows)
  if P is None:
    P = rows[0].numel()
  device = rows[0].device if rows else torch.device("cuda", torch.cuda.current_device())
  dq = float(step if dequant_step is None else dequant_step)
  if multi is None:
    multi = is_multi(group)
  batch = None
  out = None
  if not multi and rows and codec.pipeline_wanted(len(rows), P):
    # one process: the round in two client halves, the first half's decode beside the
    # second half's encode; an overflowed capacity falls back to the checked path below
    rnd = codec.PipelinedRound(P, list(caps) if caps is not None else [codec.default_capacity(P)] * len(rows),
                               device)
    ptrs = torch.tensor([r.data_ptr() for r in rows], dtype=torch.int64, device=device)
    noise = codec.noise_sum(local_seeds, P, device) if mode == _lib.DITHERED else None
    out = torch.empty(P, dtype=torch.float32, device=device)
    perr = codec.encode_decode_pipelined(
        ptrs, P, step, local_seeds, mode, rnd, out=out, dq_step=dq, noise_sum=noise,
        norms=norms, prescale=None if prescale is None else torch.as_tensor(prescale).reshape(-1, 2).to(device))
    if not len(rnd.overflowed()):
      if int(perr.item()):
        raise RuntimeError("malformed run-length gamma code")
      parts = [client_measurements(b, P) for b in rnd.batches]
      distortion, sparsity, bits = (np.concatenate([p_[i] for p_ in parts]) for i in range(3))
      meas = collections.OrderedDict(
          avg_bitrate=np.float64(np.mean(bits) / np.float64(P)) if P else np.float64(0.0),
          avg_distortion=F32(np.mean(distortion, dtype=np.float32)),
          avg_sparsity=F32(np.mean(sparsity, dtype=np.float32)))
      return RoundOutput(out, rnd, meas)
    out = None
  if rows:
    batch = codec.quantize_encode_checked(rows, step, local_seeds, mode, norms=norms, caps=caps,
                                          prescale=prescale)
  err = torch.zeros(1, dtype=torch.int32, device=device)
  if not multi:
    out = (torch.empty if batch is not None else torch.zeros)(P, dtype=torch.float32, device=device)
    if batch is not None:
      noise = codec.noise_sum(local_seeds, P, device) if mode == _lib.DITHERED else None
      codec.decode_accumulate(batch, want_sum=False, out=out, step=dq, noise_sum=noise, err=err)
  else:
    isum = torch.zeros(P, dtype=torch.int32, device=device)
    works = []
    bounds = slab_bounds(codec.num_tiles(P), slabs)
    for k in range(len(bounds) - 1):
      if batch is not None:
        codec.decode_accumulate(batch, sum_out=isum, err=err, tiles=(bounds[k], bounds[k + 1]))
      lo, hi = slab_elements(bounds, k, P)
      works.append(dist.all_reduce(isum[lo:hi], op=dist.ReduceOp.SUM, group=group, async_op=True))
    noise = None
    if mode == _lib.DITHERED:
      noise = (codec.noise_sum(local_seeds, P, device) if rows
               else torch.zeros(P, dtype=torch.float32, device=device))
      works.append(dist.all_reduce(noise, op=dist.ReduceOp.SUM, group=group, async_op=True))
    for w in works:
      w.wait()
    out = codec.dequantize(isum, dq, noise)
  # multi-rank: a malformed code is flagged through the measurement all-reduce
  # below, so every rank raises (a rank raising alone would leave the others
  # blocked in the next collective)
  bad = bool(int(err.item()))
  if bad and not multi:
    raise RuntimeError("malformed run-length gamma code")
  if batch is not None:
    distortion, sparsity, bits = client_measurements(batch, P)
  else:
    distortion = sparsity = np.zeros(0, np.float32)
    bits = np.zeros(0, np.float64)
  if not multi:  # single process: float32 means, as the factory always computed them
    meas = collections.OrderedDict(
        avg_bitrate=np.float64(np.mean(bits) / np.float64(P)) if P else np.float64(0.0),
        avg_distortion=F32(np.mean(distortion, dtype=np.float32)),
        avg_sparsity=F32(np.mean(sparsity, dtype=np.float32)))
  else:
    (mbits, mdist, mspars, nbad), _ = global_means(
        [bits.sum(), distortion.astype(np.float64).sum(), sparsity.astype(np.float64).sum(), float(bad)],
        len(rows), device, group)
    if nbad > 0:  # (only a rank holding clients decodes, so the count is > 0 then)
      raise RuntimeError("malformed run-length gamma code (on at least one rank)")
    meas = collections.OrderedDict(
        avg_bitrate=np.float64(mbits / np.float64(P)) if P else np.float64(0.0),
        avg_distortion=F32(mdist), avg_sparsity=F32(mspars))
  return RoundOutput(out, batch, meas)


def onebit_round(local_rows, threshold=0.0, group=None, P=None, slabs=1, multi=None):
  """Config 5's one-bit SGD round (one_bit_sgd.py:45-112) over this rank's clients.

  Each rank encodes its clients (fc_onebit_encode: masks + two means), decodes
  and sums them in client order in float32 (fc_onebit_decode_sum), and the
  ranks' float32 partial sums are all-reduced (RCCL) -- in `slabs` element
  ranges, each all-reduced while the next one is summed.  Measurements: the
  fixed bitrate (P + 64) / P and the global mean of the clients' distortions.
  Returns RoundOutput(result float32 [P] on every rank, None, measurements).
  """
  rows = list(local_rows)
  if P is None:
    P = rows[0].numel()
  device = rows[0].device if rows else torch.device("cuda", torch.cuda.current_device())
  if multi is None:
    multi = is_multi(group)
  out = torch.zeros(P, dtype=torch.float32, device=device)
  dists = np.zeros(0, np.float32)
  size = F32(P)
  if rows:
    masks, means, dist_ = codec.onebit_encode(rows, threshold)
    dists = (dist_.cpu().numpy().astype(np.float32) / size).astype(np.float32)
  works = []
  nw = (P + 31) // 32
  bounds = slab_bounds(nw, slabs if multi else 1)
  for k in range(len(bounds) - 1):
    lo, hi = bounds[k] * 32, min(P, bounds[k + 1] * 32)
    if rows:
      codec.onebit_decode_sum(masks, means, len(rows), P, out=out, words=(bounds[k], bounds[k + 1]))
    if multi:
      works.append(dist.all_reduce(out[lo:hi], op=dist.ReduceOp.SUM, group=group, async_op=True))
  for w in works:
    w.wait()
  bitrate = F32((size + F32(64.0)) / size)
  if not multi:
    avg_d = F32(np.mean(dists, dtype=np.float32))
  else:
    (m,), _ = global_means([dists.astype(np.float64).sum()], len(rows), device, group)
    avg_d = F32(m)
  return RoundOutput(out, None, collections.OrderedDict(avg_bitrate=bitrate, avg_distortion=avg_d))
