"""Client-sharded multi-GPU aggregation (one process per GPU, RCCL over xGMI).

A round's clients are independent until the server sum
(``federated_aggregate`` accumulate/merge, elias_gamma_encode.py:63-88), and
the sum is an associative int32 sum.  So each rank encodes and decodes its
contiguous block of clients and the ranks' int32 partial sums are combined
with ONE all-reduce (backend "nccl" = RCCL on ROCm; "gloo" in CPU tests).
Integer addition is exact and order-independent, so the result is bit-identical
to the single-GPU sum for any world size or ring order.  The dequantise then
runs once, on every rank (each rank holds the server result).
"""
import torch
import torch.distributed as dist

from federated_amd import _lib
from federated_amd import codec


def client_shard(nclients, world, rank):
  """Contiguous block [lo, hi) of clients for `rank` (sizes differ by <= 1)."""
  base, extra = divmod(int(nclients), int(world))
  lo = rank * base + min(rank, extra)
  return lo, lo + base + (1 if rank < extra else 0)


def allreduce_sum_(t, group=None):
  """In-place SUM all-reduce of an integer (or float) tensor; no-op at world 1."""
  if dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1:
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


def aggregate_round(local_rows, step, local_seeds, mode, group=None, prescale=None, slabs=4):
  """Encode + decode this rank's clients, all-reduce the int32 sums, dequantise.

  The decode runs in `slabs` tile ranges (fc_decode_accumulate_tiles, shrinking
  ones: slab_bounds); each range's sum is all-reduced asynchronously (the
  collective's stream waits for that range's decode) while the next range
  decodes.  Integer sums make the
  result independent of the range split and of the ring order.
  Returns (float32 result [P], local EncodedBatch).  Dithered mode also
  all-reduces the float32 noise sum (tolerance, as TFF's federated_sum).
  """
  batch = codec.quantize_encode_checked(local_rows, step, local_seeds, mode, prescale=prescale)
  P = batch.P
  isum = torch.empty(P, dtype=torch.int32, device=batch.device)
  err = torch.zeros(1, dtype=torch.int32, device=batch.device)
  multi = dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1
  bounds = slab_bounds(codec.num_tiles(P), slabs if multi else 1)
  works = []
  for k in range(len(bounds) - 1):
    codec.decode_accumulate(batch, sum_out=isum, err=err, tiles=(bounds[k], bounds[k + 1]))
    if multi:
      lo, hi = slab_elements(bounds, k, P)
      works.append(dist.all_reduce(isum[lo:hi], op=dist.ReduceOp.SUM, group=group, async_op=True))
  for w in works:
    w.wait()
  if int(err.item()):
    raise RuntimeError("malformed run-length gamma code")
  noise = None
  if mode == _lib.DITHERED:
    noise = codec.noise_sum(local_seeds, batch.P, isum.device)
    allreduce_sum_(noise, group)
  return codec.dequantize(isum, step, noise), batch
