"""Headline benchmark: device-resident encode+decode GiB/s on 25M-fp32 client deltas.

BASELINE.json metric: "device-resident encode+decode GiB/s on 25M-fp32 deltas
at 1/2/4/8 MI355X".  One step = one aggregation round of the
compressed_communication/ codec over a batch of C client deltas of P = 25,000,000
float32 each (BASELINE.md headline: C = 1024, stochastic rounding, step 0.5,
sigma = 1): per client quantise + run-length Elias-gamma encode (HIP
k_encode), then decode + int32 client sum (HIP k_decode), then dequantise of the
sum.  Multi-GPU: the C clients are split across ranks (strong scaling), each
rank encodes/decodes its share and the int32 partial sums are all-reduced with
RCCL (backend "nccl") before the dequantise.

value = C * P * 4 bytes / t_step / 2^30 (GiB/s of fp32 deltas consumed),
t_step = max over ranks of the timed region.  Inputs are synthetic, generated
on device, and resident in HBM before the timed region starts; the delta pool
(by default a distinct 100 MB delta per client, 102 GB at C = 1024) is far
beyond the 256 MiB Infinity Cache, so every client streams from HBM.

Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--clients C]
       [--mode stochastic|uniform|dithered] [--no-cpu-baseline] [--slabs S]
       [--dump-result PATH]

N > 1: each rank decodes its clients in S tile ranges and all-reduces each range
while the next decodes.  Rehearsal on a 1-GPU box (never used by the driver):
FEDCODEC_BENCH_BACKEND=gloo FEDCODEC_BENCH_ONE_DEVICE=1 with --dump-result, see
tools/rehearse_multigpu.sh.
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from federated_amd import _lib  # noqa: E402
from federated_amd import codec  # noqa: E402

HBM_PEAK = 8.0e12  # MI355X HBM3E spec, bytes/s (MI355X_MICROARCH.md)
MODES = {"uniform": _lib.UNIFORM, "stochastic": _lib.STOCHASTIC, "dithered": _lib.DITHERED}


def parse():
  ap = argparse.ArgumentParser()
  ap.add_argument("--gpus", type=int, default=1)
  ap.add_argument("--steps", type=int, default=5)
  ap.add_argument("--warmup", type=int, default=2)
  ap.add_argument("--clients", type=int, default=1024, help="clients per round (all ranks)")
  ap.add_argument("--P", type=int, default=25_000_000)
  ap.add_argument("--mode", default="stochastic", choices=list(MODES))
  ap.add_argument("--step-size", type=float, default=0.5)
  ap.add_argument("--sigma", type=float, default=1.0)
  ap.add_argument("--pool", type=int, default=0,
                  help="distinct delta buffers cycled over clients (0 = one per client)")
  ap.add_argument("--cap-bytes-per-elem", type=float, default=1.0)
  ap.add_argument("--no-cpu-baseline", action="store_true")
  ap.add_argument("--cpu-sample-clients", type=int, default=32)
  ap.add_argument("--dump-result", default="",
                  help="rank 0 saves the round's dequantised sum (.npy) to compare world sizes")
  ap.add_argument("--slabs", type=int, default=4,
                  help="N > 1: tile ranges decoded in turn, each all-reduced while the next decodes")
  return ap.parse_args()


def setup_dist(args):
  world = int(os.environ.get("WORLD_SIZE", "1"))
  rank = int(os.environ.get("RANK", "0"))
  local = int(os.environ.get("LOCAL_RANK", "0"))
  if world > 1:
    import torch.distributed as dist  # pylint: disable=g-import-not-at-top
    # rehearsal knobs for a 1-GPU box (never set by the driver): every rank on one
    # device, gloo instead of RCCL
    backend = os.environ.get("FEDCODEC_BENCH_BACKEND", "nccl")
    if os.environ.get("FEDCODEC_BENCH_ONE_DEVICE"):
      local = 0
    torch.cuda.set_device(local)
    if backend == "nccl":
      dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
      dist.init_process_group(backend)
  else:
    torch.cuda.set_device(0)
  return rank, world


def cpu_baseline(args):
  """Oracle "port" of the reference TF-CPU path on a bounded sample (rank 0, N=1).

  Per client: numpy quantise (TF's multi-pass elementwise structure) + the
  scalar C run-length-gamma encoder, then decode-accumulate, clients spread over
  a thread pool (numpy ufuncs and the C codec release the GIL).
  """
  from concurrent.futures import ThreadPoolExecutor  # pylint: disable=g-import-not-at-top
  from oracle import codec as ocodec  # pylint: disable=g-import-not-at-top
  from oracle import quantize_utils as oq  # pylint: disable=g-import-not-at-top
  n = args.cpu_sample_clients
  P = args.P
  rng = np.random.default_rng(1)
  xs = [(rng.standard_normal(P, dtype=np.float32) * np.float32(args.sigma)) for _ in range(n)]
  qfn = {"uniform": lambda x, s, sd: oq.uniform_quantize(x, s), "stochastic": oq.stochastic_quantize,
         "dithered": oq.dithered_quantize}[args.mode]
  ocodec.lib()
  cores = min(n, 16, len(os.sched_getaffinity(0)))  # the GPU box grants 16 CPUs per GPU

  def one(c):
    q = qfn(xs[c], np.float32(args.step_size), (c, c))
    code, _ = ocodec.run_length_gamma_encode(q)
    return code

  t0 = time.perf_counter()
  with ThreadPoolExecutor(cores) as ex:
    codes = list(ex.map(one, range(n)))
  acc = np.zeros(P, np.int32)
  for code in codes:  # federated_aggregate accumulate: sequential on the server
    ocodec.decode_accumulate(code, acc)
  _ = oq.uniform_dequantize(acc, args.step_size)
  t = time.perf_counter() - t0
  return {"value": n * P * 4 / t / 2**30, "unit": "GiB/s", "cores": cores, "kind": "port",
          "sample": "%d clients x %d fp32, %s step %g: numpy quantise + C rlgamma encode on a %d-thread "
                    "pool, sequential decode-accumulate, dequantise; %.1f s" % (
                        n, P, args.mode, args.step_size, cores, t)}


def measured_traffic(args, C):
  """Per-launch HBM bytes of k_encode from the latest committed PMC profile of this exact
  workload (profiles/*/traffic.json, written from tools/profile_bench.sh's FETCH_SIZE and
  WRITE_SIZE passes with the gfx950 correction), else None."""
  import glob  # pylint: disable=g-import-not-at-top
  best = None
  for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "*", "traffic.json"))):
    try:
      with open(f) as fh:
        d = json.load(fh)
    except (OSError, ValueError):
      continue
    cfg = d.get("config", {})
    if (cfg.get("clients"), cfg.get("P"), cfg.get("mode"), cfg.get("step")) == (C, args.P, args.mode,
                                                                               args.step_size):
      best = (f, d)
  if best is None:
    return None, None
  return best[1]["k_encode"]["hbm_bytes_corrected"], os.path.relpath(best[0], ROOT)


def main():
  args = parse()
  rank, world = setup_dist(args)
  dev = torch.device("cuda", torch.cuda.current_device())
  P = args.P
  C = args.clients
  assert C % world == 0, "clients must divide evenly over ranks"
  Cg = C // world
  mode = MODES[args.mode]

  # ---- synthetic inputs, resident in HBM before timing ----
  g = torch.Generator(device=dev)
  g.manual_seed(20251015 + rank)
  npool = args.pool if args.pool > 0 else Cg
  pool = []
  for i in range(npool):
    if npool == Cg:  # a delta per client, seeded by its global index: any --gpus N sums the same round
      g.manual_seed(20251015 + rank * Cg + i)
    t = torch.randn(P, generator=g, device=dev, dtype=torch.float32)
    pool.append(t.mul_(args.sigma))
  rows = [pool[c % npool] for c in range(Cg)]
  ptrs = torch.tensor([r.data_ptr() for r in rows], dtype=torch.int64, device=dev)
  base = 1000 + rank * Cg
  seeds = torch.tensor([[base + c, base + c] for c in range(Cg)], dtype=torch.int64, device=dev)
  cap = codec._round_up(int(P * args.cap_bytes_per_elem) + 256, 64)
  batch = codec.EncodedBatch(P, Cg, [cap] * Cg, dev)
  out = torch.empty(P, dtype=torch.float32, device=dev)
  isum = torch.empty(P, dtype=torch.int32, device=dev)
  err = torch.zeros(1, dtype=torch.int32, device=dev)
  stream = torch.cuda.current_stream()
  if world > 1:
    import torch.distributed as dist  # pylint: disable=g-import-not-at-top

  T = codec.num_tiles(P)
  nslab = max(1, min(args.slabs, T))
  bounds = [T * k // nslab for k in range(nslab + 1)]

  def step():
    codec.quantize_encode(None, args.step_size, seeds, mode, ptrs=ptrs, P=P, out=batch,
                          stream=stream)
    if world == 1:
      codec.decode_accumulate(batch, want_sum=False, out=out, step=args.step_size, err=err,
                              stream=stream)
    else:
      # decode tile range k, then all-reduce it (RCCL on its own stream, ordered after
      # the decode) while range k+1 decodes; the int32 sum is exact in any order
      err.zero_()
      works = []
      for k in range(nslab):
        codec.decode_accumulate(batch, sum_out=isum, err=err, stream=stream,
                                tiles=(bounds[k], bounds[k + 1]))
        lo, hi = bounds[k] * 1024, min(P, bounds[k + 1] * 1024)
        works.append(dist.all_reduce(isum[lo:hi], async_op=True))
      for w in works:
        w.wait()
      _lib.call("fc_dequantize", _lib.ptr(isum), P, float(args.step_size), None, _lib.ptr(out),
                _lib.stream_handle(stream))

  for _ in range(args.warmup):
    step()
  torch.cuda.synchronize()
  ovf = codec.check_overflow(batch)
  if len(ovf):
    raise SystemExit("stream capacity too small for %d clients; raise --cap-bytes-per-elem" % len(ovf))
  if int(err.item()):
    raise SystemExit("decoder reported a malformed stream")

  # ---- timed region ----
  if world > 1:
    dist.barrier()
  torch.cuda.synchronize()
  t0 = time.perf_counter()
  ev0 = torch.cuda.Event(enable_timing=True)
  ev1 = torch.cuda.Event(enable_timing=True)
  ev0.record(stream)
  for _ in range(args.steps):
    step()
  ev1.record(stream)
  torch.cuda.synchronize()
  if world > 1:
    dist.barrier()
  wall = time.perf_counter() - t0
  t_dev = ev0.elapsed_time(ev1) / 1e3
  if args.dump_result and rank == 0:
    np.save(args.dump_result, out.cpu().numpy())
  t = torch.tensor([max(wall, t_dev)], dtype=torch.float64, device=dev)
  if world > 1:
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
  t_step = float(t.item()) / args.steps

  # ---- per-kernel timing of the dominant kernel (HIP events on its stream) ----
  nbytes = batch.nbytes().astype(np.float64)
  S = float(nbytes.sum())
  e = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
  reps = max(2, min(args.steps, 5))
  t_enc = t_dec = 0.0
  for _ in range(reps):
    e[0].record(stream)
    codec.quantize_encode(None, args.step_size, seeds, mode, ptrs=ptrs, P=P, out=batch, stream=stream)
    e[1].record(stream)
    codec.decode_accumulate(batch, want_sum=False, out=out, step=args.step_size, err=err, stream=stream)
    e[2].record(stream)
    torch.cuda.synchronize()
    t_enc += e[0].elapsed_time(e[1]) / 1e3
    t_dec += e[1].elapsed_time(e[2]) / 1e3
  t_enc /= reps
  t_dec /= reps
  enc_bytes = Cg * 4.0 * P + S  # fp32 read + code write
  dec_bytes = S + 4.0 * P  # code read + f32 result write
  step_bytes = Cg * 4.0 * P + 2 * S + 12.0 * P  # BASELINE.md B_alg per GPU

  result = None
  traffic, traffic_src = measured_traffic(args, C) if world == 1 else (None, None)
  if rank == 0:
    value = C * P * 4.0 / t_step / 2**30
    result = {
        "metric": "device-resident encode+decode GiB/s on 25M-fp32 deltas",
        "value": round(value, 3),
        "unit": "GiB/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(t_step * 1e3, 3),
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "f32->int32 (u8 bitstream)",
        "data": "synthetic: sigma*N(0,1) fp32 deltas generated on device, %s" % (
            "a distinct delta per client (%.1f GB resident)" % (npool * P * 4 / 1e9)
            if npool == Cg else "%d-buffer pool cycled over clients" % npool),
        "config": {"workload": "%d clients x %d fp32 deltas, %s rounding step %g, run-length Elias-gamma "
                               "code, decode + int32 client sum + dequantise" % (C, P, args.mode,
                                                                                 args.step_size),
                   "clients_per_gpu": Cg, "parallelism": "client-sharded dp%d + RCCL int32 all-reduce"
                   % world if world > 1 else "1 GPU"},
        "roofline": {"bound": "hbm", "kernel": "k_encode",
                     "achieved": round(enc_bytes / t_enc / 1e9, 1),
                     "peak": HBM_PEAK / 1e9, "unit": "GB/s",
                     "frac": round(enc_bytes / t_enc / HBM_PEAK, 4),
                     "traffic": round(traffic) if traffic else None,
                     "traffic_source": traffic_src,
                     "alg_bytes_per_launch": enc_bytes, "launch_ms": round(t_enc * 1e3, 3)},
        "decode": {"kernel": "k_decode", "launch_ms": round(t_dec * 1e3, 3),
                   "alg_GBps": round(dec_bytes / t_dec / 1e9, 1)},
        "step_roofline": {"alg_bytes_per_gpu": step_bytes,
                          "achieved_GBps": round(step_bytes / t_step / 1e9, 1),
                          "frac": round(step_bytes / t_step / HBM_PEAK, 4)},
        "bits_per_element": round(8 * S / (Cg * P), 4),
    }
    if world == 1 and not args.no_cpu_baseline:
      result["cpu_baseline"] = cpu_baseline(args)
    print(json.dumps(result), flush=True)
  if world > 1:
    dist.barrier()
    dist.destroy_process_group()
  return result


if __name__ == "__main__":
  main()
