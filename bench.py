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

At N = 1 the same JSON line also carries ``workloads``: one object per other
single-GPU workload BASELINE.json / BASELINE.md name, each with its own
HIP-event kernel timings and roofline (dominant kernel's algorithmic bytes per
launch / its launch time vs the 8 TB/s HBM peak):
  headline_uniform  the trainer's default rounding (trainer.py:63-65) on the headline round
  trainer_round     the trainer-default builder round at 1024 x 25 M: fused
                    L2 + Linf wrapper-norm pass, clip x weight pre-scale fused
                    into the encoder, decode, weighted mean (builder.py:77-117)
  trainer_round_c128  the same round on one GPU's 8-GPU share (128 x 25 M)
  config2           128 x 2^20, stochastic step 1/127, sigma 0.25 ("8-bit")
  config3           256 x 4,050,748 (StackOverflow LSTM), stochastic step 1.0
  bare_decode       the reference's wire path at the headline: the server holds only the
                    clients' TFC byte strings (elias_gamma_encode.py:97-109) and decodes them
                    (run_length_gamma_decode, :69-73): fc_build_index rebuilds the decoder
                    index from the bytes on the device, then decode + dequantise
  config4_share     one GPU's share of config 4 (512 x 11 M over 8 GPUs): 64 x 11 M,
                    stochastic step 0.5 (sigma 1)
  config4_full      config 4's whole round on one GPU (512 x 11 M): the N = 1
                    denominator of the driver's 8-GPU config-4 run
  headline_c128     one GPU's share of the 8-GPU headline: 128 x 25 M
  onebit            config 5's codec: 1024 x 25 M one-bit SGD (one_bit_sgd.py:45-112)
  copy              a 16-byte-per-lane HBM copy (the achievable streaming rate)
``--workload NAME`` runs one of them alone (for rocprofv3 passes of one workload).

Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--clients C]
       [--mode stochastic|uniform|dithered] [--no-cpu-baseline] [--slabs S]
       [--workload all|headline|NAME] [--dump-result PATH]

N > 1: each rank decodes its clients in S tile ranges and all-reduces each range
while the next decodes.  `python bench.py --gpus N` (no WORLD_SIZE in the
environment) starts its N ranks itself -- `torch.distributed.run` as a child
process, before this process touches the GPU -- and exits with the child's
code; under a launcher (WORLD_SIZE set) WORLD_SIZE must equal --gpus.
`--workload onebit` at N > 1 times config 5's sharded one-bit round
(distributed.onebit_round: float32 partial sums all-reduced).  Rehearsal on a
1-GPU box (never used by the driver): FEDCODEC_BENCH_BACKEND=gloo
FEDCODEC_BENCH_ONE_DEVICE=1 with --dump-result, see tools/rehearse_multigpu.sh.
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from federated_amd import _lib  # noqa: E402
from federated_amd import codec  # noqa: E402
from federated_amd import distributed  # noqa: E402

HBM_PEAK = 8.0e12  # MI355X HBM3E spec, bytes/s (MI355X_MICROARCH.md)
MODES = {"uniform": _lib.UNIFORM, "stochastic": _lib.STOCHASTIC, "dithered": _lib.DITHERED}
EXTRA = ["headline_uniform", "trainer_round", "trainer_round_c128", "bare_decode", "config2", "config3",
         "config4_share", "config4_full", "headline_c128", "onebit", "onebit_c128", "copy"]


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
  ap.add_argument("--cap-bytes-per-elem", type=float, default=0.0,
                  help="stream capacity per element; 0: sized as QuantizeEncodeFactory does "
                       "(codec.CapacityHint from an untimed probe round)")
  ap.add_argument("--no-cpu-baseline", action="store_true")
  ap.add_argument("--cpu-sample-clients", type=int, default=32)
  ap.add_argument("--dump-result", default="",
                  help="rank 0 saves the round's dequantised sum (.npy) to compare world sizes")
  ap.add_argument("--slabs", type=int, default=4,
                  help="N > 1: tile ranges decoded in turn, each all-reduced while the next decodes")
  ap.add_argument("--workload", default="all", choices=["all", "headline"] + EXTRA,
                  help="all (N=1 default): headline line + every extra workload; headline: the "
                       "headline only; NAME: that workload alone (profiling)")
  ap.add_argument("--extra-steps", type=int, default=5, help="timed steps per extra workload")
  return ap.parse_args()


def free_port():
  s = socket.socket()
  s.bind(("127.0.0.1", 0))
  port = s.getsockname()[1]
  s.close()
  return port


def launcher_cmd(argv, gpus, port):
  """The torch.distributed.run command that starts `gpus` ranks of this script."""
  return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(int(gpus)),
          "--master-addr", "127.0.0.1", "--master-port", str(int(port)), os.path.abspath(__file__)] + list(argv)


def check_world(args, environ=None):
  """Returns "spawn" when this process must start --gpus ranks itself (no
  launcher, --gpus > 1), else None.  Raises SystemExit when a launcher's
  WORLD_SIZE disagrees with --gpus.  Touches nothing on the GPU."""
  env = os.environ if environ is None else environ
  if "WORLD_SIZE" not in env:
    if args.gpus < 1:
      raise SystemExit("bench.py: --gpus must be >= 1")
    return "spawn" if args.gpus > 1 else None
  world = int(env["WORLD_SIZE"])
  if world != args.gpus:
    raise SystemExit("bench.py: WORLD_SIZE=%d from the launcher but --gpus %d" % (world, args.gpus))
  return None


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


def rccl_version():
  """RCCL's version as torch reports it (torch.cuda.nccl on ROCm), or None."""
  try:
    return ".".join(str(v) for v in torch.cuda.nccl.version())
  except Exception:  # pylint: disable=broad-except
    return None


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


def measured_traffic(workload, kernel):
  """Per-launch HBM bytes of `kernel` in `workload` from the latest committed PMC
  profile (profiles/*/traffic_<workload>.json, written by tools/make_profile_record.py
  from separate FETCH_SIZE / WRITE_SIZE passes with the gfx950 correction), else None."""
  import glob  # pylint: disable=g-import-not-at-top
  best = None
  for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "*", "traffic_%s.json" % workload))):
    try:
      with open(f) as fh:
        d = json.load(fh)
    except (OSError, ValueError):
      continue
    if kernel in d:
      best = (f, d)
  if best is None:
    return None, None
  return best[1][kernel]["hbm_bytes_corrected"], os.path.relpath(best[0], ROOT)


class Timer:
  """HIP events around named phases on one stream (the stream the kernels run on)."""

  def __init__(self, stream):
    self.stream = stream
    self.acc = {}
    self.n = {}

  def phase(self, name, fn):
    e0 = torch.cuda.Event(enable_timing=True)
    e1 = torch.cuda.Event(enable_timing=True)
    e0.record(self.stream)
    r = fn()
    e1.record(self.stream)
    self.acc.setdefault(name, []).append((e0, e1))
    return r

  def ms(self):
    torch.cuda.synchronize()
    return {k: sum(a.elapsed_time(b) for a, b in v) / len(v) for k, v in self.acc.items()}


def roofline(kernel, alg_bytes, launch_ms, workload):
  traffic, src = measured_traffic(workload, kernel)
  return {"bound": "hbm", "kernel": kernel, "achieved": round(alg_bytes / launch_ms / 1e6, 1),
          "peak": HBM_PEAK / 1e9, "unit": "GB/s", "frac": round(alg_bytes / launch_ms / 1e-3 / HBM_PEAK, 4),
          "traffic": round(traffic) if traffic else None, "traffic_source": src,
          "alg_bytes_per_launch": alg_bytes, "launch_ms": round(launch_ms, 3)}


PROBE_SEED_OFFSET = 7919


def probe_seeds(seeds):
  """The untimed probe round's seeds: other Philox streams than the timed round's."""
  return seeds + PROBE_SEED_OFFSET


def sized_batch(P, C, dev, encode, cap_per_elem=0.0):
  """The round's EncodedBatch with capacities as the factory sizes them: an
  untimed probe round (1 byte per element), then codec.CapacityHint (largest
  client code + 1/8 + 4 KiB) -- what QuantizeEncodeFactory uses from its second
  round on.  The probe encodes with other seeds (``probe_seeds``) than the timed
  round, as the factory only knows the previous round's sizes (uniform rounding
  draws no stream: there the probe's codes equal the timed ones).
  cap_per_elem > 0: that fixed capacity instead."""
  if cap_per_elem > 0:
    return codec.EncodedBatch(P, C, [codec._round_up(int(P * cap_per_elem) + 256, 64)] * C, dev)  # pylint: disable=protected-access
  probe = codec.EncodedBatch(P, C, [codec._round_up(P + 256, 64)] * C, dev)  # pylint: disable=protected-access
  encode(probe)
  hint = codec.CapacityHint()
  hint.update(probe)
  del probe
  torch.cuda.empty_cache()
  return codec.EncodedBatch(P, C, hint.caps(P, C), dev)


def make_deltas(C, P, sigma, dev, seed0):
  g = torch.Generator(device=dev)
  rows = []
  for i in range(C):
    g.manual_seed(seed0 + i)
    rows.append(torch.randn(P, generator=g, device=dev, dtype=torch.float32).mul_(sigma))
  return rows


def codec_round(name, rows, ptrs, P, step, mode, steps, warmup, stream, workload=None):
  """Encode + decode + dequantise rounds of one codec configuration; HIP-event timed."""
  C = len(rows)
  dev = rows[0].device
  seeds = torch.tensor([[500 + c, 500 + c] for c in range(C)], dtype=torch.int64, device=dev)
  batch = sized_batch(P, C, dev, lambda b: codec.quantize_encode(None, step, probe_seeds(seeds), mode, ptrs=ptrs, P=P, out=b,
                                                                  stream=stream))
  out = torch.empty(P, dtype=torch.float32, device=dev)
  err = torch.zeros(1, dtype=torch.int32, device=dev)
  tm = Timer(stream)
  for i in range(warmup + steps):
    t = tm if i >= warmup else Timer(stream)
    t.phase("k_encode", lambda: codec.quantize_encode(None, step, seeds, mode, ptrs=ptrs, P=P, out=batch,
                                                      stream=stream))
    t.phase("k_decode", lambda: codec.decode_accumulate(batch, want_sum=False, out=out, step=step, err=err,
                                                        stream=stream))
    # a segmented batch's stitch runs on a second stream beside the decode: the
    # round ends when it has (the wait's phase is the stitch's time past the decode)
    t.phase("stitch_join", lambda: batch.join(stream))
  ms = tm.ms()
  if len(codec.check_overflow(batch)) or int(err.item()):
    raise SystemExit("%s: overflow or malformed stream" % name)
  S = float(batch.nbytes().astype(np.float64).sum())
  t_step = ms["k_encode"] + ms["k_decode"] + ms["stitch_join"]
  return {
      "workload": name, "clients": C, "P": P, "mode": [k for k, v in MODES.items() if v == mode][0],
      "step_size": step, "ms_per_step": round(t_step, 3),
      "value_GiBps": round(C * P * 4.0 / (t_step * 1e-3) / 2**30, 2),
      "bits_per_element": round(8 * S / (C * P), 4),
      "roofline": roofline("k_encode", C * 4.0 * P + S, ms["k_encode"], workload or name),
      "decode": {"kernel": "k_decode", "launch_ms": round(ms["k_decode"], 3),
                 "alg_GBps": round((S + 4.0 * P) / (ms["k_decode"] * 1e-3) / 1e9, 1)},
      "step_roofline_frac": round((C * 4.0 * P + 2 * S + 12.0 * P) / (t_step * 1e-3) / HBM_PEAK, 4),
  }


def w_trainer_round(rows, ptrs, P, steps, warmup, stream, name="trainer_round"):
  """Trainer-default builder round (uniform, step 0.5, clipping + zeroing, weighted),
  device part as builder.WrappedAggregationFactory runs it: ONE fused L2 + Linf norm
  pass, host scalars for the wrapper scales (one 8-KB D2H), the clip scale x weight
  pre-scale fused into the encoder, decode + dequantise, divide by the weight sum."""
  C = len(rows)
  dev = rows[0].device
  step = 0.5
  w = torch.arange(200, 200 + C, dtype=torch.float32)  # example counts
  seeds = torch.tensor([[9 + c, 9 + c] for c in range(C)], dtype=torch.int64, device=dev)
  batch = None  # sized by the first round (below)
  out = torch.empty(P, dtype=torch.float32, device=dev)
  err = torch.zeros(1, dtype=torch.int32, device=dev)
  denom = torch.full((1,), float(w.sum()), dtype=torch.float32, device=dev)
  norms = torch.empty(2 * C, dtype=torch.float32, device=dev)
  clip, zero_thr = np.float32(1.0), np.float32(21.0)

  def norm_pass():
    _lib.call("fc_client_norms_scaled", _lib.ptr(ptrs), C, P, _lib.NORM_L2_LINF, None, _lib.ptr(norms),
              _lib.stream_handle(stream))

  tm = Timer(stream)
  t_wall = []
  for i in range(warmup + steps):
    t = tm if i >= warmup else Timer(stream)
    torch.cuda.synchronize()
    w0 = time.perf_counter()
    t.phase("k_client_norms", norm_pass)
    nh = norms.cpu().numpy().reshape(2, C)  # the wrapper scales are host scalars (sync)
    l2, linf = nh[0], nh[1]
    keep = ~(linf > zero_thr)
    l2 = np.where(keep, l2, np.float32(0.0)).astype(np.float32)
    with np.errstate(divide="ignore"):
      inv = np.where(l2 > 0, np.float32(1.0) / l2, np.float32(np.inf)).astype(np.float32)
    s0 = np.where(keep, clip * np.minimum(inv, np.float32(1.0) / clip), np.float32(0.0)).astype(np.float32)
    pre = torch.from_numpy(np.stack([s0, w.numpy()], 1).astype(np.float32)).to(dev, non_blocking=True)
    if batch is None:
      batch = sized_batch(P, C, dev, lambda b: codec.quantize_encode(None, step, probe_seeds(seeds), _lib.UNIFORM, ptrs=ptrs, P=P,
                                                                      out=b, stream=stream, prescale=pre))
    t.phase("k_encode", lambda: codec.quantize_encode(None, step, seeds, _lib.UNIFORM, ptrs=ptrs, P=P, out=batch,
                                                      stream=stream, prescale=pre))
    t.phase("k_decode", lambda: codec.decode_accumulate(batch, want_sum=False, out=out, step=step, err=err,
                                                        stream=stream))
    t.phase("mean", lambda: out.div_(denom))
    torch.cuda.synchronize()
    if i >= warmup:
      t_wall.append(time.perf_counter() - w0)
  ms = tm.ms()
  if len(codec.check_overflow(batch)) or int(err.item()):
    raise SystemExit("%s: overflow or malformed stream" % name)
  S = float(batch.nbytes().astype(np.float64).sum())
  t_round = float(np.mean(t_wall)) * 1e3
  return {
      "workload": name, "clients": C, "P": P, "mode": "uniform", "step_size": step,
      "clipping": True, "zeroing": True, "weighted": True,
      "ms_per_step": round(t_round, 3), "value_GiBps": round(C * P * 4.0 / (t_round * 1e-3) / 2**30, 2),
      "kernels_ms": {k: round(v, 3) for k, v in ms.items()},
      "bits_per_element": round(8 * S / (C * P), 4),
      "roofline": roofline("k_encode", C * 4.0 * P + S, ms["k_encode"], name),
      "norms_roofline": roofline("k_client_norms", C * 4.0 * P, ms["k_client_norms"], name),
  }


def w_onebit(rows, ptrs, P, steps, warmup, stream, name="onebit"):
  """Config 5's codec on one GPU: 1024 x 25 M one-bit SGD encode + client-order decode-sum
  (name "onebit_c128": one GPU's 128-client share of config 5's 8-GPU run)."""
  C = len(rows)
  dev = rows[0].device
  nw = (P + 31) // 32
  masks = torch.empty(C * nw, dtype=torch.int32, device=dev)
  means = torch.empty(2 * C, dtype=torch.float32, device=dev)
  dist = torch.empty(C, dtype=torch.float64, device=dev)
  out = torch.empty(P, dtype=torch.float32, device=dev)
  h = _lib.stream_handle(stream)
  tm = Timer(stream)
  for i in range(warmup + steps):
    t = tm if i >= warmup else Timer(stream)
    t.phase("k_mask_encode", lambda: _lib.call("fc_onebit_encode", _lib.ptr(ptrs), C, P, 0.0, _lib.ptr(masks),
                                                _lib.ptr(means), _lib.ptr(dist), h))
    t.phase("k_onebit_decode_sum", lambda: _lib.call("fc_onebit_decode_sum", _lib.ptr(masks), _lib.ptr(means), C,
                                                      P, _lib.ptr(out), h))
  ms = tm.ms()
  t_step = ms["k_mask_encode"] + ms["k_onebit_decode_sum"]
  enc_bytes = C * 4.0 * P + C * 4.0 * nw
  return {
      "workload": name, "clients": C, "P": P, "codec": "one-bit SGD, threshold 0",
      "ms_per_step": round(t_step, 3), "value_GiBps": round(C * P * 4.0 / (t_step * 1e-3) / 2**30, 2),
      "roofline": roofline("k_mask_encode", enc_bytes, ms["k_mask_encode"], name),
      "decode": {"kernel": "k_onebit_decode_sum", "launch_ms": round(ms["k_onebit_decode_sum"], 3),
                 "alg_GBps": round((C * 4.0 * nw + 4.0 * P) / (ms["k_onebit_decode_sum"] * 1e-3) / 1e9, 1)},
  }


def w_bare_decode(rows, ptrs, P, steps, warmup, stream):
  """Server decode of bare TFC strings at the headline (stochastic, step 0.5): the
  headline round's codes are encoded once (untimed); a step is fc_build_index over
  the streams' bytes alone (the encoder's index is overwritten) + k_decode + the
  dequantise epilogue.  The result is checked equal to the decode with the
  encoder's own index."""
  C = len(rows)
  dev = rows[0].device
  step = 0.5
  seeds = torch.tensor([[1000 + c, 1000 + c] for c in range(C)], dtype=torch.int64, device=dev)
  batch = sized_batch(P, C, dev, lambda b: codec.quantize_encode(None, step, probe_seeds(seeds), _lib.STOCHASTIC,
                                                                  ptrs=ptrs, P=P, out=b, stream=stream))
  codec.quantize_encode(None, step, seeds, _lib.STOCHASTIC, ptrs=ptrs, P=P, out=batch, stream=stream)
  if len(codec.check_overflow(batch)):
    raise SystemExit("bare_decode: overflow")
  batch.join(stream)
  ref = torch.empty(P, dtype=torch.float32, device=dev)
  out = torch.empty(P, dtype=torch.float32, device=dev)
  err = torch.zeros(1, dtype=torch.int32, device=dev)
  codec.decode_accumulate(batch, want_sum=False, out=ref, step=step, err=err, stream=stream)
  nb = batch.nbytes()
  nbytes = torch.from_numpy(nb.astype(np.int64)).to(dev)
  maxb = int(nb.max())
  ierr = []
  tm = Timer(stream)
  for i in range(warmup + steps):
    t = tm if i >= warmup else Timer(stream)
    ierr.append(t.phase("fc_build_index", lambda: codec.index_codes(batch, nbytes, maxb, stream=stream, check=False)))
    t.phase("k_decode", lambda: codec.decode_accumulate(batch, want_sum=False, out=out, step=step, err=err,
                                                        stream=stream))
  ms = tm.ms()
  if int(err.item()) or any(int(e.item()) for e in ierr) or not bool(torch.equal(out, ref)):
    raise SystemExit("bare_decode: index rebuild or decode differs from the encoder-index decode")
  S = float(nb.astype(np.float64).sum())
  t_step = ms["fc_build_index"] + ms["k_decode"]
  return {
      "workload": "bare_decode", "clients": C, "P": P, "mode": "stochastic", "step_size": step,
      "ms_per_step": round(t_step, 3), "code_GB": round(S / 1e9, 3),
      "value_GiBps": round(C * P * 4.0 / (t_step * 1e-3) / 2**30, 2),
      "index_rebuild": {"kernels": "fc_build_index (k_idx_spec/sync/fix/scan/emit/check)",
                        "launch_ms": round(ms["fc_build_index"], 3),
                        "code_GBps": round(S / (ms["fc_build_index"] * 1e-3) / 1e9, 1)},
      "decode": {"kernel": "k_decode", "launch_ms": round(ms["k_decode"], 3),
                 "alg_GBps": round((S + 4.0 * P) / (ms["k_decode"] * 1e-3) / 1e9, 1)},
      "note": "value counts the clients' fp32 deltas the decoded round stands for, over the server side only",
  }


def w_copy(dev, stream, steps=10):
  n = 4 << 30
  a = torch.empty(n, dtype=torch.uint8, device=dev)
  b = torch.empty(n, dtype=torch.uint8, device=dev)
  a.fill_(1)
  h = _lib.stream_handle(stream)
  tm = Timer(stream)
  for i in range(2 + steps):
    t = tm if i >= 2 else Timer(stream)
    t.phase("k_copy_f4", lambda: _lib.call("fc_copy", _lib.ptr(b), _lib.ptr(a), n, h))
  ms = tm.ms()["k_copy_f4"]
  gbps = 2.0 * n / (ms * 1e-3) / 1e9
  del a, b
  return {"workload": "copy", "bytes_moved_per_launch": 2 * n, "launch_ms": round(ms, 3),
          "achieved_GBps": round(gbps, 1), "frac_of_8TBps": round(gbps * 1e9 / HBM_PEAK, 4)}


def run_extra(name, args, dev, stream, head_rows, head_ptrs):
  steps, warmup = args.extra_steps, 2
  P = args.P
  if name == "headline_uniform":
    return codec_round(name, head_rows, head_ptrs, P, 0.5, _lib.UNIFORM, steps, warmup, stream)
  if name == "trainer_round":
    return w_trainer_round(head_rows, head_ptrs, P, steps, warmup, stream)
  if name == "trainer_round_c128":  # the first 128 of the headline's client deltas
    return w_trainer_round(head_rows[:128], head_ptrs[:128], P, max(steps, 10), warmup, stream,
                           name="trainer_round_c128")
  if name == "onebit":
    return w_onebit(head_rows, head_ptrs, P, steps, warmup, stream)
  if name == "onebit_c128":  # config 5's per-GPU share at 8 GPUs: the first 128 client deltas
    return w_onebit(head_rows[:128], head_ptrs[:128], P, max(steps, 10), warmup, stream, name="onebit_c128")
  if name == "copy":
    return w_copy(dev, stream)
  if name == "bare_decode":
    return w_bare_decode(head_rows, head_ptrs, P, steps, warmup, stream)
  if name == "headline_c128":  # the first 128 of the headline's client deltas
    return codec_round(name, head_rows[:128], head_ptrs[:128], P, 0.5, _lib.STOCHASTIC, max(steps, 10), warmup,
                       stream)
  if name == "config2":
    rows = make_deltas(128, 1 << 20, 0.25, dev, 7000)
    step = 1.0 / 127
  elif name == "config4_share":
    rows = make_deltas(64, 11_000_000, 1.0, dev, 11000)
    step = 0.5
  elif name == "config4_full":
    rows = make_deltas(512, 11_000_000, 1.0, dev, 11000)  # the share's 64 deltas are its first 64
    step = 0.5
  else:  # config3
    rows = make_deltas(256, 4_050_748, 1.0, dev, 9000)
    step = 1.0
  ptrs = torch.tensor([r.data_ptr() for r in rows], dtype=torch.int64, device=dev)
  r = codec_round(name, rows, ptrs, rows[0].numel(), step, _lib.STOCHASTIC, max(steps, 10), warmup, stream)
  del rows
  return r


def onebit_sharded(args, rank, world, dev, stream):
  """Config 5 on N GPUs: C clients x P one-bit SGD (one_bit_sgd.py:45-112),
  C / N clients per rank.  A step: fc_onebit_encode of the rank's clients, the
  client-order float32 decode-sum in `--slabs` element ranges, each range's
  float32 sum all-reduced (RCCL) while the next is summed."""
  import torch.distributed as dist  # pylint: disable=g-import-not-at-top
  P, C = args.P, args.clients
  assert C % world == 0, "clients must divide evenly over ranks"
  Cg = C // world
  g = torch.Generator(device=dev)
  rows = []
  for i in range(Cg):
    g.manual_seed(20251015 + rank * Cg + i)  # a delta per client, seeded by its global index
    rows.append(torch.randn(P, generator=g, device=dev, dtype=torch.float32).mul_(args.sigma))
  ptrs = torch.tensor([r.data_ptr() for r in rows], dtype=torch.int64, device=dev)
  nw = (P + 31) // 32
  masks = torch.empty(Cg * nw, dtype=torch.int32, device=dev)
  means = torch.empty(2 * Cg, dtype=torch.float32, device=dev)
  dist_ = torch.empty(Cg, dtype=torch.float64, device=dev)
  out = torch.empty(P, dtype=torch.float32, device=dev)
  h = _lib.stream_handle(stream)
  bounds = distributed.slab_bounds(nw, args.slabs)

  def step():
    _lib.call("fc_onebit_encode", _lib.ptr(ptrs), Cg, P, 0.0, _lib.ptr(masks), _lib.ptr(means), _lib.ptr(dist_), h)
    works = []
    for k in range(len(bounds) - 1):
      _lib.call("fc_onebit_decode_sum_range", _lib.ptr(masks), _lib.ptr(means), Cg, P, bounds[k], bounds[k + 1],
                _lib.ptr(out), h)
      lo, hi = bounds[k] * 32, min(P, bounds[k + 1] * 32)
      works.append(dist.all_reduce(out[lo:hi], async_op=True))
    for w in works:
      w.wait()

  for _ in range(args.warmup):
    step()
  torch.cuda.synchronize()
  dist.barrier()
  torch.cuda.synchronize()
  t0 = time.perf_counter()
  for _ in range(args.steps):
    step()
  torch.cuda.synchronize()
  dist.barrier()
  wall = time.perf_counter() - t0
  if args.dump_result and rank == 0:
    np.save(args.dump_result, out.cpu().numpy())
  t = torch.tensor([wall], dtype=torch.float64, device=dev)
  dist.all_reduce(t, op=dist.ReduceOp.MAX)
  t_step = float(t.item()) / args.steps
  tm = Timer(stream)
  for _ in range(max(2, min(args.steps, 5))):
    tm.phase("k_mask_encode", lambda: _lib.call("fc_onebit_encode", _lib.ptr(ptrs), Cg, P, 0.0, _lib.ptr(masks),
                                                 _lib.ptr(means), _lib.ptr(dist_), h))
  ms = tm.ms()
  result = None
  if rank == 0:
    enc_bytes = Cg * 4.0 * P + Cg * 4.0 * nw
    result = {
        "metric": "device-resident encode+decode GiB/s on 25M-fp32 deltas",
        "value": round(C * P * 4.0 / t_step / 2**30, 3), "unit": "GiB/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(t_step * 1e3, 3),
        "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "f32 (1-bit masks)",
        "data": "synthetic: sigma*N(0,1) fp32 deltas generated on device, a distinct delta per client",
        "config": {"workload": "config 5: %d clients x %d fp32 deltas, one-bit SGD (threshold 0), client-order "
                               "float32 decode-sum + RCCL float32 all-reduce" % (C, P),
                   "clients_per_gpu": Cg, "world_size": world, "backend": dist.get_backend(),
                   "rccl_version": rccl_version(),
                   "parallelism": "client-sharded dp%d + float32 all-reduce in %d slabs" % (world, len(bounds) - 1)},
        "roofline": roofline("k_mask_encode", enc_bytes, ms["k_mask_encode"], "none"),
    }
    print(json.dumps(result), flush=True)
  dist.barrier()
  dist.destroy_process_group()
  return result


def main():
  args = parse()
  if check_world(args) == "spawn":
    # N ranks under torch.distributed.run, started before this process touches the GPU
    sys.exit(subprocess.call(launcher_cmd(sys.argv[1:], args.gpus, free_port())))
  rank, world = setup_dist(args)
  dev = torch.device("cuda", torch.cuda.current_device())
  stream = torch.cuda.current_stream()
  P = args.P
  C = args.clients
  assert C % world == 0, "clients must divide evenly over ranks"
  Cg = C // world
  mode = MODES[args.mode]
  single = args.workload not in ("all", "headline")
  if world > 1 and args.workload == "onebit":
    return onebit_sharded(args, rank, world, dev, stream)
  if world > 1 and single:
    raise SystemExit("bench.py: --workload %s runs on one GPU only (N > 1: headline, onebit)" % args.workload)

  # ---- synthetic inputs, resident in HBM before timing ----
  g = torch.Generator(device=dev)
  g.manual_seed(20251015 + rank)
  npool = args.pool if args.pool > 0 else Cg
  pool = []
  need_head = not single or args.workload in ("headline_uniform", "trainer_round", "trainer_round_c128",
                                              "bare_decode", "onebit", "headline_c128", "onebit_c128")
  for i in range(npool if need_head else 0):
    if npool == Cg:  # a delta per client, seeded by its global index: any --gpus N sums the same round
      g.manual_seed(20251015 + rank * Cg + i)
    t = torch.randn(P, generator=g, device=dev, dtype=torch.float32)
    pool.append(t.mul_(args.sigma))
  rows = [pool[c % npool] for c in range(Cg)] if pool else []
  ptrs = torch.tensor([r.data_ptr() for r in rows], dtype=torch.int64, device=dev) if rows else None

  if single:  # one extra workload alone (profiling runs)
    r = run_extra(args.workload, args, dev, stream, rows, ptrs)
    print(json.dumps(r), flush=True)
    return r

  base = 1000 + rank * Cg
  seeds = torch.tensor([[base + c, base + c] for c in range(Cg)], dtype=torch.int64, device=dev)
  batch = sized_batch(P, Cg, dev, lambda b: codec.quantize_encode(None, args.step_size, probe_seeds(seeds), mode, ptrs=ptrs, P=P,
                                                                   out=b, stream=stream), args.cap_bytes_per_elem)
  out = torch.empty(P, dtype=torch.float32, device=dev)
  isum = torch.empty(P, dtype=torch.int32, device=dev)
  err = torch.zeros(1, dtype=torch.int32, device=dev)
  if world > 1:
    import torch.distributed as dist  # pylint: disable=g-import-not-at-top

  bounds = distributed.slab_bounds(codec.num_tiles(P), args.slabs)  # shrinking: the last is smallest
  # one GPU: the round in two client halves, the first half's decode beside the second
  # half's encode (codec.encode_decode_pipelined; same int32 sum)
  pipelined = world == 1 and codec.pipeline_wanted(Cg, P)
  rnd = codec.PipelinedRound(P, list(batch.caps_host), dev) if pipelined else None

  def step():
    if pipelined:
      codec.encode_decode_pipelined(ptrs, P, args.step_size, seeds, mode, rnd, out=out, stream=stream)
      return
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
      for k in range(len(bounds) - 1):
        codec.decode_accumulate(batch, sum_out=isum, err=err, stream=stream,
                                tiles=(bounds[k], bounds[k + 1]))
        lo, hi = distributed.slab_elements(bounds, k, P)
        works.append(dist.all_reduce(isum[lo:hi], async_op=True))
      for w in works:
        w.wait()
      _lib.call("fc_dequantize", _lib.ptr(isum), P, float(args.step_size), None, _lib.ptr(out),
                _lib.stream_handle(stream))
    batch.join(stream)  # a segmented batch's stitch (second stream) is part of the round

  for _ in range(args.warmup):
    step()
  torch.cuda.synchronize()
  ovf = rnd.overflowed() if pipelined else codec.check_overflow(batch)
  if len(ovf):
    raise SystemExit("stream capacity too small for %d clients; raise --cap-bytes-per-elem" % len(ovf))
  if int((rnd.err if pipelined else err).item()):
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
  tm = Timer(stream)
  reps = max(2, min(args.steps, 5))
  for _ in range(reps):
    tm.phase("k_encode", lambda: codec.quantize_encode(None, args.step_size, seeds, mode, ptrs=ptrs, P=P,
                                                       out=batch, stream=stream))
    tm.phase("k_decode", lambda: codec.decode_accumulate(batch, want_sum=False, out=out, step=args.step_size,
                                                         err=err, stream=stream))
    batch.join(stream)
  ms = tm.ms()
  enc_bytes = Cg * 4.0 * P + S  # fp32 read + code write
  dec_bytes = S + 4.0 * P  # code read + f32 result write
  step_bytes = Cg * 4.0 * P + 2 * S + 12.0 * P  # BASELINE.md B_alg per GPU

  result = None
  if rank == 0:
    value = C * P * 4.0 / t_step / 2**30
    headline_name = "headline" if (args.mode, args.step_size, C, P) == ("stochastic", 0.5, 1024, 25_000_000) \
        else "custom"
    rl = roofline("k_encode", enc_bytes, ms["k_encode"], headline_name if world == 1 else "none")
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
                   "clients_per_gpu": Cg, "world_size": world,
                   "backend": dist.get_backend() if world > 1 else None,
                   "rccl_version": rccl_version(),
                   "stream_capacity": "CapacityHint from an untimed probe round with other seeds" if not
                   args.cap_bytes_per_elem else "%g bytes per element" % args.cap_bytes_per_elem,
                   "parallelism": "client-sharded dp%d + RCCL int32 all-reduce"
                   % world if world > 1 else "1 GPU",
                   "schedule": "two client halves: the first half's decode on a side stream beside the second "
                               "half's encode" if pipelined else "encode, then decode"},
        "roofline": rl,
        "decode": {"kernel": "k_decode", "launch_ms": round(ms["k_decode"], 3),
                   "alg_GBps": round(dec_bytes / (ms["k_decode"] * 1e-3) / 1e9, 1)},
        "step_roofline": {"alg_bytes_per_gpu": step_bytes,
                          "achieved_GBps": round(step_bytes / t_step / 1e9, 1),
                          "frac": round(step_bytes / t_step / HBM_PEAK, 4)},
        "bits_per_element": round(8 * S / (Cg * P), 4),
    }
  if world == 1 and args.workload == "all":
    extras = {}
    for name in EXTRA:
      torch.cuda.synchronize()
      extras[name] = run_extra(name, args, dev, stream, rows, ptrs)
      torch.cuda.empty_cache()
    result["workloads"] = extras
  if rank == 0:
    if world == 1 and not args.no_cpu_baseline:
      result["cpu_baseline"] = cpu_baseline(args)
    print(json.dumps(result), flush=True)
  if world > 1:
    dist.barrier()
    dist.destroy_process_group()
  return result


if __name__ == "__main__":
  main()
