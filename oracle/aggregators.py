"""Round semantics of the reference aggregation processes (TEST INFRASTRUCTURE ONLY).

Each function restates one ``next_fn`` of compressed_communication/ in numpy +
the C run-length-gamma restatement, for a list of client values:

* ``quantize_encode_next``   aggregators/quantize_encode.py:139-211
* ``elias_gamma_sum_next``   aggregators/elias_gamma_encode.py:63-114
* ``stochastic_quantize_next`` aggregators/stochastic_quantize.py:57-88 (SumFactory inner)
* ``one_bit_sgd_next``       aggregators/comparison_methods/one_bit_sgd.py:45-112
* ``qsgd_next``              aggregators/comparison_methods/qsgd.py:62-146
* ``client_lambda_next``     aggregators/quantize_encode_client_lambda.py:97-182
* ``drive_next``             aggregators/comparison_methods/drive.py:48-124
* ``hadamard_forward/inverse`` the randomized Hadamard rotation builder.py:68-69 wraps
  (tff.aggregators.HadamardTransformFactory; TFF absent: sign stream unpinned)

Float reductions (distortion, 1-bit means, one-bit decoded sums) follow TF's
float32 semantics up to summation order; tests compare them with tolerances.
"""
import collections

import numpy as np

from oracle import codec
from oracle import quantize_utils as qu

F32 = np.float32

_Q = {"uniform": lambda x, s, seed: qu.uniform_quantize(x, s), "stochastic": qu.stochastic_quantize,
      "dithered": qu.dithered_quantize}
_NORM = {"constant": lambda x: F32(1.0), "mean_magnitude": qu.mean_magnitude,
         "max_magnitude": qu.max_magnitude, "dimensionless_norm": qu.dimensionless_norm}


def wrap_i32(a):
  return ((np.asarray(a, np.int64) + 2**31) % 2**32 - 2**31).astype(np.int32)


def quantize_encode_next(client_values, step_size, rounding_type="uniform", seeds=None,
                         normalization_type="constant"):
  """One round of QuantizeEncodeFactory: returns (result, measurements, codes)."""
  xs = [np.asarray(v, np.float32).reshape(-1) for v in client_values]
  P = xs[0].size
  step_size = F32(step_size)
  if seeds is None:
    seeds = [(c, c) for c in range(len(xs))]
  acc = np.zeros(P, np.int64)
  noise_sum = np.zeros(P, np.float32)
  dists, sps, lengths, codes = [], [], [], []
  for c, x in enumerate(xs):
    step = F32(_NORM[normalization_type](x) * step_size)                 # :145
    q = _Q[rounding_type](x, step, tuple(seeds[c]))                        # :146
    if rounding_type == "dithered":
      noise = qu.generate_noise(tuple(seeds[c]), P)                        # :147
      deq = qu.dithered_dequantize(q, step, noise)                         # :148-149
      noise_sum = (noise_sum + noise).astype(np.float32)                   # :183
    else:
      deq = qu.uniform_dequantize(q, step)
    d = qu.ftz(x) - deq
    dists.append(F32(np.sum(d.astype(np.float64) ** 2) / P))             # :150-152
    sps.append(F32((F32(P) - F32(np.count_nonzero(q))) / F32(P)))        # :153-155
    code, _ = codec.run_length_gamma_encode(q)                             # e_g_e.py:97-99
    codes.append(code)
    lengths.append(codec.get_bitstring_length(code))                      # e_g_e.py:100-101
    acc += q
  isum = wrap_i32(acc)                                                     # e_g_e.py:63-88
  if rounding_type == "dithered":
    result = qu.dithered_dequantize(isum, step_size, noise_sum)           # :189-190
  else:
    result = qu.uniform_dequantize(isum, step_size)
  measurements = collections.OrderedDict(
      avg_bitrate=np.float64(np.mean(lengths) / np.float64(P)),           # e_g_e.py:102-108
      avg_distortion=F32(np.mean(dists)),
      avg_sparsity=F32(np.mean(sps)),
      step_size=step_size)
  return result, measurements, codes


def elias_gamma_sum_next(client_values):
  """EliasGammaEncodedSumFactory round: (int32 sum, avg_bitrate, codes)."""
  qs = [np.asarray(v, np.int32).reshape(-1) for v in client_values]
  acc = np.zeros(qs[0].size, np.int32)
  codes = []
  for q in qs:
    code, _ = codec.run_length_gamma_encode(q)
    codes.append(code)
    codec.decode_accumulate(code, acc)
  bits = [codec.get_bitstring_length(c) for c in codes]
  return acc, np.float64(np.mean(bits) / np.float64(qs[0].size)), codes


def stochastic_quantize_next(client_values, scale_factor, seeds):
  qs = [qu.stochastic_quantize(np.asarray(v, np.float32), scale_factor, tuple(s))
        for v, s in zip(client_values, seeds)]
  s = wrap_i32(np.sum(np.stack(qs).astype(np.int64), axis=0))
  return qu.uniform_dequantize(s, scale_factor), s


def one_bit_sgd_next(client_values, threshold=0.0):
  """OneBitSGDFactory round: (float32 result, measurements)."""
  xs = [np.asarray(v, np.float32).reshape(-1) for v in client_values]
  P = xs[0].size
  acc = np.zeros(P, np.float32)
  dists = []
  for x in xs:
    above = (x >= F32(threshold)).astype(np.float32)                        # :58-61
    below = F32(1.0) - above
    # :63-68: float32 reduce_sum (restated as the correctly rounded float32 of the
    # float64 sum) divided in float32 by the float32 count
    mb = F32(F32(np.sum(x * below, dtype=np.float64)) / F32(max(np.sum(below), 1.0)))
    ma = F32(F32(np.sum(x * above, dtype=np.float64)) / F32(max(np.sum(above), 1.0)))
    dec = (above * ma + (F32(1.0) - above) * mb).astype(np.float32)         # :45-54
    # :76-78
    dists.append(F32(np.sum((x - dec).astype(np.float64) ** 2) / P))
    acc = (acc + dec).astype(np.float32)                                     # :97-100
  return acc, collections.OrderedDict(avg_bitrate=F32((F32(P) + F32(64.0)) / F32(P)),
                                      avg_distortion=F32(np.mean(dists)))


def l2_norm(x):
  """tf.norm(value, ord=2) (qsgd.py:66): TF reduces in float32 in an unspecified
  order; restated as the correctly rounded float32 of a float64 sum (the HIP
  path's fc_client_norms does the same), so q can be compared bit-exactly."""
  x = qu.ftz(np.asarray(x, np.float32)).astype(np.float64)
  return F32(np.sqrt(np.sum(x * x)))


def qsgd_next(client_values, num_steps, seeds):
  """QSGDFactory round: (float32 result, measurements, codes)."""
  xs = [np.asarray(v, np.float32).reshape(-1) for v in client_values]
  P = xs[0].size
  acc = np.zeros(P, np.float32)                                              # :88-89
  dists, sps, lengths, codes = [], [], [], []
  for c, x in enumerate(xs):
    norm = l2_norm(x)                                                         # :66
    with np.errstate(divide="ignore", invalid="ignore"):
      step = F32(norm / F32(num_steps))                                       # :67
    q = qu.stochastic_quantize(x, step, tuple(seeds[c]))                      # :68-69
    deq = qu.uniform_dequantize(q, step)                                      # :70-71
    d = qu.ftz(x) - deq
    dists.append(F32(np.sum(d.astype(np.float64) ** 2) / P))                 # :72-74
    sps.append(F32((F32(P) - F32(np.count_nonzero(q))) / F32(P)))            # :75-77
    code, _ = codec.run_length_gamma_encode(q)                                # :78
    codes.append(code)
    lengths.append(np.float64(32.0 + 8.0 * len(code)))                        # :27-32
    acc = (acc + deq).astype(np.float32)                                      # :92-97 (client order)
  measurements = collections.OrderedDict(
      avg_bitrate=np.float64(np.mean(lengths) / np.float64(P)),              # :127-134
      avg_distortion=F32(np.mean(dists)),
      avg_sparsity=F32(np.mean(sps)))
  return acc, measurements, codes


def vote_step_size(x, options, lagrange_multiplier, rounding_type, seed):
  """quantize_encode_client_lambda.py:105-130 for one client: (one-hot int32, losses)."""
  x = np.asarray(x, np.float32).reshape(-1)
  P = x.size
  noise = qu.generate_noise(tuple(seed), P) if rounding_type == "dithered" else None
  losses = []
  for step in options:
    step = F32(step)
    q = _Q[rounding_type](x, step, tuple(seed))                                    # :114
    deq = (qu.dithered_dequantize(q, step, noise) if rounding_type == "dithered"
           else qu.uniform_dequantize(q, step))                                     # :115-116
    d = qu.ftz(x) - deq
    distortion = F32(F32(np.sum(d.astype(np.float64) ** 2)) / F32(P))              # :118-120
    code, _ = codec.run_length_gamma_encode(q)
    rate = F32(F32(codec.get_bitstring_length(code)) / F32(P))                      # :121-124
    losses.append(F32(distortion + F32(lagrange_multiplier) * rate))                # :126
  onehot = np.zeros(len(options), np.int32)
  onehot[int(np.argmin(losses))] = 1                                                # :129-130
  return onehot, np.array(losses, np.float32)


def client_lambda_next(client_values, lagrange_multiplier, step_size, options,
                       rounding_type="uniform", seeds=None, vote_seeds=None):
  """QuantizeEncodeClientLambdaFactory round: (result, measurements, next_step)."""
  xs = [np.asarray(v, np.float32).reshape(-1) for v in client_values]
  if seeds is None:
    seeds = [(c, c) for c in range(len(xs))]
  if vote_seeds is None:
    vote_seeds = seeds
  result, _, _ = quantize_encode_next(xs, step_size, rounding_type, seeds=seeds)    # :152-159
  counts = np.zeros(len(options), np.int32)
  for c, x in enumerate(xs):
    onehot, _ = vote_step_size(x, options, lagrange_multiplier, rounding_type, vote_seeds[c])
    counts += onehot                                                                # :161-162
  next_step = F32(np.asarray(options, np.float32)[int(np.argmax(counts))])           # :163-166
  measurements = collections.OrderedDict(step_size=F32(step_size), step_size_options=list(options),
                                         step_size_vote_counts=counts)
  return result, measurements, next_step


def drive_next(client_values, scaling_factor="unbiased"):
  """DRIVEFactory round: (float32 result, measurements)."""
  xs = [qu.ftz(np.asarray(v, np.float32).reshape(-1)) for v in client_values]
  P = xs[0].size
  acc = np.zeros(P, np.float32)
  dists = []
  for x in xs:
    neg = x < F32(0.0)                                                         # :59
    norm1 = F32(np.sum(np.abs(x).astype(np.float64)))
    if scaling_factor == "min_distortion":
      scale = F32(norm1 / F32(P))                                              # :61-62
    else:
      norm2 = F32(np.sqrt(np.sum(x.astype(np.float64) ** 2)))
      sq = F32(norm2 * norm2)
      scale = F32(0.0) if norm1 == 0 else F32(sq / norm1)                      # :63-65
    dec = np.where(neg, -scale, scale).astype(np.float32)                      # :48-56
    dists.append(F32(np.sum((x - dec).astype(np.float64) ** 2) / P))          # :69-70
    acc = (acc + dec).astype(np.float32)                                       # :88-90
  return acc, collections.OrderedDict(avg_bitrate=F32((F32(P) + F32(32.0)) / F32(P)),
                                      avg_distortion=F32(np.mean(dists)))


def rademacher(n, seed):
  """Signs of the rotation: bit 31 of the Philox stream of `seed` (element i ->
  output word i % 4 of counter i / 4), as fc_hadamard draws them."""
  from oracle import philox  # pylint: disable=g-import-not-at-top
  bits = philox.random_bits(n, tuple(seed))
  return np.where(bits >> 31, F32(-1.0), F32(1.0)).astype(np.float32)


def fwht(x):
  """Unnormalised fast Walsh-Hadamard transform (float64) of a power-of-two vector."""
  y = np.asarray(x, np.float64).copy()
  h = 1
  while h < y.size:
    y = y.reshape(-1, 2, h)
    y = np.stack([y[:, 0] + y[:, 1], y[:, 0] - y[:, 1]], axis=1).reshape(-1)
    h *= 2
  return y


def hadamard_forward(x, seed):
  x = np.asarray(x, np.float32).reshape(-1)
  n = 1 << max(0, (x.size - 1).bit_length())
  v = np.zeros(n, np.float32)
  v[:x.size] = x
  return fwht(v * rademacher(n, seed)) / np.sqrt(n)


def hadamard_inverse(y, seed, P):
  n = y.size
  return (fwht(y) / np.sqrt(n) * rademacher(n, seed))[:P]


def dft_forward(x, seed):
  """DiscreteFourierTransformFactory's rotation as restated (builder.py:70-71; TFF's
  own real/imaginary pairing unpinned): zero-pad to even n, signs D, then the unitary
  DFT of the n/2 complex numbers x[:n/2] + i x[n/2:], (real, imaginary) halves."""
  x = np.asarray(x, np.float32).reshape(-1)
  n = x.size + (x.size % 2)
  v = np.zeros(n, np.float64)
  v[:x.size] = x
  v *= rademacher(n, seed)
  h = n // 2
  z = np.fft.fft(v[:h] + 1j * v[h:], norm="ortho")
  return np.concatenate([z.real, z.imag])


def dft_inverse(y, seed, P):
  y = np.asarray(y, np.float64).reshape(-1)
  h = y.size // 2
  z = np.fft.ifft(y[:h] + 1j * y[h:], norm="ortho")
  return (np.concatenate([z.real, z.imag]) * rademacher(y.size, seed))[:P]


# --- the trainer's aggregator across rounds (VERDICT r05 "next" 6) -------------------------------
def quantile_update(estimate, norms, target_quantile, learning_rate):
  """``PrivateQuantileEstimationProcess.no_noise`` (tensorflow_privacy's
  ``QuantileEstimatorQuery`` without noise, geometric update; builder.py:104-117):
  the fraction of clients whose norm is <= the raw estimate X moves X by
  X * exp(-lr * (fraction - target)).  TFF is absent: parity unpinned."""
  below = F32(np.mean((np.asarray(norms, np.float32) <= F32(estimate)).astype(np.float32)))
  return F32(F32(estimate) * np.exp(-F32(learning_rate) * (below - F32(target_quantile))))


def trainer_aggregator_init(step_size):
  """The initial state of build_quantization_encode_aggregator's process
  (builder.py:104-117 initial estimates; quantize_encode.py:161-166)."""
  return collections.OrderedDict(zeroing_norm=F32(10.0), clipping_norm=F32(1.0), round_num=F32(0.0),
                                 step_size=F32(step_size))


def trainer_aggregator_next(state, client_values, weights, seeds, rounding_type, schedule_fn):
  """One round of ``build_quantization_encode_aggregator`` (builder.py:453-525) with
  the wrappers of ``configure_aggregator`` (builder.py:100-117) in their order:
  zeroing (a client whose max |x| > 2 X + 1 contributes zeros), clipping
  (``tf.clip_by_global_norm`` to C: scale C * min(1 / ||x||, 1 / C)), the weighted
  mean (value * weight summed by QuantizeEncodeFactory, / sum(weight)), then the
  estimates' and the codec's next state (quantize_encode.py:192-201:
  round_num + 1, step = schedule(round_num + 1)).  Returns (result, measurements,
  next_state)."""
  xs = [qu.ftz(np.asarray(v, np.float32).reshape(-1)) for v in client_values]
  w = np.asarray(weights, np.float32)
  linf = np.array([np.max(np.abs(x)) for x in xs], np.float32)
  zero_thr = F32(F32(state["zeroing_norm"]) * F32(2.0) + F32(1.0))
  keep = ~(linf > zero_thr)
  l2 = np.array([np.sqrt(np.sum(x.astype(np.float64) ** 2)) for x in xs], np.float32)
  l2 = np.where(keep, l2, F32(0.0)).astype(np.float32)
  clip = F32(state["clipping_norm"])
  with np.errstate(divide="ignore"):
    inv = np.where(l2 > 0, F32(1.0) / l2, np.float32(np.inf)).astype(np.float32)
  scale = np.where(keep, clip * np.minimum(inv, F32(1.0) / clip), F32(0.0)).astype(np.float32)
  pre = [((x * scale[c]) * w[c]).astype(np.float32) for c, x in enumerate(xs)]
  res, meas, _ = quantize_encode_next(pre, state["step_size"], rounding_type, seeds=seeds)
  denom = F32(np.sum(w, dtype=np.float32))
  res = (res / denom).astype(np.float32) if denom != 0 else np.zeros_like(res)
  nr = F32(state["round_num"] + F32(1.0))
  nxt = collections.OrderedDict(
      zeroing_norm=quantile_update(state["zeroing_norm"], linf, 0.98, np.log(10.0)),
      clipping_norm=quantile_update(state["clipping_norm"], l2, 0.8, 0.2),
      round_num=nr, step_size=F32(schedule_fn(nr)))
  measurements = collections.OrderedDict(zeroing_norm=zero_thr, clipping_norm=clip, mean_value=meas)
  return res, measurements, nxt
