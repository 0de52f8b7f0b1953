"""The trainer's aggregator across rounds (VERDICT r05 "next" 6).

The reference drives its aggregator with ``tff.simulation.run_training_process``
(trainer.py:345-354): every round's state feeds the next -- the codec's round
number and step schedule (quantize_encode.py:192-201) and the adaptive clipping and
zeroing estimates (builder.py:104-117) -- and the program state is checkpointed
every ``rounds_per_checkpoint`` rounds (trainer.py:108; utils/training_utils.py:
26-55).  Here R = 6 rounds of ``build_quantization_encode_aggregator`` with an
exponentially decaying stochastic step, clipping, zeroing and client weights run
on the HIP path, against ``oracle.aggregators.trainer_aggregator_next`` chained
over the same rounds: each round's result bit for bit, its measurements, and the
next state.  After round 3 the state is saved with ``FileProgramStateManager``
(the checkpoint stand-in), a NEW process is built from a new factory and loaded
from the file, and the remaining rounds continue from it.
"""
import numpy as np
import pytest

from federated_amd import builder
from federated_amd import tff_compat as tc
from oracle import aggregators as oagg
from oracle import quantize_utils as oq

pytestmark = pytest.mark.gpu

F32 = np.float32
R, C, P = 6, 12, 200_003
STEP0, MIN_STEP, HPARAM = 0.5, 0.05, 0.25


def _round_inputs(r):
  rng = np.random.default_rng(1000 + r)
  # norms straddling the clipping estimate (l2 ~ 0.3 .. 3), example-count weights
  xs = [(rng.standard_normal(P) * (rng.uniform(0.3, 3.0) / np.sqrt(P))).astype(np.float32) for _ in range(C)]
  if r % 2 == 0:
    xs[r % C] = (xs[r % C] * F32(1e4)).astype(np.float32)  # max |x| far above 2 X + 1: zeroed
  w = rng.integers(50, 500, C).astype(np.float32)
  seeds = np.array([[7919 * r + c, 31 * c + r] for c in range(C)], np.int64)
  return xs, w, seeds


def _factory():
  return builder.build_quantization_encode_aggregator(
      step_size=STEP0, rounding_type="stochastic", step_size_sched="exponential_decay",
      step_size_sched_hparam=HPARAM, min_step_size=MIN_STEP)


def _sched(nr):
  return oq.exponential_decay(STEP0, MIN_STEP, nr, HPARAM)


def test_round_chain_with_checkpoint(gpu, tmp_path):
  process = _factory().create((np.float32, (P,)), (np.float32, ()))
  state = process.initialize()
  ostate = oagg.trainer_aggregator_init(STEP0)
  manager = tc.FileProgramStateManager(str(tmp_path / "checkpoints"))
  zeroed_rounds = 0
  for r in range(R):
    xs, w, seeds = _round_inputs(r)
    out = process.next(state, xs, weight=w, seeds=seeds)
    want, wmeas, onext = oagg.trainer_aggregator_next(ostate, xs, w, seeds, "stochastic", _sched)
    np.testing.assert_array_equal(out.result, want)
    m = out.measurements
    assert m["zeroing_norm"] == wmeas["zeroing_norm"] and m["clipping_norm"] == wmeas["clipping_norm"]
    mv, wv = m["mean_value"], wmeas["mean_value"]
    assert mv["avg_bitrate"] == wv["avg_bitrate"] and mv["avg_sparsity"] == wv["avg_sparsity"]
    assert mv["step_size"] == wv["step_size"] == ostate["step_size"]
    np.testing.assert_allclose(mv["avg_distortion"], wv["avg_distortion"], rtol=1e-5)
    st = out.state
    assert st["zeroing_norm"] == onext["zeroing_norm"] and st["clipping_norm"] == onext["clipping_norm"]
    assert st["inner_state"]["round_num"] == onext["round_num"] == F32(r + 1)
    assert st["inner_state"]["step_size"] == onext["step_size"]
    zeroed_rounds += int(np.max(np.abs(xs[r % C])) > wmeas["zeroing_norm"])
    state, ostate = st, onext
    if r == 2:  # checkpoint, then continue in a new process object from the file
      manager.save(state, r + 1)
      process = _factory().create((np.float32, (P,)), (np.float32, ()))
      state, version = manager.load_latest(process.initialize())
      assert version == 3
      assert state["inner_state"]["round_num"] == F32(3.0)
      assert state["clipping_norm"] == ostate["clipping_norm"]
  assert zeroed_rounds >= 2  # the zeroing path ran
  assert ostate["step_size"] < F32(STEP0)  # the schedule decayed
