"""CPU oracle for the compressed_communication client-update codec.

TEST INFRASTRUCTURE ONLY.  Nothing under ``oracle/`` is part of the product
path.  Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s
``cpu_baseline`` leg may import it, and only as the checker (or as the timed
CPU restatement of the reference semantics), never as the thing measured on
the GPU.  The product package ``federated_amd`` must never import it.

Contents (each function cites the reference file:line it restates):

* ``philox``          TF ``stateless_random_uniform`` (Philox4x32-10, TF seed
                      scramble, ``Uint32ToFloat``) -- external TF semantics.
* ``quantize_utils``  ``compressed_communication/aggregators/utils/quantize_utils.py``
                      with TF-CPU numerics (FTZ/DAZ, round-half-even, x86
                      float->int32 conversion).
* ``codec``           ctypes binding of ``rlgamma.c``: tensorflow-compression's
                      ``run_length_gamma_encode/decode`` restated in C
                      (single-threaded scalar bit writer/reader per client).
* ``aggregators``     ``QuantizeEncodeFactory.next`` / ``EliasGammaEncodedSumFactory``
                      / ``StochasticQuantizeFactory`` / ``OneBitSGDFactory`` round
                      semantics in numpy + the C codec.

Parity pinning (see DESIGN.md "Oracle"):

* pinned by the reference's own known-answer tests (bit lengths, byte rounding,
  quantised values, schedules, 1-bit codec values) and by the Random123
  Philox4x32-10 known-answer vectors;
* **parity unpinned** for: TF's seed->(key, counter) scramble and
  ``Uint32ToFloat`` (restated from upstream TF, not present in this image),
  and the tensorflow-compression bit order inside bytes (restated as classic
  MSB-first Elias gamma, sign bit 1 = positive).  Lengths and round trips are
  pinned; byte images are not.
"""
