/* fedcodec: MI355X-native client-update codec for compressed_communication/.
 *
 * C ABI of libfedcodec.so (federated_amd/csrc/fedcodec.hip, gfx950 only).
 * Plain pointers and sizes; every device pointer is caller-owned HBM; every
 * entry is asynchronous on the given hipStream_t (passed as void*).  Two
 * library-owned exceptions, both outside steady state: fc_client_norms(_scaled),
 * fc_onebit_encode and fc_drive_encode keep a small grow-only partials buffer per
 * (device, stream), allocated on the first call of a size (a call under graph
 * capture that would have to grow it fails with -1: warm it uncaptured); the
 * encoders write their look-back spin limit (a device global) on the first call
 * per device.  Return 0 on success, a negative code on a rejected argument
 * (message from fc_last_error(), thread-local); no C++ exception crosses the ABI.
 *
 * Reference interfaces replaced (file:line under google-research/federated):
 *   fc_quantize            quantize_utils.uniform_quantize / stochastic_quantize /
 *                          dithered_quantize (+ generate_noise)
 *                          aggregators/utils/quantize_utils.py:33-36, 46-53, 57-66
 *   fc_dequantize          quantize_utils.uniform_dequantize / dithered_dequantize
 *                          quantize_utils.py:39-42, 69-84; QuantizeEncodeFactory
 *                          server `dequantize` aggregators/quantize_encode.py:169-171
 *   fc_quantize_encode     QuantizeEncodeFactory client `quantize` tf_computation
 *                          quantize_encode.py:139-156 fused with
 *                          tfc.run_length_gamma_encode (elias_gamma_encode.py:97-99),
 *                          batched over a round's clients
 *   fc_rlgamma_encode      tfc.run_length_gamma_encode(int32) (elias_gamma_encode.py:98)
 *   fc_decode_accumulate   EliasGammaEncodedSumFactory federated_aggregate
 *                          accumulate/merge (elias_gamma_encode.py:63-88) =
 *                          tfc.run_length_gamma_decode + int32 sum, optionally fused
 *                          with the server dequantize (quantize_encode.py:189-190)
 *   fc_decode_accumulate_scaled  QSGDFactory sum_encoded_value accumulate
 *                          (comparison_methods/qsgd.py:85-112): decode + per-client
 *                          dequantize(norm / num_steps) + float32 sum
 *   fc_vote_lengths        QuantizeEncodeClientLambdaFactory vote_step_size: per
 *                          option quantize + dequantize distortion + code length
 *                          (quantize_encode_client_lambda.py:105-130), lengths only
 *   fc_noise_sum           federated_sum(noise) for dithered mode (quantize_encode.py:183)
 *   fc_client_norms(_scaled) normalize_fn: mean_magnitude / max_magnitude /
 *                          dimensionless_norm (quantize_utils.py:20-29,
 *                          quantize_encode.py:79-90, 145); the clipping / zeroing
 *                          wrapper norms of builder.py:100-117 (one fused pass)
 *   fc_finalize            avg_distortion / avg_sparsity / bit lengths per client
 *                          (quantize_encode.py:150-155, elias_gamma_encode.py:22-24, 100-108)
 *   fc_drive_encode        DRIVEFactory encode (comparison_methods/drive.py:58-76); its
 *                          server sum is fc_onebit_decode_sum with (-scale, +scale)
 *   fc_hadamard            tff.aggregators.HadamardTransformFactory rotation that
 *                          builder.py:68-71 wraps around a codec (randomized FWHT)
 *   fc_dft_rotate          tff.aggregators.DiscreteFourierTransformFactory rotation
 *                          (builder.py:70-71): sign flip + unitary DFT (Stockham /
 *                          Bluestein FFT)
 *   fc_onebit_encode/_decode_sum  OneBitSGDFactory encode/decode_and_sum
 *                          (comparison_methods/one_bit_sgd.py:45-81, 87-112)
 *
 * Bitstream layout (per client): tensorflow-compression run-length gamma
 * (protocol at elias_gamma_encode.py:30-45), MSB-first within bytes, sign bit 1
 * = positive; byte length = ceil(bits / 8), last byte zero padded.
 */
#ifndef FEDCODEC_H_
#define FEDCODEC_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Rounding modes (QuantizeEncodeFactory rounding_type, quantize_encode.py:92-107). */
#define FC_UNIFORM 0
#define FC_STOCHASTIC 1
#define FC_DITHERED 2

/* Normalisations (quantize_encode.py:79-90). */
#define FC_NORM_MEAN_MAGNITUDE 1
#define FC_NORM_MAX_MAGNITUDE 2
#define FC_NORM_DIMENSIONLESS 3
/* Norms of the TFF wrappers restated by the builder (builder.py:104-117). */
#define FC_NORM_L2 4   /* tf.linalg.global_norm: clipping_factory */
#define FC_NORM_LINF 5 /* max |x|: zeroing_factory (norm_order=inf) */
#define FC_NORM_L2_LINF 6 /* both wrapper norms in one pass: norms[c] = L2, norms[nclients + c] = LINF */

#define FC_TILE_ELEMS 1024       /* encoder tile (one wavefront) = decoder index granularity */
#define FC_MAX_ELEMS 1006632960LL    /* P limit: 2^30 - 2^26 elements per client tensor -- every code
                                        then fits the decoder index's 36-bit bit offsets (<= 65 bits
                                        per element).  The index holds 1 + the last nonzero modulo
                                        2^28: a reader recovers it from the unit it decodes (the
                                        first code's nonzero lies in that unit) */
#define FC_MAX_ROW_ELEMS 67108863LL  /* one encoder row (26-bit positions in the look-back status):
                                        fc_quantize_encode(_hinted / _quarters) and fc_rlgamma_encode
                                        take P <= 2^26 - 1; fc_quantize_encode_segmented cuts longer
                                        tensors into rows of at most this many elements */

/* overflow[] flags of the encoders. */
#define FC_OVERFLOW_CAPACITY 1
#define FC_OVERFLOW_STALL 2

const char* fc_last_error(void);
const char* fc_version(void);

/* Number of encoder tiles for P elements: ceil(P / FC_TILE_ELEMS). */
int64_t fc_num_tiles(int64_t P);

/* Host copy of the decoder's compile-time tables (diagnostics and CPU tests; no
 * GPU call): lut[i] = the up-to-two codes the 12 window bits i begin, glut[i] =
 * the structure of the one code they begin (k_decode's layouts; the decode of
 * tfc.run_length_gamma_decode, elias_gamma_encode.py:71-72).  n = entries the
 * buffers hold; returns the table size (4096), or -1 when n is smaller. */
int32_t fc_decode_tables(uint32_t* lut, uint16_t* glut, int32_t n);

/* Device workspace bytes fc_quantize_encode / fc_rlgamma_encode need for a batch
 * of `nclients` clients of P elements each.  16-byte aligned pointer required. */
int64_t fc_encode_workspace_bytes(int32_t nclients, int64_t P);

/* Elementwise quantiser of one tensor: q[i] from x[i] (and noise[i] when
 * noise != NULL; dithered/stochastic draw the TF stateless_uniform stream of
 * `seed`).  step is the already-normalised step size. */
int fc_quantize(const float* x, int64_t P, float step, int64_t seed0, int64_t seed1,
                int mode, int32_t* q, float* noise, void* stream);

/* Fused client-side quantise + run-length-gamma encode for a batch of clients.
 *   xs          device array of nclients device pointers to float32[P]
 *   norms       nullable device float[nclients]: client step = norms[c] * step
 *   prescale    nullable device float[2 * nclients]: x -> (x * prescale[2c]) *
 *               prescale[2c+1] before quantising (the TFF clipping_factory scale,
 *               then the MeanFactory client weight; builder.py:100-109)
 *   seeds       device int64[2 * nclients] (TF stateless seed per client)
 *   stream_buf  device byte buffer; client c's code starts at stream_off[c]
 *               (16-byte aligned) with room for stream_cap[c] bytes
 *   idx         device uint64[nclients * (fc_num_tiles(P) + 1)]: decoder index
 *   total_bits  device int64[nclients]: exact code length in bits
 *   dist_part   device float[nclients * tiles]: per-tile sum (x - deq)^2
 *   nnz_part    device int32[nclients * tiles]: per-tile nonzero count
 *   overflow    device int32[nclients], bit flags (zeroed by the call):
 *               FC_OVERFLOW_CAPACITY when stream_cap[c] is too small (the code is
 *               then incomplete; total_bits is still exact); FC_OVERFLOW_STALL when
 *               a look-back of this launch hit its spin limit and client c was
 *               re-encoded on the exact path (the code is complete and exact; the
 *               flag reports lost progress, DESIGN.md §2 "Ticket streams")
 * Bit-exact on q and on the bitstream vs the oracle's restatement. */
int fc_quantize_encode(const float* const* xs, int32_t nclients, int64_t P, float step,
                       const float* norms, const float* prescale, const int64_t* seeds, int mode,
                       uint8_t* stream_buf, const int64_t* stream_off,
                       const int64_t* stream_cap, uint64_t* idx, int64_t* total_bits,
                       float* dist_part, int32_t* nnz_part, int32_t* overflow,
                       void* workspace, int64_t workspace_bytes, void* stream);

/* fc_quantize_encode with a host-side hint: max_cap = the largest stream_cap[c]
 * (bytes; <= 0 unknown).  Same results bit for bit; the hint picks the encoder's
 * ticket size: codes expected within 6.5 bits per element take four-tile
 * tickets (per-ticket work and look-back once per 4096 elements), denser or
 * unknown ones two (a four-tile window overflow is correct but slow: the client
 * goes to the exact path). */
int fc_quantize_encode_hinted(const float* const* xs, int32_t nclients, int64_t P, float step,
                              const float* norms, const float* prescale, const int64_t* seeds,
                              int mode, uint8_t* stream_buf, const int64_t* stream_off,
                              const int64_t* stream_cap, uint64_t* idx, int64_t* total_bits,
                              float* dist_part, int32_t* nnz_part, int32_t* overflow,
                              void* workspace, int64_t workspace_bytes, int64_t max_cap,
                              void* stream);

/* Segmented quantise + encode (few clients per GPU; same results as
 * fc_quantize_encode, bit for bit).  Each client is cut into nseg element
 * segments (a multiple of 2048 elements each, plus a remainder) encoded as
 * independent rows -- each continuing its client's Philox stream -- then
 * stitched into the client's canonical stream (first run codes rebased on the
 * client's previous nonzero, per-segment trailing codes dropped, bits moved),
 * with the decoder index and the measurement partials rebased.  max_cap: the
 * largest stream_cap (sizes the segments' staging).  Workspace:
 * fc_segmented_workspace_bytes (256-byte aligned); -1 there means the
 * segmentation is not possible (segments under 2048 elements).  Replaces the
 * same reference call as fc_quantize_encode (quantize_encode.py:139-156 +
 * elias_gamma_encode.py:97-99). */
int64_t fc_segmented_workspace_bytes(int32_t nclients, int64_t P, int32_t nseg, int64_t max_cap);
int fc_quantize_encode_segmented(const float* const* xs, int32_t nclients, int64_t P, float step,
                                 const float* norms, const float* prescale, const int64_t* seeds,
                                 int mode, int32_t nseg, int64_t max_cap, uint8_t* stream_buf,
                                 const int64_t* stream_off, const int64_t* stream_cap, uint64_t* idx,
                                 int64_t* total_bits, float* dist_part, int32_t* nnz_part,
                                 int32_t* overflow, void* workspace, int64_t workspace_bytes,
                                 void* stream);

/* fc_quantize_encode_segmented with the stitch on a second stream: the segments'
 * encode and the plan (total_bits, overflow) run on `stream`; the bit moves into
 * the canonical streams, the canonical idx and the per-tile partials on
 * `stitch_stream` (ordered after the plan; the caller joins it before reading
 * stream_buf, idx, dist_part or nnz_part).  Meanwhile
 * fc_decode_accumulate_segmented can decode the unstitched segments on `stream`
 * from the same workspace (kept unchanged until both are done).  stitch_stream ==
 * stream or NULL: exactly fc_quantize_encode_segmented. */
int fc_quantize_encode_segmented_split(const float* const* xs, int32_t nclients, int64_t P, float step,
                                       const float* norms, const float* prescale, const int64_t* seeds,
                                       int mode, int32_t nseg, int64_t max_cap, uint8_t* stream_buf,
                                       const int64_t* stream_off, const int64_t* stream_cap,
                                       uint64_t* idx, int64_t* total_bits, float* dist_part,
                                       int32_t* nnz_part, int32_t* overflow, void* workspace,
                                       int64_t workspace_bytes, void* stream, void* stitch_stream);

/* Decode + client sum of a segmented batch straight from its segments (the
 * workspace of the fc_quantize_encode_segmented(_split) call that made them, same
 * nclients / P / nseg / max_cap): each segment's code and index are the client's
 * code and index for its element range, so the results equal
 * fc_decode_accumulate_tiles on the stitched batch bit for bit.  Tile range and
 * err as fc_decode_accumulate_tiles (err is OR'ed into). */
int fc_decode_accumulate_segmented(const void* workspace, int64_t workspace_bytes, int32_t nclients,
                                   int64_t P, int32_t nseg, int64_t max_cap, int32_t tile_begin,
                                   int32_t tile_end, const int32_t* sum_in, int32_t* sum_out,
                                   float* out, float step, const float* noise_sum, int32_t* err,
                                   void* stream);

/* fc_quantize_encode plus a quarter-tile decoder index: idxq = device
 * uint64[nclients * fc_num_tiles(P) * 3], entry 3 (c * tiles + t) + s - 1 = the
 * decoder entry (bit offset | 1 + last nonzero before, << 36) of elements
 * [1024 t + 256 s, ...) for s = 1..3.  Same codes, index and measurements bit for
 * bit; the extra entries let fc_decode_accumulate_quarters run four lane segments
 * per tile and client (few clients with dense codes: each segment's serial decode
 * chain, not memory, bounds the decoder).  Replaces the same reference call as
 * fc_quantize_encode (quantize_encode.py:139-156 + elias_gamma_encode.py:97-99). */
int fc_quantize_encode_quarters(const float* const* xs, int32_t nclients, int64_t P, float step,
                                const float* norms, const float* prescale, const int64_t* seeds,
                                int mode, uint8_t* stream_buf, const int64_t* stream_off,
                                const int64_t* stream_cap, uint64_t* idx, uint64_t* idxq,
                                int64_t* total_bits, float* dist_part, int32_t* nnz_part,
                                int32_t* overflow, void* workspace, int64_t workspace_bytes,
                                void* stream);

/* tfc.run_length_gamma_encode over int32 inputs (same batch layout as above,
 * qs = device array of device pointers to int32[P]). */
int fc_rlgamma_encode(const int32_t* const* qs, int32_t nclients, int64_t P,
                      uint8_t* stream_buf, const int64_t* stream_off,
                      const int64_t* stream_cap, uint64_t* idx, int64_t* total_bits,
                      int32_t* overflow, void* workspace, int64_t workspace_bytes,
                      void* stream);

/* fc_rlgamma_encode of tensors longer than one encoder row (P up to
 * FC_MAX_ELEMS): nseg segments per client (each at most FC_MAX_ROW_ELEMS and at
 * least 2048 elements) encoded as rows and stitched into each client's one canonical
 * code -- byte-identical to coding the tensor in one piece.  Workspace:
 * fc_segmented_workspace_bytes(nclients, P, nseg, max_cap), 256-byte aligned. */
int fc_rlgamma_encode_segmented(const int32_t* const* qs, int32_t nclients, int64_t P, int32_t nseg, int64_t max_cap,
                                uint8_t* stream_buf, const int64_t* stream_off, const int64_t* stream_cap, uint64_t* idx,
                                int64_t* total_bits, int32_t* overflow, void* workspace, int64_t workspace_bytes,
                                void* stream);

/* Decode nclients codes (layout as produced above) and sum them over clients.
 *   sum_in     nullable int32[P]: running sum to add to (multi-batch rounds)
 *   sum_out    nullable int32[P]: integer client sum (RCCL all-reduce input)
 *   out        nullable float[P]: dequantised sum (float(sum) [+ noise_sum]) * step
 *   noise_sum  nullable float[P] (dithered)
 *   err        device int32[1]: set nonzero on a malformed stream */
int fc_decode_accumulate(const uint8_t* stream_buf, const int64_t* stream_off,
                         const int64_t* stream_cap, const uint64_t* idx, int32_t nclients,
                         int64_t P, const int32_t* sum_in, int32_t* sum_out, float* out,
                         float step, const float* noise_sum, int32_t* err, void* stream);

/* Decoder index of BARE run-length gamma codes: the reference server decodes a
 * client's message with tfc.run_length_gamma_decode(code, shape) -- the byte
 * string alone (elias_gamma_encode.py:69-73; the client message is that single
 * tf.string, :97-109) -- so codes from a stock TFC client come without the
 * encoder's index.  fc_build_index rebuilds it on the device from the bytes:
 * idx (and, when idxq != NULL, the quarter index of fc_quantize_encode_quarters)
 * and total_bits, bit for bit what the encoder writes, after which
 * fc_decode_accumulate(_tiles / _quarters) decode the batch as usual.
 *   stream_off  device int64[nclients]: client c's code at stream_buf + stream_off[c]
 *               (16-byte aligned; readable up to the next 16-byte boundary past its end)
 *   nbytes      device int64[nclients]: each code's byte length (the tf.string's length)
 *   max_bytes   host: >= every nbytes[c] (sizes the work; fc_index_workspace_bytes)
 *   err         device int32[1]: cleared, then set nonzero on a malformed code (a code
 *               that does not parse, holds more or fewer than P elements, or whose
 *               byte length is not ceil(bits / 8))
 * Each lane parses a chunk of a code (2048, 4096 or 8192 bits, chosen from nclients
 * and max_bytes) from a guessed start; the parses resynchronise within a few codes
 * and are stitched.  The workspace size depends on the same choice:
 * take it from fc_index_workspace_bytes with the same nclients and max_bytes. */
int64_t fc_index_workspace_bytes(int32_t nclients, int64_t max_bytes);
int fc_build_index(const uint8_t* stream_buf, const int64_t* stream_off, const int64_t* nbytes, int32_t nclients,
                   int64_t P, int64_t max_bytes, uint64_t* idx, uint64_t* idxq, int64_t* total_bits, int32_t* err,
                   void* workspace, int64_t workspace_bytes, void* stream);

/* fc_decode_accumulate restricted to tiles [tile_begin, tile_end) of 1024
 * elements: only elements [1024 * tile_begin, min(P, 1024 * tile_end)) of
 * sum_out / out are written.  err is OR'ed into, not cleared (zero it before the
 * first range).  Lets a multi-GPU round all-reduce finished tile ranges while
 * later ranges decode (same accumulate/merge as fc_decode_accumulate). */
int fc_decode_accumulate_tiles(const uint8_t* stream_buf, const int64_t* stream_off,
                               const int64_t* stream_cap, const uint64_t* idx, int32_t nclients,
                               int64_t P, int32_t tile_begin, int32_t tile_end,
                               const int32_t* sum_in, int32_t* sum_out, float* out, float step,
                               const float* noise_sum, int32_t* err, void* stream);

/* fc_decode_accumulate_tiles over a batch encoded with fc_quantize_encode_quarters:
 * lane segments of 256 elements (entries from idxq).  Same results bit for bit;
 * err is OR'ed into, not cleared.  Replaces elias_gamma_encode.py:118-120's decode
 * + the int32 sum (quantize_encode.py:169-171) like fc_decode_accumulate. */
int fc_decode_accumulate_quarters(const uint8_t* stream_buf, const int64_t* stream_off,
                                  const int64_t* stream_cap, const uint64_t* idx,
                                  const uint64_t* idxq, int32_t nclients, int64_t P,
                                  int32_t tile_begin, int32_t tile_end, const int32_t* sum_in,
                                  int32_t* sum_out, float* out, float step, const float* noise_sum,
                                  int32_t* err, void* stream);

/* QSGD server side (qsgd.py:85-112 sum_encoded_value): acc = fsum_in[i] (or 0),
 * then acc = acc + float(q_c[i]) * client_scale[c] for c = 0 .. nclients-1 in
 * order, float32 -- the reference's client-order sum, deterministic and bit for
 * bit.  The clients are decoded in groups into int32 q rows in `workspace`
 * (16-byte aligned; fc_decode_scaled_workspace_bytes gives the size for groups of
 * up to 1 GiB of rows, at least one client row is required). */
int64_t fc_decode_scaled_workspace_bytes(int32_t nclients, int64_t P);
int fc_decode_accumulate_scaled(const uint8_t* stream_buf, const int64_t* stream_off,
                                const int64_t* stream_cap, const uint64_t* idx, int32_t nclients,
                                int64_t P, const float* client_scale, const float* fsum_in,
                                float* out, int32_t* err, void* workspace, int64_t workspace_bytes,
                                void* stream);

/* fc_decode_accumulate_scaled with a caller-guaranteed bound qmax on every |q|
 * (QSGD: num_steps + 1, since |x| <= ||x||_2).  qmax in [1, 127]: the client q rows
 * are int8 (a quarter of the rows' memset / write / read traffic; a decoded value
 * beyond 127 sets err); otherwise (qmax <= 0 or > 127) exactly
 * fc_decode_accumulate_scaled.  Same float32 client-order sum bit for bit. */
int fc_decode_accumulate_scaled_bounded(const uint8_t* stream_buf, const int64_t* stream_off,
                                        const int64_t* stream_cap, const uint64_t* idx,
                                        int32_t nclients, int64_t P, const float* client_scale,
                                        const float* fsum_in, float* out, int32_t* err, int32_t qmax,
                                        void* workspace, int64_t workspace_bytes, void* stream);

/* Step-size vote: for each client c and option k (steps = device float[K]),
 * bits[c*K + k] = exact run-length-gamma code length (bits) of quantizing x_c
 * with steps[k] (rounding `mode`, TF stream of seeds[c], the same draw for every
 * option) and dist[c*K + k] = sum (x - dequantize(q))^2 (float64 accumulation
 * of float32 tile partials).  Nothing is packed. */
int64_t fc_vote_workspace_bytes(int32_t nclients, int64_t P, int32_t K);
int fc_vote_lengths(const float* const* xs, int32_t nclients, int64_t P, const float* steps,
                    int32_t K, const int64_t* seeds, int mode, int64_t* bits, double* dist,
                    void* workspace, int64_t workspace_bytes, void* stream);

/* out = (float(sum) [+ noise_sum]) * step (FTZ as TF-CPU). */
int fc_dequantize(const int32_t* sum, int64_t P, float step, const float* noise_sum,
                  float* out, void* stream);

/* noise_sum[i] = sum over clients (in client order, float32) of the dither noise
 * TF's generate_noise(seed_c) draws for element i. */
int fc_noise_sum(const int64_t* seeds, int32_t nclients, int64_t P, float* noise_sum,
                 void* stream);

/* norms[c] = normalize_fn(x_c) (or the wrapper norms) as float32, kind in FC_NORM_*;
 * float64 accumulation in a fixed order.  nclients <= 65535.  With few clients each
 * client's row is split over several workgroups (about two per CU in all), whose
 * float64 partials a second kernel adds in order; the partials live in a small
 * library-owned device buffer per (device, stream). */
int fc_client_norms(const float* const* xs, int32_t nclients, int64_t P, int kind,
                    float* norms, void* stream);

/* fc_client_norms of the pre-scaled values (x * prescale[2c]) * prescale[2c+1]
 * (prescale nullable, the same per-client pre-scales fc_quantize_encode takes):
 * QuantizeEncode's normalize_fn sees the value after the TFF clipping and mean
 * wrappers (builder.py:100-109 around quantize_encode.py:145).  kind
 * FC_NORM_L2_LINF writes 2 * nclients floats. */
int fc_client_norms_scaled(const float* const* xs, int32_t nclients, int64_t P, int kind,
                           const float* prescale, float* norms, void* stream);

/* Per-client reduction of the encoder's per-tile partials:
 * dist[c] = sum_t dist_part (float64), nnz[c] = sum_t nnz_part (int64). */
int fc_finalize(const float* dist_part, const int32_t* nnz_part, int32_t nclients, int64_t P,
                double* dist, int64_t* nnz, void* stream);

/* One-bit SGD (comparison_methods/one_bit_sgd.py): per client the above/below
 * threshold masks (bit-packed, 1 = x >= threshold), the two means and the
 * distortion; decode_sum adds every client's decoded tensor in client order.
 * nclients <= 65535; rows split over workgroups as fc_client_norms (fc_drive_encode too). */
int fc_onebit_encode(const float* const* xs, int32_t nclients, int64_t P, float threshold,
                     uint32_t* masks, float* means, double* dist, void* stream);
int fc_onebit_decode_sum(const uint32_t* masks, const float* means, int32_t nclients,
                         int64_t P, float* out, void* stream);
/* The same over mask words [word_begin, word_end) only (elements 32 word_begin ..
 * min(P, 32 word_end)): the multi-GPU round sums one element range while the
 * previous range's float32 all-reduce runs (one_bit_sgd.py:87-112 per range). */
int fc_onebit_decode_sum_range(const uint32_t* masks, const float* means, int32_t nclients,
                               int64_t P, int64_t word_begin, int64_t word_end, float* out,
                               void* stream);

/* DRIVE: masks bit set = x >= 0 (not negative), means[2c] = -scale, means[2c+1] =
 * +scale with scale = ||x||_2^2 / ||x||_1 (min_distortion = 0, divide_no_nan) or
 * ||x||_1 / P (min_distortion = 1), dist[c] = sum (x - decode)^2. */
int fc_drive_encode(const float* const* xs, int32_t nclients, int64_t P, int min_distortion,
                    uint32_t* masks, float* means, double* dist, void* stream);

/* In-place randomized Hadamard transform of nclients rows of n = 2^k floats:
 * forward y = H D x / sqrt(n), inverse (inverse = 1) x = D H y / sqrt(n), with D
 * the Rademacher signs of the Philox stream of (seed0, seed1). */
int fc_hadamard(float* const* rows, int32_t nclients, int64_t n, int inverse, int64_t seed0,
                int64_t seed1, void* stream);

/* In place x *= D for nclients rows of n floats, D the Rademacher signs of the
 * Philox stream of (seed0, seed1) (the stream fc_hadamard uses): the sign step of
 * tff.aggregators.DiscreteFourierTransformFactory, which builder.py:70-71 wraps
 * around a codec (the FFT itself is a library transform, rocFFT). */
int fc_sign_flip(float* const* rows, int32_t nclients, int64_t n, int64_t seed0, int64_t seed1, void* stream);

/* The DFT rotation of tff.aggregators.DiscreteFourierTransformFactory (builder.py:70-71),
 * in place on nclients device rows of an even length n (rows: device array of row
 * pointers), one row at a time: forward x <- F(D x), inverse (inverse = 1) x <- D F^-1(x),
 * with D = fc_sign_flip's signs and F the unitary DFT of the n / 2 complex numbers
 * x[k] + i x[k + n/2], written back as (real, imaginary) halves.  Hand-written FFT
 * (Stockham radix-16 passes; Bluestein's chirp-z convolution for lengths other than
 * powers of two).  workspace: fc_dft_workspace_bytes(n), 16-byte aligned. */
int64_t fc_dft_workspace_bytes(int64_t n);
int fc_dft_rotate(float* const* rows, int32_t nclients, int64_t n, int inverse, int64_t seed0,
                  int64_t seed1, void* workspace, int64_t workspace_bytes, void* stream);

/* Measurement utility (not a reference interface): dst <- src, nbytes a multiple
 * of 16, 16-byte aligned pointers; a grid-stride 16-byte-per-lane copy whose rate
 * bench.py reports as the achievable HBM streaming peak beside the codec kernels. */
int fc_copy(void* dst, const void* src, int64_t nbytes, void* stream);

/* Test utility (not a reference interface): occupy every CU of the XCDs whose bit
 * is set in xcd_mask (bits 0..7 = HW_REG_XCC_ID) for `microseconds` (<= 5 s) with
 * one workgroup per CU that holds all of its LDS, so that concurrent kernels on
 * other streams cannot use those CUs meanwhile (tests/test_gpu_progress.py: the
 * encoder's ticket streams make progress on the remaining XCDs).  `held`
 * (nullable device int32) is incremented once per workgroup that held a CU. */
int fc_diag_occupy(uint32_t xcd_mask, int64_t microseconds, int32_t* held, void* stream);

/* Measurement utility (not a reference interface): the encoder's arithmetic floor
 * -- read every x, draw TF's Philox4x32-10 stream, apply the exact quantiser
 * (uniform or stochastic, power-of-two step) and sum the distortion and nonzeros
 * per 1024-element tile into dist_part / nnz_part (layout of fc_quantize_encode's),
 * with no run-length gamma coding.  workspace >= 16 * nclients bytes (16-byte
 * aligned).  bench / DESIGN.md compare fc_quantize_encode's time with it. */
int fc_quantize_floor(const float* const* xs, int32_t nclients, int64_t P, float step, const int64_t* seeds, int mode,
                      float* dist_part, int32_t* nnz_part, void* workspace, int64_t workspace_bytes, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* FEDCODEC_H_ */
