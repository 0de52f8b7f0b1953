/* tensorflow-compression run-length Elias-gamma coder restated in C.
 *
 * TEST INFRASTRUCTURE ONLY: the CPU oracle and the CPU baseline ("port").
 * Never linked into the product library.
 *
 * Reference call sites: compressed_communication/aggregators/elias_gamma_encode.py:71-72
 * (tfc.run_length_gamma_decode) and :97-99 (tfc.run_length_gamma_encode); the
 * protocol is the docstring at elias_gamma_encode.py:30-45.  The kernel itself
 * lives in tensorflow-compression (RunLengthGammaEncodeOp/DecodeOp, version
 * unpinned in compressed_communication/requirements.txt:5) which is not in
 * this image, so its published algorithm is restated:
 *
 *   zc = 1
 *   for v in data:              # flattened int32
 *     if v == 0: zc += 1; continue
 *     Gamma(zc); Bit(v > 0); Gamma(|v|); zc = 1
 *   if zc > 1: Gamma(zc)        # trailing zero run (pinned by
 *                               # elias_gamma_encode_test.py:32-37)
 *   Gamma(d) = floor(log2 d) zeros, then d in floor(log2 d)+1 bits.
 *   output = ceil(bits / 8) bytes, last byte zero padded.
 *
 * Pinned by the reference tests: bit counts and byte counts.  Unpinned: the
 * bit order inside bytes.  This restatement (and the HIP kernels) use classic
 * MSB-first order: stream bit k is bit (7 - k % 8) of byte k / 8, sign bit 1 =
 * positive.  |INT32_MIN| is coded as the 32-bit magnitude 2^31.
 */
#include <stdint.h>
#include <string.h>

typedef struct {
  uint8_t* out;
  int64_t cap;
  int64_t nbytes;
  uint64_t acc;
  int nacc;
  int overflow;
} bitwriter;

static inline void bw_put(bitwriter* w, uint64_t v, int n) { /* n <= 32 */
  w->acc = (w->acc << n) | v;
  w->nacc += n;
  while (w->nacc >= 8) {
    w->nacc -= 8;
    if (w->nbytes < w->cap) w->out[w->nbytes] = (uint8_t)(w->acc >> w->nacc);
    else w->overflow = 1;
    w->nbytes++;
  }
}

static inline int ilog2_u64(uint64_t d) { return 63 - __builtin_clzll(d); }

static inline void bw_gamma(bitwriter* w, uint64_t d) { /* 1 <= d < 2^32 */
  int n = ilog2_u64(d);
  if (n) bw_put(w, 0, n);
  bw_put(w, d, n + 1);
}

static inline int64_t gamma_len(uint64_t d) { return 2 * (int64_t)ilog2_u64(d) + 1; }

/* Length in bits of the code for q[0..n). */
int64_t rlg_encoded_bits(const int32_t* q, int64_t n) {
  int64_t bits = 0;
  uint64_t zc = 1;
  for (int64_t i = 0; i < n; ++i) {
    int32_t v = q[i];
    if (v == 0) { ++zc; continue; }
    uint32_t mag = v < 0 ? (uint32_t)0 - (uint32_t)v : (uint32_t)v;
    bits += gamma_len(zc) + 1 + gamma_len(mag);
    zc = 1;
  }
  if (zc > 1) bits += gamma_len(zc);
  return bits;
}

/* Encode q[0..n) into out (capacity cap bytes).  Returns the bit length, or -1
 * if the capacity was too small. */
int64_t rlg_encode(const int32_t* q, int64_t n, uint8_t* out, int64_t cap) {
  bitwriter w = {out, cap, 0, 0, 0, 0};
  uint64_t zc = 1;
  int64_t bits = 0;
  for (int64_t i = 0; i < n; ++i) {
    int32_t v = q[i];
    if (v == 0) { ++zc; continue; }
    uint32_t mag = v < 0 ? (uint32_t)0 - (uint32_t)v : (uint32_t)v;
    bw_gamma(&w, zc);
    bw_put(&w, v > 0 ? 1u : 0u, 1);
    bw_gamma(&w, mag);
    bits += gamma_len(zc) + 1 + gamma_len(mag);
    zc = 1;
  }
  if (zc > 1) { bw_gamma(&w, zc); bits += gamma_len(zc); }
  if (w.nacc > 0) bw_put(&w, 0, 8 - w.nacc); /* zero-pad the final byte */
  return w.overflow ? -1 : bits;
}

typedef struct {
  const uint8_t* in;
  int64_t nbytes;
  int64_t next;
  uint64_t buf; /* next bits, MSB aligned */
  int nbuf;
} bitreader;

static inline void br_refill(bitreader* r) {
  while (r->nbuf <= 56 && r->next < r->nbytes) {
    r->buf |= (uint64_t)r->in[r->next++] << (56 - r->nbuf);
    r->nbuf += 8;
  }
}

static inline int br_bits(bitreader* r, int n, uint64_t* v) { /* 1 <= n <= 32 */
  br_refill(r);
  if (r->nbuf < n) return -1;
  *v = r->buf >> (64 - n);
  r->buf <<= n;
  r->nbuf -= n;
  return 0;
}

static inline int br_gamma(bitreader* r, uint64_t* d) {
  br_refill(r);
  int n = 0;
  for (;;) { /* count leading zeros, possibly across refills */
    if (r->nbuf == 0) return -1;
    if (r->buf) {
      int z = __builtin_clzll(r->buf);
      if (z >= r->nbuf) { n += r->nbuf; r->buf = 0; r->nbuf = 0; br_refill(r); continue; }
      n += z;
      r->buf <<= z;
      r->nbuf -= z;
      break;
    }
    n += r->nbuf;
    r->nbuf = 0;
    br_refill(r);
  }
  if (n > 31) return -2;
  return br_bits(r, n + 1, d);
}

/* Decode exactly n values.  Returns 0 on success, <0 on a malformed stream. */
int rlg_decode(const uint8_t* code, int64_t nbytes, int64_t n, int32_t* out) {
  bitreader r = {code, nbytes, 0, 0, 0};
  int64_t i = 0;
  while (i < n) {
    uint64_t zc, sign, mag;
    if (br_gamma(&r, &zc)) return -1;
    if ((int64_t)(zc - 1) > n - i) return -3;
    memset(out + i, 0, (size_t)(zc - 1) * sizeof(int32_t));
    i += (int64_t)(zc - 1);
    if (i >= n) break; /* trailing zero run */
    if (br_bits(&r, 1, &sign)) return -1;
    if (br_gamma(&r, &mag)) return -1;
    uint32_t m = (uint32_t)mag;
    out[i++] = (int32_t)(sign ? m : (uint32_t)0 - m);
  }
  return 0;
}

/* Decode and add into acc (int32, wrapping) -- the federated_aggregate
 * accumulate step of elias_gamma_encode.py:69-73, without a temporary. */
int rlg_decode_accumulate(const uint8_t* code, int64_t nbytes, int64_t n, int32_t* acc) {
  bitreader r = {code, nbytes, 0, 0, 0};
  int64_t i = 0;
  while (i < n) {
    uint64_t zc, sign, mag;
    if (br_gamma(&r, &zc)) return -1;
    if ((int64_t)(zc - 1) > n - i) return -3;
    i += (int64_t)(zc - 1);
    if (i >= n) break;
    if (br_bits(&r, 1, &sign)) return -1;
    if (br_gamma(&r, &mag)) return -1;
    uint32_t m = (uint32_t)mag;
    acc[i] = (int32_t)((uint32_t)acc[i] + (sign ? m : (uint32_t)0 - m));
    ++i;
  }
  return 0;
}
