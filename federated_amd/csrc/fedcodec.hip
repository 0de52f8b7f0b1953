// fedcodec: MI355X (gfx950 / CDNA4) kernels for the compressed_communication/
// client-update codec, exported through the C ABI in include/fedcodec.h.
//
// Hot path (DESIGN.md "Kernels"):
//   k_encode  one pass over the fp32 client deltas: quantise (TF-CPU numerics,
//             Philox4x32-10 stochastic rounding), per-element run-length Elias
//             gamma code lengths, wavefront scans, single-pass decoupled
//             look-back across 4096-element tiles, LDS-staged MSB-first bit
//             packing, owner-writes-word stores (no memset, no global atomics on
//             the stream), per-tile decoder index.
//   k_decode  per 4096-element tile, one lane per client: sequential gamma
//             decode of that client's tile segment from the encoder index,
//             LDS int32 accumulation, fused dequantise epilogue.
//
// Compiled with -fgpu-flush-denormals-to-zero -ffp-contract=off: TF-CPU runs
// its Eigen kernels with FTZ/DAZ and without FMA contraction of these ops.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstring>
#include <cstdlib>
#include <algorithm>
#include <cmath>
#include <string>

#include "../../include/fedcodec.h"

namespace {

constexpr int kTE = FC_TILE_ELEMS;  // elements per tile
constexpr int kThreads = 256;       // 4 waves of 64
constexpr int kWinWords = 2048;     // LDS bit window (64 Kbit = 16 bits/element)
constexpr uint32_t kNoPos = 0x1FFF; // "no nonzero" in a 13-bit tile-relative field

// ---------------------------------------------------------------------------
// Philox4x32-10 and TF's stateless seed scramble (see oracle/philox.py).
// ---------------------------------------------------------------------------
struct Key4 {
  uint32_t k0, k1, c2, c3;
};

__host__ __device__ __forceinline__ void philox10(uint32_t& c0, uint32_t& c1, uint32_t& c2,
                                                  uint32_t& c3, uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const uint64_t p0 = (uint64_t)0xD2511F53u * c0;
    const uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
    const uint32_t n0 = (uint32_t)(p1 >> 32) ^ c1 ^ k0;
    const uint32_t n2 = (uint32_t)(p0 >> 32) ^ c3 ^ k1;
    c1 = (uint32_t)p1;
    c3 = (uint32_t)p0;
    c0 = n0;
    c2 = n2;
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
}

__host__ __device__ __forceinline__ Key4 tf_seed_scramble(int64_t s0, int64_t s1) {
  uint32_t c0 = (uint32_t)(uint64_t)s0, c1 = (uint32_t)((uint64_t)s0 >> 32);
  uint32_t c2 = (uint32_t)(uint64_t)s1, c3 = (uint32_t)((uint64_t)s1 >> 32);
  philox10(c0, c1, c2, c3, 0x3EC8F720u, 0x02461E29u);
  return Key4{c0, c1, c2, c3};
}

// Random uint32 for the 4-element group g (element 4g + lane).
__device__ __forceinline__ uint4 philox_group(const Key4& k, uint32_t g) {
  uint32_t c0 = g, c1 = 0, c2 = k.c2, c3 = k.c3;
  philox10(c0, c1, c2, c3, k.k0, k.k1);
  return make_uint4(c0, c1, c2, c3);
}

__device__ __forceinline__ float u01(uint32_t r) {  // TF Uint32ToFloat
  return __uint_as_float((r & 0x7FFFFFu) | 0x3F800000u) - 1.0f;
}

// x86 cvttps2dq: out-of-range and NaN -> INT32_MIN (TF-CPU tf.cast).
__device__ __forceinline__ int32_t f2i_x86(float r) {
  return (r >= -2147483648.0f && r < 2147483648.0f) ? (int32_t)r : (int32_t)0x80000000;
}

// quantize_utils.py:33-36 / 46-53 / 62-66 for one element.  Returns q and the
// client-side dequantised value (quantize_encode.py:148-149).  RCP: step is a
// power of two, so x / step == x * (1 / step) exactly (FTZ included).
template <int MODE, bool RCP = false>
__device__ __forceinline__ int32_t quantize_one(float x, float step, float rcp, uint32_t rbits,
                                                float& deq, float& noise) {
  const float sc = RCP ? x * rcp : x / step;  // IEEE-correct division, FTZ/DAZ
  float r;
  noise = 0.0f;
  if (MODE == FC_UNIFORM) {
    r = rintf(sc);
  } else if (MODE == FC_STOCHASTIC) {
    const float fl = floorf(sc);
    const float prob = sc - fl;
    r = (u01(rbits) <= prob) ? ceilf(sc) : fl;
  } else {
    noise = u01(rbits) - 0.5f;
    r = rintf(sc - noise);
  }
  const int32_t q = f2i_x86(r);
  deq = (MODE == FC_DITHERED) ? ((float)q + noise) * step : (float)q * step;
  return q;
}

// ---------------------------------------------------------------------------
// Elias gamma helpers (MSB-first: the code of d is d in 2*floor(log2 d)+1 bits).
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint32_t ilog2_u32(uint32_t d) { return 31u - __clz(d); }
__device__ __forceinline__ uint32_t glen(uint32_t d) { return 2u * ilog2_u32(d) + 1u; }
__device__ __forceinline__ uint32_t mag_u32(int32_t v) {
  return v < 0 ? 0u - (uint32_t)v : (uint32_t)v;
}

// Look-back monoid element: a run of tiles' code, with positions absolute in
// the client tensor.  body = bits after the segment's first run code (for a
// root segment, which starts at stream bit 0, first = -1 and body = all bits).
// tail = low 32 bits of body (stream order: bit 0 is the last stream bit).
struct Seg {
  uint32_t has_nz;
  int32_t first, last;
  uint64_t body;
  uint32_t tail;
};

__device__ __forceinline__ uint64_t shl_lt64(uint64_t x, uint64_t s) { return s >= 64 ? 0 : x << s; }

__device__ __forceinline__ Seg seg_combine(const Seg& a, const Seg& b) {
  if (!b.has_nz) return a;
  if (!a.has_nz) return b;
  const uint32_t d = (uint32_t)(b.first - a.last);
  const uint32_t rl = glen(d);
  Seg r;
  r.has_nz = 1;
  r.first = a.first;
  r.last = b.last;
  r.body = a.body + rl + b.body;
  const uint64_t t = shl_lt64(a.tail, (uint64_t)rl + b.body) | shl_lt64(d, b.body) | b.tail;
  r.tail = (uint32_t)t;
  return r;
}

// Status words (two self-tagged 8-byte granules per tile, agent-scope atomics):
//  w1: [63:62] flag (1 aggregate, 2 inclusive prefix)
//      aggregate: [61:49] first_rel  [48:36] last_rel  [35:0] body bits
//      prefix:    [61:36] last+1     [35:0] bits
//  w2: [63:62] flag  [31:0] tail
constexpr uint64_t kFlagAgg = 1ull << 62;
constexpr uint64_t kFlagPre = 2ull << 62;
constexpr uint64_t kMask36 = (1ull << 36) - 1;

__device__ __forceinline__ Seg seg_from_status(uint64_t w1, uint64_t w2, int64_t tile_base) {
  Seg s;
  if ((w1 >> 62) == 2) {
    s.has_nz = 1;
    s.first = -1;
    s.last = (int32_t)((w1 >> 36) & ((1u << 26) - 1)) - 1;
    s.body = w1 & kMask36;
  } else {
    const uint32_t fr = (uint32_t)(w1 >> 49) & 0x1FFF;
    const uint32_t lr = (uint32_t)(w1 >> 36) & 0x1FFF;
    s.has_nz = fr != kNoPos;
    s.first = (int32_t)(tile_base + fr);
    s.last = (int32_t)(tile_base + lr);
    s.body = w1 & kMask36;
  }
  s.tail = (uint32_t)w2;
  return s;
}

__device__ __forceinline__ uint64_t ld_agent(const uint64_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_agent(uint64_t* p, uint64_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ uint32_t bswap32(uint32_t v) { return __builtin_bswap32(v); }

// ---------------------------------------------------------------------------
// Wave-level scans (64 lanes).
// ---------------------------------------------------------------------------
__device__ __forceinline__ int32_t wave_incl_max(int32_t v, int lane) {
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int32_t t = __shfl_up(v, o, 64);
    if (lane >= o) v = max(v, t);
  }
  return v;
}
__device__ __forceinline__ uint32_t wave_incl_sum(uint32_t v, int lane) {
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t t = __shfl_up(v, o, 64);
    if (lane >= o) v += t;
  }
  return v;
}
__device__ __forceinline__ int32_t wave_min(int32_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = min(v, __shfl_xor(v, o, 64));
  return v;
}

// ---------------------------------------------------------------------------
// Encoder.
// ---------------------------------------------------------------------------
struct EncodeArgs {
  const void* const* xs;  // float* or int32* per client
  int32_t nclients;
  int64_t P;
  int32_t T;  // tiles per client
  float step;
  float rcp;  // 1 / step when step is a power of two (exact reciprocal path)
  const float* norms;
  const float* prescale;  // nullable [2*C]: x -> (x * clip) * weight before quantising
  const int64_t* seeds;
  uint8_t* stream_buf;
  const int64_t* stream_off;
  const int64_t* stream_cap;
  uint64_t* idx;
  int64_t* total_bits;
  float* dist_part;
  int32_t* nnz_part;
  int32_t* overflow;
  uint64_t* status;   // [nclients * T][2]
  uint32_t* counter;  // ticket counter (zeroed per launch)
  uint32_t* spin_err;
};

struct EncShared {
  uint32_t win[kWinWords];  // LDS bit window (MSB-first words)
  int32_t wave_last[4];
  int32_t wave_first[4];
  uint32_t wave_bits[4];
  float wave_dist[4];
  int32_t wave_nnz[4];
  uint32_t tail;
  uint32_t ticket;
  uint32_t next_ticket;
  uint32_t slow;  // tile needs the slow (re-quantise) emission path
  // look-back results broadcast to the workgroup
  uint64_t b0;
  int32_t last_before;
  uint32_t tail_before;
  uint32_t r0_R0;      // stream-window bit where the body starts = (b0 % 32) + R0
  uint32_t nwin_bits;  // bits in the stream window (incl. trailing code on the last tile)
  uint64_t trail;      // trailing run code value
  uint32_t trail_len;
};

// Emit a piece of <= 32 bits at window bit position wp into the LDS window
// covering window words [pass_lo, pass_lo + kWinWords).
__device__ __forceinline__ void win_emit32(uint32_t* win, uint32_t v, uint32_t L, uint32_t wp,
                                           uint32_t pass_lo) {
  if (L == 0) return;
  const uint32_t o = wp & 31;
  const uint64_t X = (uint64_t)v << (64 - o - L);
  const uint32_t hi = (uint32_t)(X >> 32), lo = (uint32_t)X;
  const int32_t i0 = (int32_t)(wp >> 5) - (int32_t)pass_lo;
  if ((uint32_t)i0 < (uint32_t)kWinWords && hi) atomicOr(&win[i0], hi);
  if (o + L > 32 && (uint32_t)(i0 + 1) < (uint32_t)kWinWords && lo) atomicOr(&win[i0 + 1], lo);
}

__device__ __forceinline__ void win_emit(uint32_t* win, uint64_t v, uint32_t L, uint32_t wp,
                                         uint32_t pass_lo) {
  if (L > 32) {
    win_emit32(win, (uint32_t)(v >> 32), L - 32, wp, pass_lo);
    win_emit32(win, (uint32_t)v, 32, wp + (L - 32), pass_lo);
  } else {
    win_emit32(win, (uint32_t)v, L, wp, pass_lo);
  }
}

// Bits of stream word k covered by a piece (v, L) starting at bit p (MSB-first).
__device__ __forceinline__ uint32_t piece_word(uint64_t v, uint32_t L, uint32_t p, uint32_t k) {
  const int32_t lo = 32 * (int32_t)k, end = (int32_t)(p + L);
  if (L == 0 || end <= lo || (int32_t)p >= lo + 32) return 0;
  const int32_t sh = lo + 32 - end;
  return sh >= 0 ? (uint32_t)(sh >= 64 ? 0 : v << sh) : (uint32_t)(-sh >= 64 ? 0 : v >> -sh);
}

// OR the part of a piece (ending at body position `end`) that falls in the last
// 32 body bits into the tail word.
__device__ __forceinline__ void tail_emit(uint32_t* tailw, uint64_t v, uint32_t L, uint32_t end,
                                          uint32_t body) {
  const uint32_t s = body - end;
  if (s < 32 && L) {
    const uint32_t c = (uint32_t)(v << s);
    if (c) atomicOr(tailw, c);
  }
}

__device__ __forceinline__ Seg seg_identity() {
  Seg s;
  s.has_nz = 0;
  s.first = s.last = 0;
  s.body = 0;
  s.tail = 0;
  return s;
}

// ---------------------------------------------------------------------------
// DPP wavefront scans (GFX9 row_shr / row_bcast / wave_shr; VALU, no LDS).
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint32_t dpp_incl_sum(uint32_t x) {
  x += __builtin_amdgcn_update_dpp(0u, x, 0x111, 0xf, 0xf, false);  // row_shr:1
  x += __builtin_amdgcn_update_dpp(0u, x, 0x112, 0xf, 0xf, false);  // row_shr:2
  x += __builtin_amdgcn_update_dpp(0u, x, 0x114, 0xf, 0xf, false);  // row_shr:4
  x += __builtin_amdgcn_update_dpp(0u, x, 0x118, 0xf, 0xf, false);  // row_shr:8
  x += __builtin_amdgcn_update_dpp(0u, x, 0x142, 0xa, 0xf, false);  // row_bcast:15
  x += __builtin_amdgcn_update_dpp(0u, x, 0x143, 0xc, 0xf, false);  // row_bcast:31
  return x;
}
__device__ __forceinline__ int32_t dpp_incl_max(int32_t x) {
  const int32_t id = (int32_t)0x80000000;
  x = max(x, __builtin_amdgcn_update_dpp(id, x, 0x111, 0xf, 0xf, false));
  x = max(x, __builtin_amdgcn_update_dpp(id, x, 0x112, 0xf, 0xf, false));
  x = max(x, __builtin_amdgcn_update_dpp(id, x, 0x114, 0xf, 0xf, false));
  x = max(x, __builtin_amdgcn_update_dpp(id, x, 0x118, 0xf, 0xf, false));
  x = max(x, __builtin_amdgcn_update_dpp(id, x, 0x142, 0xa, 0xf, false));
  x = max(x, __builtin_amdgcn_update_dpp(id, x, 0x143, 0xc, 0xf, false));
  return x;
}
__device__ __forceinline__ int32_t dpp_shr1(int32_t x, int32_t fill) {  // wave_shr:1
  return __builtin_amdgcn_update_dpp(fill, x, 0x138, 0xf, 0xf, false);
}
__device__ __forceinline__ int32_t lane63(int32_t x) { return __builtin_amdgcn_readlane(x, 63); }

// Decoupled look-back for tile t of one client, run by one full wave.  Returns
// the exclusive prefix (a root segment: body = stream bits before tile t).
__device__ __forceinline__ Seg lookback(const uint64_t* status_c, int32_t t, int lane,
                                        uint32_t* spin_err) {
  Seg S = seg_identity();
  int64_t base = (int64_t)t - 1;
  for (;;) {
    const int64_t ti = base - lane;
    uint64_t w1 = kFlagPre, w2 = kFlagPre;  // ti < 0: virtual root prefix
    bool valid = ti < 0;
    int k;
    uint32_t spins = 0;
    for (;;) {
      if (!valid) {
        w1 = ld_agent(status_c + 2 * ti);
        w2 = ld_agent(status_c + 2 * ti + 1);
        valid = (w1 >> 62) != 0 && (w1 >> 62) == (w2 >> 62);
      }
      const uint64_t pre = __ballot(valid && (w1 >> 62) == 2);
      const uint64_t val = __ballot(valid);
      k = pre ? __builtin_ctzll(pre) : 64;
      const uint64_t need = k >= 63 ? ~0ull : ((2ull << k) - 1);
      if ((val & need) == need) break;
      __builtin_amdgcn_s_sleep(1);
      if (++spins > (1u << 24)) {  // safety net only: tickets guarantee progress
        if (lane == 0) atomicOr(spin_err, 1u);
        k = 0;
        w1 = kFlagPre;
        w2 = kFlagPre;
        break;
      }
    }
    Seg v = (lane <= k && ti >= -1) ? seg_from_status(w1, w2, ti * kTE) : seg_identity();
    // suffix scan over lanes 0..k: lane 0 ends with the combination of the window
    const int kk = k < 63 ? k : 63;
    for (int d = 1; d <= kk; d <<= 1) {
      Seg o;
      o.has_nz = __shfl_down(v.has_nz, d, 64);
      o.first = __shfl_down(v.first, d, 64);
      o.last = __shfl_down(v.last, d, 64);
      o.body = __shfl_down(v.body, d, 64);
      o.tail = __shfl_down(v.tail, d, 64);
      if (lane + d >= 64) o.has_nz = 0;
      v = seg_combine(o, v);
    }
    Seg W;
    W.has_nz = __builtin_amdgcn_readfirstlane(v.has_nz);
    W.first = __builtin_amdgcn_readfirstlane(v.first);
    W.last = __builtin_amdgcn_readfirstlane(v.last);
    W.body = ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(v.body >> 32)) << 32) |
             __builtin_amdgcn_readfirstlane((uint32_t)v.body);
    W.tail = __builtin_amdgcn_readfirstlane(v.tail);
    S = seg_combine(W, S);
    if (k < 64) break;
    base -= 64;
  }
  return S;
}

// Raw 4x4 input words (float or int32 bit patterns) of one thread's chunks.
template <bool INT_IN>
__device__ __forceinline__ void load_raw(const EncodeArgs& a, uint32_t ticket, int wv, int lane,
                                         uint32_t (&raw)[4][4]) {
  const int32_t t = (int32_t)(ticket / (uint32_t)a.nclients);
  const int32_t c = (int32_t)(ticket - (uint32_t)t * (uint32_t)a.nclients);
  const int64_t tile_base = (int64_t)t * kTE;
  const uint32_t* xp = (const uint32_t*)a.xs[c];
  const bool aligned = (((uintptr_t)xp) & 15) == 0;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int64_t e0 = tile_base + 1024 * wv + 256 * j + 4 * lane;
    if (aligned && e0 + 3 < a.P) {
      const uint4 v = *(const uint4*)(xp + e0);
      raw[j][0] = v.x; raw[j][1] = v.y; raw[j][2] = v.z; raw[j][3] = v.w;
    } else {
#pragma unroll
      for (int k = 0; k < 4; ++k) raw[j][k] = (e0 + k < a.P) ? xp[e0 + k] : 0u;
    }
  }
}

struct ClientQ {
  float step;
  float rcp;
  float s0, s1;  // pre-scales (TFF clipping factor, MeanFactory weight)
  bool pre;
  Key4 key;
};

template <int MODE, bool INT_IN>
__device__ __forceinline__ ClientQ client_q(const EncodeArgs& a, int32_t c) {
  ClientQ r;
  r.step = a.step;
  if (!INT_IN && a.norms) r.step = a.norms[c] * a.step;
  r.rcp = a.rcp;
  r.pre = !INT_IN && a.prescale != nullptr;
  r.s0 = r.pre ? a.prescale[2 * c] : 1.0f;
  r.s1 = r.pre ? a.prescale[2 * c + 1] : 1.0f;
  r.key = Key4{0, 0, 0, 0};
  if (!INT_IN && MODE != FC_UNIFORM) r.key = tf_seed_scramble(a.seeds[2 * c], a.seeds[2 * c + 1]);
  return r;
}

// Quantise one chunk of 4 consecutive elements starting at e0.
template <int MODE, bool INT_IN, bool RCP>
__device__ __forceinline__ void quant_chunk(const ClientQ& cq, int64_t e0, int64_t P,
                                            const uint32_t (&r4)[4], int32_t (&q4)[4],
                                            float& dist) {
  if (INT_IN) {
#pragma unroll
    for (int k = 0; k < 4; ++k) q4[k] = (int32_t)r4[k];
  } else {
    uint4 rb = make_uint4(0, 0, 0, 0);
    if (MODE != FC_UNIFORM) rb = philox_group(cq.key, (uint32_t)(e0 >> 2));
    const uint32_t rr[4] = {rb.x, rb.y, rb.z, rb.w};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      float deq, noise;
      float xv = __uint_as_float(r4[k]);
      if (cq.pre) xv = (xv * cq.s0) * cq.s1;  // clipping_factory, then MeanFactory weight
      const int32_t qq = quantize_one<MODE, RCP>(xv, cq.step, cq.rcp, rr[k], deq, noise);
      const bool valid = e0 + k < P;
      q4[k] = valid ? qq : 0;
      const float dd = xv - deq;
      dist = valid ? fmaf(dd, dd, dist) : dist;
    }
  }
}

// Run-length gamma code of one chunk of 4 consecutive elements (branch-free),
// built right after the chunk is quantised so the int32 values never stay live:
// acc holds the concatenated codes after the chunk's first nonzero's run code
// (that one depends on the previous chunks and is prepended in phase C).
struct ChunkCode {
  uint64_t acc;
  uint32_t len;
  uint32_t lng;   // a code > 32 bits or more than 64 bits in the chunk
  int32_t first;  // tile-relative first nonzero of the chunk, or -1
  int32_t last;   // tile-relative last nonzero of the chunk, or -1
};

__device__ __forceinline__ ChunkCode chunk_local(const int32_t (&q4)[4], int32_t rel0) {
  ChunkCode r;
  r.acc = 0;
  r.len = 0;
  r.lng = 0;
  r.first = -1;
  int32_t pk = -1;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int32_t v = q4[k];
    const bool nz = v != 0;
    const uint32_t m = mag_u32(v);
    const uint32_t ml = 2u * (31u - __clz(m | 1u)) + 1u;
    const uint32_t d = (uint32_t)(k - pk);
    const uint32_t rl = pk >= 0 ? 2u * (31u - __clz(d)) + 1u : 0u;
    const uint32_t L = rl + 1u + ml;
    const uint32_t code = ((pk >= 0 && L <= 32u) ? (d << (1u + ml)) : 0u) | ((uint32_t)(v > 0) << ml) | m;
    r.lng |= (nz && L > 32u) ? 1u : 0u;
    r.acc = nz ? (r.acc << L) | code : r.acc;
    r.len += nz ? L : 0u;
    r.first = (r.first < 0 && nz) ? rel0 + k : r.first;
    pk = nz ? k : pk;
  }
  r.last = pk >= 0 ? rel0 + pk : -1;
  r.lng |= r.len > 64u ? 1u : 0u;
  return r;
}

// Prepend the run code of the chunk's first nonzero once the last nonzero
// before the chunk (prev, tile-relative, -1 = none in this tile) is known.
__device__ __forceinline__ void chunk_prepend(ChunkCode& r, int32_t prev) {
  if (r.first >= 0 && prev >= 0) {
    const uint32_t d = (uint32_t)(r.first - prev);
    const uint32_t rl = 2u * (31u - __clz(d)) + 1u;
    r.lng |= (r.len + rl > 64u) ? 1u : 0u;
    r.acc = (r.len + rl > 64u) ? 0 : (((uint64_t)d << r.len) | r.acc);
    r.len += rl;
  }
}

template <int MODE, bool INT_IN, bool RCP>
__device__ __forceinline__ void quantize_tile(const EncodeArgs& a, int32_t c, int64_t tile_base,
                                              int wv, int lane, const uint32_t (&raw)[4][4],
                                              ChunkCode (&cc)[4], float& dist, int32_t& nnz) {
  const ClientQ cq = client_q<MODE, INT_IN>(a, c);
  dist = 0.0f;
  nnz = 0;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int32_t rel0 = 1024 * wv + 256 * j + 4 * lane;
    int32_t q4[4];
    quant_chunk<MODE, INT_IN, RCP>(cq, tile_base + rel0, a.P, raw[j], q4, dist);
#pragma unroll
    for (int k = 0; k < 4; ++k) nnz += q4[k] != 0;
    cc[j] = chunk_local(q4, rel0);
  }
}

// Re-read and re-quantise one chunk (slow path: tiles with codes > 32 bits or
// a body larger than the LDS window).
template <int MODE, bool INT_IN, bool RCP>
__device__ __forceinline__ void reload_chunk(const EncodeArgs& a, const ClientQ& cq, int32_t c,
                                             int64_t e0, int32_t (&q4)[4]) {
  const uint32_t* xp = (const uint32_t*)a.xs[c];
  uint32_t r4[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) r4[k] = (e0 + k < a.P) ? xp[e0 + k] : 0u;
  float dd = 0.0f;
  quant_chunk<MODE, INT_IN, RCP>(cq, e0, a.P, r4, q4, dd);
}

#ifdef FC_STAMPS
__device__ unsigned long long g_stamps[8];
#define STAMP(i)                                               \
  do {                                                         \
    if (tid == 0) {                                            \
      const uint64_t now_ = __builtin_amdgcn_s_memtime();      \
      st_acc[i] += now_ - st_last;                             \
      st_last = now_;                                          \
    }                                                          \
  } while (0)
#else
#define STAMP(i) do {} while (0)
#endif

template <int MODE, bool INT_IN, bool RCP>
__global__ __launch_bounds__(kThreads, 4) void k_encode(EncodeArgs a) {
  __shared__ EncShared sh;
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wv = tid >> 6;
  const uint32_t total_tiles = (uint32_t)a.nclients * (uint32_t)a.T;
#ifdef FC_STAMPS
  uint64_t st_acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  uint64_t st_last = __builtin_amdgcn_s_memtime();
#endif

  for (int i = tid; i < kWinWords; i += kThreads) sh.win[i] = 0;
  if (tid == 0) sh.ticket = atomicAdd(a.counter, 1u);
  __syncthreads();
  uint32_t ticket = sh.ticket;
  uint32_t raw[4][4];
  if (ticket < total_tiles) load_raw<INT_IN>(a, ticket, wv, lane, raw);

  while (ticket < total_tiles) {
    STAMP(0);
    if (tid == 0) {
      sh.next_ticket = atomicAdd(a.counter, 1u);  // read after the first barrier
      sh.tail = 0;
      sh.slow = 0;
    }
    // tickets interleave clients (tile-major) so each client has few tiles in
    // flight and the look-back almost always finds a prefix at distance 1
    const int32_t t = (int32_t)(ticket / (uint32_t)a.nclients);
    const int32_t c = (int32_t)(ticket - (uint32_t)t * (uint32_t)a.nclients);
    const int64_t P = a.P;
    const int64_t tile_base = (int64_t)t * kTE;
    const bool last_tile = (t == a.T - 1);

    // ---- phase A: quantise + chunk-local codes (4 chunks of 4 consecutive elements) ----
    ChunkCode cc[4];
    float dist;
    int32_t nnz;
    quantize_tile<MODE, INT_IN, RCP>(a, c, tile_base, wv, lane, raw, cc, dist, nnz);
    STAMP(1);

    // ---- phase B: wave max-scan of the chunks' last nonzero ----
    int32_t chunk_prev[4];  // last nonzero before the chunk (tile-relative), or -1
    int32_t carry = -1, wfirst = 0x7FFFFFFF;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      wfirst = min(wfirst, cc[j].first >= 0 ? cc[j].first : 0x7FFFFFFF);
      const int32_t incl = dpp_incl_max(cc[j].last);
      chunk_prev[j] = max(dpp_shr1(incl, -1), carry);
      carry = max(carry, lane63(incl));
    }
    {
      float d = dist;
      int32_t n = nnz;
      int32_t f = wfirst;
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) {
        d += __shfl_xor(d, o, 64);
        n += __shfl_xor(n, o, 64);
        f = min(f, __shfl_xor(f, o, 64));
      }
      if (lane == 0) {
        sh.wave_dist[wv] = d;
        sh.wave_nnz[wv] = n;
        sh.wave_last[wv] = carry;
        sh.wave_first[wv] = f;
      }
    }
    __syncthreads();
    STAMP(2);
    int32_t wave_in = -1;
    for (int w = 0; w < wv; ++w) wave_in = max(wave_in, sh.wave_last[w]);
    int32_t tile_first = 0x7FFFFFFF, tile_last = -1;
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      tile_first = min(tile_first, sh.wave_first[w]);
      tile_last = max(tile_last, sh.wave_last[w]);
    }
    if (tid == 0) {
      const float d = ((sh.wave_dist[0] + sh.wave_dist[1]) + sh.wave_dist[2]) + sh.wave_dist[3];
      const int32_t n = sh.wave_nnz[0] + sh.wave_nnz[1] + sh.wave_nnz[2] + sh.wave_nnz[3];
      if (a.dist_part) a.dist_part[(int64_t)c * a.T + t] = d;
      if (a.nnz_part) a.nnz_part[(int64_t)c * a.T + t] = n;
    }
    const uint32_t next = sh.next_ticket;

    // ---- phase C: complete the chunk codes, sum-scan of their lengths ----
    uint64_t cacc[4];
    uint32_t chunk_off[4], clen[4];
    uint32_t wbits = 0, lng = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      chunk_prev[j] = max(chunk_prev[j], wave_in);
      chunk_prepend(cc[j], chunk_prev[j]);
      cacc[j] = cc[j].acc;
      clen[j] = cc[j].len;
      lng |= cc[j].lng;
      const uint32_t incl = dpp_incl_sum(cc[j].len);
      chunk_off[j] = wbits + incl - cc[j].len;
      wbits += (uint32_t)lane63((int32_t)incl);
    }
    if (lane == 0) sh.wave_bits[wv] = wbits;
    if (lng) sh.slow = 1;
    __syncthreads();
    STAMP(3);
    uint32_t woff = 0, body = 0;
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      woff += (w < wv) ? sh.wave_bits[w] : 0u;
      body += sh.wave_bits[w];
    }
    // fast path: no code > 32 bits and the body (+ trailing code + one funnel
    // word) fits the LDS window
    const bool fast = !sh.slow && body + 64u <= 32u * (kWinWords - 1);

    // ---- phase D: emit the body at body-relative bit offsets (fast path), or
    //      compute just its last 32 bits (slow path); prefetch the next tile ----
    if (fast) {
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if (clen[j]) win_emit(sh.win, cacc[j], clen[j], woff + chunk_off[j], 0);
    } else {
      // slow tile: recompute codes element by element (any length) for the tail
      const ClientQ cq = client_q<MODE, INT_IN>(a, c);
#pragma unroll 1
      for (int j = 0; j < 4; ++j) {
        const uint32_t off = woff + (j == 0 ? chunk_off[0] : j == 1 ? chunk_off[1] : j == 2 ? chunk_off[2] : chunk_off[3]);
        const uint32_t cl = (j == 0 ? clen[0] : j == 1 ? clen[1] : j == 2 ? clen[2] : clen[3]);
        if (off + cl + 32 < body || cl == 0) continue;
        const int32_t rel0 = 1024 * wv + 256 * j + 4 * lane;
        int32_t qv[4];
        reload_chunk<MODE, INT_IN, RCP>(a, cq, c, tile_base + rel0, qv);
        int32_t prev = (j == 0 ? chunk_prev[0] : j == 1 ? chunk_prev[1] : j == 2 ? chunk_prev[2] : chunk_prev[3]);
        uint32_t pos = off;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const int32_t v = qv[k];
          if (v == 0) continue;
          if (prev >= 0) {
            const uint32_t d = (uint32_t)(rel0 + k - prev);
            const uint32_t rl = glen(d);
            pos += rl;
            tail_emit(&sh.tail, d, rl, pos, body);
          }
          const uint32_t m = mag_u32(v);
          const uint32_t ml = glen(m);
          const uint64_t sm = ((uint64_t)(v > 0) << ml) | m;
          pos += 1 + ml;
          tail_emit(&sh.tail, sm, 1 + ml, pos, body);
          prev = rel0 + k;
        }
      }
    }
    if (next < total_tiles) load_raw<INT_IN>(a, next, wv, lane, raw);
    __syncthreads();
    STAMP(4);

    // ---- phase E: publish aggregate, decoupled look-back (wave 0) ----
    if (wv == 0) {
      uint64_t* st = a.status + 2 * ((int64_t)c * a.T + t);
      Seg agg;
      agg.has_nz = tile_last >= 0;
      agg.first = agg.has_nz ? (int32_t)(tile_base + tile_first) : 0;
      agg.last = agg.has_nz ? (int32_t)(tile_base + tile_last) : 0;
      agg.body = body;
      if (fast) {
        uint32_t tl = 0;
        if (body >= 32) {
          const uint32_t s = body - 32, w = s >> 5, o = s & 31;
          tl = o ? (sh.win[w] << o) | (sh.win[w + 1] >> (32 - o)) : sh.win[w];
        } else if (body) {
          tl = sh.win[0] >> (32 - body);
        }
        agg.tail = tl;
      } else {
        agg.tail = sh.tail;
      }
      Seg excl;
      if (t == 0) {
        excl.has_nz = 1;
        excl.first = -1;
        excl.last = -1;
        excl.body = 0;
        excl.tail = 0;
      } else {
        if (lane == 0) {
          const uint64_t fr = agg.has_nz ? (uint64_t)tile_first : kNoPos;
          const uint64_t lr = agg.has_nz ? (uint64_t)tile_last : kNoPos;
          st_agent(st + 1, kFlagAgg | agg.tail);
          st_agent(st, kFlagAgg | (fr << 49) | (lr << 36) | (uint64_t)body);
        }
        excl = lookback(a.status + 2 * (int64_t)c * a.T, t, lane, a.spin_err);
      }
      const Seg incl = seg_combine(excl, agg);
      if (lane == 0) {
        st_agent(st + 1, kFlagPre | incl.tail);
        st_agent(st, kFlagPre | ((uint64_t)(incl.last + 1) << 36) | (incl.body & kMask36));
        const int64_t ib = (int64_t)c * (a.T + 1);
        a.idx[ib + t] = (excl.body & kMask36) | ((uint64_t)(excl.last + 1) << 36);
        sh.b0 = excl.body;
        sh.last_before = excl.last;
        sh.tail_before = excl.tail;
        const uint32_t r0 = (uint32_t)(excl.body & 31);
        uint32_t R0 = 0;
        if (agg.has_nz) R0 = glen((uint32_t)(agg.first - excl.last));
        sh.r0_R0 = r0 + R0;
        uint32_t tl = 0;
        uint64_t tv = 0;
        if (last_tile) {
          const int64_t zc = P - 1 - (int64_t)incl.last;  // trailing zeros
          if (zc > 0) {
            tv = (uint64_t)(zc + 1);
            tl = 2u * (63u - (uint32_t)__clzll(tv)) + 1u;
            if (fast) win_emit(sh.win, tv, tl, body, 0);  // body-relative
          }
          a.idx[ib + a.T] = (incl.body & kMask36) | ((uint64_t)(incl.last + 1) << 36);
          a.total_bits[c] = (int64_t)incl.body + tl;
        }
        sh.trail = tv;
        sh.trail_len = tl;
        sh.nwin_bits = r0 + R0 + body + tl;
      }
    }
    __syncthreads();
    STAMP(5);

    // ---- phase F: store the words this tile owns ----
    const uint64_t b0 = sh.b0;
    const uint32_t bstart = sh.r0_R0;
    const uint32_t nwin_bits = sh.nwin_bits;
    const int32_t last_before = sh.last_before;
    const uint32_t nwords_owned = last_tile ? (nwin_bits + 31) / 32 : nwin_bits / 32;
    const int64_t cap = a.stream_cap[c];
    uint32_t* out32 = (uint32_t*)(a.stream_buf + a.stream_off[c]);
    const uint64_t w0 = b0 >> 5;
    const uint32_t r0 = (uint32_t)(b0 & 31);
    if (tid == 0 && (int64_t)(w0 + nwords_owned) * 4 > cap) atomicOr((uint32_t*)&a.overflow[c], 1u);
    if (fast) {
      const uint32_t dfirst = tile_last >= 0 ? (uint32_t)(tile_base + tile_first - last_before) : 0u;
      const uint32_t R0 = bstart - r0;
      const uint32_t tb = sh.tail_before & (r0 ? ((1u << r0) - 1u) : 0u);
      for (uint32_t k = tid; k < nwords_owned; k += kThreads) {
        // stream-window bits [32k, 32k+32) = body bits [32k - bstart, ...)
        const int32_t s = 32 * (int32_t)k - (int32_t)bstart;
        uint32_t wv32;
        if (s >= 0) {
          const uint32_t w = (uint32_t)s >> 5, o = (uint32_t)s & 31;
          wv32 = o ? (sh.win[w] << o) | (sh.win[w + 1] >> (32 - o)) : sh.win[w];
        } else {
          wv32 = (-s < 32) ? (sh.win[0] >> -s) : 0u;
          wv32 |= piece_word(tb, r0, 0, k) | piece_word(dfirst, R0, r0, k);
        }
        if ((int64_t)(w0 + k + 1) * 4 <= cap) out32[w0 + k] = bswap32(wv32);
      }
      __syncthreads();
      const uint32_t nt = min((uint32_t)kWinWords, (body + sh.trail_len + 31) / 32 + 1);
      for (uint32_t i = tid; i < nt; i += kThreads) sh.win[i] = 0;
    } else {
      // slow path (a code > 32 bits, or a body larger than the LDS window):
      // re-read and re-quantise this tile one chunk at a time and emit
      // stream-relative in window passes
      const ClientQ cq = client_q<MODE, INT_IN>(a, c);
      const uint32_t npass = (nwords_owned + kWinWords - 1) / kWinWords;
      for (uint32_t pass = 0; pass < npass; ++pass) {
        const uint32_t plo = pass * kWinWords;
        if (tid == 0) {
          if (r0) win_emit32(sh.win, sh.tail_before & ((1u << r0) - 1u), r0, 0, plo);
          if (tile_last >= 0) {
            const uint32_t d = (uint32_t)(tile_base + tile_first - last_before);
            win_emit(sh.win, d, glen(d), r0, plo);
          }
          if (sh.trail_len) win_emit(sh.win, sh.trail, sh.trail_len, bstart + body, plo);
        }
#pragma unroll 1
        for (int j = 0; j < 4; ++j) {
          const int32_t rel0 = 1024 * wv + 256 * j + 4 * lane;
          int32_t prev = j == 0 ? chunk_prev[0] : j == 1 ? chunk_prev[1] : j == 2 ? chunk_prev[2] : chunk_prev[3];
          uint32_t pos = bstart + woff +
                         (j == 0 ? chunk_off[0] : j == 1 ? chunk_off[1] : j == 2 ? chunk_off[2] : chunk_off[3]);
          int32_t q4[4];
          reload_chunk<MODE, INT_IN, RCP>(a, cq, c, tile_base + rel0, q4);
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            const int32_t v = q4[k];
            if (v == 0) continue;
            const uint32_t m = mag_u32(v);
            const uint32_t ml = glen(m);
            const uint64_t sm = ((uint64_t)(v > 0) << ml) | m;
            if (prev >= 0) {
              const uint32_t d = (uint32_t)(rel0 + k - prev);
              const uint32_t rl = glen(d);
              win_emit32(sh.win, d, rl, pos, plo);
              pos += rl;
            }
            win_emit(sh.win, sm, 1 + ml, pos, plo);
            pos += 1 + ml;
            prev = rel0 + k;
          }
        }
        __syncthreads();
        const uint32_t nw = min((uint32_t)kWinWords, nwords_owned - plo);
        for (uint32_t i = tid; i < nw; i += kThreads) {
          const uint64_t wi = w0 + plo + i;
          if ((int64_t)(wi + 1) * 4 <= cap) out32[wi] = bswap32(sh.win[i]);
        }
        __syncthreads();
        const uint32_t nt = min((uint32_t)kWinWords, (nwin_bits + 31) / 32 - plo);
        for (uint32_t i = tid; i < nt; i += kThreads) sh.win[i] = 0;
        __syncthreads();
      }
    }
    STAMP(6);
    ticket = next;
  }
#ifdef FC_STAMPS
  if (tid == 0)
    for (int i = 0; i < 8; ++i) atomicAdd(&g_stamps[i], (unsigned long long)st_acc[i]);
#endif
}

// ---------------------------------------------------------------------------
// Decoder: one workgroup per (group of) 4096-element tile(s), one lane per client.
// ---------------------------------------------------------------------------
struct DecodeArgs {
  const uint8_t* stream_buf;
  const int64_t* stream_off;
  const int64_t* stream_cap;
  const uint64_t* idx;
  int32_t nclients;
  int64_t P;
  int32_t T;
  int32_t lanes_per_tile;  // power of two, divides 256
  const int32_t* sum_in;
  int32_t* sum_out;
  float* out;
  float step;
  const float* noise_sum;
  int32_t* err;
};

// MSB-first bit reader over one client's code: a 64-bit window plus one
// prefetched 32-bit word, so each refill's load is issued ~one refill early.
struct BitReader {
  const uint4* p;    // next 16-byte block to fetch
  const uint4* end;  // first block beyond the client's region
  uint4 nxt;         // prefetched raw block, consumed one reservoir later
  uint32_t nxtok;    // nxt lies inside the region
  uint64_t rhi, rlo; // reservoir: next 128 bits after the window, MSB aligned
  int rbits;         // valid bits in the reservoir (multiple of 32)
  uint64_t win;      // next bits, MSB aligned
  int nwin;          // valid bits in win (>= 32 after refill)

  __device__ __forceinline__ void prefetch() {
    nxtok = p < end;
    nxt = *(nxtok ? p : end - 1);  // unconditional 16-byte load: no branch, no early wait
    ++p;
  }
  __device__ __forceinline__ void load_reservoir() {
    const uint4 b = nxtok ? nxt : make_uint4(0, 0, 0, 0);
    rhi = ((uint64_t)bswap32(b.x) << 32) | bswap32(b.y);
    rlo = ((uint64_t)bswap32(b.z) << 32) | bswap32(b.w);
    rbits = 128;
    prefetch();
  }
  __device__ __forceinline__ uint32_t next_word() {
    if (rbits == 0) load_reservoir();
    const uint32_t w = (uint32_t)(rhi >> 32);
    rhi = (rhi << 32) | (rlo >> 32);
    rlo <<= 32;
    rbits -= 32;
    return w;
  }
  __device__ __forceinline__ void init(const uint8_t* base, int64_t cap, uint64_t bit) {
    p = (const uint4*)base + (bit >> 7);
    end = (const uint4*)base + (cap >> 4);
    prefetch();
    load_reservoir();
    for (int i = (int)((bit >> 5) & 3); i > 0; --i) (void)next_word();
    win = ((uint64_t)next_word() << 32);
    win |= next_word();
    const int skip = (int)(bit & 31);
    win <<= skip;
    nwin = 64 - skip;
  }
  __device__ __forceinline__ void refill() {
    if (nwin <= 32) {
      win |= (uint64_t)next_word() << (32 - nwin);
      nwin += 32;
    }
  }
  // Consume n <= 32 bits (caller guarantees nwin >= n).
  __device__ __forceinline__ uint32_t take(int n) {
    const uint32_t v = (uint32_t)(win >> (64 - n));
    win = n >= 64 ? 0 : win << n;
    nwin -= n;
    refill();
    return v;
  }
  // Gamma-coded value (1 .. 2^32-1), general path.  Returns 0 on a malformed code.
  __device__ __forceinline__ uint32_t gamma() {
    int zeros = 0;
    for (;;) {
      int zz = win ? (int)__clzll(win) : 64;
      if (zz >= nwin) {  // the whole window is zeros
        zeros += nwin;
        win = 0;
        nwin = 0;
        refill();
        if (zeros > 31) return 0;
        continue;
      }
      zeros += zz;
      win <<= zz;
      nwin -= zz;
      refill();
      break;
    }
    if (zeros > 31) return 0;
    return take(zeros + 1);
  }
};

__device__ __forceinline__ uint64_t shl64(uint64_t x, uint32_t n) { return n >= 64 ? 0 : x << n; }

// One nonzero's code: run gamma d, sign bit, magnitude gamma m.  Returns the
// bits consumed (0 on a malformed code).
__device__ __forceinline__ uint32_t decode_code(BitReader& br, uint32_t& d, int32_t& val) {
  const uint64_t w = br.win;
  const uint32_t z1 = w ? (uint32_t)__clzll(w) : 64u;
  const uint32_t L1 = 2u * z1 + 1u;
  const uint64_t w3 = shl64(w, L1 + 1u);
  const uint32_t z2 = w3 ? (uint32_t)__clzll(w3) : 64u;
  const uint32_t L2 = 2u * z2 + 1u;
  const uint32_t L = L1 + 1u + L2;
  if (L <= (uint32_t)br.nwin && L1 <= 32u && L2 <= 32u) {  // fast path: whole code in the window
    d = (uint32_t)(w >> (64u - L1));
    const uint32_t s = (uint32_t)(shl64(w, L1) >> 63);
    const uint32_t m = (uint32_t)(w3 >> (64u - L2));
    val = (int32_t)(s ? m : 0u - m);
    br.win = shl64(w3, L2);
    br.nwin -= (int)L;
    br.refill();
    return L;
  }
  d = br.gamma();
  const uint32_t s = br.take(1);
  const uint32_t m = br.gamma();
  val = (int32_t)(s ? m : 0u - m);
  if (d == 0 || m == 0) return 0;
  return 2u * (31u - __clz(d)) + 1u + 1u + 2u * (31u - __clz(m)) + 1u;
}

__global__ __launch_bounds__(kThreads) void k_decode(DecodeArgs a) {
  extern __shared__ int32_t acc[];  // [tiles_per_wg][kTE]
  const int tid = threadIdx.x;
  const int tiles_per_wg = kThreads / a.lanes_per_tile;
  const int64_t t0 = (int64_t)blockIdx.x * tiles_per_wg;
  for (int i = tid; i < tiles_per_wg * kTE; i += kThreads) acc[i] = 0;
  __syncthreads();
  const int sub = tid / a.lanes_per_tile;
  const int l = tid - sub * a.lanes_per_tile;
  const int64_t t = t0 + sub;
  int32_t* my = acc + sub * kTE;
  if (t < a.T) {
    const int64_t tile_base = t * kTE;
    for (int c = l; c < a.nclients; c += a.lanes_per_tile) {
      const int64_t ib = (int64_t)c * (a.T + 1) + t;
      const uint64_t e0 = a.idx[ib], e1 = a.idx[ib + 1];
      const uint64_t bstart = e0 & kMask36, bend = e1 & kMask36;
      if (bend <= bstart) continue;
      int32_t rel = (int32_t)((int64_t)(e0 >> 36) - 1 - tile_base);  // last nonzero, tile-relative
      BitReader br;
      br.init(a.stream_buf + a.stream_off[c], a.stream_cap[c], bstart);
      int64_t rem = (int64_t)(bend - bstart);
      while (rem > 0) {
        uint32_t d;
        int32_t v;
        const uint32_t L = decode_code(br, d, v);
        rel += (int32_t)d;
        if (L == 0 || (uint32_t)rel >= (uint32_t)kTE) {
          atomicOr(a.err, 1);
          break;
        }
        atomicAdd(&my[rel], v);
        rem -= L;
      }
    }
  }
  __syncthreads();
  for (int i = tid; i < tiles_per_wg * kTE; i += kThreads) {
    const int64_t e = t0 * kTE + i;
    if (e >= a.P) break;
    int32_t v = acc[i];
    if (a.sum_in) v = (int32_t)((uint32_t)v + (uint32_t)a.sum_in[e]);
    if (a.sum_out) a.sum_out[e] = v;
    if (a.out) {
      float f = (float)v;
      if (a.noise_sum) f = f + a.noise_sum[e];
      a.out[e] = f * a.step;
    }
  }
}

// ---------------------------------------------------------------------------
// Elementwise kernels.
// ---------------------------------------------------------------------------
template <int MODE>
__global__ void k_quantize(const float* __restrict__ x, int64_t P, float step, Key4 key,
                           int32_t* __restrict__ q, float* __restrict__ noise) {
  const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t e0 = g * 4;
  if (e0 >= P) return;
  uint4 rb = make_uint4(0, 0, 0, 0);
  if (MODE != FC_UNIFORM) rb = philox_group(key, (uint32_t)g);
  const uint32_t rr[4] = {rb.x, rb.y, rb.z, rb.w};
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    if (e0 + k < P) {
      float deq, nz;
      q[e0 + k] = quantize_one<MODE>(x[e0 + k], step, 0.0f, rr[k], deq, nz);
      if (noise) noise[e0 + k] = (MODE == FC_UNIFORM) ? 0.0f : (MODE == FC_DITHERED ? nz : u01(rr[k]) - 0.5f);
    }
  }
}

__global__ void k_dequantize(const int32_t* __restrict__ s, int64_t P, float step,
                             const float* __restrict__ noise_sum, float* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= P) return;
  float f = (float)s[i];
  if (noise_sum) f = f + noise_sum[i];
  out[i] = f * step;
}

__global__ void k_noise_sum(const int64_t* __restrict__ seeds, int32_t n, int64_t P,
                            float* __restrict__ out) {
  const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t e0 = g * 4;
  if (e0 >= P) return;
  float s[4] = {0.f, 0.f, 0.f, 0.f};
  for (int c = 0; c < n; ++c) {
    const Key4 key = tf_seed_scramble(seeds[2 * c], seeds[2 * c + 1]);
    const uint4 rb = philox_group(key, (uint32_t)g);
    s[0] = s[0] + (u01(rb.x) - 0.5f);
    s[1] = s[1] + (u01(rb.y) - 0.5f);
    s[2] = s[2] + (u01(rb.z) - 0.5f);
    s[3] = s[3] + (u01(rb.w) - 0.5f);
  }
#pragma unroll
  for (int k = 0; k < 4; ++k)
    if (e0 + k < P) out[e0 + k] = s[k];
}

// Per-client norm: one workgroup per client, float64 accumulation, fixed order.
__global__ __launch_bounds__(kThreads) void k_client_norms(const float* const* xs, int64_t P,
                                                           int kind, float* norms) {
  __shared__ double red[kThreads];
  const int c = blockIdx.x;
  const float* x = xs[c];
  double acc = 0.0;
  for (int64_t i = threadIdx.x; i < P; i += kThreads) {
    const float v = x[i] + 0.0f;  // DAZ
    const double a = fabs((double)v);
    if (kind == FC_NORM_MAX_MAGNITUDE || kind == FC_NORM_LINF) acc = a > acc ? a : acc;
    else if (kind == FC_NORM_MEAN_MAGNITUDE) acc += a;
    else acc += a * a;
  }
  red[threadIdx.x] = acc;
  __syncthreads();
  for (int o = kThreads / 2; o > 0; o >>= 1) {
    if (threadIdx.x < o) {
      const double b = red[threadIdx.x + o];
      red[threadIdx.x] = (kind == FC_NORM_MAX_MAGNITUDE || kind == FC_NORM_LINF) ? fmax(red[threadIdx.x], b)
                                                                               : red[threadIdx.x] + b;
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    double r = red[0];
    if (kind == FC_NORM_MEAN_MAGNITUDE) r = r / (double)P;
    if (kind == FC_NORM_DIMENSIONLESS) r = sqrt(r / (double)P);
    if (kind == FC_NORM_L2) r = sqrt(r);
    norms[c] = (float)r;
  }
}

__global__ __launch_bounds__(kThreads) void k_finalize(const float* dist_part, const int32_t* nnz_part,
                                                       int32_t T, double* dist, int64_t* nnz) {
  __shared__ double rd[kThreads];
  __shared__ long long rn[kThreads];
  const int c = blockIdx.x;
  double d = 0.0;
  long long n = 0;
  for (int t = threadIdx.x; t < T; t += kThreads) {
    if (dist_part) d += (double)dist_part[(int64_t)c * T + t];
    if (nnz_part) n += nnz_part[(int64_t)c * T + t];
  }
  rd[threadIdx.x] = d;
  rn[threadIdx.x] = n;
  __syncthreads();
  for (int o = kThreads / 2; o > 0; o >>= 1) {
    if (threadIdx.x < o) {
      rd[threadIdx.x] += rd[threadIdx.x + o];
      rn[threadIdx.x] += rn[threadIdx.x + o];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    if (dist) dist[c] = rd[0];
    if (nnz) nnz[c] = rn[0];
  }
}

// One-bit SGD (one_bit_sgd.py:56-81): pass 1 = masks + masked sums per client.
__global__ __launch_bounds__(kThreads) void k_onebit_encode(const float* const* xs, int64_t P,
                                                            float thr, uint32_t* masks, float* means,
                                                            double* dist) {
  __shared__ double r0[kThreads], r1[kThreads], r2[kThreads], r3[kThreads];
  const int c = blockIdx.x;
  const float* x = xs[c];
  const int64_t nw = (P + 31) / 32;
  uint32_t* m = masks + (int64_t)c * nw;
  double sb = 0, sa = 0, nb = 0, na = 0;
  for (int64_t w = threadIdx.x; w < nw; w += kThreads) {
    uint32_t bits = 0;
    for (int k = 0; k < 32; ++k) {
      const int64_t i = w * 32 + k;
      if (i >= P) break;
      const float v = x[i] + 0.0f;
      if (v < thr) {
        sb += v;
        nb += 1;
      } else {
        sa += v;
        na += 1;
        bits |= 1u << k;
      }
    }
    m[w] = bits;
  }
  r0[threadIdx.x] = sb; r1[threadIdx.x] = sa; r2[threadIdx.x] = nb; r3[threadIdx.x] = na;
  __syncthreads();
  for (int o = kThreads / 2; o > 0; o >>= 1) {
    if (threadIdx.x < o) {
      r0[threadIdx.x] += r0[threadIdx.x + o];
      r1[threadIdx.x] += r1[threadIdx.x + o];
      r2[threadIdx.x] += r2[threadIdx.x + o];
      r3[threadIdx.x] += r3[threadIdx.x + o];
    }
    __syncthreads();
  }
  __shared__ float mb_s, ma_s;
  if (threadIdx.x == 0) {
    const float mb = (float)r0[0] / fmaxf((float)r2[0], 1.0f);
    const float ma = (float)r1[0] / fmaxf((float)r3[0], 1.0f);
    means[2 * c] = mb;
    means[2 * c + 1] = ma;
    mb_s = mb;
    ma_s = ma;
  }
  __syncthreads();
  double dd = 0;
  for (int64_t i = threadIdx.x; i < P; i += kThreads) {
    const float v = x[i] + 0.0f;
    const float dec = (v < thr) ? mb_s : ma_s;
    const float e = v - dec;
    dd += (double)(e * e);
  }
  r0[threadIdx.x] = dd;
  __syncthreads();
  for (int o = kThreads / 2; o > 0; o >>= 1) {
    if (threadIdx.x < o) r0[threadIdx.x] += r0[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) dist[c] = r0[0];
}

__global__ void k_onebit_decode_sum(const uint32_t* masks, const float* means, int32_t n,
                                    int64_t P, float* out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= P) return;
  const int64_t nw = (P + 31) / 32;
  float s = 0.0f;
  for (int c = 0; c < n; ++c) {
    const uint32_t bit = (masks[(int64_t)c * nw + (i >> 5)] >> (i & 31)) & 1u;
    const float above = bit ? 1.0f : 0.0f;
    const float dec = above * means[2 * c + 1] + (1.0f - above) * means[2 * c];
    s = s + dec;
  }
  out[i] = s;
}

// ---------------------------------------------------------------------------
// Host side.
// ---------------------------------------------------------------------------
thread_local std::string g_err;

int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

int check_launch(const char* what) {
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return fail(-10, std::string(what) + ": " + hipGetErrorString(e));
  return 0;
}

int64_t tiles_for(int64_t P) { return (P + kTE - 1) / kTE; }

int64_t enc_status_bytes(int32_t n, int64_t P) { return ((int64_t)n * tiles_for(P) * 16 + 64 + 255) & ~255LL; }

int encode_common(const void* const* xs, int32_t nclients, int64_t P, float step, const float* norms,
                  const float* prescale, const int64_t* seeds, int mode, bool int_in, uint8_t* stream_buf,
                  const int64_t* stream_off, const int64_t* stream_cap, uint64_t* idx,
                  int64_t* total_bits, float* dist_part, int32_t* nnz_part, int32_t* overflow,
                  void* workspace, int64_t workspace_bytes, void* stream) {
  if (nclients <= 0) return fail(-1, "nclients must be > 0");
  if (P <= 0 || P > FC_MAX_ELEMS) return fail(-1, "P must be in [1, 2^26 - 1]");
  if (!xs || !stream_buf || !stream_off || !stream_cap || !idx || !total_bits || !overflow)
    return fail(-1, "null required pointer");
  if (!int_in && mode != FC_UNIFORM && !seeds) return fail(-1, "seeds required for stochastic/dithered");
  if (mode < 0 || mode > 2) return fail(-1, "mode must be 0 (uniform), 1 (stochastic) or 2 (dithered)");
  if (!int_in && !(step > 0.0f) && !norms) return fail(-1, "step must be > 0");
  const int64_t need = fc_encode_workspace_bytes(nclients, P);
  if (!workspace || workspace_bytes < need || ((uintptr_t)workspace & 15))
    return fail(-1, "workspace too small or misaligned");
  hipStream_t s = (hipStream_t)stream;
  const int64_t T = tiles_for(P);
  const int64_t sb = enc_status_bytes(nclients, P);
  if (hipMemsetAsync(workspace, 0, sb, s) != hipSuccess) return fail(-10, "memset status");
  if (hipMemsetAsync(overflow, 0, sizeof(int32_t) * nclients, s) != hipSuccess) return fail(-10, "memset overflow");
  EncodeArgs a;
  a.xs = xs;
  a.nclients = nclients;
  a.P = P;
  a.T = (int32_t)T;
  a.step = step;
  a.norms = norms;
  a.prescale = int_in ? nullptr : prescale;
  a.seeds = seeds;
  a.stream_buf = stream_buf;
  a.stream_off = stream_off;
  a.stream_cap = stream_cap;
  a.idx = idx;
  a.total_bits = total_bits;
  a.dist_part = dist_part;
  a.nnz_part = nnz_part;
  a.overflow = overflow;
  a.status = (uint64_t*)workspace;
  a.counter = (uint32_t*)((uint8_t*)workspace + (int64_t)nclients * T * 16);
  a.spin_err = a.counter + 4;
  int dev = 0, ncu = 256;
  (void)hipGetDevice(&dev);
  (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
  const int64_t total = (int64_t)nclients * T;
  // few clients: cap the tiles in flight per client so look-back windows stay short
  int64_t max_grid = std::min<int64_t>((int64_t)ncu * 8, std::max<int64_t>(128, 64LL * nclients));
  if (const char* g = getenv("FEDCODEC_ENC_GRID")) max_grid = std::max(1L, atol(g));  // test knob
  const int grid = (int)std::min<int64_t>(total, max_grid);
  // power-of-two step (no per-client normalisation): x / step == x * (1 / step)
  int ex = 0;
  const bool pow2 = !int_in && !norms && std::frexp(step, &ex) == 0.5f && std::isnormal(1.0f / step);
  a.rcp = pow2 ? 1.0f / step : 0.0f;
  const dim3 g(grid), b(kThreads);
  if (int_in) {
    hipLaunchKernelGGL((k_encode<FC_UNIFORM, true, false>), g, b, 0, s, a);
  } else if (mode == FC_UNIFORM) {
    if (pow2) hipLaunchKernelGGL((k_encode<FC_UNIFORM, false, true>), g, b, 0, s, a);
    else hipLaunchKernelGGL((k_encode<FC_UNIFORM, false, false>), g, b, 0, s, a);
  } else if (mode == FC_STOCHASTIC) {
    if (pow2) hipLaunchKernelGGL((k_encode<FC_STOCHASTIC, false, true>), g, b, 0, s, a);
    else hipLaunchKernelGGL((k_encode<FC_STOCHASTIC, false, false>), g, b, 0, s, a);
  } else {
    if (pow2) hipLaunchKernelGGL((k_encode<FC_DITHERED, false, true>), g, b, 0, s, a);
    else hipLaunchKernelGGL((k_encode<FC_DITHERED, false, false>), g, b, 0, s, a);
  }
  return check_launch("k_encode");
}

}  // namespace

extern "C" {

const char* fc_last_error(void) { return g_err.c_str(); }
const char* fc_version(void) { return "fedcodec 0.1 gfx950"; }
#ifdef FC_STAMPS
int fc_debug_stamps(unsigned long long* host8, int reset) {
  if (hipMemcpyFromSymbol(host8, HIP_SYMBOL(g_stamps), sizeof(unsigned long long) * 8) != hipSuccess) return -1;
  if (reset) {
    unsigned long long z[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_stamps), z, sizeof(z)) != hipSuccess) return -1;
  }
  return 0;
}
#endif
int64_t fc_num_tiles(int64_t P) { return P <= 0 ? 0 : tiles_for(P); }
int64_t fc_encode_workspace_bytes(int32_t nclients, int64_t P) {
  if (nclients <= 0 || P <= 0) return 256;
  return enc_status_bytes(nclients, P);
}

int fc_quantize(const float* x, int64_t P, float step, int64_t seed0, int64_t seed1, int mode,
                int32_t* q, float* noise, void* stream) {
  if (P < 0 || P > FC_MAX_ELEMS) return fail(-1, "P out of range");
  if (P == 0) return 0;
  if (!x || !q) return fail(-1, "null pointer");
  if (mode < 0 || mode > 2) return fail(-1, "bad mode");
  const Key4 key = tf_seed_scramble(seed0, seed1);
  const int64_t groups = (P + 3) / 4;
  const dim3 grid((unsigned)((groups + 255) / 256));
  hipStream_t s = (hipStream_t)stream;
  if (mode == FC_UNIFORM) hipLaunchKernelGGL((k_quantize<FC_UNIFORM>), grid, dim3(256), 0, s, x, P, step, key, q, noise);
  else if (mode == FC_STOCHASTIC) hipLaunchKernelGGL((k_quantize<FC_STOCHASTIC>), grid, dim3(256), 0, s, x, P, step, key, q, noise);
  else hipLaunchKernelGGL((k_quantize<FC_DITHERED>), grid, dim3(256), 0, s, x, P, step, key, q, noise);
  return check_launch("k_quantize");
}

int fc_quantize_encode(const float* const* xs, int32_t nclients, int64_t P, float step,
                       const float* norms, const float* prescale, const int64_t* seeds, int mode, uint8_t* stream_buf,
                       const int64_t* stream_off, const int64_t* stream_cap, uint64_t* idx,
                       int64_t* total_bits, float* dist_part, int32_t* nnz_part, int32_t* overflow,
                       void* workspace, int64_t workspace_bytes, void* stream) {
  return encode_common((const void* const*)xs, nclients, P, step, norms, prescale, seeds, mode, false, stream_buf,
                       stream_off, stream_cap, idx, total_bits, dist_part, nnz_part, overflow, workspace,
                       workspace_bytes, stream);
}

int fc_rlgamma_encode(const int32_t* const* qs, int32_t nclients, int64_t P, uint8_t* stream_buf,
                      const int64_t* stream_off, const int64_t* stream_cap, uint64_t* idx,
                      int64_t* total_bits, int32_t* overflow, void* workspace, int64_t workspace_bytes,
                      void* stream) {
  return encode_common((const void* const*)qs, nclients, P, 1.0f, nullptr, nullptr, nullptr, FC_UNIFORM, true,
                       stream_buf, stream_off, stream_cap, idx, total_bits, nullptr, nullptr, overflow,
                       workspace, workspace_bytes, stream);
}

int fc_decode_accumulate(const uint8_t* stream_buf, const int64_t* stream_off, const int64_t* stream_cap,
                         const uint64_t* idx, int32_t nclients, int64_t P, const int32_t* sum_in,
                         int32_t* sum_out, float* out, float step, const float* noise_sum, int32_t* err,
                         void* stream) {
  if (nclients <= 0) return fail(-1, "nclients must be > 0");
  if (P <= 0 || P > FC_MAX_ELEMS) return fail(-1, "P must be in [1, 2^26 - 1]");
  if (!stream_buf || !stream_off || !stream_cap || !idx || !err) return fail(-1, "null required pointer");
  if (!sum_out && !out) return fail(-1, "one of sum_out / out required");
  DecodeArgs a;
  a.stream_buf = stream_buf;
  a.stream_off = stream_off;
  a.stream_cap = stream_cap;
  a.idx = idx;
  a.nclients = nclients;
  a.P = P;
  a.T = (int32_t)tiles_for(P);
  int lpt = 256;
  while (lpt > 64 && lpt / 2 >= nclients) lpt /= 2;
  a.lanes_per_tile = lpt;
  a.sum_in = sum_in;
  a.sum_out = sum_out;
  a.out = out;
  a.step = step;
  a.noise_sum = noise_sum;
  a.err = err;
  const int tpw = kThreads / lpt;
  const dim3 grid((unsigned)((a.T + tpw - 1) / tpw));
  hipStream_t s = (hipStream_t)stream;
  if (hipMemsetAsync(err, 0, sizeof(int32_t), s) != hipSuccess) return fail(-10, "memset err");
  hipLaunchKernelGGL(k_decode, grid, dim3(kThreads), (size_t)tpw * kTE * sizeof(int32_t), s, a);
  return check_launch("k_decode");
}

int fc_dequantize(const int32_t* sum, int64_t P, float step, const float* noise_sum, float* out,
                  void* stream) {
  if (P < 0) return fail(-1, "P < 0");
  if (P == 0) return 0;
  if (!sum || !out) return fail(-1, "null pointer");
  hipLaunchKernelGGL(k_dequantize, dim3((unsigned)((P + 255) / 256)), dim3(256), 0, (hipStream_t)stream, sum, P,
                     step, noise_sum, out);
  return check_launch("k_dequantize");
}

int fc_noise_sum(const int64_t* seeds, int32_t nclients, int64_t P, float* noise_sum, void* stream) {
  if (P < 0 || nclients < 0) return fail(-1, "bad sizes");
  if (P == 0) return 0;
  if (!seeds || !noise_sum) return fail(-1, "null pointer");
  const int64_t groups = (P + 3) / 4;
  hipLaunchKernelGGL(k_noise_sum, dim3((unsigned)((groups + 255) / 256)), dim3(256), 0, (hipStream_t)stream, seeds,
                     nclients, P, noise_sum);
  return check_launch("k_noise_sum");
}

int fc_client_norms(const float* const* xs, int32_t nclients, int64_t P, int kind, float* norms, void* stream) {
  if (nclients <= 0 || P <= 0) return fail(-1, "bad sizes");
  if (kind < 1 || kind > 5) return fail(-1, "bad norm kind");
  if (!xs || !norms) return fail(-1, "null pointer");
  hipLaunchKernelGGL(k_client_norms, dim3(nclients), dim3(kThreads), 0, (hipStream_t)stream, xs, P, kind, norms);
  return check_launch("k_client_norms");
}

int fc_finalize(const float* dist_part, const int32_t* nnz_part, int32_t nclients, int64_t P, double* dist,
                int64_t* nnz, void* stream) {
  if (nclients <= 0 || P <= 0) return fail(-1, "bad sizes");
  hipLaunchKernelGGL(k_finalize, dim3(nclients), dim3(kThreads), 0, (hipStream_t)stream, dist_part, nnz_part,
                     (int32_t)tiles_for(P), dist, nnz);
  return check_launch("k_finalize");
}

int fc_onebit_encode(const float* const* xs, int32_t nclients, int64_t P, float threshold, uint32_t* masks,
                     float* means, double* dist, void* stream) {
  if (nclients <= 0 || P <= 0) return fail(-1, "bad sizes");
  if (!xs || !masks || !means || !dist) return fail(-1, "null pointer");
  hipLaunchKernelGGL(k_onebit_encode, dim3(nclients), dim3(kThreads), 0, (hipStream_t)stream, xs, P, threshold,
                     masks, means, dist);
  return check_launch("k_onebit_encode");
}

int fc_onebit_decode_sum(const uint32_t* masks, const float* means, int32_t nclients, int64_t P, float* out,
                         void* stream) {
  if (nclients <= 0 || P <= 0) return fail(-1, "bad sizes");
  if (!masks || !means || !out) return fail(-1, "null pointer");
  hipLaunchKernelGGL(k_onebit_decode_sum, dim3((unsigned)((P + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                     masks, means, nclients, P, out);
  return check_launch("k_onebit_decode_sum");
}

}  // extern "C"
