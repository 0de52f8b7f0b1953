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
#include <string>

#include "../../include/fedcodec.h"

namespace {

constexpr int kTE = FC_TILE_ELEMS;  // elements per tile
constexpr int kThreads = 256;       // 4 waves of 64
constexpr int kWinWords = 2048;     // LDS bit window per emission pass (64 Kbit)
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
// client-side dequantised value (quantize_encode.py:148-149).
template <int MODE>
__device__ __forceinline__ int32_t quantize_one(float x, float step, uint32_t rbits,
                                                float& deq, float& noise) {
  const float sc = x / step;  // IEEE-correct division, FTZ/DAZ
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
  const float* norms;
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
  uint32_t win[kWinWords];
  int32_t wave_last[4];
  int32_t wave_first[4];
  uint32_t wave_bits[4];
  float wave_dist[4];
  int32_t wave_nnz[4];
  uint32_t tail;
  uint32_t ticket;
  // look-back results broadcast to the workgroup
  uint64_t b0;
  int32_t last_before;
  uint32_t tail_before;
  uint32_t r0_R0;      // window bit where the body starts = (b0 % 32) + R0
  uint32_t nwin_bits;  // bits in the window (incl. trailing code on the last tile)
  uint64_t trail;      // trailing run code value
  uint32_t trail_len;
};

// Emit a piece of <= 32 bits at window bit position wp into the LDS window for
// pass `pass` (window words [pass*kWinWords, (pass+1)*kWinWords)).
__device__ __forceinline__ void win_emit32(uint32_t* win, uint32_t v, uint32_t L, uint64_t wp,
                                           uint64_t pass_lo) {
  if (L == 0) return;
  const uint64_t w = wp >> 5;
  const uint32_t o = (uint32_t)(wp & 31);
  const uint64_t X = (uint64_t)v << (64 - o - L);
  const uint32_t hi = (uint32_t)(X >> 32), lo = (uint32_t)X;
  const int64_t i0 = (int64_t)w - (int64_t)pass_lo;
  if (i0 >= 0 && i0 < kWinWords && hi) atomicOr(&win[i0], hi);
  if (o + L > 32 && i0 + 1 >= 0 && i0 + 1 < kWinWords && lo) atomicOr(&win[i0 + 1], lo);
}

__device__ __forceinline__ void win_emit(uint32_t* win, uint64_t v, uint32_t L, uint64_t wp,
                                         uint64_t pass_lo) {
  if (L > 32) {
    win_emit32(win, (uint32_t)(v >> 32), L - 32, wp, pass_lo);
    win_emit32(win, (uint32_t)v, 32, wp + (L - 32), pass_lo);
  } else {
    win_emit32(win, (uint32_t)v, L, wp, pass_lo);
  }
}

// OR the part of a piece (ending at body position `end`) that falls in the last
// 32 body bits into the tail word.
__device__ __forceinline__ void tail_emit(uint32_t* tailw, uint64_t v, uint32_t L, uint64_t end,
                                          uint64_t body) {
  const uint64_t s = body - end;
  if (s < 32 && L) {
    const uint32_t c = (uint32_t)(v << s);
    if (c) atomicOr(tailw, c);
  }
}

template <int MODE, bool INT_IN>
__global__ __launch_bounds__(kThreads) void k_encode(EncodeArgs a) {
  __shared__ EncShared sh;
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wv = tid >> 6;
  const uint32_t total_tiles = (uint32_t)a.nclients * (uint32_t)a.T;

  for (int i = tid; i < kWinWords; i += kThreads) sh.win[i] = 0;

  for (;;) {
    if (tid == 0) sh.ticket = atomicAdd(a.counter, 1u);
    __syncthreads();
    const uint32_t ticket = sh.ticket;
    if (ticket >= total_tiles) break;
    const int32_t c = (int32_t)(ticket / (uint32_t)a.T);
    const int32_t t = (int32_t)(ticket - (uint32_t)c * (uint32_t)a.T);
    const int64_t P = a.P;
    const int64_t tile_base = (int64_t)t * kTE;
    const bool last_tile = (t == a.T - 1);

    // ---- load + quantise: thread owns 4 chunks of 4 consecutive elements ----
    int32_t q[4][4];
    float dist = 0.0f;
    int32_t nnz = 0;
    {
      float step = a.step;
      if (!INT_IN && a.norms) step = a.norms[c] * a.step;
      Key4 key{0, 0, 0, 0};
      if (!INT_IN && MODE != FC_UNIFORM) key = tf_seed_scramble(a.seeds[2 * c], a.seeds[2 * c + 1]);
      const void* xp = a.xs[c];
      const bool aligned = (((uintptr_t)xp) & 15) == 0;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int64_t e0 = tile_base + 1024 * wv + 256 * j + 4 * lane;
        if (INT_IN) {
          const int32_t* qp = (const int32_t*)xp;
          if (aligned && e0 + 3 < P) {
            const int4 v = *(const int4*)(qp + e0);
            q[j][0] = v.x; q[j][1] = v.y; q[j][2] = v.z; q[j][3] = v.w;
          } else {
#pragma unroll
            for (int k = 0; k < 4; ++k) q[j][k] = (e0 + k < P) ? qp[e0 + k] : 0;
          }
        } else {
          const float* fp = (const float*)xp;
          float xv[4];
          if (aligned && e0 + 3 < P) {
            const float4 v = *(const float4*)(fp + e0);
            xv[0] = v.x; xv[1] = v.y; xv[2] = v.z; xv[3] = v.w;
          } else {
#pragma unroll
            for (int k = 0; k < 4; ++k) xv[k] = (e0 + k < P) ? fp[e0 + k] : 0.0f;
          }
          uint4 rb = make_uint4(0, 0, 0, 0);
          if (MODE != FC_UNIFORM) rb = philox_group(key, (uint32_t)(e0 >> 2));
          const uint32_t rr[4] = {rb.x, rb.y, rb.z, rb.w};
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            float deq, noise;
            const int32_t qq = quantize_one<MODE>(xv[k], step, rr[k], deq, noise);
            const bool valid = e0 + k < P;
            q[j][k] = valid ? qq : 0;
            const float dd = xv[k] - deq;
            dist += valid ? dd * dd : 0.0f;
          }
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) nnz += q[j][k] != 0;
      }
    }

    // ---- max-scan of nonzero positions (tile-relative), wave level ----
    int32_t chunk_prev[4];  // last nonzero before this chunk within the wave, or -1
    int32_t carry = -1, wfirst = 0x7FFFFFFF;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int32_t rel0 = 1024 * wv + 256 * j + 4 * lane;
      int32_t cl = -1, cf = 0x7FFFFFFF;
#pragma unroll
      for (int k = 3; k >= 0; --k)
        if (q[j][k] != 0) cf = rel0 + k;
#pragma unroll
      for (int k = 0; k < 4; ++k)
        if (q[j][k] != 0) cl = rel0 + k;
      wfirst = min(wfirst, cf);
      const int32_t incl = wave_incl_max(cl, lane);
      int32_t excl = __shfl_up(incl, 1, 64);
      if (lane == 0) excl = -1;
      chunk_prev[j] = max(excl, carry);
      carry = max(carry, __shfl(incl, 63, 64));
    }
    wfirst = wave_min(wfirst);
    if (lane == 0) {
      sh.wave_last[wv] = carry;
      sh.wave_first[wv] = wfirst;
    }
    __syncthreads();
    int32_t wave_in = -1;
    for (int w = 0; w < wv; ++w) wave_in = max(wave_in, sh.wave_last[w]);
    int32_t tile_first = 0x7FFFFFFF, tile_last = -1;
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      tile_first = min(tile_first, sh.wave_first[w]);
      tile_last = max(tile_last, sh.wave_last[w]);
    }

    // ---- code lengths of the body and wave-level sum-scan ----
    uint32_t chunk_off[4];
    uint32_t wbits = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int32_t rel0 = 1024 * wv + 256 * j + 4 * lane;
      int32_t prev = max(chunk_prev[j], wave_in);
      uint32_t bits = 0;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int32_t v = q[j][k];
        if (v != 0) {
          const uint32_t rl = prev >= 0 ? glen((uint32_t)(rel0 + k - prev)) : 0u;
          bits += rl + 1u + glen(mag_u32(v));
          prev = rel0 + k;
        }
      }
      const uint32_t incl = wave_incl_sum(bits, lane);
      chunk_off[j] = wbits + incl - bits;
      wbits += __shfl(incl, 63, 64);
    }
    if (lane == 0) sh.wave_bits[wv] = wbits;
    // per-wave measurement partials
    {
      float d = dist;
      int32_t n = nnz;
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) {
        d += __shfl_xor(d, o, 64);
        n += __shfl_xor(n, o, 64);
      }
      if (lane == 0) {
        sh.wave_dist[wv] = d;
        sh.wave_nnz[wv] = n;
      }
    }
    if (tid == 0) sh.tail = 0;
    __syncthreads();
    uint32_t woff = 0, body = 0;
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      woff += (w < wv) ? sh.wave_bits[w] : 0u;
      body += sh.wave_bits[w];
    }
    if (tid == 0) {
      const float d = ((sh.wave_dist[0] + sh.wave_dist[1]) + sh.wave_dist[2]) + sh.wave_dist[3];
      const int32_t n = sh.wave_nnz[0] + sh.wave_nnz[1] + sh.wave_nnz[2] + sh.wave_nnz[3];
      if (a.dist_part) a.dist_part[(int64_t)c * a.T + t] = d;
      if (a.nnz_part) a.nnz_part[(int64_t)c * a.T + t] = n;
    }

    // ---- tail: last 32 bits of the body ----
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const uint32_t off = woff + chunk_off[j];
      if (off + 4 * 89 + 32 < body) continue;  // cannot reach the last 32 bits
      const int32_t rel0 = 1024 * wv + 256 * j + 4 * lane;
      int32_t prev = max(chunk_prev[j], wave_in);
      uint64_t pos = off;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int32_t v = q[j][k];
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
    __syncthreads();

    // ---- publish aggregate, decoupled look-back (wave 0) ----
    uint64_t* st = a.status + 2 * ((int64_t)c * a.T + t);
    if (wv == 0) {
      Seg agg;
      agg.has_nz = tile_last >= 0;
      agg.first = agg.has_nz ? (int32_t)(tile_base + tile_first) : 0;
      agg.last = agg.has_nz ? (int32_t)(tile_base + tile_last) : 0;
      agg.body = body;
      agg.tail = sh.tail;
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
        Seg S;
        S.has_nz = 0;
        S.first = S.last = 0;
        S.body = 0;
        S.tail = 0;
        int64_t base = (int64_t)t - 1;
        for (;;) {
          const int64_t ti = base - lane;
          uint64_t w1 = kFlagPre, w2 = kFlagPre;  // ti < 0: virtual root prefix
          if (ti >= 0) {
            const uint64_t* sp = a.status + 2 * ((int64_t)c * a.T + ti);
            uint32_t spins = 0;
            for (;;) {
              w1 = ld_agent(sp);
              w2 = ld_agent(sp + 1);
              if ((w1 >> 62) != 0 && (w1 >> 62) == (w2 >> 62)) break;
              __builtin_amdgcn_s_sleep(1);
              if (++spins > (1u << 26)) {
                atomicOr(a.spin_err, 1u);
                w1 = kFlagPre;
                w2 = kFlagPre;
                break;
              }
            }
          }
          const bool is_pre = (w1 >> 62) == 2;
          const uint64_t pm = __ballot(is_pre);
          const int k = pm ? __builtin_ctzll(pm) : 64;
          Seg v;
          if (lane <= k && ti >= -1) {
            v = seg_from_status(w1, w2, ti * kTE);
          } else {
            v.has_nz = 0;
            v.first = v.last = 0;
            v.body = 0;
            v.tail = 0;
          }
          // suffix scan: lane l <- combine(lanes [l+d ...], lane l)
#pragma unroll
          for (int d = 1; d < 64; d <<= 1) {
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
          W.has_nz = __shfl(v.has_nz, 0, 64);
          W.first = __shfl(v.first, 0, 64);
          W.last = __shfl(v.last, 0, 64);
          W.body = __shfl(v.body, 0, 64);
          W.tail = __shfl(v.tail, 0, 64);
          S = seg_combine(W, S);
          if (k < 64) break;
          base -= 64;
        }
        excl = S;
      }
      // excl is a root segment: body = stream bits before this tile.
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
        uint64_t nbits = (uint64_t)r0 + R0 + body;
        uint32_t tl = 0;
        uint64_t tv = 0;
        if (last_tile) {
          const int64_t zc = P - 1 - (int64_t)incl.last;  // trailing zeros
          if (zc > 0) {
            tv = (uint64_t)(zc + 1);
            tl = 2u * (63u - (uint32_t)__clzll(tv)) + 1u;
          }
          a.idx[ib + a.T] = (incl.body & kMask36) | ((uint64_t)(incl.last + 1) << 36);
          a.total_bits[c] = (int64_t)incl.body + tl;
        }
        sh.trail = tv;
        sh.trail_len = tl;
        sh.nwin_bits = (uint32_t)(nbits + tl);
      }
    }
    __syncthreads();

    // ---- emit the code into the LDS window, then store owned words ----
    const uint64_t b0 = sh.b0;
    const uint32_t bstart = sh.r0_R0;
    const uint32_t nwin_bits = sh.nwin_bits;
    const int32_t last_before = sh.last_before;
    const uint32_t nwords_owned = last_tile ? (nwin_bits + 31) / 32 : nwin_bits / 32;
    const uint32_t npass = (nwords_owned + kWinWords - 1) / kWinWords;
    const int64_t cap = a.stream_cap[c];
    uint32_t* out32 = (uint32_t*)(a.stream_buf + a.stream_off[c]);
    const uint64_t w0 = b0 >> 5;
    if (tid == 0 && (int64_t)(w0 + nwords_owned) * 4 > cap) atomicOr((uint32_t*)&a.overflow[c], 1u);
    for (uint32_t pass = 0; pass < npass; ++pass) {
      const uint64_t plo = (uint64_t)pass * kWinWords;
      if (tid == 0) {
        const uint32_t r0 = (uint32_t)(b0 & 31);
        if (r0) win_emit32(sh.win, sh.tail_before & ((1u << r0) - 1u), r0, 0, plo);
        if (tile_last >= 0) {
          const uint32_t d = (uint32_t)(tile_base + tile_first - last_before);
          win_emit(sh.win, d, glen(d), r0, plo);
        }
        if (sh.trail_len) win_emit(sh.win, sh.trail, sh.trail_len, (uint64_t)bstart + body, plo);
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int32_t rel0 = 1024 * wv + 256 * j + 4 * lane;
        int32_t prev = max(chunk_prev[j], wave_in);
        uint64_t pos = (uint64_t)bstart + woff + chunk_off[j];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const int32_t v = q[j][k];
          if (v == 0) continue;
          const uint32_t m = mag_u32(v);
          const uint32_t ml = glen(m);
          const uint64_t sm = ((uint64_t)(v > 0) << ml) | m;
          if (prev >= 0) {
            const uint32_t d = (uint32_t)(rel0 + k - prev);
            const uint32_t rl = glen(d);
            if (rl + 1 + ml <= 32) {
              win_emit32(sh.win, (uint32_t)(((uint64_t)d << (1 + ml)) | sm), rl + 1 + ml, pos, plo);
            } else {
              win_emit32(sh.win, d, rl, pos, plo);
              win_emit(sh.win, sm, 1 + ml, pos + rl, plo);
            }
            pos += rl + 1 + ml;
          } else {
            win_emit(sh.win, sm, 1 + ml, pos, plo);
            pos += 1 + ml;
          }
          prev = rel0 + k;
        }
      }
      __syncthreads();
      const uint32_t nw = min((uint32_t)kWinWords, nwords_owned - pass * kWinWords);
      for (uint32_t i = tid; i < nw; i += kThreads) {
        const uint64_t wi = w0 + plo + i;
        if ((int64_t)(wi + 1) * 4 <= cap) out32[wi] = bswap32(sh.win[i]);
      }
      __syncthreads();
      for (uint32_t i = tid; i < kWinWords; i += kThreads) sh.win[i] = 0;
      // the next ticket's __syncthreads (or the next pass's) orders this clear
      if (pass + 1 < npass) __syncthreads();
    }
  }
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

struct BitReader {
  const uint4* p;    // next 16-byte block to fetch
  const uint4* end;  // first block beyond the client's region
  uint4 nxt;         // prefetched block
  uint32_t blk[4];   // current block
  int bi;            // next word index in blk
  uint64_t win;      // next bits, MSB aligned
  int nwin;          // valid bits in win

  __device__ __forceinline__ uint4 fetch() {
    uint4 r = make_uint4(0, 0, 0, 0);
    if (p < end) r = *p;
    ++p;
    return r;
  }
  __device__ __forceinline__ void init(const uint8_t* base, int64_t cap, uint64_t bit) {
    const uint64_t blk_i = bit >> 7;
    p = (const uint4*)base + blk_i;
    end = (const uint4*)base + (cap >> 4);
    const uint4 b = fetch();
    nxt = fetch();
    blk[0] = bswap32(b.x); blk[1] = bswap32(b.y); blk[2] = bswap32(b.z); blk[3] = bswap32(b.w);
    const int wi = (int)((bit >> 5) & 3);
    bi = wi;
    win = 0;
    nwin = 0;
    refill();
    refill();
    const int skip = (int)(bit & 31);
    win <<= skip;
    nwin -= skip;
  }
  __device__ __forceinline__ uint32_t next_word() {
    if (bi == 4) {
      const uint4 b = nxt;
      nxt = fetch();
      blk[0] = bswap32(b.x); blk[1] = bswap32(b.y); blk[2] = bswap32(b.z); blk[3] = bswap32(b.w);
      bi = 0;
    }
    uint32_t w;
    switch (bi) {
      case 0: w = blk[0]; break;
      case 1: w = blk[1]; break;
      case 2: w = blk[2]; break;
      default: w = blk[3]; break;
    }
    ++bi;
    return w;
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
    win <<= n;
    nwin -= n;
    refill();
    return v;
  }
  // Gamma-coded value (1 .. 2^32-1).  Returns 0 on a malformed code.
  __device__ __forceinline__ uint32_t gamma() {
    int z = win ? __clzll(win) : 64;
    if (z > nwin) z = nwin;
    if (2 * z + 1 <= nwin) {
      const int L = 2 * z + 1;
      const uint32_t v = (uint32_t)(win >> (64 - L));
      win <<= L;
      nwin -= L;
      refill();
      return v;
    }
    // long code: consume the zeros first (at most 31 of them)
    int zeros = 0;
    for (;;) {
      int zz = win ? __clzll(win) : 64;
      if (zz > nwin) zz = nwin;
      zeros += zz;
      win = zz >= 64 ? 0 : win << zz;
      nwin -= zz;
      refill();
      if (zz < 32 || zeros > 31) break;
    }
    if (zeros > 31) return 0;
    return take(zeros + 1);
  }
};

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
      int64_t pos = (int64_t)(e0 >> 36) - 1;  // last nonzero before the tile
      BitReader br;
      br.init(a.stream_buf + a.stream_off[c], a.stream_cap[c], bstart);
      uint64_t consumed = bstart;
      while (consumed < bend) {
        const uint32_t d = br.gamma();
        const uint32_t s = br.take(1);
        const uint32_t m = br.gamma();
        consumed += 2 * (31 - __clz(d | 1)) + 1 + 1 + 2 * (31 - __clz(m | 1)) + 1;
        pos += d;
        const int64_t rel = pos - tile_base;
        if (d == 0 || m == 0 || rel < 0 || rel >= kTE) {
          atomicOr(a.err, 1);
          break;
        }
        atomicAdd(&my[rel], (int32_t)(s ? m : 0u - m));
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
      q[e0 + k] = quantize_one<MODE>(x[e0 + k], step, rr[k], deq, nz);
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
    if (kind == FC_NORM_MAX_MAGNITUDE) acc = a > acc ? a : acc;
    else if (kind == FC_NORM_MEAN_MAGNITUDE) acc += a;
    else acc += a * a;
  }
  red[threadIdx.x] = acc;
  __syncthreads();
  for (int o = kThreads / 2; o > 0; o >>= 1) {
    if (threadIdx.x < o) {
      const double b = red[threadIdx.x + o];
      red[threadIdx.x] = (kind == FC_NORM_MAX_MAGNITUDE) ? fmax(red[threadIdx.x], b) : red[threadIdx.x] + b;
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    double r = red[0];
    if (kind == FC_NORM_MEAN_MAGNITUDE) r = r / (double)P;
    if (kind == FC_NORM_DIMENSIONLESS) r = sqrt(r / (double)P);
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
                  const int64_t* seeds, int mode, bool int_in, uint8_t* stream_buf,
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
  const int grid = (int)std::min<int64_t>(total, (int64_t)ncu * 8);
  if (int_in) {
    hipLaunchKernelGGL((k_encode<FC_UNIFORM, true>), dim3(grid), dim3(kThreads), 0, s, a);
  } else if (mode == FC_UNIFORM) {
    hipLaunchKernelGGL((k_encode<FC_UNIFORM, false>), dim3(grid), dim3(kThreads), 0, s, a);
  } else if (mode == FC_STOCHASTIC) {
    hipLaunchKernelGGL((k_encode<FC_STOCHASTIC, false>), dim3(grid), dim3(kThreads), 0, s, a);
  } else {
    hipLaunchKernelGGL((k_encode<FC_DITHERED, false>), dim3(grid), dim3(kThreads), 0, s, a);
  }
  return check_launch("k_encode");
}

}  // namespace

extern "C" {

const char* fc_last_error(void) { return g_err.c_str(); }
const char* fc_version(void) { return "fedcodec 0.1 gfx950"; }
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
                       const float* norms, const int64_t* seeds, int mode, uint8_t* stream_buf,
                       const int64_t* stream_off, const int64_t* stream_cap, uint64_t* idx,
                       int64_t* total_bits, float* dist_part, int32_t* nnz_part, int32_t* overflow,
                       void* workspace, int64_t workspace_bytes, void* stream) {
  return encode_common((const void* const*)xs, nclients, P, step, norms, seeds, mode, false, stream_buf,
                       stream_off, stream_cap, idx, total_bits, dist_part, nnz_part, overflow, workspace,
                       workspace_bytes, stream);
}

int fc_rlgamma_encode(const int32_t* const* qs, int32_t nclients, int64_t P, uint8_t* stream_buf,
                      const int64_t* stream_off, const int64_t* stream_cap, uint64_t* idx,
                      int64_t* total_bits, int32_t* overflow, void* workspace, int64_t workspace_bytes,
                      void* stream) {
  return encode_common((const void* const*)qs, nclients, P, 1.0f, nullptr, nullptr, FC_UNIFORM, true,
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
  if (kind < 1 || kind > 3) return fail(-1, "bad norm kind");
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
