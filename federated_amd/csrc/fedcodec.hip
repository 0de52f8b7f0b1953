// fedcodec: MI355X (gfx950 / CDNA4) kernels for the compressed_communication/
// client-update codec, exported through the C ABI in include/fedcodec.h.
//
// Hot path (DESIGN.md "Kernels"):
//   k_encode  one pass over the fp32 client deltas: quantise (TF-CPU numerics,
//             Philox4x32-10 stochastic rounding), per-element run-length Elias
//             gamma code lengths, wavefront scans, single-pass decoupled
//             look-back across 1024-element tiles, LDS-staged MSB-first bit
//             packing, owner-writes-word stores (no memset, no global atomics on
//             the stream), per-tile decoder index.
//   k_decode  per 1024-element tile, one lane per client: sequential gamma
//             decode of that client's tile segment from the encoder index,
//             LDS int32 accumulation, fused dequantise epilogue.
//
// Compiled with -fgpu-flush-denormals-to-zero -ffp-contract=off: TF-CPU runs
// its Eigen kernels with FTZ/DAZ and without FMA contraction of these ops.
#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <cstdlib>
#include <algorithm>
#include <cmath>
#include <map>
#include <mutex>
#include <string>
#include <utility>

#include "../../include/fedcodec.h"

// Diagnostic ablation bits (performance experiments only; 0 in every real build):
//   1 skip LDS emission  2 skip stream stores  4 skip look-back  8 skip quantise math
#ifndef FC_ENC_WAVES
#define FC_ENC_WAVES 4  // encoder waves per SIMD the register budget is sized for (LDS: 4 per SIMD)
#endif
#ifndef FC_CHUNK_BARRIER
#define FC_CHUNK_BARRIER __builtin_amdgcn_sched_barrier(0)
#endif
#ifndef FC_ABL
#define FC_ABL 0
#endif

namespace {

constexpr int kTE = FC_TILE_ELEMS;  // elements per tile
constexpr int kThreads = 256;       // 4 waves of 64 (decoder and small kernels)
constexpr int kEncThreads = 64;     // encoder workgroup = one wavefront = one tile at a time
constexpr int kChunks = kTE / (4 * kEncThreads);  // 4 chunks of 4 elements per lane
#ifndef FC_WIN_WORDS
#define FC_WIN_WORDS 544
#endif
constexpr int kWinWords = FC_WIN_WORDS;  // per-wave LDS bit window (17 Kbit, ~16.9 bits/element)
constexpr uint32_t kNoPos = 0x3FFF; // "no nonzero" in a 14-bit (super-)tile-relative field
// Ticket streams: one device-scope atomic word saturates near 90 dequeues/us
// (MI355X_MICROARCH.md "dequeue"), so tickets come from kTicketShards counters,
// one 64-B line each; stream k hands out tickets k, k + K, k + 2K, ... in order.
constexpr int kTicketShards = 32;
constexpr int kShardStride = 16;  // uint32 words between counters (64 B)
// A wave's stream comes from its START ORDER, not from its blockIdx.  Progress: the
// smallest ticket m nobody has taken belongs to stream s; every wave of stream s
// holds only tickets below m, whose predecessors are all taken, so (by induction on
// m) they finish and one of them takes m -- provided stream s has a wave that has
// started, and a started wave stays resident until its stream is exhausted.
// With blockIdx streams (round 5) a stream whose workgroups were not resident --
// another kernel holding their CUs, e.g. a second process's persistent encoder on
// the same GPU -- left every resident wave spinning in the look-back until the spin
// limit (DESIGN.md §2 "Ticket streams and progress").
// Start order is counted on kStartHeads heads (64-B lines), head h = a hash of the
// wave's index: its n-th started wave takes stream (h + n) mod K.  One head per
// launch (any K started waves cover all K streams) or one per XCD cost 60-70 us per
// encoder launch in contention at configs 3 and 4 (one dequeue word saturates near
// 90/us, MI355X_MICROARCH.md "dequeue"; profiles/r06/diag_start_heads.txt); 32 heads
// cost nothing measurable.  A head with K started waves covers every stream, so any
// kStartHeads * K started waves suffice (pigeonhole: a quarter of an idle chip's
// grid), and fewer usually do (waves of one XCD land on heads spread over all
// offsets).  Below that the spin limit remains the safety net: the client goes to
// the exact path and the launch reports FC_OVERFLOW_STALL.
// FEDCODEC_TICKET_BLOCKIDX=1 restores round 5's mapping for the regression demo only.
constexpr int kStartHeads = 32;
__device__ __forceinline__ uint32_t ticket_stream(uint32_t* started, uint32_t b, uint32_t w, uint32_t wpg,
                                                  uint32_t nshards, uint32_t by_block, int lane) {
  const uint32_t g = b * wpg + w;
  if (by_block) return g % nshards;
  const uint32_t h = (g + (g >> 5)) % (uint32_t)kStartHeads;
  uint32_t r = 0;
  if (lane == 0) r = atomicAdd(started + kShardStride * h, 1u);
  r = __builtin_amdgcn_readfirstlane(r);
  return (r + h) % nshards;
}
#ifndef FC_STORE_ALIGN
#define FC_STORE_ALIGN 1
#endif
// Code-word stores line-aligned: lane l of a store instruction writes the word
// at lane offset l from the 128-B line holding the ticket's first word, so each
// instruction covers two whole lines instead of straddling three (the encoder's
// WRITE_SIZE was 1.15x the code bytes with unaligned 256-B store instructions).
constexpr bool kStoreAlign = FC_STORE_ALIGN;
#ifndef FC_LOOKBACK_WIN
#define FC_LOOKBACK_WIN 0  // 0: chosen per launch from the tiles in flight per client
#endif
constexpr int kLookbackWin = FC_LOOKBACK_WIN;  // statuses prefetched for the vector look-back

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

// Philox4x32-10 with a wave-uniform key (the encoder's per-client key lives in
// SGPRs): each round's two 3-input xors are one gfx950 v_bitop3_b32 each
// (truth table 0x96 = a ^ b ^ c), which the compiler does not form by itself.
__device__ __forceinline__ uint32_t xor3_vvs(uint32_t a, uint32_t b, uint32_t s) {
  uint32_t r;
  asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x96" : "=v"(r) : "v"(a), "v"(b), "s"(s));
  return r;
}
#ifndef FC_PHILOX_R2S
#define FC_PHILOX_R2S 1  // round 2's n2 xor with the scalar c3 ^ k1 (A/B knob)
#endif
// Rounds 0-1 stay plain C: with a lane-varying c0 only, half of their products
// and xors are wave-uniform and the compiler moves them to the scalar unit.
__device__ __forceinline__ void philox10_ukey(uint32_t& c0, uint32_t& c1, uint32_t& c2,
                                              uint32_t& c3, uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const uint64_t p0 = (uint64_t)0xD2511F53u * c0;
    const uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
    // round keys recomputed on the scalar unit at each use (volatile: not hoisted
    // across chunks, where 20 live key SGPRs would spill into VGPR lanes)
    uint32_t kk0, kk1;
    // (readfirstlane: a no-op on the SGPR key, and a guard should the register
    // allocator ever hand the key over in a VGPR)
    asm volatile("s_add_u32 %0, %1, %2" : "=s"(kk0) : "s"(__builtin_amdgcn_readfirstlane(k0)),
                 "i"(0x9E3779B9u * (uint32_t)r));
    asm volatile("s_add_u32 %0, %1, %2" : "=s"(kk1) : "s"(__builtin_amdgcn_readfirstlane(k1)),
                 "i"(0xBB67AE85u * (uint32_t)r));
    const uint32_t n0 = r < 2 ? (uint32_t)(p1 >> 32) ^ c1 ^ kk0 : xor3_vvs((uint32_t)(p1 >> 32), c1, kk0);
    // (round 2: c3 is still wave-uniform -- the low product of round 1's uniform
    // c0 -- so c3 ^ kk1 is one scalar xor and n2 one v_xor, no v_mov + v_bitop3)
    const uint32_t n2 = r < 2 + FC_PHILOX_R2S ? (uint32_t)(p0 >> 32) ^ (c3 ^ kk1) : xor3_vvs((uint32_t)(p0 >> 32), c3, kk1);
    c1 = (uint32_t)p1;
    c3 = (uint32_t)p0;
    c0 = n0;
    c2 = n2;
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

// Same, for a key that is uniform across the wave (k_encode's per-client key).
__device__ __forceinline__ uint4 philox_group_u(const Key4& k, uint32_t g) {
  uint32_t c0 = g, c1 = 0, c2 = k.c2, c3 = k.c3;
  philox10_ukey(c0, c1, c2, c3, k.k0, k.k1);
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
//      aggregate: [61:48] first_rel  [47:34] last_rel  [33:0] body bits (< 2^32)
//      prefix:    [61:36] last+1     [35:0] bits
//  w2: [63:62] flag  [31:0] tail
constexpr uint64_t kFlagAgg = 1ull << 62;
constexpr uint64_t kFlagPre = 2ull << 62;
constexpr uint64_t kFlagSlow = 3ull << 62;  // tile left to the exact kernel (terminal)
constexpr uint64_t kMask36 = (1ull << 36) - 1;
constexpr int kAggFirstShift = 48, kAggLastShift = 34;  // aggregate position fields
__device__ __forceinline__ uint64_t agg_word(uint64_t fr, uint64_t lr, uint32_t body) {
  return kFlagAgg | (fr << kAggFirstShift) | (lr << kAggLastShift) | (uint64_t)body;
}
// Decoder index entries hold (1 + the last nonzero before the unit) modulo 2^28 in
// bits [63:36] (writers shift a wider value left by 36: the high bits drop).
constexpr uint32_t kIdxLastMask = (1u << 28) - 1;
__host__ __device__ __forceinline__ int32_t sext28(uint32_t x) { return ((int32_t)(x << 4)) >> 4; }

__device__ __forceinline__ Seg seg_from_status(uint64_t w1, uint64_t w2, int64_t tile_base) {
  Seg s;
  if ((w1 >> 62) == 2) {
    s.has_nz = 1;
    s.first = -1;
    s.last = (int32_t)((w1 >> 36) & ((1u << 26) - 1)) - 1;
    s.body = w1 & kMask36;
  } else {
    const uint32_t fr = (uint32_t)(w1 >> kAggFirstShift) & kNoPos;
    const uint32_t lr = (uint32_t)(w1 >> kAggLastShift) & kNoPos;
    s.has_nz = fr != kNoPos;
    s.first = (int32_t)(tile_base + fr);
    s.last = (int32_t)(tile_base + lr);
    s.body = w1 & ((1ull << kAggLastShift) - 1);
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

// Both granules of a look-back status in one 16-byte store (readers accept a
// status only once both carry the same flag, so the granule order is free).
__device__ __forceinline__ void st_agent2(uint64_t* p, uint64_t g0, uint64_t g1) {
  typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
  const u32x4 v = {(uint32_t)g0, (uint32_t)(g0 >> 32), (uint32_t)g1, (uint32_t)(g1 >> 32)};
  // `s_nop 1` inside the statement: a store of more than 8 bytes reads its data
  // VGPRs after issue, and the compiler does not see the store to pad the VALU
  // write that may follow (a gfx9 hazard: a status could go out with half-overwritten
  // words; no instance was found in the listings, but nothing prevented one -- DESIGN
  // §2 "Ticket streams and progress")
  asm volatile("global_store_dwordx4 %0, %1, off sc1\n\ts_nop 1" ::"v"(p), "v"(v) : "memory");
}

__device__ __forceinline__ uint32_t bswap32(uint32_t v) { return __builtin_bswap32(v); }

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
  uint32_t* counter;  // kTicketShards ticket counters, 64 B apart (zeroed per launch)
  uint32_t nshards;   // ticket streams in use: min(kTicketShards, grid)
  uint32_t by_block;  // regression-test knob: streams by blockIdx (round 5) instead of start order
  uint32_t* started;  // waves started (start order -> ticket stream)
  uint32_t* spin_err;
  const void* cparams;   // ClientParam[nclients] (workspace)
  uint32_t* slow_count;  // clients handed to the exact kernel
  int32_t* slow_flag;    // [nclients] (zeroed per launch)
  int32_t* slow_list;    // [nclients]
  uint32_t* counter2;    // exact kernel's ticket counter
  uint32_t div_m, div_l;  // ticket / nclients by multiply-high (Granlund-Montgomery)
  int32_t lb_lane0;       // first lane whose status the look-back prefetches (64 - window)
  int32_t T2;             // super-tiles (two tiles) per client: k_encode2's tickets and statuses
  const int64_t* elem_off;  // nullable [C]: element offset (multiple of 4) of row c in its client's
                            // tensor -- the row is a segment; its Philox stream continues there
  uint64_t* idxq;           // nullable [C * T][3]: quarter-tile decoder entries (k_encode and the
                            // exact path write them tile-relative, k_quarter_index rebases them)
};

// Quarter-tile entries (elements 256 s of a tile, s = 1..3), tile-relative as the
// encoder writes them: [0, 24) body bits before the quarter's first code (after the
// tile's leading run code), [24, 35) 1 + the tile's last nonzero before the quarter
// (0: none), [35, 46) 1 + the tile's first nonzero.  k_quarter_index turns them into
// decoder entries (absolute bit offset | 1 + last nonzero before << 36).
__device__ __forceinline__ uint64_t quarter_rel(uint32_t off, int32_t prev, int32_t first) {
  return (uint64_t)(off & 0xFFFFFFu) | ((uint64_t)(uint32_t)(prev + 1) << 24) |
         ((uint64_t)(uint32_t)(first + 1) << 35);
}

// The launch's EncodeArgs re-read from the kernarg segment (k_encode and
// k_encode_exact take EncodeArgs as their only argument, at offset 0).  The
// opaque asm makes every use a fresh scalar load, so fields needed only on rare
// paths (slow tiles, overflow, spin errors, a client's last tile) do not hold
// SGPRs for the whole persistent loop.
// (Kernels only: LLVM lowers __builtin_amdgcn_kernarg_segment_ptr() to NULL in any
// function that is not a kernel, so an out-of-line callee -- lookback_deep,
// lookback_vec_wait -- that read the arguments this way dereferenced address 0:
// the round-5 fault in its spin-timeout branch, and round 6's first build on every
// poll.  The out-of-line look-backs read their spin limit from g_spin_limit and
// report a timeout through their result (kSegTimeout); the kernels set spin_err.
// tests/test_kernarg_use.py checks the compiled IR.)
__device__ __forceinline__ const EncodeArgs& enc_args_fresh() {
  const EncodeArgs* p = (const EncodeArgs*)__builtin_amdgcn_kernarg_segment_ptr();
  asm volatile("" : "+s"(p));
  return *p;
}

// Polls before a fast-kernel look-back gives up (the client then goes to the exact
// path and the launch reports FC_OVERFLOW_STALL): a device global, so the
// out-of-line look-backs need no argument for it (test knob FEDCODEC_SPIN_LIMIT).
// In the constant address space, so it is a scalar load, and read once per call
// before the poll loop: as a plain global it compiled to a vector load plus a
// `vmcnt(0)` in every poll -- waiting on the wave's pending code stores and staging
// loads each time (+8-10 % encode time at configs 2-4, profiles/r06/diag_spin_limit_ab.txt).
__constant__ uint32_t g_spin_limit = 1u << 24;

__device__ __forceinline__ uint32_t div_clients(const EncodeArgs& a, uint32_t n) {
  if (a.div_l == 0) return n;  // nclients == 1
  const uint32_t t1 = __umulhi(n, a.div_m);
  return (t1 + ((n - t1) >> 1)) >> (a.div_l - 1);
}

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
__device__ __forceinline__ uint32_t dpp_incl_or(uint32_t x) {
  x |= __builtin_amdgcn_update_dpp(0u, x, 0x111, 0xf, 0xf, false);  // row_shr:1
  x |= __builtin_amdgcn_update_dpp(0u, x, 0x112, 0xf, 0xf, false);  // row_shr:2
  x |= __builtin_amdgcn_update_dpp(0u, x, 0x114, 0xf, 0xf, false);  // row_shr:4
  x |= __builtin_amdgcn_update_dpp(0u, x, 0x118, 0xf, 0xf, false);  // row_shr:8
  x |= __builtin_amdgcn_update_dpp(0u, x, 0x142, 0xa, 0xf, false);  // row_bcast:15
  x |= __builtin_amdgcn_update_dpp(0u, x, 0x143, 0xc, 0xf, false);  // row_bcast:31
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
// Whole-wave reductions through the inclusive DPP scans (no ds_bpermute address registers).
__device__ __forceinline__ float wave_sum_f(float x) {
  uint32_t b = __float_as_uint(x);
  float v = x;
  v += __uint_as_float(__builtin_amdgcn_update_dpp(0u, b, 0x111, 0xf, 0xf, false));
  b = __float_as_uint(v);
  v += __uint_as_float(__builtin_amdgcn_update_dpp(0u, b, 0x112, 0xf, 0xf, false));
  b = __float_as_uint(v);
  v += __uint_as_float(__builtin_amdgcn_update_dpp(0u, b, 0x114, 0xf, 0xf, false));
  b = __float_as_uint(v);
  v += __uint_as_float(__builtin_amdgcn_update_dpp(0u, b, 0x118, 0xf, 0xf, false));
  b = __float_as_uint(v);
  v += __uint_as_float(__builtin_amdgcn_update_dpp(0u, b, 0x142, 0xa, 0xf, false));
  b = __float_as_uint(v);
  v += __uint_as_float(__builtin_amdgcn_update_dpp(0u, b, 0x143, 0xc, 0xf, false));
  return __uint_as_float((uint32_t)lane63((int32_t)__float_as_uint(v)));
}
__device__ __forceinline__ int32_t wave_sum_i(int32_t x) { return lane63((int32_t)dpp_incl_sum((uint32_t)x)); }
__device__ __forceinline__ int32_t wave_min_i(int32_t x) { return -lane63(dpp_incl_max(-x)); }
__device__ __forceinline__ uint32_t uniform(uint32_t x) { return __builtin_amdgcn_readfirstlane(x); }

// Decoupled look-back for tile t of one client, run by one full wave.  Returns
// the exclusive prefix (a root segment: body = stream bits before tile t).
// pre1/pre2 (optional): this lane's status of tile t-1-lane, loaded earlier.
template <int SPAN = kTE>  // elements per status slot (tile, or super-tile)
__device__ __forceinline__ Seg lookback(const uint64_t* status_c, int32_t t, int lane,
                                        bool& slow, bool& timeout, uint32_t limit, bool have_pre = false,
                                        uint64_t pre1 = 0, uint64_t pre2 = 0) {
  Seg S = seg_identity();
  int64_t base = (int64_t)t - 1;
  for (;;) {
    const int64_t ti = base - lane;
    uint64_t w1 = kFlagPre, w2 = kFlagPre;  // ti < 0: virtual root prefix
    bool valid = ti < 0;
    if (have_pre && base == (int64_t)t - 1 && !valid) {
      w1 = pre1;
      w2 = pre2;
      valid = (w1 >> 62) != 0 && (w1 >> 62) == (w2 >> 62);
    }
    int k;
    uint32_t spins = 0;
    for (;;) {
      if (!valid) {
        w1 = ld_agent(status_c + 2 * ti);
        w2 = ld_agent(status_c + 2 * ti + 1);
        valid = (w1 >> 62) != 0 && (w1 >> 62) == (w2 >> 62);
      }
      const uint64_t pre = __ballot(valid && (w1 >> 62) >= 2);  // prefix or slow: terminal
      const uint64_t val = __ballot(valid);
      k = pre ? __builtin_ctzll(pre) : 64;
      const uint64_t need = k >= 63 ? ~0ull : ((2ull << k) - 1);
      if ((val & need) == need) break;
      __builtin_amdgcn_s_sleep(1);
      if (++spins > limit) {  // safety net only: tickets guarantee progress
        // (a timed-out look-back's fold is not a prefix: `slow` makes the caller re-encode the
        // client -- k_encode_exact's callers through the overflow flag; the fold itself runs on,
        // which keeps this cold path from changing the encoders' register allocation)
        timeout = true;
        slow = true;
        k = 0;
        w1 = kFlagPre;
        w2 = kFlagPre;
        break;
      }
    }
    // fold lanes k (farthest, or 63) .. 0 (nearest) serially in scalar registers
    Seg W = seg_identity();
    const int kk = k < 63 ? k : 63;
    const uint32_t w1lo = (uint32_t)w1, w1hi = (uint32_t)(w1 >> 32), w2lo = (uint32_t)w2,
                   w2hi = (uint32_t)(w2 >> 32);
    if (k < 64 && (__builtin_amdgcn_readlane(w1hi, k) >> 30) == 3u) {  // a slow tile: give up
      slow = true;
      return S;
    }
    for (int i = kk; i >= 0; --i) {
      const int64_t tii = base - i;
      if (tii < -1) continue;
      const uint64_t a1 = ((uint64_t)__builtin_amdgcn_readlane(w1hi, i) << 32) | __builtin_amdgcn_readlane(w1lo, i);
      const uint64_t a2 = ((uint64_t)__builtin_amdgcn_readlane(w2hi, i) << 32) | __builtin_amdgcn_readlane(w2lo, i);
      W = seg_combine(W, seg_from_status(a1, a2, tii * SPAN));
    }
    S = seg_combine(W, S);
    if (k < 64) break;
    base -= 64;
  }
  return S;
}

#ifdef FC_STAMPS
__device__ unsigned long long g_stamps[16];
#define FC_COUNT(i, v) do { if (threadIdx.x == 0) atomicAdd(&g_stamps[i], (unsigned long long)(v)); } while (0)
#else
#define FC_COUNT(i, v) do {} while (0)
#endif
// Multi-window vector look-back, for when the 64 tiles before t hold no
// inclusive prefix (few clients: many tiles of one client in flight).  Lane i
// holds tile wbase+i of the current 64-tile window.  A window of 64 aggregates
// is folded with the same DPP scans as lookback_vec into a segment of its own
// and the walk moves 64 tiles back, until a window holds a prefix.  A window's
// tail is its newest tile's tail whenever that tile's body has >= 32 bits;
// otherwise the scalar lookback() does the whole fold (rare: a nearly empty
// tile).  Out of line: it keeps its registers off the common path.
constexpr uint32_t kSegSlow = 0xFFFFFFFFu;     // lookback_deep's "a slow tile" result (has_nz)
constexpr uint32_t kSegTimeout = 0xFFFFFFFEu;  // ... "gave up polling" (slow too; the kernel reports it)
template <int SPAN = kTE>
__device__ __noinline__ Seg lookback_deep(const uint64_t* status_c, int32_t t, int lane,
                                          uint64_t pre1, uint64_t pre2) {
  // Everything on 32-bit halves: h = granule bits [63:32] (flag in [31:30]),
  // l = bits [31:0].  ti < 0: the virtual root prefix (last + 1 = 0, body 0).
  Seg S = seg_identity();  // fold of the newer windows already walked
  const uint32_t lim = g_spin_limit;
  int32_t wbase = t - 64;
  uint32_t h1 = (uint32_t)(pre1 >> 32), l1 = (uint32_t)pre1, h2 = (uint32_t)(pre2 >> 32), l2 = (uint32_t)pre2;
  for (;;) {
    const int32_t ti = wbase + lane;
    if (ti < 0) {
      h1 = h2 = 0x80000000u;
      l1 = l2 = 0u;
    }
    // a status is readable once both granules carry the same nonzero flag
    bool valid = h1 >= 0x40000000u && (h1 ^ h2) < 0x40000000u;
    uint32_t spins = 0;
    uint64_t pre;
    for (;;) {
      pre = __ballot(valid && h1 >= 0x80000000u);  // inclusive prefix (or slow)
      const uint64_t val = __ballot(valid);
      const uint64_t need = pre ? ~0ull << (63 - (int)__clzll(pre)) : ~0ull;
      if ((val & need) == need) break;
      __builtin_amdgcn_s_sleep(1);
      if (++spins > lim) {  // (safety net) the client goes to the exact path
        Seg r = seg_identity();
        r.has_nz = kSegTimeout;
        return r;
      }
      if (!valid) {
        const uint64_t w1 = ld_agent(status_c + 2 * (int64_t)ti);
        const uint64_t w2 = ld_agent(status_c + 2 * (int64_t)ti + 1);
        h1 = (uint32_t)(w1 >> 32);
        l1 = (uint32_t)w1;
        h2 = (uint32_t)(w2 >> 32);
        l2 = (uint32_t)w2;
        valid = h1 >= 0x40000000u && (h1 ^ h2) < 0x40000000u;
      }
    }
    const int p = pre ? 63 - (int)__clzll(pre) : -1;  // nearest (newest) prefix, -1: none in this window
    uint32_t ph = 0;
    if (p >= 0) {
      ph = __builtin_amdgcn_readlane(h1, p);
      if (ph >= 0xC0000000u) {  // a slow tile: give up
        Seg r = seg_identity();
        r.has_nz = kSegSlow;
        return r;
      }
    }
    Seg r;
    r.has_nz = 1;
    r.first = -1;
    // prefix at lane p: [61:36] last + 1, [35:0] bits
    const int32_t plast = (int32_t)((ph >> 4) & ((1u << 26) - 1)) - 1;
    const uint64_t pbody = p >= 0 ? ((uint64_t)(ph & 0xFu) << 32) | __builtin_amdgcn_readlane(l1, p) : 0ull;
    if (p == 63) {  // the newest tile's own inclusive prefix
      r.last = plast;
      r.body = pbody;
      r.tail = __builtin_amdgcn_readlane(l2, 63);
      return seg_combine(r, S);
    }
    // aggregates above the prefix: [61:48] first_rel, [47:34] last_rel, body < 2^32
    const bool agg = lane > p;
    const uint32_t fr = (h1 >> (kAggFirstShift - 32)) & kNoPos, lr = (h1 >> (kAggLastShift - 32)) & kNoPos;
    const bool nz = agg && fr != kNoPos;
    const int32_t tb = ti * SPAN;
    int32_t lastv = agg ? -1 : (lane == p ? plast : -1);
    lastv = nz ? tb + (int32_t)lr : lastv;
    const int32_t M = dpp_incl_max(lastv);
    const int32_t Mx = dpp_shr1(M, -1);  // last nonzero before this tile (-1: none in the window)
    uint32_t contrib = agg ? l1 : 0u;
    // no prefix: the window's first nonzero has no run code yet (seg_combine adds it)
    if (nz && (p >= 0 || Mx >= 0)) contrib += glen((uint32_t)(tb + (int32_t)fr - Mx));
    const uint32_t csum = (uint32_t)wave_sum_i((int32_t)contrib);
    if (__builtin_amdgcn_readlane(l1, 63) < 32u) {  // short newest body: exact scalar fold
      bool slow = false;
      bool to = false;
      Seg r2 = lookback<SPAN>(status_c, t, lane, slow, to, lim);
      if (slow) r2.has_nz = to ? kSegTimeout : kSegSlow;
      return r2;
    }
    r.tail = __builtin_amdgcn_readlane(l2, 63);  // the newest body holds the last 32 bits
    r.body = pbody + csum;
    if (p >= 0) {
      r.last = lane63(M);
      return seg_combine(r, S);
    }
    // 64 aggregates and no prefix: fold them into a segment, walk 64 tiles back
    const uint64_t nzm = __ballot(nz);
    r.has_nz = nzm != 0;
    r.first = nzm ? __builtin_amdgcn_readlane(tb + (int32_t)fr, (int)__builtin_ctzll(nzm)) : 0;
    r.last = lane63(M);
    if (r.has_nz) S = seg_combine(r, S);
    wbase -= 64;
    const int32_t tn = wbase + lane;
    h1 = h2 = l1 = l2 = 0u;  // unreadable until loaded (ti < 0: root, set above)
    if (tn >= 0) {
      const uint64_t w1 = ld_agent(status_c + 2 * (int64_t)tn);
      const uint64_t w2 = ld_agent(status_c + 2 * (int64_t)tn + 1);
      h1 = (uint32_t)(w1 >> 32);
      l1 = (uint32_t)w1;
      h2 = (uint32_t)(w2 >> 32);
      l2 = (uint32_t)w2;
    }
  }
}

// Vectorised look-back (the encoder's common case).  Lane i holds tile
// t-64+i (lane 63 = t-1); pre1/pre2 are those statuses, loaded earlier.  Once
// the nearest inclusive prefix p and every aggregate after it are visible, the
// fold is two DPP scans instead of a serial scalar walk: the last nonzero
// before each aggregate (max-scan of the aggregates' last positions), its
// first run code length, and the sum of bodies.  The combined tail is the
// newest tile's tail whenever that tile's body has >= 32 bits; otherwise the
// scalar lookback() does the fold.  No prefix within 64 tiles: lookback_deep().
template <int SPAN>
__device__ __noinline__ Seg lookback_vec_wait(const uint64_t* status_c, int32_t t, int lane, uint64_t pre1,
                                              uint64_t pre2);
template <bool WAIT, int SPAN>
__device__ __forceinline__ Seg lookback_vec_impl(const uint64_t* status_c, int32_t t, int lane,
                                                 bool& slow, bool& timeout, uint64_t pre1,
                                                 uint64_t pre2) {
  // Everything on 32-bit halves: h = granule bits [63:32] (flag in [31:30]),
  // l = bits [31:0].  ti < 0: the virtual root prefix (last + 1 = 0, body 0).
  const int32_t ti = t - 64 + lane;
  uint32_t h1 = (uint32_t)(pre1 >> 32), l1 = (uint32_t)pre1, h2 = (uint32_t)(pre2 >> 32), l2 = (uint32_t)pre2;
  if (ti < 0) {
    h1 = h2 = 0x80000000u;
    l1 = l2 = 0u;
  }
  // a status is readable once both granules carry the same nonzero flag
  bool valid = h1 >= 0x40000000u && (h1 ^ h2) < 0x40000000u;
  int p;
  if (!WAIT) {
    // common case: the prefetched window already holds a prefix and every
    // aggregate after it (no loop, so no lane-mask phi in the caller's loop)
    const uint64_t pre = __ballot(valid && h1 >= 0x80000000u);
    const uint64_t val = __ballot(valid);
    p = pre ? 63 - (int)__clzll(pre) : 0;
    const uint64_t need = ~0ull << p;
    if (pre == 0 || (val & need) != need) {
      Seg r = lookback_vec_wait<SPAN>(status_c, t, lane, pre1, pre2);
      if (r.has_nz >= kSegTimeout) {
        slow = true;
        timeout = r.has_nz == kSegTimeout;
        r = seg_identity();
      }
      return r;
    }
  }
  uint32_t spins = 0;
  const uint32_t lim = WAIT ? g_spin_limit : 0u;
  for (; WAIT;) {
    const uint64_t pre = __ballot(valid && h1 >= 0x80000000u);  // inclusive prefix (or slow)
    const uint64_t val = __ballot(valid);
    if (pre == 0) {  // no prefix in the window: walk 64-tile windows
      FC_COUNT(10, 1);
      Seg r = lookback_deep<SPAN>(status_c, t, lane, pre1, pre2);
      if (r.has_nz >= kSegTimeout) {
        slow = true;
        timeout = r.has_nz == kSegTimeout;
        r = seg_identity();
      }
      return r;
    }
    p = 63 - (int)__clzll(pre);  // nearest (newest) prefix
    const uint64_t need = ~0ull << p;
    if ((val & need) == need) break;
    FC_COUNT(9, 1);
    __builtin_amdgcn_s_sleep(1);
    if (++spins > lim) {  // (safety net) the client goes to the exact path
      timeout = true;
      slow = true;
      return seg_identity();
    }
    if (!valid) {
      const uint64_t w1 = ld_agent(status_c + 2 * (int64_t)ti);
      const uint64_t w2 = ld_agent(status_c + 2 * (int64_t)ti + 1);
      h1 = (uint32_t)(w1 >> 32);
      l1 = (uint32_t)w1;
      h2 = (uint32_t)(w2 >> 32);
      l2 = (uint32_t)w2;
      valid = h1 >= 0x40000000u && (h1 ^ h2) < 0x40000000u;
    }
  }
  const uint32_t ph = __builtin_amdgcn_readlane(h1, p);
  if (ph >= 0xC0000000u) {  // a slow tile: give up
    slow = true;
    return seg_identity();
  }
  Seg r;
  r.has_nz = 1;
  r.first = -1;
  // prefix at lane p: [61:36] last + 1, [35:0] bits
  const int32_t plast = (int32_t)((ph >> 4) & ((1u << 26) - 1)) - 1;
  const uint64_t pbody = ((uint64_t)(ph & 0xFu) << 32) | __builtin_amdgcn_readlane(l1, p);
  FC_COUNT(8, 1);
  FC_COUNT(13, 63 - p);
  if (p == 63) {  // the predecessor's own inclusive prefix
    FC_COUNT(12, 1);
    r.last = plast;
    r.body = pbody;
    r.tail = __builtin_amdgcn_readlane(l2, 63);
    return r;
  }
  // aggregates above the prefix: [61:48] first_rel, [47:34] last_rel, body < 2^32
  const bool agg = lane > p;
  const uint32_t fr = (h1 >> (kAggFirstShift - 32)) & kNoPos, lr = (h1 >> (kAggLastShift - 32)) & kNoPos;
  const bool nz = agg && fr != kNoPos;
  const int32_t tb = ti * SPAN;
  int32_t lastv = agg ? -1 : (lane == p ? plast : -1);
  lastv = nz ? tb + (int32_t)lr : lastv;
  const int32_t M = dpp_incl_max(lastv);
  const int32_t Mx = dpp_shr1(M, -1);  // last nonzero before this tile
  uint32_t contrib = agg ? l1 : 0u;
  const uint32_t dfirst = (uint32_t)(tb + (int32_t)fr - Mx);  // nz lanes: their first run value
  if (nz) contrib += glen(dfirst);
  const uint32_t incl = dpp_incl_sum(contrib);
  const uint32_t csum = (uint32_t)lane63((int32_t)incl);
  r.last = lane63(M);
  r.body = pbody + csum;
  if (__builtin_amdgcn_readlane(l1, 63) >= 32u) {  // the newest body holds the last 32 bits
    r.tail = __builtin_amdgcn_readlane(l2, 63);
    return r;
  }
  // short newest body (nearly empty tiles, e.g. sparse clients): the last 32 bits
  // gather from several pieces.  Piece i (lanes >= p) is lane i's run code + body
  // (the prefix lane: its stream tail); S = csum - incl bits follow it; a piece with
  // S < 32 contributes (its low bits << S), and the pieces' bits are disjoint, so
  // the tail is the OR over lanes.  (A piece's tail holds its last <= 32 body bits,
  // zero above a shorter body.)
  FC_COUNT(11, 1);
  const uint32_t S = csum - incl;
  uint64_t v = (uint64_t)l2;
  if (nz && l1 < 32u) v |= (uint64_t)dfirst << l1;
  const uint32_t cpart = (lane >= p && S < 32u) ? (uint32_t)(v << S) : 0u;
  r.tail = (uint32_t)lane63((int32_t)dpp_incl_or(cpart));
  return r;
}

// The waiting variant, out of line (a re-poll, or no prefix in the window).
template <int SPAN>
__device__ __noinline__ Seg lookback_vec_wait(const uint64_t* status_c, int32_t t, int lane, uint64_t pre1,
                                              uint64_t pre2) {
  bool slow = false, to = false;
  Seg r = lookback_vec_impl<true, SPAN>(status_c, t, lane, slow, to, pre1, pre2);
  if (slow) r.has_nz = to ? kSegTimeout : kSegSlow;
  return r;
}
template <int SPAN = kTE>
__device__ __forceinline__ Seg lookback_vec(const uint64_t* status_c, int32_t t, int lane, bool& slow,
                                            bool& timeout, uint64_t pre1, uint64_t pre2) {
  return lookback_vec_impl<false, SPAN>(status_c, t, lane, slow, timeout, pre1, pre2);
}

// Runtime-indexed read of a small register array without scratch (select chain).
template <typename T, int N>
__device__ __forceinline__ T pick(const T (&arr)[N], int j) {
  T v = arr[0];
#pragma unroll
  for (int i = 1; i < N; ++i) v = (j == i) ? arr[i] : v;
  return v;
}

struct ClientQ {
  float step;
  float rcp;
  float s0, s1;  // pre-scales (TFF clipping factor, MeanFactory weight)
  bool pre;
  Key4 key;
  uint32_t gofs;  // Philox group of the row's element 0 (a segment of a longer client)
};

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
    if (MODE != FC_UNIFORM) rb = philox_group(cq.key, (uint32_t)(e0 >> 2) + cq.gofs);
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

__device__ __forceinline__ float vmax3_abs(float a, float b, float c) {
  float r;
  asm("v_max3_f32 %0, |%1|, |%2|, |%3|" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}

// Fused quantise + chunk-local code of one chunk of 4 in-range float
// elements (the fast path's inner loop).  The rounded value stays a float (an
// exact integer when |r| < 8192): m = |r| by one conversion, floor(log2 m) is
// its exponent, and the in-chunk run lengths come from select chains on the
// nonzero flags.  |r| >= 8192, Inf or NaN marks the chunk long; the slow path
// then recomputes the tile exactly (TF cast semantics, codes of any length).
// DIV: how x / step is formed (all three equal to TF-CPU's IEEE division on the
// fast path's range): 0 the IEEE division; 1 step a power of two, x * (1 / step)
// is exact; 2 step known to the host with a significand other than all ones:
// q0 = x * y, r = x - q0 * step (exact, one FMA), q = RN(q0 + r * y) with
// y = RN(1 / step) -- Markstein's theorem makes q the correctly rounded quotient
// (normal range; quotients beyond the fast path's |q| < 8192 or under 2^-125 do
// not change q and the exact path recomputes anything it marks long).
template <int DIV>
__device__ __forceinline__ float div_step(float x, float step, float y) {
  if (DIV == 1) return x * y;
  if (DIV == 2) {
    const float q0 = x * y;
    return fmaf(fmaf(-q0, step, x), y, q0);
  }
  return x / step;
}

#ifndef FC_NZ_BITS
#define FC_NZ_BITS 1  // chunk first / last nonzero by bit scans of a nonzero mask (0: select chains)
#endif
#ifndef FC_NZ_ADDC
#define FC_NZ_ADDC 1  // that mask by add-with-carry steps from the nonzero lane masks (0: selects and ORs)
#endif
template <int MODE, int DIV, bool PRE, bool MASK = false, bool PAIR = false>
__device__ __forceinline__ ChunkCode quant_code_fast(const ClientQ& cq, uint32_t g,
                                                     const uint32_t (&r4)[4], int32_t rel0,
                                                     float& dist, int32_t& nnz, const uint32_t* clut,
                                                     int32_t nvalid = 4, const uint32_t* plut = nullptr) {
  uint4 rb = make_uint4(0, 0, 0, 0);
  if (FC_ABL & 8) {  // diagnostics: a cheap hash instead of Philox
    rb.x = g * 2654435761u; rb.y = rb.x ^ 0x9E3779B9u; rb.z = rb.x + cq.key.k0; rb.w = rb.y ^ cq.key.k1;
  } else if (MODE != FC_UNIFORM) {
    rb = philox_group_u(cq.key, g);
  }
  const uint32_t rbits[4] = {rb.x, rb.y, rb.z, rb.w};
  float q[4];
  bool nz[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    float xv = __uint_as_float(r4[k]);
    if (PRE) xv = (xv * cq.s0) * cq.s1;
    const float sc = div_step<DIV>(xv, cq.step, cq.rcp);
    float r, noise = 0.0f;
    if (MODE == FC_UNIFORM) {
      r = rintf(sc);
    } else if (MODE == FC_STOCHASTIC) {
      const float fl = floorf(sc);
      r = (u01(rbits[k]) <= sc - fl) ? ceilf(sc) : fl;
    } else {
      noise = u01(rbits[k]) - 0.5f;
      r = rintf(sc - noise);
    }
    // pow2 step (RCP): sc = x / step exactly, so x - deq = step * (sc - r') exactly
    // (r' = r, or RN(r + noise) dithered) and every squared term and partial sum is
    // the unscaled one times step^2 -- k_encode multiplies the tile sum by step^2
    const float rq = (MODE == FC_DITHERED) ? (r + noise) : r;
    const float dd = DIV == 1 ? sc - rq : xv - rq * cq.step;
    // zero padding past P quantises to 0; only dithering's noise would count
    dist = (!MASK || k < nvalid) ? fmaf(dd, dd, dist) : dist;
    q[k] = r;
    nz[k] = r != 0.0f;
    nnz += (int32_t)__popcll(__ballot(nz[k]));  // wave total, scalar unit
  }
  // the chunk's first / last nonzero, as selects here, before the code paths
  // branch (computed after them the compiler turned the chains into branches)
#if FC_NZ_BITS
  // from a 4-bit mask of the nonzeros, by bit scans: the select chains below came
  // out as divergent branches (exec-mask juggling around single adds)
#if FC_NZ_ADDC
  // the mask from the nonzero tests' lane masks (the SGPR pairs the nnz ballots
  // already hold): one select and three add-with-carry steps, m = 2m + carry_k,
  // instead of four selects and the ORs
  uint32_t nzm;
  {
    const uint64_t b0 = __ballot(nz[0]), b1 = __ballot(nz[1]), b2 = __ballot(nz[2]), b3 = __ballot(nz[3]);
    uint64_t cj;
    nzm = nz[3] ? 1u : 0u;
    asm volatile("v_addc_co_u32_e64 %0, %1, %2, %2, %3" : "=v"(nzm), "=s"(cj) : "v"(nzm), "s"(b2));
    asm volatile("v_addc_co_u32_e64 %0, %1, %2, %2, %3" : "=v"(nzm), "=s"(cj) : "v"(nzm), "s"(b1));
    asm volatile("v_addc_co_u32_e64 %0, %1, %2, %2, %3" : "=v"(nzm), "=s"(cj) : "v"(nzm), "s"(b0));
  }
#else
  uint32_t nzm = (nz[0] ? 1u : 0u) | (nz[1] ? 2u : 0u) | (nz[2] ? 4u : 0u) | (nz[3] ? 8u : 0u);
  asm volatile("" : "+v"(nzm));
#endif
#if FC_ABL & 8192  // diagnostics: no chunk first / last nonzero (wrong stream)
  int32_t cfirst = rel0 + (int32_t)(nzm & 1u), clast = rel0 + 3;
#else
  int32_t cfirst = nzm ? rel0 + (int32_t)__builtin_ctz(nzm) : -1;
  int32_t clast = nzm ? rel0 + 31 - (int32_t)__builtin_clz(nzm) : -1;
#endif
  asm volatile("" : "+v"(cfirst), "+v"(clast));
#else
  int32_t cfirst = nz[0] ? rel0 : (nz[1] ? rel0 + 1 : (nz[2] ? rel0 + 2 : (nz[3] ? rel0 + 3 : -1)));
  int32_t clast = nz[3] ? rel0 + 3 : (nz[2] ? rel0 + 2 : (nz[1] ? rel0 + 1 : (nz[0] ? rel0 : -1)));
  asm volatile("" : "+v"(cfirst), "+v"(clast));
#endif
  ChunkCode r;
  r.acc = 0;
  r.len = 0;
  if (FC_ABL & 128) {  // diagnostics: no code construction (stand-in codes, wrong stream)
    r.acc = __float_as_uint(q[0]) ^ __float_as_uint(q[1]) ^ __float_as_uint(q[2]) ^ __float_as_uint(q[3]);
    r.len = 12;
    r.first = rel0;
    r.last = rel0 + 3;
    r.lng = 0;
    return r;
  }
  // max |r| of the chunk: two v_max3_f32 with |.| source modifiers.  A NaN may
  // drop out of the max, but a NaN or infinite r always makes the distortion
  // non-finite, which k_encode checks per tile before trusting the fast path.
  const float mabs = vmax3_abs(q[0], q[1], vmax3_abs(q[2], q[3], 0.0f));
  const bool bad = !(mabs < 8192.0f);
  // small values across the wave (|q| <= 31, the common case): one table read per element
  const bool big = !(mabs <= 31.0f);
  if (PAIR && __ballot(!(mabs <= 7.0f)) == 0) {
    // |q| <= 7 across the wave: one pair-table read per two elements.  Byte offset
    // 4 * ((qb & 15) << 4 | (qa & 15)): q * 4 (q * 64) + 1.5 * 2^23 is exact and its
    // low bits are 4q mod 64 (64q mod 1024); the second pair's table region is the
    // run state the first pair's entry hands on (bits 31:30 -> byte offset 1024 s)
    const uint32_t a0 = __float_as_uint(fmaf(q[0], 4.0f, 12582912.0f));
    const uint32_t b0 = __float_as_uint(fmaf(q[1], 64.0f, 12582912.0f));
    const uint32_t e0 = *(const uint32_t*)((const char*)plut + ((a0 & 0x3Cu) | (b0 & 0x3C0u)));
    const uint32_t a1 = __float_as_uint(fmaf(q[2], 4.0f, 12582912.0f));
    const uint32_t b1 = __float_as_uint(fmaf(q[3], 64.0f, 12582912.0f));
    const uint32_t e1 =
        *(const uint32_t*)((const char*)plut + ((a1 & 0x3Cu) | (b1 & 0x3C0u) | ((e0 >> 20) & 0xC00u)));
    const uint32_t l1 = (e1 >> 18) & 31u;
    r.acc = ((uint64_t)(e0 & 0x3FFFFu) << l1) | (e1 & 0x3FFFFu);
    r.len = ((e0 >> 18) & 31u) + l1;
  } else {
  // run code (value dv in rl bits) before element k, from the previous nonzero in the chunk
  const uint32_t dv1 = nz[0] ? 1u : 0u;
  const uint32_t dv2 = nz[1] ? 1u : (nz[0] ? 2u : 0u);
  const uint32_t rl2 = nz[1] ? 1u : (nz[0] ? 3u : 0u);
  const uint32_t dv3 = nz[2] ? 1u : (nz[1] ? 2u : (nz[0] ? 3u : 0u));
  const uint32_t rl3 = nz[2] ? 1u : ((nz[1] || nz[0]) ? 3u : 0u);
  const uint32_t dv[4] = {0u, dv1, dv2, dv3};
  const uint32_t rl[4] = {0u, dv1, rl2, rl3};
  if (__ballot(big) == 0) {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      // byte offset 4 * ((dv << 6) | (q & 63)): q * 4 + 1.5 * 2^23 is exact for |q| <= 31
      // and its low 8 bits are 4q mod 256 -- one FMA instead of a float->int conversion
      const uint32_t qb = __float_as_uint(fmaf(q[k], 4.0f, 12582912.0f)) & 0xFCu;
      const uint32_t e = *(const uint32_t*)((const char*)clut + ((dv[k] << 8) | qb));  // zero -> empty code
      const uint32_t L = e >> 16;
      r.acc = k == 0 ? (uint64_t)(e & 0xFFFFu) : ((r.acc << L) | (e & 0xFFFFu));
      r.len += L;
    }
  } else {
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const uint32_t m = (uint32_t)fabsf(q[k]);
    const uint32_t ml = 2u * ((__float_as_uint(q[k]) >> 23) & 0xFFu) - 253u;  // 2 floor(log2 m) + 1
    const uint32_t t = 2u * dv[k] + (q[k] > 0.0f ? 1u : 0u);                     // run code, sign bit
    // zero elements emit nothing: masked, not branched (keeps the wave convergent)
    uint32_t mk = nz[k] ? 0xFFFFFFFFu : 0u;
    asm volatile("" : "+v"(mk));
    const uint32_t code = ((t << ml) | m) & mk;
    const uint32_t L = (rl[k] + ml + 1u) & mk;
    r.acc = k == 0 ? (uint64_t)code : ((r.acc << L) | code);
    r.len += L;
  }
  }
  }
  r.first = cfirst;
  r.last = clast;
  r.lng = (bad || r.len > 64u) ? 1u : 0u;
  return r;
}

// Chunk code table: entry (ds << 6) | (q & 63) for |q| <= 31 is the code of a
// nonzero q whose in-chunk run value is ds (0: the chunk's first nonzero, whose
// run code is prepended later) -- [15:0] code bits, [31:16] length; q = 0 -> 0.
constexpr int kCodeLut = 256;
__device__ __forceinline__ uint32_t code_lut_entry(uint32_t i) {
  const uint32_t ds = i >> 6;
  const int32_t q = ((int32_t)(i << 26)) >> 26;  // sign-extend 6 bits
  if (q == 0 || ds > 3) return 0u;
  const uint32_t m = (uint32_t)(q < 0 ? -q : q);
  const uint32_t ml = glen(m);
  uint32_t code = ((uint32_t)(q > 0) << ml) | m, L = 1u + ml;
  if (ds) {
    code |= ds << L;
    L += glen(ds);
  }
  return code | (L << 16);
}

// Pair table (k_encode2): entry (s << 8) | ((qb & 15) << 4) | (qa & 15) for two
// consecutive elements qa, qb with |q| <= 7 and run state s -- the distance from
// the chunk's last nonzero before the pair to qa (0: none; the pair's first
// nonzero is then the chunk's first, whose run code is prepended later) --
// holds [17:0] the pair's code, [22:18] its length, [31:30] the state for the
// next pair (1 if qb is nonzero, 2 if only qa is, else 0).
constexpr int kPairLut = 768;
__device__ __forceinline__ uint32_t pair_lut_entry(uint32_t i) {
  const uint32_t s = i >> 8;
  const int32_t qa = ((int32_t)(i << 28)) >> 28, qb = ((int32_t)(i << 24)) >> 28;
  if (qa < -7 || qb < -7) return 0u;  // |q| = 8: never looked up
  uint32_t code = 0, len = 0;
  const int32_t qs[2] = {qa, qb};
  uint32_t run = s;  // distance from the last nonzero to the next element (0: none)
  for (int k = 0; k < 2; ++k) {
    const int32_t q = qs[k];
    if (q != 0) {
      const uint32_t m = (uint32_t)(q < 0 ? -q : q);
      const uint32_t ml = glen(m);
      uint32_t c = ((uint32_t)(q > 0) << ml) | m, L = 1u + ml;
      if (run) {
        c |= run << L;
        L += glen(run);
      }
      code = (code << L) | c;
      len += L;
      run = 1;
    } else if (run) {
      ++run;
    }
  }
  const uint32_t snext = qb != 0 ? 1u : (qa != 0 ? 2u : 0u);
  return code | (len << 18) | (snext << 30);
}

// Prepend the run code of the chunk's first nonzero once the last nonzero
// before the chunk (prev, tile-relative, -1 = none in this tile) is known.
__device__ __forceinline__ void chunk_prepend(ChunkCode& r, int32_t prev) {
  if (r.first >= 0 && prev >= 0) {
    const uint32_t d = (uint32_t)(r.first - prev);           // >= 1
    const uint32_t rl = 63u - 2u * (uint32_t)__builtin_clz(d);  // glen(d)
    // past 64 bits the chunk is long: the tile takes the exact path, acc is then unused
    r.lng |= (r.len + rl > 64u) ? 1u : 0u;
    r.acc |= (uint64_t)d << (r.len & 63u);
    r.len += rl;
  }
}

// Chained pair table (k_encode2, FC_PAIR_CHAIN): the run state crosses the
// lane's chunks, so a chunk's first nonzero takes its run code from the table
// like every other nonzero, and no per-chunk first / last nonzero or prepend is
// computed.  Entry (s << 8) | ((qa + 16 qb) & 255) -- one index for |qa|, |qb| <= 7,
// formed by two FMAs on the rounded floats -- with s = distance from the
// lane's last nonzero to qa, 1..6; 0 no nonzero yet in the lane (the lane's first
// run code comes from the wave scan); 7 "far" (>= 7: a nonzero here is coded
// without its run code and flagged, and the caller prepends the exact one).
// [31:14] code, [13] flag, [12:10] the state for the next pair (already the
// byte offset of its table region), [9:8] the pair's nonzero pattern (bit 8: qa,
// bit 9: qb), [4:0] length (bits 7:5 zero: two entries' lengths add in one op).
constexpr int kChainStates = 8;
constexpr uint32_t kChainFar = 7;
constexpr int kChainLut = kChainStates * 256;
constexpr uint32_t kChainFlag = 1u << 13;
constexpr uint32_t kChainState = 7u << 10;
__device__ __forceinline__ uint32_t pair_chain_entry(uint32_t i) {
  const uint32_t s = i >> 8;
  const int32_t qa = ((int32_t)(i << 28)) >> 28;
  const int32_t qb = ((int32_t)((((i & 255u) - (uint32_t)qa) & 255u) << 24)) >> 28;
  if (qa < -7 || qb < -7) return 0u;  // |q| = 8: never looked up
  uint32_t code = 0, len = 0, flag = 0;
  const int32_t qs[2] = {qa, qb};
  uint32_t run = s;
  for (int k = 0; k < 2; ++k) {
    const int32_t q = qs[k];
    if (q != 0) {
      const uint32_t m = (uint32_t)(q < 0 ? -q : q);
      const uint32_t ml = glen(m);
      uint32_t c = ((uint32_t)(q > 0) << ml) | m, L = 1u + ml;
      if (run == kChainFar) {
        flag = 1;  // the caller prepends the exact run code (only a chunk's first nonzero can be far)
      } else if (run) {
        c |= run << L;
        L += glen(run);
      }
      code = (code << L) | c;
      len += L;
      run = 1;
    } else if (run) {
      run = min(run + 1u, kChainFar);
    }
  }
  const uint32_t nzp = (qa != 0 ? 1u : 0u) | (qb != 0 ? 2u : 0u);
  return (code << 14) | (flag << 13) | (run << 10) | (nzp << 8) | len;
}

// The super-tile encoder's distortion sum.  FC_DIST_MFMA: each element slot's
// squared errors added by one v_mfma_f32_16x16x4_f32 with the errors as both
// operands -- its diagonal D[i][i] gathers sum_k dd(lane 16k + i)^2, so the
// diagonal's total is the wave's sum -- on the matrix pipe instead of one VALU
// FMA per element (the wave total is read off the diagonal once per ticket).
#ifndef FC_DIST_MFMA
#define FC_DIST_MFMA 0  // measured: +17 % stochastic, +4 % uniform (the dependent MFMA chain stalls the wave; profiles/r05/diag_enc_dist_mfma_ab.txt)
#endif
typedef float f32x4_t __attribute__((ext_vector_type(4)));
struct DistAcc {
  float s;
  f32x4_t m;
  __device__ __forceinline__ void zero() {
    s = 0.0f;
    m = f32x4_t{0.0f, 0.0f, 0.0f, 0.0f};
  }
  __device__ __forceinline__ void add(float dd) {
    if (FC_DIST_MFMA) m = __builtin_amdgcn_mfma_f32_16x16x4f32(dd, dd, m, 0, 0, 0);
    else s = fmaf(dd, dd, s);
  }
  // the wave's total (every lane); D[i][j] sits in lane j + 16 (i / 4), register i % 4
  __device__ __forceinline__ float wave_total(int lane) const {
    if (!FC_DIST_MFMA) return wave_sum_f(s);
    const int a = lane & 15, b = lane >> 4;
    const float d = (a & 3) == 0 ? m.x : (a & 3) == 1 ? m.y : (a & 3) == 2 ? m.z : m.w;
    return wave_sum_f((a >> 2) == b ? d : 0.0f);
  }
};

struct ChainCode {
  uint64_t acc;
  uint32_t len;
  uint32_t lng;  // a code > 32 bits, |r| >= 8192 / Inf / NaN, or more than 64 bits
  uint32_t nzm;  // nonzero mask of the chunk (bit k: element k)
  uint32_t pre;   // the chunk's first nonzero still needs its run code (a nonzero before it in the lane)
  uint64_t prem;  // the wave's lanes with pre: a scalar mask across the two code paths
};

// quant_code_fast for the chained table: the same quantiser, numerics and
// counts; sst holds the run state as a byte offset into the chained table
// (state << 10) and is advanced past the chunk.
#ifndef FC_PK
#define FC_PK 0  // packed float32 pairs in quant_code_chain (1): fewer instructions, 2.5 % slower stochastic encode (profiles/r05/diag_enc_pk_ab.txt)
#endif
constexpr bool PK = FC_PK;
template <int MODE, int DIV, bool PRE, bool MASK = false>
__device__ __forceinline__ void quant_chain4(const ClientQ& cq, uint32_t g, const uint32_t (&r4)[4], DistAcc& dist,
                                             float (&q)[4], int32_t nvalid = 4) {
  // Philox + the exact quantiser + the distortion terms of one chunk (its codes:
  // code_chain)
  uint4 rb = make_uint4(0, 0, 0, 0);
  if (FC_ABL & 8) {
    rb.x = g * 2654435761u; rb.y = rb.x ^ 0x9E3779B9u; rb.z = rb.x + cq.key.k0; rb.w = rb.y ^ cq.key.k1;
  } else if (MODE != FC_UNIFORM) {
    rb = philox_group_u(cq.key, g);
  }
  const uint32_t rbits[4] = {rb.x, rb.y, rb.z, rb.w};
  if (PK && DIV == 1 && !MASK && MODE != FC_DITHERED) {
    // the same arithmetic with the elementwise multiplies, subtractions and the
    // distortion terms as packed float32 pairs (v_pk_mul / v_pk_add / v_pk_fma_f32:
    // one instruction per two elements; IEEE per lane, FTZ as the scalar forms)
    typedef float f2 __attribute__((ext_vector_type(2)));
    f2 x01 = {__uint_as_float(r4[0]), __uint_as_float(r4[1])};
    f2 x23 = {__uint_as_float(r4[2]), __uint_as_float(r4[3])};
    if (PRE) {
      const f2 s0 = {cq.s0, cq.s0}, s1 = {cq.s1, cq.s1};
      x01 = (x01 * s0) * s1;
      x23 = (x23 * s0) * s1;
    }
    const f2 rc = {cq.rcp, cq.rcp};
    const f2 sc01 = x01 * rc, sc23 = x23 * rc;
    const float sc[4] = {sc01.x, sc01.y, sc23.x, sc23.y};
    f2 r01, r23;
    if (MODE == FC_UNIFORM) {
      r01 = f2{rintf(sc[0]), rintf(sc[1])};
      r23 = f2{rintf(sc[2]), rintf(sc[3])};
    } else {
      const f2 fl01 = {floorf(sc[0]), floorf(sc[1])}, fl23 = {floorf(sc[2]), floorf(sc[3])};
      const f2 p01 = sc01 - fl01, p23 = sc23 - fl23;
      const f2 one = {1.0f, 1.0f};
      const f2 u01v = f2{__uint_as_float((rbits[0] & 0x7FFFFFu) | 0x3F800000u),
                         __uint_as_float((rbits[1] & 0x7FFFFFu) | 0x3F800000u)} - one;
      const f2 u23v = f2{__uint_as_float((rbits[2] & 0x7FFFFFu) | 0x3F800000u),
                         __uint_as_float((rbits[3] & 0x7FFFFFu) | 0x3F800000u)} - one;
      r01 = f2{u01v.x <= p01.x ? ceilf(sc[0]) : fl01.x, u01v.y <= p01.y ? ceilf(sc[1]) : fl01.y};
      r23 = f2{u23v.x <= p23.x ? ceilf(sc[2]) : fl23.x, u23v.y <= p23.y ? ceilf(sc[3]) : fl23.y};
    }
    const f2 dd01 = sc01 - r01, dd23 = sc23 - r23;
    dist.add(dd01.x);
    dist.add(dd01.y);
    dist.add(dd23.x);
    dist.add(dd23.y);
    q[0] = r01.x; q[1] = r01.y; q[2] = r23.x; q[3] = r23.y;
  } else {
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    float xv = __uint_as_float(r4[k]);
    if (PRE) xv = (xv * cq.s0) * cq.s1;
    const float sc = div_step<DIV>(xv, cq.step, cq.rcp);
    float r, noise = 0.0f;
    if (MODE == FC_UNIFORM) {
      r = rintf(sc);
    } else if (MODE == FC_STOCHASTIC) {
      const float fl = floorf(sc);
      r = (u01(rbits[k]) <= sc - fl) ? ceilf(sc) : fl;
    } else {
      noise = u01(rbits[k]) - 0.5f;
      r = rintf(sc - noise);
    }
    const float rq = (MODE == FC_DITHERED) ? (r + noise) : r;
    const float dd = DIV == 1 ? sc - rq : xv - rq * cq.step;
    dist.add((!MASK || k < nvalid) ? dd : 0.0f);
    q[k] = r;
  }
  }
}

// The codes of one chunk from its quantised values (the chained pair table when
// |q| <= 7 across the wave -- TAB: the caller has checked that for the whole tile --
// else the code table / exponent paths); sst carries the run state.
template <bool TAB = false>
__device__ __forceinline__ ChainCode code_chain(const float (&q)[4], const uint32_t* clut, const uint32_t* plut,
                                                uint32_t& sst) {
  // r.nzm: the chunk's nonzero mask (the caller counts the lane's nonzeros from the
  // masks once per tile); on the pair-table path it comes from the table entries, so
  // no per-element compares are issued there
  ChainCode r;
  const float mabs = vmax3_abs(q[0], q[1], vmax3_abs(q[2], q[3], 0.0f));
  const bool bad = !(mabs < 8192.0f);
  r.acc = 0;
  r.len = 0;
  if (TAB || __ballot(!(mabs <= 7.0f)) == 0) {
    // |q| <= 7 across the wave: two chained pair-table reads
    // 1.5 * 2^23 + 4 qa + 64 qb is an exact float integer whose low 10 bits are
    // 4 * ((qa + 16 qb) mod 256): the pair's byte offset in a state region
    const uint32_t t0 = __float_as_uint(fmaf(q[1], 64.0f, fmaf(q[0], 4.0f, 12582912.0f)));
    const uint32_t e0 = *(const uint32_t*)((const char*)plut + ((t0 & 0x3FCu) | sst));
    const uint32_t t1 = __float_as_uint(fmaf(q[3], 64.0f, fmaf(q[2], 4.0f, 12582912.0f)));
    const uint32_t e1 = *(const uint32_t*)((const char*)plut + ((t1 & 0x3FCu) | (e0 & kChainState)));
    sst = e1 & kChainState;
    const uint32_t l1 = e1 & 31u;
    r.acc = ((uint64_t)(e0 >> 14) << l1) | (e1 >> 14);
    r.len = (e0 + e1) & 63u;  // bits 7:5 are zero: the two lengths add without interference
    r.pre = (e0 | e1) & kChainFlag;
    r.prem = __ballot(r.pre != 0u);
    r.nzm = __builtin_amdgcn_ubfe(e0, 8, 2) | (__builtin_amdgcn_ubfe(e1, 8, 2) << 2);
    r.lng = 0;  // |q| <= 7: at most 36 bits
    return r;
  } else {
    bool nz[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) nz[k] = q[k] != 0.0f;
    r.nzm = (nz[0] ? 1u : 0u) | (nz[1] ? 2u : 0u) | (nz[2] ? 4u : 0u) | (nz[3] ? 8u : 0u);
    // codes without the chunk's first run code, as quant_code_fast; the caller
    // prepends it when the lane had a nonzero before the chunk
    const uint32_t dv1 = nz[0] ? 1u : 0u;
    const uint32_t dv2 = nz[1] ? 1u : (nz[0] ? 2u : 0u);
    const uint32_t rl2 = nz[1] ? 1u : (nz[0] ? 3u : 0u);
    const uint32_t dv3 = nz[2] ? 1u : (nz[1] ? 2u : (nz[0] ? 3u : 0u));
    const uint32_t rl3 = nz[2] ? 1u : ((nz[1] || nz[0]) ? 3u : 0u);
    const uint32_t dv[4] = {0u, dv1, dv2, dv3};
    const uint32_t rl[4] = {0u, dv1, rl2, rl3};
    const bool big = !(mabs <= 31.0f);
    if (__ballot(big) == 0) {
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const uint32_t qb = __float_as_uint(fmaf(q[k], 4.0f, 12582912.0f)) & 0xFCu;
        const uint32_t e = *(const uint32_t*)((const char*)clut + ((dv[k] << 8) | qb));
        const uint32_t L = e >> 16;
        r.acc = k == 0 ? (uint64_t)(e & 0xFFFFu) : ((r.acc << L) | (e & 0xFFFFu));
        r.len += L;
      }
    } else {
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const uint32_t m = (uint32_t)fabsf(q[k]);
        const uint32_t ml = 2u * ((__float_as_uint(q[k]) >> 23) & 0xFFu) - 253u;
        const uint32_t t = 2u * dv[k] + (q[k] > 0.0f ? 1u : 0u);
        uint32_t mk = nz[k] ? 0xFFFFFFFFu : 0u;
        asm volatile("" : "+v"(mk));
        const uint32_t code = ((t << ml) | m) & mk;
        const uint32_t L = (rl[k] + ml + 1u) & mk;
        r.acc = k == 0 ? (uint64_t)code : ((r.acc << L) | code);
        r.len += L;
      }
    }
    const uint32_t nzm = r.nzm;
    r.pre = (nzm != 0u && sst != 0u) ? 1u : 0u;
    r.prem = __ballot(r.pre != 0u);
    // the state after the chunk: distance from its last nonzero to the next chunk
    const uint32_t far = kChainFar << 10;
    sst = nzm ? (4u - (31u - (uint32_t)__builtin_clz(nzm))) << 10 : (sst ? min(sst + (4u << 10), far) : 0u);
  }
  r.lng = (bad || r.len > 64u) ? 1u : 0u;
  return r;
}

template <int MODE, int DIV, bool PRE, bool MASK = false>
__device__ __forceinline__ ChainCode quant_code_chain(const ClientQ& cq, uint32_t g, const uint32_t (&r4)[4],
                                                      DistAcc& dist, const uint32_t* clut,
                                                      const uint32_t* plut, uint32_t& sst, int32_t nvalid = 4) {
  float q[4];
  quant_chain4<MODE, DIV, PRE, MASK>(cq, g, r4, dist, q, nvalid);
  return code_chain(q, clut, plut, sst);
}

// Re-read and re-quantise one chunk (slow path: tiles with codes > 32 bits or
// a body larger than the LDS window).
template <int MODE, bool INT_IN, bool RCP>
__device__ __forceinline__ void reload_chunk(const EncodeArgs& a, const ClientQ& cq, int32_t c,
                                             int64_t e0, int32_t (&q4)[4], float& dist) {
  const uint32_t* xp = (const uint32_t*)a.xs[c];
  uint32_t r4[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) r4[k] = (e0 + k < a.P) ? xp[e0 + k] : 0u;
  quant_chunk<MODE, INT_IN, RCP>(cq, e0, a.P, r4, q4, dist);
}

template <typename T, int N>
__device__ __forceinline__ void put(T (&arr)[N], int j, T v) {
#pragma unroll
  for (int i = 0; i < N; ++i) arr[i] = (j == i) ? v : arr[i];
}

#ifdef FC_STAMPS
#define STAMP(i)                                               \
  do {                                                         \
    if (lane == 0) {                                           \
      const uint64_t now_ = __builtin_amdgcn_s_memtime();      \
      st_acc[i] += now_ - st_last;                             \
      st_last = now_;                                          \
    }                                                          \
  } while (0)
#else
#define STAMP(i) do {} while (0)
#endif

// Per-client encoder parameters, computed once per launch (k_client_params)
// and read by k_encode with one scalar load per tile.
struct alignas(64) ClientParam {
  float step, rcp, s0, s1;   // step (x norm), 1/step (pow2 path), pre-scales
  uint32_t k0, k1, c2, c3;   // scrambled Philox key / counter words (TF seed)
  const uint32_t* x;         // the client's float32 (or int32) values
  uint32_t* out;             // stream_buf + stream_off[c]
  int64_t cap;               // stream_cap[c] (bytes)
  int64_t gofs;              // Philox group of x[0]: elem_off[c] / 4 (segments), else 0
};

// Also zeroes the launch's look-back statuses, ticket counters and slow-client flags
// (nzero16 16-byte words from `zero`): one prologue launch instead of a memset plus
// this kernel.
__global__ void k_client_params(EncodeArgs a, ClientParam* cp, int need_key, uint4* zero, int64_t nzero16) {
  const int64_t i0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (int64_t i = i0; i < nzero16; i += (int64_t)gridDim.x * blockDim.x) zero[i] = make_uint4(0, 0, 0, 0);
  const int c = (int)i0;
  if (c >= a.nclients) return;
  ClientParam p;
  p.step = a.norms ? a.norms[c] * a.step : a.step;
  p.rcp = a.rcp;
  p.s0 = a.prescale ? a.prescale[2 * c] : 1.0f;
  p.s1 = a.prescale ? a.prescale[2 * c + 1] : 1.0f;
  Key4 k{0, 0, 0, 0};
  if (need_key) k = tf_seed_scramble(a.seeds[2 * c], a.seeds[2 * c + 1]);
  p.k0 = k.k0;
  p.k1 = k.k1;
  p.c2 = k.c2;
  p.c3 = k.c3;
  p.x = (const uint32_t*)a.xs[c];
  p.out = (uint32_t*)(a.stream_buf + a.stream_off[c]);
  p.cap = a.stream_cap[c];
  p.gofs = a.elem_off ? a.elem_off[c] >> 2 : 0;
  cp[c] = p;
  a.overflow[c] = 0;  // (instead of a memset launch: this kernel runs before every encoder kernel)
}

typedef const __attribute__((address_space(4))) ClientParam* ConstParamPtr;

// Field-wise read through the constant address space: one s_load per tile.
__device__ __forceinline__ ClientParam ld_param(ConstParamPtr p) {
  ClientParam r;
  r.step = p->step;
  r.rcp = p->rcp;
  r.s0 = p->s0;
  r.s1 = p->s1;
  r.k0 = p->k0;
  r.k1 = p->k1;
  r.c2 = p->c2;
  r.c3 = p->c3;
  r.x = p->x;
  r.out = p->out;
  r.cap = p->cap;
  r.gofs = p->gofs;
  return r;
}

__device__ __forceinline__ ClientQ client_q_of(const ClientParam& p, bool pre) {
  ClientQ r;
  r.step = p.step;
  r.rcp = p.rcp;
  r.s0 = p.s0;
  r.s1 = p.s1;
  r.pre = pre;
  r.key = Key4{p.k0, p.k1, p.c2, p.c3};
  r.gofs = (uint32_t)p.gofs;
  return r;
}

// Window layout: body bit b of the current tile lives at window bit kPre + b;
// the tile's leading pieces (previous tile's partial word, first run code) are
// placed just before it once the look-back has resolved them.
constexpr uint32_t kPre = 96;

// OR a code of len <= 64 bits (right-aligned in acc) into the window at bit
// position wp: three ds_or_b32 (zero pieces of a nonempty code are harmless);
// positions past the window land in the guard words (the tile then takes the
// slow path anyway).  Empty codes are skipped: an LDS atomic to one address
// from many lanes serialises, and the lanes of an empty stretch (zero runs,
// sparse clients) all sit at the same window position -- unconditional ORs made
// an all-zero round 2.5x slower than a dense one (81 vs 32 ms at 1024 x 25 M;
// skipping each word a code does not reach costs 2 % more on dense data).
#ifndef FC_EMIT_BRANCH
#define FC_EMIT_BRANCH 1  // empty codes skip their ORs by a branch (0: their zero ORs go to lane-spread words)
#endif
// The window ORs as inline asm (FC_EMIT_ASM): the compiler's wait-count pass
// otherwise puts an s_waitcnt vmcnt(0) in front of the first OR of a tile -- it
// cannot tell the window from the staging buffer the next tile's LDS-DMA is
// filling -- so the emission waited for that DMA (and every pending store).  LDS
// operations of one wave complete in order, so the later window reads see the ORs.
#ifndef FC_EMIT_ASM
#define FC_EMIT_ASM 0  // measured even (profiles/r05/diag_enc_nt_ab.txt, easm)
#endif
typedef __attribute__((address_space(3))) uint32_t* lds_uptr;
template <int OFS>
__device__ __forceinline__ void lds_or(uint32_t* p, uint32_t v) {
  if (FC_EMIT_ASM) asm volatile("ds_or_b32 %0, %1 offset:%2" ::"v"((lds_uptr)p), "v"(v), "i"(OFS) : "memory");
  else atomicOr(p + OFS / 4, v);
}
template <uint32_t W = kWinWords, bool CLAMP = true>  // CLAMP false: the caller keeps wp inside the window
__device__ __forceinline__ void emit64(uint32_t* win, uint64_t acc, uint32_t len, uint32_t wp) {
  const uint64_t X = acc << ((64u - len) & 63u);  // MSB-aligned (len 0: acc is 0)
  const uint32_t o = wp & 31u;
  uint32_t i0 = CLAMP ? min(wp >> 5, W) : wp >> 5;
  const uint32_t hi = (uint32_t)(X >> 32), lo = (uint32_t)X;
  if (!FC_EMIT_BRANCH) i0 = len ? i0 : (uint32_t)__lane_id();  // OR of zeros: any word, one per lane
  if (!FC_EMIT_BRANCH || len) {
    lds_or<0>(win + i0, hi >> o);
    lds_or<4>(win + i0, __builtin_amdgcn_alignbit(hi, lo, o));
    lds_or<8>(win + i0, __builtin_amdgcn_alignbit(lo, 0u, o));
  }
}

// Same for a code of len <= 32 bits: two ds_or_b32.
template <uint32_t W = kWinWords, bool CLAMP = true>
__device__ __forceinline__ void emit32(uint32_t* win, uint32_t v, uint32_t len, uint32_t wp) {
  const uint32_t X = (uint32_t)((uint64_t)v << ((32u - len) & 63u));  // MSB-aligned (len 0: v is 0)
  const uint32_t o = wp & 31u;
  uint32_t i0 = CLAMP ? min(wp >> 5, W) : wp >> 5;
  if (!FC_EMIT_BRANCH) i0 = len ? i0 : (uint32_t)__lane_id();
  if (!FC_EMIT_BRANCH || len) {
    lds_or<0>(win + i0, X >> o);
    lds_or<4>(win + i0, __builtin_amdgcn_alignbit(X, 0u, o));
  }
}

// 32 window bits starting at window bit s (any s; reads words s>>5, +1).
__device__ __forceinline__ uint32_t win_bits32(const uint32_t* win, uint32_t s) {
  const uint32_t w = s >> 5, o = s & 31u;
  const uint64_t pair = ((uint64_t)win[w] << 32) | win[w + 1];
  return (uint32_t)(pair >> (32u - o));
}


// Exact path (clients with a rare tile: a code past the fast path's limits or
// a body larger than the LDS window), run by k_encode_exact after k_encode so
// its registers do not weigh on the fast kernel.  slow_scan recomputes the tile exactly (TF cast semantics, codes of any
// length): chunk predecessors and offsets, counts, distortion and the body's
// last 32 bits.  slow_emit re-quantises again and emits stream-relative in
// window passes.
struct SlowScan {
  int32_t chunk_prev[kChunks];
  uint32_t chunk_off[kChunks];
  uint32_t body;
  int32_t carry, wfirst;
  float dist;
  int32_t nnz;
  uint32_t tail;
};

template <int MODE, bool INT_IN, bool RCP>
__device__ __forceinline__ void slow_scan(const EncodeArgs& a, const ClientQ& cq, int32_t c,
                                                    int64_t tile_base, uint32_t* win, uint32_t* tailw,
                                                    SlowScan& o) {
  const int lane = threadIdx.x;
  for (int i = lane; i < kWinWords; i += kEncThreads) win[i] = 0;
  int32_t carry = -1, wfirst = 0x7FFFFFFF, nnz = 0;
  uint32_t body = 0;
  float dist = 0.0f;
  int32_t chunk_prev[kChunks] = {-1, -1, -1, -1};
  uint32_t chunk_off[kChunks] = {0, 0, 0, 0};
#pragma unroll 1
  for (int j = 0; j < kChunks; ++j) {
    const int32_t rel0 = 256 * j + 4 * lane;
    int32_t q4[4];
    reload_chunk<MODE, INT_IN, RCP>(a, cq, c, tile_base + rel0, q4, dist);
#pragma unroll
    for (int k = 0; k < 4; ++k) nnz += q4[k] != 0;
    ChunkCode cj = chunk_local(q4, rel0);
    wfirst = min(wfirst, cj.first >= 0 ? cj.first : 0x7FFFFFFF);
    const int32_t imax = dpp_incl_max(cj.last);
    const int32_t prev = max(dpp_shr1(imax, -1), carry);
    carry = max(carry, lane63(imax));
    chunk_prepend(cj, prev);
    const uint32_t isum = dpp_incl_sum(cj.len);
    put(chunk_prev, j, prev);
    put(chunk_off, j, body + isum - cj.len);
    body += (uint32_t)lane63((int32_t)isum);
  }
  if (lane == 0) *tailw = 0;
#pragma unroll 1
  for (int j = 0; j < kChunks; ++j) {
    const int32_t rel0 = 256 * j + 4 * lane;
    int32_t qv[4];
    float dd = 0.0f;
    reload_chunk<MODE, INT_IN, RCP>(a, cq, c, tile_base + rel0, qv, dd);
    int32_t prev = pick(chunk_prev, j);
    uint32_t pos = pick(chunk_off, j);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int32_t v = qv[k];
      if (v == 0) continue;
      if (prev >= 0) {
        const uint32_t d = (uint32_t)(rel0 + k - prev);
        const uint32_t rl = glen(d);
        pos += rl;
        tail_emit(tailw, d, rl, pos, body);
      }
      const uint32_t m = mag_u32(v);
      const uint32_t ml = glen(m);
      const uint64_t sm = ((uint64_t)(v > 0) << ml) | m;
      pos += 1 + ml;
      tail_emit(tailw, sm, 1 + ml, pos, body);
      prev = rel0 + k;
    }
  }
  for (int j = 0; j < kChunks; ++j) {
    o.chunk_prev[j] = chunk_prev[j];
    o.chunk_off[j] = chunk_off[j];
  }
  o.body = body;
  o.carry = carry;
  o.wfirst = wfirst;
  o.dist = dist;
  o.nnz = nnz;
  o.tail = uniform(*tailw);
}

struct SlowEmit {
  uint32_t r0, tb, R0, dfirst, bstart, body, trail_len, nwords_owned, nwin_bits;
  int32_t tile_last;
  uint64_t trail, w0;
  uint32_t* out32;
  int64_t cap;
};

template <int MODE, bool INT_IN, bool RCP>
__device__ __forceinline__ void slow_emit(const EncodeArgs& a, const ClientQ& cq, int32_t c,
                                                    int64_t tile_base, uint32_t* win, const SlowScan& sc,
                                                    const SlowEmit& e) {
  const int lane = threadIdx.x;
  const uint32_t npass = (e.nwords_owned + kWinWords - 1) / kWinWords;
  for (uint32_t pass = 0; pass < npass; ++pass) {
    const uint32_t plo = pass * kWinWords;
    if (lane == 0) {
      if (e.r0) win_emit32(win, e.tb, e.r0, 0, plo);
      if (e.tile_last >= 0) win_emit(win, e.dfirst, e.R0, e.r0, plo);
      if (e.trail_len) win_emit(win, e.trail, e.trail_len, e.bstart + e.body, plo);
    }
#pragma unroll 1
    for (int j = 0; j < kChunks; ++j) {
      const int32_t rel0 = 256 * j + 4 * lane;
      int32_t prev = sc.chunk_prev[j];
      uint32_t pos = e.bstart + sc.chunk_off[j];
      int32_t q4[4];
      float dd = 0.0f;
      reload_chunk<MODE, INT_IN, RCP>(a, cq, c, tile_base + rel0, q4, dd);
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
          win_emit32(win, d, rl, pos, plo);
          pos += rl;
        }
        win_emit(win, sm, 1 + ml, pos, plo);
        pos += 1 + ml;
        prev = rel0 + k;
      }
    }
    const uint32_t nw = min((uint32_t)kWinWords, e.nwords_owned - plo);
    for (uint32_t i = lane; i < nw; i += kEncThreads) {
      const uint64_t wi = e.w0 + plo + i;
      if ((int64_t)(wi + 1) * 4 <= e.cap) e.out32[wi] = bswap32(win[i]);
    }
    const uint32_t nt = min((uint32_t)kWinWords, (e.nwin_bits + 31) / 32 - plo);
    for (uint32_t i = lane; i < nt; i += kEncThreads) win[i] = 0;
  }
}

// s_waitcnt immediates (gfx9 encoding): vmcnt(0) alone / lgkmcnt(0) alone.
constexpr int kWaitVm0 = 0x0F70;

// Tile staging through LDS-DMA (global_load_lds_dwordx4).  DMA instruction b
// (b = 0..3) fetches the tile's 1-KiB global block b -- coalesced -- into staging
// words [256 b, +256), permuted inside the block so that lane l's chunk j
// (tile elements [16 l + 4 j, +4)) lands at word 256 (l >> 4) + 64 j + 4 ((l + 4 j) & 15):
// the four ds_read_b128 that hand each lane its 16 consecutive elements are then
// bank-conflict-free (every 16-lane group of a ds_read_b128 covers all 64 banks).
// Only full tiles of 16-B-aligned rows are staged; returns whether it issued.
#ifndef FC_STAGE_AUX
#define FC_STAGE_AUX 2  // cache policy of the encoders' LDS-DMA staging loads (2: nt; the rows are read once): with FC_CODE_NT -1.3 % stochastic, -3 % uniform (profiles/r05/diag_enc_nt_ab.txt)
#endif
constexpr int kStageAux = FC_STAGE_AUX;
#ifndef FC_CODE_NT
#define FC_CODE_NT 1  // the encoders' code-word stores non-temporal (0: default policy)
#endif
__device__ __forceinline__ void code_store(uint32_t* p, uint32_t v) {
  if (FC_CODE_NT) __builtin_nontemporal_store(v, p);
  else *p = v;
}
__device__ __forceinline__ bool stage_tile(const EncodeArgs& a, ConstParamPtr cparams, uint32_t ticket,
                                           uint32_t* stg, int lane) {
  const int32_t t = (int32_t)div_clients(a, ticket);
  const int32_t c = (int32_t)(ticket - (uint32_t)t * (uint32_t)a.nclients);
  const int64_t tile_base = (int64_t)t * kTE;
  const uint32_t* x = cparams[c].x;
  if (tile_base + kTE > a.P || ((uintptr_t)x & 15u) || (FC_ABL & 64)) return false;
  const uint32_t j = (uint32_t)lane >> 4, q = (uint32_t)lane & 15u;
  // one lane address for all four: the instruction offset (1 KiB * b) applies to
  // both the global and the LDS address, and the LDS base stays the staging array
  // (typed pointers: generic ones cost a null-checked M0 and a 64-bit add per DMA)
  typedef __attribute__((address_space(1))) void* gvptr;
  typedef __attribute__((address_space(3))) void* lvptr;
  const uint32_t lane_bytes = 4u * (16u * ((q - 4u * j) & 15u) + 4u * j);
  const gvptr src = (gvptr)((const char*)(x + tile_base) + lane_bytes);
  const lvptr dst = (lvptr)stg;
  __builtin_amdgcn_global_load_lds(src, dst, 16, 0, kStageAux);
  __builtin_amdgcn_global_load_lds(src, dst, 16, 1024, kStageAux);
  __builtin_amdgcn_global_load_lds(src, dst, 16, 2048, kStageAux);
  __builtin_amdgcn_global_load_lds(src, dst, 16, 3072, kStageAux);
  return true;
}
__device__ __forceinline__ int stage_pos(int lane, int j) {
  return 256 * (lane >> 4) + 64 * j + 4 * ((lane + 4 * j) & 15);
}
// The staging reads are inline asm: the compiler's wait-count pass treats any
// ds_read of a buffer an LDS-DMA wrote as waiting on that DMA, and would otherwise
// drain vmcnt -- including the next tile's DMA and the pending tile's stores -- at
// every tile start.  The four reads and their lgkmcnt wait are ONE statement with
// early-clobber outputs: the compiler sees the registers written only once the
// data has landed, so it cannot copy, spill or reuse them before.
typedef uint32_t u32x4_t __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void stage_read4(const uint32_t* stg, int lane, uint32_t (&raw)[kChunks][4]) {
  static_assert(kChunks == 4, "four staging reads per lane");
  typedef const __attribute__((address_space(3))) uint32_t* lds_cptr;
  u32x4_t v0, v1, v2, v3;
  asm volatile(
      "ds_read_b128 %0, %4\n\t"
      "ds_read_b128 %1, %5\n\t"
      "ds_read_b128 %2, %6\n\t"
      "ds_read_b128 %3, %7\n\t"
      "s_waitcnt lgkmcnt(0)"
      : "=&v"(v0), "=&v"(v1), "=&v"(v2), "=&v"(v3)
      : "v"((lds_cptr)(stg + stage_pos(lane, 0))), "v"((lds_cptr)(stg + stage_pos(lane, 1))),
        "v"((lds_cptr)(stg + stage_pos(lane, 2))), "v"((lds_cptr)(stg + stage_pos(lane, 3)))
      : "memory");
  raw[0][0] = v0.x; raw[0][1] = v0.y; raw[0][2] = v0.z; raw[0][3] = v0.w;
  raw[1][0] = v1.x; raw[1][1] = v1.y; raw[1][2] = v1.z; raw[1][3] = v1.w;
  raw[2][0] = v2.x; raw[2][1] = v2.y; raw[2][2] = v2.z; raw[2][3] = v2.w;
  raw[3][0] = v3.x; raw[3][1] = v3.y; raw[3][2] = v3.z; raw[3][3] = v3.w;
}

// One wavefront = one workgroup = one 1024-element tile at a time: no barriers,
// every cross-lane step is DPP / ballot / readlane, the bit window is the
// wave's own LDS.  Software-pipelined over the wave's tiles: tile n is
// quantised, coded and its aggregate published, then tile n-1 (whose
// predecessor status was fetched before tile n's work) finishes its look-back
// and stores its words -- so the look-back's memory round trip overlaps a
// whole tile of compute instead of stalling the wave.
template <int MODE, bool INT_IN, int DIV, bool PRE>
__global__ __launch_bounds__(kEncThreads, FC_ENC_WAVES) void k_encode(EncodeArgs a) {
  __shared__ uint32_t wins[2][kWinWords + 3];  // double-buffered; + guard words
  __shared__ uint32_t clut[kCodeLut];
  __shared__ __attribute__((aligned(16))) uint32_t stg[kTE];  // LDS-DMA staging of the next tile
  const int lane = threadIdx.x;
  for (int i = lane; i < kCodeLut; i += kEncThreads) clut[i] = code_lut_entry((uint32_t)i);
  const uint32_t total_tiles = (uint32_t)a.nclients * (uint32_t)a.T;
  const ConstParamPtr cparams = (ConstParamPtr)a.cparams;
  constexpr bool pre = PRE;
  const int64_t P = a.P;
#ifdef FC_STAMPS
  uint64_t st_acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  uint64_t st_last = __builtin_amdgcn_s_memtime();
#endif
  for (int i = lane; i < 2 * (kWinWords + 3); i += kEncThreads) (&wins[0][0])[i] = 0;
  const uint32_t shard = ticket_stream(a.started, blockIdx.x, 0, 1, a.nshards, a.by_block, lane);
  uint32_t* my_counter = a.counter + kShardStride * shard;
  // Tickets run two ahead: the tile after the current one is known when the
  // current one starts, so its values are staged into LDS (LDS-DMA) while the
  // current tile computes.
  uint32_t tk = 0;
  if (lane == 0) tk = atomicAdd(my_counter, 1u);
  uint32_t ticket = shard + a.nshards * uniform(tk);
  uint32_t tk1 = 0;
  if (ticket < total_tiles && lane == 0) tk1 = atomicAdd(my_counter, 1u);
  uint32_t ticket1 = ticket < total_tiles ? shard + a.nshards * uniform(tk1) : ticket;
  bool staged = ticket < total_tiles && stage_tile(a, cparams, ticket, stg, lane);
  __builtin_amdgcn_s_waitcnt(kWaitVm0);
  // the pending tile (coded, aggregate published, words not yet stored)
  bool pv = false;
  int32_t pt = 0, pc = 0, pfirst = 0, plast = -1;
  uint32_t pbody = 0, ptail = 0;
  uint32_t buf = 0;

  for (;;) {
    const bool have = ticket < total_tiles;
    if (!have && !pv) break;
    STAMP(0);
    uint32_t ntk = 0;  // the ticket after next: requested once the next tile is staged (below)
    // the pending tile's look-back window (lane i: tile pt-64+i), fetched now and
    // used after this tile's work
    uint64_t pw1 = 0, pw2 = 0;  // not fetched: unreadable (lookback_vec re-polls it if needed)
    // only the nearest statuses are fetched (window chosen per launch): every fetched
    // status is a coherent read, so with few clients -- many tiles of one client in
    // flight -- a short window is cheaper even when the nearest inclusive prefix
    // lies beyond it (lookback_vec then polls further back itself)
    if (!(FC_ABL & 16) && pv && pt + lane >= 64 && lane >= a.lb_lane0) {
      const uint64_t* sp = a.status + 2 * ((int64_t)pc * a.T + pt - 64 + lane);
      pw1 = ld_agent(sp);
      pw2 = ld_agent(sp + 1);
    }
    // ---- this tile: A-D, then publish its aggregate ----
    bool nv = false;
    int32_t nt_ = 0, nc = 0, nfirst = 0, nlast = -1;
    uint32_t nbody = 0, ntail = 0;
    if (have) {
      uint32_t* win = wins[buf];
      // tickets interleave clients (tile-major) so each client has few tiles in flight
      const int32_t t = (int32_t)div_clients(a, ticket);
      const int32_t c = (int32_t)(ticket - (uint32_t)t * (uint32_t)a.nclients);
      const int64_t tile_base = (int64_t)t * kTE;
      const bool full = tile_base + kTE <= P;
      const ClientParam cp = ld_param(cparams + c);
      // raw values: lane l owns the 16 consecutive tile elements [16 l, 16 l + 16),
      // chunk j = [16 l + 4 j, +4), from the LDS staging (full, 16-B aligned
      // tiles) or loaded directly (a client's last, partial tile)
      const int32_t lrel = 16 * lane;
      uint32_t raw[kChunks][4];
      if (FC_ABL & 64) {  // diagnostics: synthetic values, no loads
#pragma unroll
        for (int j = 0; j < kChunks; ++j) {
          const uint32_t h = (uint32_t)(tile_base + lrel + 4 * j) * 2654435761u;
          raw[j][0] = __float_as_uint(((float)((h >> 28) & 15u) - 7.5f) * 0.3f);
          raw[j][1] = __float_as_uint(((float)((h >> 24) & 15u) - 7.5f) * 0.3f);
          raw[j][2] = __float_as_uint(((float)((h >> 20) & 15u) - 7.5f) * 0.3f);
          raw[j][3] = __float_as_uint(((float)((h >> 16) & 15u) - 7.5f) * 0.3f);
        }
      } else {
        if (!staged) {  // a client's last (partial) tile or an unaligned row: load into the staging
#pragma unroll
          for (int j = 0; j < kChunks; ++j) {
            const int64_t e0 = tile_base + lrel + 4 * j;
            uint4 v;
            if (full) {
              v = *(const uint4*)(cp.x + e0);
            } else {
              v.x = e0 < P ? cp.x[e0] : 0u;
              v.y = e0 + 1 < P ? cp.x[e0 + 1] : 0u;
              v.z = e0 + 2 < P ? cp.x[e0 + 2] : 0u;
              v.w = e0 + 3 < P ? cp.x[e0 + 3] : 0u;
            }
            *(uint4*)(stg + stage_pos(lane, j)) = v;
          }
        }
        stage_read4(stg, lane, raw);
      }
      // the staging is free once read: stage the next tile (waited for after part C)
      staged = ticket1 < total_tiles && stage_tile(a, cparams, ticket1, stg, lane);
      // ticket after next: its round trip completes under this tile's work (the
      // s_waitcnt after part C); requested at the loop top it made every tile wait
      // for the atomic and for the previous tile's stores
      if (ticket1 < total_tiles && lane == 0) ntk = atomicAdd(my_counter, 1u);
      // ---- A: quantise + code the lane's four chunks in order.  A chunk's first
      //      run code comes from the lane's previous nonzero when there is one;
      //      the lane's very first run code depends on earlier lanes and is
      //      resolved after the scan.
      float dist = 0.0f;
      int32_t nnz = 0;  // INT_IN and CHAIN: per lane; else the wave total
      int32_t lfirst = -1, llast = -1;  // the lane's first / last nonzero (tile-relative)
      uint32_t lng = 0, llen = 0;
      uint64_t cacc[kChunks];
      uint32_t clen[kChunks];
      {
        const ClientQ cq = client_q_of(cp, pre);
  #pragma unroll
        for (int j = 0; j < kChunks; ++j) {
          const int32_t rel0 = lrel + 4 * j;
          ChunkCode cc;
          if (INT_IN) {
            int32_t q4[4];
  #pragma unroll
            for (int k = 0; k < 4; ++k) q4[k] = (int32_t)raw[j][k];
  #pragma unroll
            for (int k = 0; k < 4; ++k) nnz += q4[k] != 0;
            cc = chunk_local(q4, rel0);
          } else {
            const uint32_t g = (uint32_t)((tile_base + rel0) >> 2) + cq.gofs;
            if (MODE == FC_DITHERED && !full)
              cc = quant_code_fast<MODE, DIV, PRE, true>(cq, g, raw[j], rel0, dist, nnz, clut,
                                                    (int32_t)min<int64_t>(4, max<int64_t>(0, P - tile_base - rel0)));
            else
              cc = quant_code_fast<MODE, DIV, PRE>(cq, g, raw[j], rel0, dist, nnz, clut);
          }
          chunk_prepend(cc, llast);  // no-op without an earlier nonzero in the lane
          lfirst = lfirst < 0 ? cc.first : lfirst;
          llast = cc.last >= 0 ? cc.last : llast;
          lng |= cc.lng;
          cacc[j] = cc.acc;
          clen[j] = cc.len;
          llen += cc.len;
          FC_CHUNK_BARRIER;
        }
      }
      // ---- B: one scan pair per tile -- last nonzero before each lane (max-scan)
      //      gives the lane's first run code, then code offsets (sum-scan)
      const int32_t im = dpp_incl_max(llast);
      const int32_t lprev = dpp_shr1(im, -1);  // -1: no nonzero in earlier lanes of this tile
      const int32_t tile_last = lane63(im);
      const bool lrun = lfirst >= 0 && lprev >= 0;
      const uint32_t dv = lrun ? (uint32_t)(lfirst - lprev) : 0u;
      const uint32_t R = lrun ? glen(dv) : 0u;
      const uint32_t ltot = R + llen;
      const uint32_t is = dpp_incl_sum(ltot);
      const uint32_t body = (uint32_t)lane63((int32_t)is);
      const uint64_t lngmask = __ballot(lng != 0);
      // ---- C: emit the lane's run code and chunks (codes past the window land in
      //      the guard words; the tile is then slow)
      if (FC_ABL & 1) {  // diagnostics: no emission
        asm volatile("" :: "v"(dv), "v"(R), "v"((uint32_t)cacc[0]), "v"((uint32_t)cacc[1]), "v"((uint32_t)cacc[2]),
                     "v"((uint32_t)cacc[3]), "v"(is));
      } else {
        uint32_t o = kPre + is - ltot;
        emit32(win, dv, R, o);
        o += R;
  #pragma unroll
        for (int j = 0; j < kChunks; ++j) {
          emit64(win, cacc[j], clen[j], o);
          o += clen[j];
        }
      }
      __builtin_amdgcn_s_waitcnt(kWaitVm0);  // next tile staged (and the look-back window loaded)
      STAMP(1);
      // fast path: no long chunk, prefix + body + trailing code + one funnel word
      // fit the wave's window, and a finite distortion (no NaN / infinite r)
      const float dsum = INT_IN ? 0.0f : wave_sum_f(dist);
      const bool fast = lngmask == 0 && kPre + body + 96u <= 32u * kWinWords &&
                        (INT_IN || dsum <= 3.4028235e38f);
      STAMP(2);

      const uint32_t agg_tail = fast ? uniform(win_bits32(win, kPre - 32u + body)) : 0u;
      const uint64_t fm = __ballot(lfirst >= 0);  // lanes are in element order
      const int32_t tile_first = fm ? __builtin_amdgcn_readlane(lfirst, (int)__builtin_ctzll(fm)) : -1;
      if (uint64_t* const iq = enc_args_fresh().idxq) {
        // quarter starts (lanes 16, 32, 48): the body offset of the lane's first code
        // and the last nonzero before it (a slow tile's client is redone by the exact path)
        const uint32_t xo = is - ltot;
        const uint64_t q1 = quarter_rel(__builtin_amdgcn_readlane(xo, 16), __builtin_amdgcn_readlane(lprev, 16),
                                        tile_first);
        const uint64_t q2 = quarter_rel(__builtin_amdgcn_readlane(xo, 32), __builtin_amdgcn_readlane(lprev, 32),
                                        tile_first);
        const uint64_t q3 = quarter_rel(__builtin_amdgcn_readlane(xo, 48), __builtin_amdgcn_readlane(lprev, 48),
                                        tile_first);
        if (lane == 0) {
          uint64_t* q = iq + 3 * ((int64_t)c * a.T + t);
          q[0] = q1;
          q[1] = q2;
          q[2] = q3;
        }
      }
      if (fast && !(FC_ABL & 32)) {
        const float d = DIV == 1 ? dsum * (cp.step * cp.step) : dsum;  // DIV 1: sums of (sc - r)^2
        const int32_t n = INT_IN ? wave_sum_i(nnz) : nnz;
        if (lane == 0) {
          if (a.dist_part) a.dist_part[(int64_t)c * a.T + t] = d;
          if (a.nnz_part) a.nnz_part[(int64_t)c * a.T + t] = n;
        }
      }
      STAMP(3);
      uint64_t* st = a.status + 2 * ((int64_t)c * a.T + t);
      if (!fast) {
        // a code past the fast path's limits or a body beyond the window: the
        // client is re-encoded by k_encode_exact
        if (lane == 0) {
          st_agent(st + 1, kFlagSlow);
          st_agent(st, kFlagSlow);
          const EncodeArgs& ka = enc_args_fresh();
          if (atomicOr(&ka.slow_flag[c], 1) == 0) ka.slow_list[atomicAdd(ka.slow_count, 1u)] = c;
        }
        for (int i = lane; i < kWinWords; i += kEncThreads) win[i] = 0;
      } else {
        if (lane == 0) {
          if (t == 0) {  // chain root: the inclusive prefix right away
            Seg root = seg_identity(), agg;
            root.has_nz = 1;
            root.first = root.last = -1;
            agg.has_nz = tile_last >= 0;
            agg.first = agg.has_nz ? tile_first : 0;
            agg.last = agg.has_nz ? tile_last : 0;
            agg.body = body;
            agg.tail = agg_tail;
            const Seg incl = seg_combine(root, agg);
            st_agent2(st, kFlagPre | ((uint64_t)(incl.last + 1) << 36) | (incl.body & kMask36), kFlagPre | incl.tail);
          } else {
            const uint64_t fr = tile_last >= 0 ? (uint64_t)tile_first : kNoPos;
            const uint64_t lr = tile_last >= 0 ? (uint64_t)tile_last : kNoPos;
            st_agent2(st, agg_word(fr, lr, body), kFlagAgg | agg_tail);
          }
        }
        nv = true;
        nt_ = t;
        nc = c;
        nfirst = tile_first;
        nlast = tile_last;
        nbody = body;
        ntail = agg_tail;
      }
    }
    STAMP(4);

    // ---- the pending tile: look-back, publish its prefix, store its words ----
    if (pv) {
      // the pending state is wave-uniform: readfirstlane keeps the bookkeeping
      // below on the scalar unit (the loop-carried copies may live in VGPRs)
      pt = (int32_t)uniform((uint32_t)pt);
      pc = (int32_t)uniform((uint32_t)pc);
      pfirst = (int32_t)uniform((uint32_t)pfirst);
      plast = (int32_t)uniform((uint32_t)plast);
      pbody = uniform(pbody);
      ptail = uniform(ptail);
      uint32_t* win = wins[buf ^ 1];
      const int64_t tile_base = (int64_t)pt * kTE;
      const bool last_tile = (pt == a.T - 1);
      uint64_t* st = a.status + 2 * ((int64_t)pc * a.T + pt);
      Seg agg;
      agg.has_nz = plast >= 0;
      agg.first = agg.has_nz ? (int32_t)(tile_base + pfirst) : 0;
      agg.last = agg.has_nz ? (int32_t)(tile_base + plast) : 0;
      agg.body = pbody;
      agg.tail = ptail;
      bool slow = false;
      Seg excl = seg_identity();
      if (pt == 0 || (FC_ABL & 4)) {
        excl.has_nz = 1;
        excl.first = excl.last = -1;
      } else {
        bool to = false;
        excl = lookback_vec(a.status + 2 * (int64_t)pc * a.T, pt, lane, slow, to, pw1, pw2);
        if (to && lane == 0) atomicOr(enc_args_fresh().spin_err, 1u);
        if (FC_ABL & 4096) {  // diagnostics: the look-back runs, its result is dropped
          asm volatile("" :: "s"((uint32_t)excl.body), "s"(excl.last), "s"(excl.tail));
          excl = seg_identity();
          excl.has_nz = 1;
          excl.first = excl.last = -1;
        }
      }
      if (slow) {
        if (lane == 0) {
          st_agent(st + 1, kFlagSlow);
          st_agent(st, kFlagSlow);
          {
            const EncodeArgs& ka = enc_args_fresh();
            if (atomicOr(&ka.slow_flag[pc], 1) == 0) ka.slow_list[atomicAdd(ka.slow_count, 1u)] = pc;
          }
        }
        for (int i = lane; i < kWinWords; i += kEncThreads) win[i] = 0;
      } else {
        const Seg incl = seg_combine(excl, agg);
        const uint32_t r0 = (uint32_t)(excl.body & 31);
        const uint32_t dfirst = agg.has_nz ? (uint32_t)(agg.first - excl.last) : 0u;
        const uint32_t R0 = agg.has_nz ? glen(dfirst) : 0u;
        const uint32_t bstart = r0 + R0;  // stream-window bit where the body starts
        const uint32_t tb = excl.tail & (r0 ? ((1u << r0) - 1u) : 0u);
        uint32_t trail_len = 0;
        uint64_t trail = 0;
        if (last_tile) {
          const int64_t zc = P - 1 - (int64_t)incl.last;  // trailing zeros
          if (zc > 0) {
            trail = (uint64_t)(zc + 1);
            trail_len = 2u * (63u - (uint32_t)__clzll(trail)) + 1u;
          }
        }
        if (lane == 0) {
          if (pt > 0) {
            st_agent2(st, kFlagPre | ((uint64_t)(incl.last + 1) << 36) | (incl.body & kMask36), kFlagPre | incl.tail);
          }
          const int64_t ib = (int64_t)pc * (a.T + 1);
          a.idx[ib + pt] = (excl.body & kMask36) | ((uint64_t)(excl.last + 1) << 36);
          if (last_tile) {
            a.idx[ib + a.T] = (incl.body & kMask36) | ((uint64_t)(incl.last + 1) << 36);
            enc_args_fresh().total_bits[pc] = (int64_t)incl.body + trail_len;
          }
          // leading pieces just before the body, trailing code after it
          emit64(win, tb, r0, kPre - bstart);
          emit64(win, dfirst, R0, kPre - R0);
          if (trail_len) emit64(win, trail, trail_len, kPre + pbody);
        }
        STAMP(5);
        const ClientParam cp = ld_param(cparams + pc);
        const uint32_t nwin_bits = bstart + pbody + trail_len;
        const uint32_t nwords_owned = last_tile ? (nwin_bits + 31) / 32 : nwin_bits / 32;
        const int64_t cap = cp.cap;
        uint32_t* out32 = cp.out;
        const uint64_t w0 = excl.body >> 5;
        if (lane == 0 && (int64_t)(w0 + nwords_owned) * 4 > cap) atomicOr((uint32_t*)&enc_args_fresh().overflow[pc], 1u);
        const uint32_t s0 = kPre - bstart;  // window bit of stream-window bit 0
        const uint32_t lead = kStoreAlign ? (uint32_t)(((uintptr_t)(out32 + w0) >> 2) & 31u) : 0u;  // lanes before the line
        // (as k_encode2: the capacity bound once, a tile-uniform funnel per word)
        const uint32_t nst = (uint32_t)max<int64_t>(0, min<int64_t>(nwords_owned, cap / 4 - (int64_t)w0));
        const uint32_t so = s0 & 31u;
        const uint32_t* const wsrc = win + (s0 >> 5);
        uint32_t* const dst = out32 + w0;
        if (!(FC_ABL & 1024))
        for (uint32_t k = lane; k < nst + lead; k += kEncThreads) {
          if (k < lead) continue;
          const uint32_t kk = k - lead;
          const uint32_t a0 = wsrc[kk], a1 = wsrc[kk + 1];
          const uint32_t wv32 = so ? __builtin_amdgcn_alignbit(a0, a1, 32u - so) : a0;
          if (FC_ABL & 2) asm volatile("" :: "v"(wv32));
          else code_store(dst + kk, bswap32(wv32));
        }
        const uint32_t nt = min((uint32_t)kWinWords, (kPre + pbody + trail_len + 31) / 32 + 1);
        if (!(FC_ABL & 1024))
        for (uint32_t i = lane; i < nt; i += kEncThreads) win[i] = 0;
      }
    }
    STAMP(6);
    pv = nv;
    pt = nt_;
    pc = nc;
    pfirst = nfirst;
    plast = nlast;
    pbody = nbody;
    ptail = ntail;
    buf ^= 1;
    if (have) {
      ticket = ticket1;
      if (ticket1 < total_tiles) ticket1 = shard + a.nshards * uniform(ntk);
    }
  }
#ifdef FC_STAMPS
  if (lane == 0)
    for (int i = 0; i < 8; ++i) atomicAdd(&g_stamps[i], (unsigned long long)st_acc[i]);
#endif
}

// Super-tile encoder: one wave codes two consecutive tiles of one client (a
// 2048-element super-tile) into one LDS window -- each half exactly as
// k_encode codes a tile, the second half's lane scans continuing from the
// first half's body and last nonzero -- and then publishes one status, runs
// one look-back and stores the super-tile's words.  The per-ticket work that
// does not grow with the elements (ticket, status prefetch and publish, look-back,
// leading pieces, store and clear set-up, reductions) is paid once per 2048
// elements.  No pending tile: the look-back window is requested when the second
// half starts, so its round trip overlaps that half's work, and the LDS holds one
// window of the super-tile's size instead of two.  Statuses are per super-tile
// (slot t2 of the client's row); the decoder index stays per 1024-element tile.
#ifndef FC_PAIR_CHAIN
#define FC_PAIR_CHAIN 1  // k_encode2: the chained pair table (run state across the lane's chunks)
#endif
#ifndef FC_ENC2_WAVES
#define FC_ENC2_WAVES 8  // k_encode2 waves per workgroup (4 or 8; two 8-wave workgroups per CU)
#endif
#ifndef FC_WIN2_WORDS
// LDS per CU (160 KiB) = workgroups x (tables + waves x (window + 4 KiB staging)):
// the chained table's 9 KiB shared by eight waves leave 1240-word windows (two
// 8-wave workgroups per CU), by four 952 (four 4-wave workgroups)
#define FC_WIN2_WORDS (FC_PAIR_CHAIN ? (FC_ENC2_WAVES == 8 ? 1240 : 952) : 2 * FC_WIN_WORDS)
#endif
constexpr uint32_t kWin2Words = FC_WIN2_WORDS;
static_assert(kWin2Words % 4 == 0, "k_encode2 zeroes its window 16 bytes at a time");
// NT-tile tickets while codes are expected within this many bits per element: a
// window holds 32 * kWin2Words - kPre - 96 bits (1240 words: ~9.6 bits per element
// for four tiles, ~4.8 for eight); the host's expectation is the caller's
// capacity hint (the last round's largest code + 1/8)
constexpr double kNt4Bits = FC_ENC2_WAVES == 8 ? 8.5 : 6.5;
constexpr double kNt8Bits = FC_ENC2_WAVES == 8 ? 4.4 : 0.0;
constexpr int kSTE = 2 * kTE;  // elements per super-tile

// LDS-DMA of one full, 16-B-aligned tile into the staging (as stage_tile).
__device__ __forceinline__ bool stage_at(const uint32_t* x, int64_t tile_base, int64_t P, uint32_t* stg,
                                         int lane) {
  if (tile_base + kTE > P || ((uintptr_t)x & 15u)) return false;
  const uint32_t j = (uint32_t)lane >> 4, q = (uint32_t)lane & 15u;
  typedef __attribute__((address_space(1))) void* gvptr;
  typedef __attribute__((address_space(3))) void* lvptr;
  const uint32_t lane_bytes = 4u * (16u * ((q - 4u * j) & 15u) + 4u * j);
  const gvptr src = (gvptr)((const char*)(x + tile_base) + lane_bytes);
  const lvptr dst = (lvptr)stg;
  __builtin_amdgcn_global_load_lds(src, dst, 16, 0, kStageAux);
  __builtin_amdgcn_global_load_lds(src, dst, 16, 1024, kStageAux);
  __builtin_amdgcn_global_load_lds(src, dst, 16, 2048, kStageAux);
  __builtin_amdgcn_global_load_lds(src, dst, 16, 3072, kStageAux);
  return true;
}

// Four independent waves per workgroup: they share the code tables (LDS per wave
// = window + staging + a quarter of the tables), nothing else -- each takes its
// own tickets; the only barrier is after the tables are built.
constexpr int kEnc2Waves = FC_ENC2_WAVES;
#ifndef FC_PAIR_LUT
#define FC_PAIR_LUT 1
#endif
#ifndef FC_LB_LATE
#define FC_LB_LATE 0  // k_encode2: look-back window loaded after the last tile's codes (A/B knob)
#endif
#ifndef FC_QUANT_FIRST
#define FC_QUANT_FIRST 0  // k_encode2: a tile's chunks quantised before any is coded (measured even: profiles/r05/diag_enc_qfirst_ab.txt)
#endif
#ifndef FC_SCAN_SKIP
#define FC_SCAN_SKIP 1  // k_encode2: no max-scan for the lanes' previous nonzero when every lane has one (-0.6 %)
#endif
#ifndef FC_RUN_MERGE
#define FC_RUN_MERGE 1  // k_encode2: the lane's run code emitted with its first chunk pair when they fit 64 bits (-1.2 %; both -1.4 %, profiles/r05/diag_enc_scan_merge_ab.txt)
#endif
#ifndef FC_FRESH_ARGS
#define FC_FRESH_ARGS 0  // k_encode2's once-per-ticket fields re-read from the kernel arguments: 0 none,
                         // 1 partials + index pointers, 2 also the status pointer and T2 (A/B knob:
                         // fewer SGPR spill reloads, but 1 / 2 took the stochastic encode +1.3 / +2 %,
                         // the scalar loads' waits: profiles/r05/diag_enc_fresh_ab.txt)
#endif
template <int MODE, bool INT_IN, int DIV, bool PRE, int NT>
__global__ __launch_bounds__(kEncThreads * kEnc2Waves, FC_ENC_WAVES) void k_encode2(EncodeArgs a) {
  constexpr int STE = NT * kTE;  // elements per super-tile (ticket)
  constexpr bool CHAIN = FC_PAIR_CHAIN && FC_PAIR_LUT && !INT_IN;
  constexpr int kPL = CHAIN ? kChainLut : kPairLut;
  // one LDS block, the code tables first: their byte offsets (< 64 KiB) fold into the
  // ds_read instruction offsets instead of an add per lookup
  struct __attribute__((aligned(16))) Lds {
    uint32_t plut[kPL];
    uint32_t clut[kCodeLut];
    uint32_t stgs[kEnc2Waves][kTE];              // LDS-DMA staging of the next tile
    uint32_t wins[kEnc2Waves][kWin2Words + 4];  // + guard words (rows 16-byte aligned)
  };
  __shared__ Lds lds;
  uint32_t* const plut = lds.plut;
  uint32_t* const clut = lds.clut;
  auto& stgs = lds.stgs;
  auto& wins = lds.wins;
  for (int i = threadIdx.x; i < kCodeLut; i += kEncThreads * kEnc2Waves) clut[i] = code_lut_entry((uint32_t)i);
  for (int i = threadIdx.x; i < kPL; i += kEncThreads * kEnc2Waves)
    plut[i] = CHAIN ? pair_chain_entry((uint32_t)i) : pair_lut_entry((uint32_t)i);
  const int wave = (int)uniform(threadIdx.x >> 6);  // wave-uniform (the compiler cannot tell)
  const int lane = (int)(threadIdx.x & 63u);
  uint32_t* win = wins[wave];
  uint32_t* stg = stgs[wave];
  for (int i = lane; i < (int)kWin2Words + 4; i += kEncThreads) win[i] = 0;
  __syncthreads();
  const uint32_t total = (uint32_t)a.nclients * (uint32_t)a.T2;
  const ConstParamPtr cparams = (ConstParamPtr)a.cparams;
  const int64_t P = a.P;
  const uint32_t shard = ticket_stream(a.started, blockIdx.x, (uint32_t)wave, kEnc2Waves, a.nshards, a.by_block, lane);
  uint32_t* my_counter = a.counter + kShardStride * shard;
  // tickets run one ahead: the next super-tile's first tile is staged while the
  // current one's second tile computes
  uint32_t tk = 0;
  if (lane == 0) tk = atomicAdd(my_counter, 1u);
  uint32_t ticket = shard + a.nshards * uniform(tk);
  uint32_t tk1 = 0;
  if (ticket < total && lane == 0) tk1 = atomicAdd(my_counter, 1u);
  uint32_t ticket1 = ticket < total ? shard + a.nshards * uniform(tk1) : ticket;
  bool staged = false;
  if (ticket < total) {
    const int32_t t2 = (int32_t)div_clients(a, ticket);
    const int32_t c = (int32_t)(ticket - (uint32_t)t2 * (uint32_t)a.nclients);
    staged = stage_at(cparams[c].x, (int64_t)t2 * STE, P, stg, lane);
  }
  __builtin_amdgcn_s_waitcnt(kWaitVm0);
#ifdef FC_STAMPS
  uint64_t st_acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  uint64_t st_last = __builtin_amdgcn_s_memtime();
#endif

  while (ticket < total) {
    STAMP(7);
    const int32_t t2 = (int32_t)div_clients(a, ticket);
    const int32_t c = (int32_t)(ticket - (uint32_t)t2 * (uint32_t)a.nclients);
    const int32_t t0 = NT * t2;  // first tile of the super-tile
    const int nt = min(NT, a.T - t0);  // tiles in this super-tile
    const int64_t sbase = (int64_t)t2 * STE;
    // the client's parameters: the quantiser and row here, the stream at the end
    // (re-read there: fewer scalar registers held across the two tiles)
    const ClientQ cq = client_q_of(ld_param(cparams + c), PRE);
    const uint32_t* xrow = cparams[c].x;
    uint32_t ntk = 0;
    uint64_t pw1 = 0, pw2 = 0;  // look-back window (lane i: super-tile t2-64+i); 0: not fetched
    float dist = 0.0f;
    DistAcc dacc;  // (the chained-table path)
    dacc.zero();
    int32_t nnz = 0;  // INT_IN and CHAIN: per lane; else the wave total
    uint32_t lng = 0;  // lane has a long chunk (either tile)
    uint32_t body = 0;
    int32_t sfirst = -1, slast = -1;  // super-tile-relative first / last nonzero
    uint32_t bodyv = 0;   // lane h: body bits before tile h
    int32_t lastv = -1;   // lane h: last nonzero before tile h (super-tile-relative, -1 none)
    for (int h = 0; h < NT; ++h) {
      if (h >= 1) {
        if (h >= nt) break;
        STAMP(0);
        __builtin_amdgcn_s_waitcnt(kWaitVm0);  // the second tile's staging has landed
        STAMP(1);
      }
      const int64_t tile_base = sbase + (int64_t)h * kTE;
      const bool full = tile_base + kTE <= P;
      const int32_t lrel = 16 * lane;
      uint32_t raw[kChunks][4];
      if (!staged && !(FC_ABL & 64)) {  // a client's last (partial) tile or an unaligned row: load into the staging
#pragma unroll
        for (int j = 0; j < kChunks; ++j) {
          const int64_t e0 = tile_base + lrel + 4 * j;
          uint4 v;
          if (full) {
            v = *(const uint4*)(xrow + e0);
          } else {
            v.x = e0 < P ? xrow[e0] : 0u;
            v.y = e0 + 1 < P ? xrow[e0 + 1] : 0u;
            v.z = e0 + 2 < P ? xrow[e0 + 2] : 0u;
            v.w = e0 + 3 < P ? xrow[e0 + 3] : 0u;
          }
          *(uint4*)(stg + stage_pos(lane, j)) = v;
        }
      }
      stage_read4(stg, lane, raw);
      if (FC_ABL & 64) {  // diagnostics: synthetic values in [-2, 2), no input loads
#pragma unroll
        for (int j = 0; j < kChunks; ++j)
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            const uint32_t hsh = ((uint32_t)tile_base + 16u * (uint32_t)lane + 4u * j + k) * 2654435761u ^ (uint32_t)c;
            raw[j][k] = __float_as_uint(__uint_as_float((hsh & 0x7FFFFFu) | 0x40000000u) - 3.0f);
          }
      }
      // the staging is free once read: stage this super-tile's next tile, or the
      // next super-tile's first (waited for before it is read)
      if (h + 1 < nt) {
        staged = stage_at(xrow, tile_base + kTE, P, stg, lane);
      } else {
        staged = false;
        if (ticket1 < total) {
          const int32_t n2 = (int32_t)div_clients(a, ticket1);
          const int32_t nc = (int32_t)(ticket1 - (uint32_t)n2 * (uint32_t)a.nclients);
          staged = stage_at(cparams[nc].x, (int64_t)n2 * STE, P, stg, lane);
          // the ticket after next: its round trip completes under this tile's work
          if (lane == 0) ntk = atomicAdd(my_counter, 1u);
        }
        // the look-back window, loaded under the last tile's work
        if (!FC_LB_LATE && t2 + lane >= 64 && lane >= a.lb_lane0) {
          const uint64_t* sp = a.status + 2 * ((int64_t)c * a.T + t2 - 64 + lane);
          pw1 = ld_agent(sp);
          pw2 = ld_agent(sp + 1);
        }
      }
      // ---- A: quantise + code the lane's four chunks (super-tile-relative positions)
      int32_t lfirst = -1, llast = -1;
      uint32_t llen = 0;
      uint64_t cacc[kChunks];
      uint32_t clen[kChunks];
      const int32_t hrel = h * kTE + lrel;
      const uint32_t gbase = (uint32_t)(tile_base >> 2) + 4u * (uint32_t)lane + cq.gofs;  // Philox counter of chunk 0
      if (CHAIN) {
        // run state across the lane's chunks: only a far run (or a chunk off the
        // pair table) needs its first run code prepended, from the lane's mask
        uint32_t sst = 0, lmask = 0;
        // FC_QUANT_FIRST: the tile's four chunks quantised first (four independent Philox
        // chains in one straight block), one |q| <= 7 test for the tile, then the codes
        float qv[kChunks][4];
        bool tab = false;
        if (FC_QUANT_FIRST && !(MODE == FC_DITHERED && !full)) {
#pragma unroll
          for (int j = 0; j < kChunks; ++j) quant_chain4<MODE, DIV, PRE>(cq, gbase + (uint32_t)j, raw[j], dacc, qv[j]);
          float m = 0.0f;
#pragma unroll
          for (int j = 0; j < kChunks; ++j) m = vmax3_abs(qv[j][0], qv[j][1], vmax3_abs(qv[j][2], qv[j][3], m));
          tab = __ballot(!(m <= 7.0f)) == 0;
        }
#pragma unroll
        for (int j = 0; j < kChunks; ++j) {
          const uint32_t g = gbase + (uint32_t)j;
          ChainCode cc;
          if (FC_QUANT_FIRST && !(MODE == FC_DITHERED && !full))
            cc = tab ? code_chain<true>(qv[j], clut, plut, sst) : code_chain(qv[j], clut, plut, sst);
          else if (MODE == FC_DITHERED && !full)
            cc = quant_code_chain<MODE, DIV, PRE, true>(
                cq, g, raw[j], dacc, clut, plut, sst,
                (int32_t)min<int64_t>(4, max<int64_t>(0, P - tile_base - lrel - 4 * j)));
          else
            cc = quant_code_chain<MODE, DIV, PRE>(cq, g, raw[j], dacc, clut, plut, sst);
          if (cc.prem != 0) {
            if (cc.pre) {  // a nonzero before it in the lane: lmask != 0
              const uint32_t d = 4u * (uint32_t)j + (uint32_t)__builtin_ctz(cc.nzm) - (31u - (uint32_t)__builtin_clz(lmask));
              const uint32_t rl = 63u - 2u * (uint32_t)__builtin_clz(d);  // glen(d)
              cc.lng |= (cc.len + rl > 64u) ? 1u : 0u;
              cc.acc |= (uint64_t)d << (cc.len & 63u);
              cc.len += rl;
            }
          }
          lmask |= cc.nzm << (4 * j);
          lng |= cc.lng;
          cacc[j] = cc.acc;
          clen[j] = cc.len;
          llen += cc.len;
          FC_CHUNK_BARRIER;
        }
        nnz += (int32_t)__popc(lmask);  // the lane's nonzeros in this tile
        lfirst = lmask ? hrel + (int32_t)__builtin_ctz(lmask) : -1;
        llast = lmask ? hrel + 31 - (int32_t)__builtin_clz(lmask) : -1;
      } else
#pragma unroll
      for (int j = 0; j < kChunks; ++j) {
        const int32_t rel0 = hrel + 4 * j;
        ChunkCode cc;
        if (INT_IN) {
          int32_t q4[4];
#pragma unroll
          for (int k = 0; k < 4; ++k) q4[k] = (int32_t)raw[j][k];
#pragma unroll
          for (int k = 0; k < 4; ++k) nnz += q4[k] != 0;
          cc = chunk_local(q4, rel0);
        } else {
          const uint32_t g = gbase + (uint32_t)j;
          if (MODE == FC_DITHERED && !full)
            cc = quant_code_fast<MODE, DIV, PRE, true, FC_PAIR_LUT>(
                cq, g, raw[j], rel0, dist, nnz, clut,
                (int32_t)min<int64_t>(4, max<int64_t>(0, P - tile_base - lrel - 4 * j)), plut);
          else
            cc = quant_code_fast<MODE, DIV, PRE, false, FC_PAIR_LUT>(cq, g, raw[j], rel0, dist, nnz, clut, 4, plut);
        }
        if (!(FC_ABL & 8192)) chunk_prepend(cc, llast);  // no-op without an earlier nonzero in the lane
        lfirst = lfirst < 0 ? cc.first : lfirst;
        llast = cc.last >= 0 ? cc.last : llast;
        lng |= cc.lng;
        cacc[j] = cc.acc;
        clen[j] = cc.len;
        llen += cc.len;
        FC_CHUNK_BARRIER;
      }
      STAMP(2);
      // the look-back window, loaded late (FC_LB_LATE): after the last tile's codes,
      // so the statuses of predecessors still coding when the tile began are
      // more likely published (fewer re-polls), under the scans and emission
      if (FC_LB_LATE && h + 1 >= nt && t2 + lane >= 64 && lane >= a.lb_lane0) {
        const uint64_t* sp = a.status + 2 * ((int64_t)c * a.T + t2 - 64 + lane);
        pw1 = ld_agent(sp);
        pw2 = ld_agent(sp + 1);
      }
      // ---- B: scans -- last nonzero before each lane (lane 0: the first half's
      //      last nonzero, or none), then code offsets after the bits so far
      int32_t lprev, hlast;
      if (FC_SCAN_SKIP && __ballot(lfirst < 0) == 0) {
        // every lane holds a nonzero (dense tiles): the lanes' last nonzeros already rise
        // with the lane, so the one before lane l is lane l - 1's (lane 0: slast)
        lprev = dpp_shr1(llast, slast);
        hlast = lane63(llast);
      } else {
        const int32_t im = dpp_incl_max(max(llast, slast));  // slast < every position of this tile
        lprev = dpp_shr1(im, slast);
        hlast = lane63(im);
      }
      const bool lrun = lfirst >= 0 && lprev >= 0;
      const uint32_t dv = lrun ? (uint32_t)(lfirst - lprev) : 0u;
      const uint32_t R = lrun ? glen(dv) : 0u;
      const uint32_t ltot = R + llen;
      const uint32_t is = dpp_incl_sum(ltot);
      const uint32_t hbody = (uint32_t)lane63((int32_t)is);
      // ---- C: emit the lane's run code and chunks
      if (!(FC_ABL & 1)) {  // (diagnostics: no emission)
        uint32_t o = kPre + body + is - ltot;
        if (FC_RUN_MERGE && __ballot(R + clen[0] + clen[1] > 64u || clen[2] + clen[3] > 64u) == 0) {
          // the run code and the chunk pairs fit 64 bits across the wave (the common
          // case): two pieces, the run code leading the first
          const uint32_t c01 = clen[0] + clen[1];
          const uint64_t a01 = ((uint64_t)dv << (c01 & 63u)) | (cacc[0] << (clen[1] & 63u)) | cacc[1];
          const uint64_t a23 = (cacc[2] << (clen[3] & 63u)) | cacc[3];
          emit64<kWin2Words>(win, a01, R + c01, o);
          emit64<kWin2Words>(win, a23, clen[2] + clen[3], o + R + c01);
        } else {
        emit32<kWin2Words>(win, dv, R, o);
        o += R;
        if (__ballot(clen[0] + clen[1] > 64u || clen[2] + clen[3] > 64u) == 0) {
          // chunk pairs fit 64 bits across the wave (the common case): two pieces, not four
          const uint64_t a01 = (cacc[0] << (clen[1] & 63u)) | cacc[1];
          const uint64_t a23 = (cacc[2] << (clen[3] & 63u)) | cacc[3];
          emit64<kWin2Words>(win, a01, clen[0] + clen[1], o);
          emit64<kWin2Words>(win, a23, clen[2] + clen[3], o + clen[0] + clen[1]);
        } else {
#pragma unroll
          for (int j = 0; j < kChunks; ++j) {
            emit64<kWin2Words>(win, cacc[j], clen[j], o);
            o += clen[j];
          }
        }
        }
      }
      if (sfirst < 0) {
        const uint64_t fm = __ballot(lfirst >= 0);  // lanes are in element order
        sfirst = fm ? __builtin_amdgcn_readlane(lfirst, (int)__builtin_ctzll(fm)) : -1;
      }
      bodyv = lane == h ? body : bodyv;
      lastv = lane == h ? slast : lastv;
      slast = hlast >= 0 ? hlast : slast;
      body += hbody;
    }
    STAMP(3);
    __builtin_amdgcn_s_waitcnt(kWaitVm0);  // next tile staged, look-back window loaded
    STAMP(4);
    // fast path: no long chunk, prefix + body + trailing code + one funnel word fit
    // the window, and a finite distortion (no NaN / infinite r)
    const float dsum = INT_IN ? 0.0f : CHAIN ? dacc.wave_total(lane) : wave_sum_f(dist);
    const bool fast = __ballot(lng != 0) == 0 && kPre + body + 96u <= 32u * kWin2Words &&
                      (INT_IN || dsum <= 3.4028235e38f);
    uint64_t* const status_f = FC_FRESH_ARGS >= 2 ? enc_args_fresh().status : a.status;
    uint64_t* st = status_f + 2 * ((int64_t)c * a.T + t2);
    if (fast) {
      const float d = DIV == 1 ? dsum * (cq.step * cq.step) : dsum;  // DIV 1: sums of (sc - r)^2
      // per-lane counts (integer input, the chained table) or the wave total
      const int32_t n = (INT_IN || CHAIN) ? wave_sum_i(nnz) : nnz;
      // one partial per super-tile (its later tiles' slots: 0), one store instruction each
      if (lane < nt) {
        // (fields used once per ticket re-read from the kernel arguments: fewer SGPRs
        // held across the loop, fewer spill reloads through VGPR lanes)
        const EncodeArgs& fa = FC_FRESH_ARGS >= 1 ? enc_args_fresh() : a;
        if (fa.dist_part) fa.dist_part[(int64_t)c * a.T + t0 + lane] = lane == 0 ? d : 0.0f;
        if (fa.nnz_part) fa.nnz_part[(int64_t)c * a.T + t0 + lane] = lane == 0 ? n : 0;
      }
    }
    const uint32_t agg_tail = fast ? uniform(win_bits32(win, kPre - 32u + body)) : 0u;
    Seg agg;
    agg.has_nz = slast >= 0;
    agg.first = agg.has_nz ? (int32_t)(sbase + sfirst) : 0;
    agg.last = agg.has_nz ? (int32_t)(sbase + slast) : 0;
    agg.body = body;
    agg.tail = agg_tail;
    bool slow = !fast;
    Seg excl = seg_identity();
    if (fast) {
      if (t2 == 0 || (FC_ABL & 4)) {  // chain root: the inclusive prefix right away (diagnostics: every super-tile)
        excl.has_nz = 1;
        excl.first = excl.last = -1;
        if (lane == 0) {
          const Seg incl = seg_combine(excl, agg);
          st_agent2(st, kFlagPre | ((uint64_t)(incl.last + 1) << 36) | (incl.body & kMask36), kFlagPre | incl.tail);
        }
      } else {
        if (lane == 0) {
          const uint64_t fr = slast >= 0 ? (uint64_t)sfirst : kNoPos;
          const uint64_t lr = slast >= 0 ? (uint64_t)slast : kNoPos;
          st_agent2(st, agg_word(fr, lr, body), kFlagAgg | agg_tail);
        }
        STAMP(5);
        bool to = false;
        excl = lookback_vec<STE>(status_f + 2 * (int64_t)c * a.T, t2, lane, slow, to, pw1, pw2);
        if (to && lane == 0) atomicOr(enc_args_fresh().spin_err, 1u);
        STAMP(6);
      }
    }
    if (slow) {
      // a code past the fast path's limits, a body beyond the window, or a slow
      // predecessor: the client is re-encoded by k_encode_exact
      if (lane == 0) {
        st_agent(st + 1, kFlagSlow);
        st_agent(st, kFlagSlow);
        const EncodeArgs& ka = enc_args_fresh();
        if (atomicOr(&ka.slow_flag[c], 1) == 0) ka.slow_list[atomicAdd(ka.slow_count, 1u)] = c;
      }
      for (int i = lane; i < (int)kWin2Words; i += kEncThreads) win[i] = 0;
    } else {
      const bool last_st = t2 == (FC_FRESH_ARGS >= 2 ? enc_args_fresh().T2 : a.T2) - 1;
      const Seg incl = seg_combine(excl, agg);
      const uint32_t r0 = (uint32_t)(excl.body & 31);
      const uint32_t dfirst = agg.has_nz ? (uint32_t)(agg.first - excl.last) : 0u;
      const uint32_t R0 = agg.has_nz ? glen(dfirst) : 0u;
      const uint32_t bstart = r0 + R0;  // stream-window bit where the body starts
      const uint32_t tb = excl.tail & (r0 ? ((1u << r0) - 1u) : 0u);
      uint32_t trail_len = 0;
      uint64_t trail = 0;
      if (last_st) {
        const int64_t zc = P - 1 - (int64_t)incl.last;  // trailing zeros
        if (zc > 0) {
          trail = (uint64_t)(zc + 1);
          trail_len = 2u * (63u - (uint32_t)__clzll(trail)) + 1u;
        }
      }
      {  // decoder index entries of the super-tile's tiles (+ the row's end entry), lane h: tile t0 + h
        // tile h: after the earlier tiles' codes (and the run code before them); tile 0
        // (lastv -1): the exclusive prefix itself
        const uint64_t off = excl.body + (lastv >= 0 ? (uint64_t)R0 + bodyv : 0u);
        const int32_t lb = lastv >= 0 ? (int32_t)(sbase + lastv) : excl.last;
        uint64_t ie = (off & kMask36) | ((uint64_t)(lb + 1) << 36);
        ie = lane == nt ? (incl.body & kMask36) | ((uint64_t)(incl.last + 1) << 36) : ie;  // (last_st only)
        if (lane < nt + (last_st ? 1 : 0)) (FC_FRESH_ARGS >= 1 ? enc_args_fresh().idx : a.idx)[(int64_t)c * (a.T + 1) + t0 + lane] = ie;
      }
      if (lane == 0) {
        if (t2 > 0)
          st_agent2(st, kFlagPre | ((uint64_t)(incl.last + 1) << 36) | (incl.body & kMask36), kFlagPre | incl.tail);
        if (last_st) enc_args_fresh().total_bits[c] = (int64_t)incl.body + trail_len;
        // leading pieces just before the body, trailing code after it
        emit64<kWin2Words>(win, tb, r0, kPre - bstart);
        emit64<kWin2Words>(win, dfirst, R0, kPre - R0);
        if (trail_len) emit64<kWin2Words>(win, trail, trail_len, kPre + body);
      }
      const uint32_t nwin_bits = bstart + body + trail_len;
      const uint32_t nwords_owned = last_st ? (nwin_bits + 31) / 32 : nwin_bits / 32;
      const ClientParam cp = ld_param(cparams + c);
      const int64_t cap = cp.cap;
      uint32_t* out32 = cp.out;
      const uint64_t w0 = excl.body >> 5;
      if (lane == 0 && (int64_t)(w0 + nwords_owned) * 4 > cap) atomicOr((uint32_t*)&enc_args_fresh().overflow[c], 1u);
      const uint32_t s0 = kPre - bstart;  // window bit of stream-window bit 0
      const uint32_t lead = kStoreAlign ? (uint32_t)(((uintptr_t)(out32 + w0) >> 2) & 31u) : 0u;  // lanes before the line
      // the words inside the stream's capacity (a client that overflows is re-encoded by
      // the caller), counted once; word kk = window bits [s0 + 32 kk, +32): a funnel of
      // window words (s0 >> 5) + kk and + 1 by the ticket-uniform s0 & 31
      const uint32_t nst = (uint32_t)max<int64_t>(0, min<int64_t>(nwords_owned, cap / 4 - (int64_t)w0));
      const uint32_t so = s0 & 31u;
      const uint32_t* const wsrc = win + (s0 >> 5);
      uint32_t* const dst = out32 + w0;
      for (uint32_t k = lane; k < nst + lead; k += kEncThreads) {
        if (k < lead) continue;
        const uint32_t kk = k - lead;
        const uint32_t a0 = wsrc[kk], a1 = wsrc[kk + 1];
        const uint32_t wv32 = so ? __builtin_amdgcn_alignbit(a0, a1, 32u - so) : a0;
        if (FC_ABL & 2) asm volatile("" :: "v"(wv32));  // diagnostics: no stream stores
        else code_store(dst + kk, bswap32(wv32));
      }
      // the dirtied window words back to zero, 16 bytes per lane and instruction
      const uint32_t nt4 = (min(kWin2Words, (kPre + body + trail_len + 31) / 32 + 1) + 3u) & ~3u;
      for (uint32_t i = 4 * lane; i < nt4; i += 4 * kEncThreads) *(uint4*)(win + i) = make_uint4(0u, 0u, 0u, 0u);
    }
    ticket = ticket1;
    if (ticket1 < total) ticket1 = shard + a.nshards * uniform(ntk);
  }
#ifdef FC_STAMPS
  if (lane == 0)
    for (int i = 0; i < 8; ++i) atomicAdd(&g_stamps[i], (unsigned long long)st_acc[i]);
#endif
}

// Reset the look-back status (and overflow flag) of the clients k_encode
// handed over, so k_encode_exact can chain them afresh.  A launch whose look-back
// hit the spin limit (spin_err) marks those clients FC_OVERFLOW_STALL: their codes
// are re-encoded exactly and valid, and the host reports the stall.
__global__ void k_zero_slow(EncodeArgs a) {
  const uint32_t n = *a.slow_count;
  const int32_t mark = *a.spin_err ? FC_OVERFLOW_STALL : 0;
  const int64_t per = 2 * (int64_t)a.T;
  const int64_t total = (int64_t)n * per;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t l = i / per;
    const int32_t c = a.slow_list[l];
    a.status[(int64_t)c * per + (i - l * per)] = 0;
    if (i - l * per == 0) a.overflow[c] = mark;
  }
}

// Exact re-encode of the handed-over clients: every tile requantised with TF
// cast semantics, codes of any length, emitted stream-relative in window
// passes; same decoupled look-back (tile-major tickets over those clients).
template <int MODE, bool INT_IN, bool RCP>
__global__ __launch_bounds__(kEncThreads) void k_encode_exact(EncodeArgs a) {
  __shared__ uint32_t win[kWinWords + 3];
  __shared__ uint32_t tailw;
  const int lane = threadIdx.x;
  const uint32_t n = *a.slow_count;
  if (n == 0) return;
  const uint32_t total_tiles = n * (uint32_t)a.T;
  const ConstParamPtr cparams = (ConstParamPtr)a.cparams;
  const bool pre = !INT_IN && a.prescale != nullptr;
  for (int i = lane; i < kWinWords + 3; i += kEncThreads) win[i] = 0;
  for (;;) {
    uint32_t tk = 0;
    if (lane == 0) tk = atomicAdd(a.counter2, 1u);
    const uint32_t ticket = uniform(tk);
    if (ticket >= total_tiles) break;
    const int32_t t = (int32_t)(ticket / n);
    const int32_t c = a.slow_list[ticket - (uint32_t)t * n];
    const int64_t P = a.P;
    const int64_t tile_base = (int64_t)t * kTE;
    const bool last_tile = (t == a.T - 1);
    const ClientParam cp = ld_param(cparams + c);
    const ClientQ cq = client_q_of(cp, pre);
    SlowScan sc;
    slow_scan<MODE, INT_IN, RCP>(a, cq, c, tile_base, win, &tailw, sc);
    const int32_t tile_last = sc.carry;
    const int32_t tile_first = wave_min_i(sc.wfirst);
    const uint32_t body = sc.body;
    if (a.idxq && lane == 0) {  // quarter j = chunk j: lane 0 holds its offset and predecessor
      uint64_t* q = a.idxq + 3 * ((int64_t)c * a.T + t);
      const int32_t f = tile_last >= 0 ? tile_first : -1;
      q[0] = quarter_rel(sc.chunk_off[1], sc.chunk_prev[1], f);
      q[1] = quarter_rel(sc.chunk_off[2], sc.chunk_prev[2], f);
      q[2] = quarter_rel(sc.chunk_off[3], sc.chunk_prev[3], f);
    }
    {
      const float d = wave_sum_f(sc.dist);
      const int32_t nz = wave_sum_i(sc.nnz);
      if (lane == 0) {
        if (a.dist_part) a.dist_part[(int64_t)c * a.T + t] = d;
        if (a.nnz_part) a.nnz_part[(int64_t)c * a.T + t] = nz;
      }
    }
    uint64_t* st = a.status + 2 * ((int64_t)c * a.T + t);
    Seg agg;
    agg.has_nz = tile_last >= 0;
    agg.first = agg.has_nz ? (int32_t)(tile_base + tile_first) : 0;
    agg.last = agg.has_nz ? (int32_t)(tile_base + tile_last) : 0;
    agg.body = body;
    agg.tail = sc.tail;
    Seg excl = seg_identity();
    if (t == 0) {
      excl.has_nz = 1;
      excl.first = -1;
      excl.last = -1;
    } else {
      if (lane == 0) {
        const uint64_t fr = agg.has_nz ? (uint64_t)tile_first : kNoPos;
        const uint64_t lr = agg.has_nz ? (uint64_t)tile_last : kNoPos;
        st_agent2(st, agg_word(fr, lr, (uint32_t)body), kFlagAgg | agg.tail);
      }
      bool slow = false;
      // (one global ticket counter: progress is unconditional here, so the test knob
      // FEDCODEC_SPIN_LIMIT does not apply; the limit stays a safety net)
      bool to = false;
      excl = lookback(a.status + 2 * (int64_t)c * a.T, t, lane, slow, to, 1u << 24);
      if (to && lane == 0) atomicOr(a.spin_err, 1u);
      // (only a timed-out look-back: every status here is the exact kernel's own) the
      // client's code is unusable; its overflow flag makes the checked caller re-encode it
      if (slow && lane == 0)
        atomicOr((uint32_t*)&enc_args_fresh().overflow[c], (uint32_t)(FC_OVERFLOW_CAPACITY | FC_OVERFLOW_STALL));
    }
    const Seg incl = seg_combine(excl, agg);
    SlowEmit e;
    e.r0 = (uint32_t)(excl.body & 31);
    e.dfirst = agg.has_nz ? (uint32_t)(agg.first - excl.last) : 0u;
    e.R0 = agg.has_nz ? glen(e.dfirst) : 0u;
    e.bstart = e.r0 + e.R0;
    e.tb = excl.tail & (e.r0 ? ((1u << e.r0) - 1u) : 0u);
    e.body = body;
    e.trail_len = 0;
    e.trail = 0;
    if (last_tile) {
      const int64_t zc = P - 1 - (int64_t)incl.last;
      if (zc > 0) {
        e.trail = (uint64_t)(zc + 1);
        e.trail_len = 2u * (63u - (uint32_t)__clzll(e.trail)) + 1u;
      }
    }
    if (lane == 0) {
      st_agent2(st, kFlagPre | ((uint64_t)(incl.last + 1) << 36) | (incl.body & kMask36), kFlagPre | incl.tail);
      const int64_t ib = (int64_t)c * (a.T + 1);
      a.idx[ib + t] = (excl.body & kMask36) | ((uint64_t)(excl.last + 1) << 36);
      if (last_tile) {
        a.idx[ib + a.T] = (incl.body & kMask36) | ((uint64_t)(incl.last + 1) << 36);
        a.total_bits[c] = (int64_t)incl.body + e.trail_len;
      }
    }
    e.nwin_bits = e.bstart + body + e.trail_len;
    e.nwords_owned = last_tile ? (e.nwin_bits + 31) / 32 : e.nwin_bits / 32;
    e.tile_last = tile_last;
    e.w0 = excl.body >> 5;
    e.out32 = cp.out;
    e.cap = cp.cap;
    if (lane == 0 && (int64_t)(e.w0 + e.nwords_owned) * 4 > e.cap) atomicOr((uint32_t*)&a.overflow[c], 1u);
    slow_emit<MODE, INT_IN, RCP>(a, cq, c, tile_base, win, sc, e);
  }
}

// ---------------------------------------------------------------------------
// Decoder: one workgroup per (group of) 1024-element tile(s), one lane per client.
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
  int32_t* plane;             // PLANE: q of each client, row c at plane + c * plane_stride (elements)
  int64_t plane_stride;
  int32_t plane8;             // the rows are int8 (|q| <= 127 declared)
  int32_t t_begin, t_end;     // tiles decoded: [t_begin, t_end)
  const uint64_t* idxq;       // nullable [nclients * T][3]: quarter-tile entries (lane segments of 256)
  // VIRT: an unstitched segmented batch -- client c's tiles [k Tv, (k + 1) Tv) are virtual client
  // c K + k's tiles (k < K), the rest virtual client C K + c's; stream_off / stream_cap are indexed
  // by virtual client, idx is unused
  const uint64_t* vidx_main;  // [C K][Tv + 1]
  const uint64_t* vidx_rem;   // [C][Tr + 1]
  int32_t vK, vTv, vTr;
};

// General decode of one code at absolute bit position pos straight from
// memory (any length; the rare path, kept out of line).  slow_code returns the
// bits consumed, 0 on a malformed code.
__device__ __forceinline__ uint32_t peek32(const uint32_t* w, uint64_t nw, uint64_t pos) {
  const uint64_t i = pos >> 5;
  const uint32_t o = (uint32_t)(pos & 31);
  const uint32_t hi = i < nw ? bswap32(w[i]) : 0u;
  const uint32_t lo = i + 1 < nw ? bswap32(w[i + 1]) : 0u;
  return (uint32_t)((((uint64_t)hi << 32) | lo) >> (32 - o));
}
// Elias-gamma value at bit q (advances q); 0 if malformed (> 31 leading zeros).
__device__ __forceinline__ uint32_t gamma_at(const uint32_t* w, uint64_t nw, uint64_t& q) {
  uint32_t zeros = 0;
  for (;;) {
    const uint32_t t = peek32(w, nw, q);
    if (t) {
      const uint32_t z = (uint32_t)__clz(t);
      zeros += z;
      q += z;
      break;
    }
    zeros += 32;
    q += 32;
    if (zeros > 31 || (q >> 5) >= nw) return 0;
  }
  if (zeros > 31) return 0;
  const uint32_t v = peek32(w, nw, q) >> (31 - zeros);  // zeros + 1 bits
  q += zeros + 1;
  return v;
}
struct CodeVal {
  uint32_t L, d;
  int32_t v;
};
__device__ __noinline__ CodeVal slow_code(const uint8_t* base, int64_t cap, uint64_t pos) {
  const uint32_t* w = (const uint32_t*)base;
  const uint64_t nw = (uint64_t)(cap >> 2);
  uint64_t q = pos;
  CodeVal r{0, 0, 0};
  const uint32_t d = gamma_at(w, nw, q);
  const uint32_t sg = peek32(w, nw, q) >> 31;
  q += 1;
  const uint32_t m = gamma_at(w, nw, q);
  if (d == 0 || m == 0) return r;
  r.L = (uint32_t)(q - pos);
  r.d = d;
  r.v = sg ? (int32_t)m : -(int32_t)m;
  return r;
}

// Bit reader of one segment: a 64-bit window (MSB-aligned, > 32 valid bits), a
// 128-bit reservoir behind it, the rest of the current chunk (kDecChunk 16-byte
// blocks, read by one lane at once) and the next chunk, requested at a batch
// point.  Whole chunks: a lane's 16-byte reads of one line, spread over many
// iterations, let the XCD's L2 (fewer lines than concurrent lane streams)
// evict the line between reads -- measured 2.7x the code bytes fetched with
// 16-byte reads.  Loads are issued only at batch points the wave reaches
// together every kDecBatch iterations, so the wave's in-order memory counter
// does not make a lane wait for loads other lanes issued an iteration ago.
#ifndef FC_DEC_ABL
#define FC_DEC_ABL 0  // decoder ablation bits (diagnostics only): 1 sums one bank per lane, 2 no sums, 8 eight clients' streams for all lanes
#endif
#ifndef FC_DEC_REPL
#define FC_DEC_REPL 1  // accumulator copies per workgroup (1, 2 or 4; A/B knob)
#endif
#ifndef FC_DEC_QTR_REPL
#define FC_DEC_QTR_REPL 4  // the same for quarter-tile segments (dense streams: lanes in step on one address;
                           // config 2 decode 0.32 -> 0.28 ms wall at 2 copies, 4 even; after the one-refill
                           // LONG loop 1 / 2 / 4 copies: 0.244 / 0.220 / 0.212 ms, profiles/r04/diag_dec_qtr_knobs.txt)
#endif
#ifndef FC_DEC_BATCH
#define FC_DEC_BATCH 4
#endif
#ifndef FC_DEC_CHUNK
#define FC_DEC_CHUNK 1
#endif
constexpr int kDecBatch = FC_DEC_BATCH;  // decode iterations between batch points (power of 2)
constexpr int kDecChunk = FC_DEC_CHUNK;  // 16-byte blocks per chunk (one 64-B line half at 4)
#ifndef FC_DEC_LONG
#define FC_DEC_LONG 4
#endif
#ifndef FC_DEC_UNROLL
#define FC_DEC_UNROLL 1  // decode_segment's loop unrolled by the batch interval: headline decode -1 %, config 2 -4 % (profiles/r05/diag_dec_unroll_ab.txt)
#endif
#ifndef FC_DEC_LONG_LANES
#define FC_DEC_LONG_LANES 16  // waiting lanes that trigger an arithmetic slot before its turn
#endif
constexpr int kDecLong = FC_DEC_LONG;  // iterations between arithmetic-decode slots (power of 2)
#ifndef FC_DEC_LONG_BITS
#define FC_DEC_LONG_BITS 9
#endif
#ifndef FC_DEC_STEP3_BITS
#define FC_DEC_STEP3_BITS 52  // 3.25 bits per element: config 3 decode -4 %, headline unchanged
#endif
// a third table step per iteration for waves whose segments all average fewer
// than this many bits per 16 elements (0: never)
constexpr int kDecStep3Bits16 = FC_DEC_STEP3_BITS;
#ifndef FC_DEC_LONG_UNROLL
#define FC_DEC_LONG_UNROLL 2
#endif
constexpr int kDecLongUnroll = FC_DEC_LONG_UNROLL;  // arithmetic decodes per iteration of that loop
#ifndef FC_DEC_LONG_R1
#define FC_DEC_LONG_R1 1  // the LONG loop refills once per iteration, not after every code (A/B knob;
                          // config 2 decode 0.27 -> 0.22 ms, profiles/r04/diag_dec_long_r1.txt)
#endif
#ifndef FC_DEC_LONG_R1_CODES
#define FC_DEC_LONG_R1_CODES 3  // codes per iteration of that loop (2 / 4: config 2 decode 0.25 / 0.23 ms)
#endif
constexpr int kDecLongR1Codes = FC_DEC_LONG_R1_CODES;
constexpr int kDecLongBits = FC_DEC_LONG_BITS;  // segment bits per element for the arithmetic-only loop (0: never)
// Batch-point loads as inline asm the compiler's wait-count pass does not see:
// a lane taking its next block would otherwise wait (in-order vmcnt) for the
// loads the whole wave issued at the latest batch point.  A batch point first
// waits for the previous one's loads (issued kDecBatch iterations earlier), so a
// block requested there is known to have landed ("ready") from then on.
#ifndef FC_DEC_ASYNC
#define FC_DEC_ASYNC 1
#endif
constexpr bool kDecAsync = FC_DEC_ASYNC && kDecChunk == 1;
// ASYNC: batch-point loads the compiler does not track (k_decode, tuned); false:
// plain loads the compiler waits for where their registers are used (the index
// rebuild's reader: its control flow leaves the register allocator free to move an
// untracked load's destination before the data lands).
template <bool ASYNC>
struct SegReaderT {
  const uint4* p;
  const uint4* end;
  uint4 cur[kDecChunk > 1 ? kDecChunk - 1 : 1];  // rest of the current chunk
  uint4 nxt[kDecChunk];                          // next chunk (requested)
  int32_t cb;                                    // blocks left in cur
  uint32_t nv;                                   // nxt holds a chunk not yet taken
  uint32_t rdy;                                  // (async) that chunk has landed
  typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
  u32x4 anx;                                     // (async) the next block, one register tuple
  uint64_t win, rh, rl;
  int32_t nwin, rb;
  int32_t vb;  // segment bits from the start of the next block taken (masks the last block)
  __device__ __forceinline__ void wait_nxt() {  // every outstanding load of the wave has landed
    if (ASYNC && kDecAsync) asm volatile("s_waitcnt vmcnt(0)" : "+v"(anx) :: "memory");
  }
  __device__ __forceinline__ void load_async() {
    const uint4* q = p < end ? p : end - 1;  // clamped
    asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(anx) : "v"(q) : "memory");
    p += 1;
  }
  __device__ __forceinline__ void load_chunk(uint4* dst) {
#pragma unroll
    for (int i = 0; i < kDecChunk; ++i) dst[i] = *(p + i < end ? p + i : end - 1);  // clamped
    p += kDecChunk;
  }
  __device__ __forceinline__ void set_res(uint4 blk) {
    rh = ((uint64_t)bswap32(blk.x) << 32) | bswap32(blk.y);
    rl = ((uint64_t)bswap32(blk.z) << 32) | bswap32(blk.w);
    rb = 128;
    if (vb < 128) {  // the segment's last block (or one past it): zero the bits after its end
      if (vb <= 64) {
        rh = vb > 0 ? rh & (~0ull << (64 - vb)) : 0ull;
        rl = 0;
      } else {
        rl &= ~0ull << (128 - vb);
      }
    }
    vb -= 128;
  }
  __device__ __forceinline__ void take_block() {
    if (kDecChunk > 1 && cb > 0) {
      set_res(cur[0]);
#pragma unroll
      for (int i = 0; i + 2 < kDecChunk; ++i) cur[i] = cur[i + 1];
      --cb;
      return;
    }
    if ((ASYNC && kDecAsync)) {
      if (!nv) {  // segment start, restart after a long code, or a lane far ahead
        load_async();
        wait_nxt();
      } else if (!rdy) {
        wait_nxt();  // requested at the latest batch point
      }
      nv = 0;
      rdy = 0;
      set_res(make_uint4(anx.x, anx.y, anx.z, anx.w));
      return;
    }
    if (!nv) load_chunk(nxt);  // segment start, restart after a long code, or a lane far ahead
    nv = 0;
    set_res(nxt[0]);
#pragma unroll
    for (int i = 0; i + 1 < kDecChunk; ++i) cur[i] = nxt[i + 1];
    cb = kDecChunk - 1;
  }
  __device__ __forceinline__ void batch() {
    if ((ASYNC && kDecAsync)) {
      wait_nxt();  // the previous batch point's loads
      rdy = nv;
      if (!nv) {
        load_async();
        nv = 1;
      }
      return;
    }
    if (!nv) {
      load_chunk(nxt);
      nv = 1;
    }
  }
  __device__ __forceinline__ uint32_t pop32() {
    const uint32_t w = (uint32_t)(rh >> 32);
    rh = (rh << 32) | (rl >> 32);
    rl <<= 32;
    rb -= 32;
    if (rb == 0) take_block();
    return w;
  }
  // left: segment bits from `bit` on -- window bits past the segment end are zeroed
  __device__ __forceinline__ void init(const uint8_t* base, int64_t cap, uint64_t bit, int32_t left) {
    p = (const uint4*)base + ((bit >> 7) & ~(uint64_t)(kDecChunk - 1));  // chunk-aligned
    end = (const uint4*)base + (cap >> 4);
    vb = (int32_t)(bit - ((bit >> 7) & ~(uint64_t)(kDecChunk - 1)) * 128) + max(left, 0);
    nv = 0;
    rdy = 0;
    cb = 0;
    take_block();
    for (int i = (int)((bit >> 5) & (4 * kDecChunk - 1)); i > 0; --i) (void)pop32();
    win = (uint64_t)pop32() << 32;
    win |= pop32();
    const int skip = (int)(bit & 31);
    win <<= skip;
    nwin = 64 - skip;
    batch();
  }
};
using SegReader = SegReaderT<true>;

// Decode table: the next 12 window bits -> up to two complete codes in one
// 32-bit word, every field out with one AND or a constant shift pair:
//   [6:0] 4*d1   [13:7] 4*d2 (0: one code)   [19:14] v1   [25:20] v2 (6-bit
//   two's complement, 0: one code)   [29:26] L = bits of the decoded codes
//   (0: the first code is longer than 12 bits -- the entry is then all zero)
#ifndef FC_LUT_BITS
#define FC_LUT_BITS 12
#endif
constexpr int kLutBits = FC_LUT_BITS;
constexpr int kLutSize = 1 << kLutBits;

// count of leading zeros, usable in constant expressions (the decode tables are
// built at compile time: g_dec_tabs)
constexpr uint32_t clz_ce(uint32_t x) {
  if (x == 0) return 32;
  uint32_t n = 0;
  if (!(x & 0xFFFF0000u)) { n += 16; x <<= 16; }
  if (!(x & 0xFF000000u)) { n += 8; x <<= 8; }
  if (!(x & 0xF0000000u)) { n += 4; x <<= 4; }
  if (!(x & 0xC0000000u)) { n += 2; x <<= 2; }
  if (!(x & 0x80000000u)) { n += 1; }
  return n;
}

constexpr uint32_t lut_entry(uint32_t i) {
  uint32_t top = i << (32 - kLutBits);
  uint32_t used = 0, e = 0;
  for (int c = 0; c < 2; ++c) {
    const uint32_t z1 = clz_ce(top);
    if (z1 > 4) break;
    const uint32_t sa = 30u - 2u * z1;
    const uint32_t rest = top << (32u - sa);
    const uint32_t z2 = clz_ce(rest);
    if (z2 > 4) break;
    const uint32_t L = 2u * (z1 + z2) + 3u;
    if (used + L > (uint32_t)kLutBits) break;
    const uint32_t d = top >> (sa + 1u);
    const uint32_t m = rest >> (31u - 2u * z2);
    const int32_t v = ((top >> sa) & 1u) ? (int32_t)m : -(int32_t)m;
    used += L;
    e |= ((4u * d) << (7 * c)) | (((uint32_t)v & 63u) << (14 + 6 * c));
    top <<= L;
  }
  return used ? (e | (used << 26)) : 0u;
}

// Single-code table (dense streams, the LONG loop): the next 12 window bits ->
// the structure of the one code they begin, whenever its run code, sign and
// magnitude prefix (up to the magnitude's leading 1) fit in them -- the
// magnitude's remaining bits are then at a known place in the window:
//   [4:0] L (0: not resolvable here -- the arithmetic decode takes the code)
//   [9:5] n = magnitude bits   [10] negative   [15:11] d (1..31)
// so m = bits [32 - L, 32 - L + n) of the window's top word (one v_bfe_u32).
// Codes of |v| < 1024 after a run d < 32 -- every code of an 8-bit-step stream.
#ifndef FC_DEC_GEN
#define FC_DEC_GEN 1  // the LONG loop (dense streams) reads the single-code table first (A/B knob)
#endif
constexpr uint32_t gen_entry(uint32_t i) {
  const uint32_t top = i << (32 - kLutBits);
  const uint32_t z1 = clz_ce(top);
  if (z1 > 4) return 0u;
  const uint32_t sa = 30u - 2u * z1;  // sign-bit position
  const uint32_t rest = top << (32u - sa);
  const uint32_t z2 = clz_ce(rest);
  if (2u * z1 + 3u + z2 > (uint32_t)kLutBits) return 0u;  // the magnitude's leading 1 is past the index bits
  const uint32_t L = 2u * (z1 + z2) + 3u;
  const uint32_t d = top >> (sa + 1u);
  const uint32_t neg = ((top >> sa) & 1u) ? 0u : 1u;
  return L | ((z2 + 1u) << 5) | (neg << 10) | (d << 11);
}

// The decode tables, computed at compile time; each k_decode workgroup copies them
// into LDS with 16-byte loads instead of building them (measured even: config 2's
// decode 0.239 -> 0.238 ms, the builds overlapped other workgroups' decoding).
// The index parse (fc_build_index) needs only a step's bits and its runs: ilut keeps
// L in [29:26] and 4 (d1 + d2) in [7:0], so the runs come out with one AND.
#ifndef FC_IDX_ILUT
#define FC_IDX_ILUT 1  // the index parse reads ilut (0: the decoder's table, two fields added per step)
#endif
// FC_DEC_TAB2: the decoder's table steps read byte fields (4 d1, 4 d2, v1, v2 as int8:
// byte selects and one arithmetic shift instead of bit-field extracts) from dlut and
// the bits consumed from a separate byte table llut (A/B knob).
#ifndef FC_DEC_TAB2
#define FC_DEC_TAB2 0
#endif
struct DecTabs {
  uint32_t lut[kLutSize];
  uint16_t glut[kLutSize];
  uint32_t ilut[kLutSize];
  uint32_t dlut[kLutSize];
  uint8_t llut[kLutSize];
};
constexpr DecTabs make_dec_tabs() {
  DecTabs t{};
  for (uint32_t i = 0; i < (uint32_t)kLutSize; ++i) {
    const uint32_t e = lut_entry(i);
    t.lut[i] = e;
    t.glut[i] = (uint16_t)gen_entry(i);
    t.ilut[i] = (e & (15u << 26)) | ((e & 0x7Fu) + ((e >> 7) & 0x7Fu));
    // 6-bit two's complement values widened to int8 bytes
    const uint32_t v1 = (e >> 14) & 63u, v2 = (e >> 20) & 63u;
    const uint32_t b1 = v1 >= 32u ? v1 | 0xC0u : v1, b2 = v2 >= 32u ? v2 | 0xC0u : v2;
    t.dlut[i] = (e & 0x7Fu) | (((e >> 7) & 0x7Fu) << 8) | (b1 << 16) | (b2 << 24);
    t.llut[i] = (uint8_t)(e >> 26);
  }
  return t;
}
__device__ const DecTabs g_dec_tabs = make_dec_tabs();
static_assert(sizeof(DecTabs) % 16 == 0 && offsetof(DecTabs, glut) % 16 == 0 && offsetof(DecTabs, ilut) % 16 == 0 &&
                  offsetof(DecTabs, dlut) % 16 == 0 && offsetof(DecTabs, llut) % 16 == 0,
              "16-byte table copies");

constexpr int kDecThreads = 256;
// Tiles per lane segment (accumulator path), chosen per launch: two with 256
// lanes per tile pair once there are >= kDecSpan2Clients clients (half the
// segment starts -- index loads and the first block's round trip -- per code:
// 1024 x 25 M decode 12.5 -> 11.3 ms); one below (config 2's 128 clients need
// every segment in flight: 0.45 vs 0.87 ms).
constexpr int kDecSpan2Clients = 256;

typedef __attribute__((address_space(3))) int32_t* lds_iptr;

// Accumulator add at LDS byte address a (int32 client sum), or (PLANE, the
// QSGD server sum) a store of the value into the client's q row at element a / 4
// of the tile -- only nonzero values (a no-op zero add may repeat the previous
// code's slot or point past the tile) inside the tile's valid bytes `hib`.
// PLANE 1: int32 rows; 2: int8 rows (|q| <= 127 declared by the caller; a larger
// value sets err).
template <int PLANE>
__device__ __forceinline__ void acc_add_at(uint32_t a, int32_t v, int32_t* ptile, uint32_t hib, int32_t* err = nullptr) {
  if (PLANE == 2) {
    if (v != 0 && a < hib) {
      if (v > 127 || v < -127) atomicOr(err, 1);
      ((int8_t*)ptile)[a >> 2] = (int8_t)v;
    }
  } else if (PLANE) {
    if (v != 0 && a < hib) ptile[a >> 2] = v;
  } else {
#if FC_DEC_ABL & 1
    a = (a & ~127u) | ((threadIdx.x & 31u) << 2);  // diagnostics: every lane its own bank
#endif
#if FC_DEC_ABL & 2
    asm volatile("" :: "v"(a), "v"(v));  // diagnostics: no accumulation
#else
    atomicAdd((int32_t*)(lds_iptr)(uintptr_t)a, v);
#endif
  }
}

// One segment = one client's code for one 1024-element tile: bits [b0, b1),
// previous nonzero at tile-relative position rel.  The accumulator position is
// kept as an LDS byte address.  An iteration makes two table steps, each taking
// the entry's codes only when they end inside the segment -- a code longer than
// 12 bits has an all-zero entry, so such a step adds 0 and consumes nothing --
// and a lane that took nothing decodes one code arithmetically from the top 32
// window bits in the next arithmetic slot (longer than 32 bits: slow_code, then
// the reader restarts).  The window holds >= 33 valid bits when an iteration
// starts.
template <int PLANE, bool LONG = false, bool STEP3 = false, bool GEN = false>
__device__ __forceinline__ void decode_segment(const uint8_t* base, int64_t cap, uint64_t b0,
                                               uint64_t b1, int32_t rel, uint32_t my_addr,
                                               const uint32_t* lut, int32_t* err, int32_t* ptile,
                                               uint32_t hib, uint32_t span = kTE,
                                               const uint16_t* glut = nullptr, const uint8_t* llut = nullptr) {
  SegReader r;
  const int32_t total = (int32_t)(b1 - b0);
  r.init(base, cap, b0, total);
  // one running count of consumed bits: the segment end and the window refill
  // compare against it (fill = cons + valid window bits)
  int32_t cons = 0;
  int32_t fill = r.nwin;
  uint32_t relb = my_addr + 4u * (uint32_t)rel;  // byte address of the previous nonzero's slot
  const uint32_t lo_addr = my_addr, hi_addr = my_addr + 4u * span;
  uint32_t bad = 0;
  uint32_t it = 0;
  // one iteration; K: its place in an unrolled group of kDecBatch (FC_DEC_UNROLL: the batch
  // points and arithmetic slots at fixed places, no iteration count through the
  // divergent loop), else the count `it`
  auto iter = [&](auto kpos) -> bool {
    constexpr int K = decltype(kpos)::value;
    constexpr bool UNR = K >= 0;
#ifdef FC_STAMPS
    {  // diagnostics (tools/diag/dec_diverge.py): wave iterations, one count per iteration the wave runs
      const uint64_t ex = __ballot(1);
      if ((uint32_t)__lane_id() == (uint32_t)__builtin_ctzll(ex)) atomicAdd(&g_stamps[15], 1ull);
    }
#endif
    // every active lane is on the same iteration: a wave-uniform count (the scalar unit
    // keeps it, not three VALU per iteration where the loop's exit is divergent)
    if (!UNR) it = __builtin_amdgcn_readfirstlane(it + 1u);
    if (UNR ? K == kDecBatch - 1 : (it & (kDecBatch - 1)) == 0) r.batch();
#if FC_DEC_ABL & 16  // diagnostics: 12 extra independent VALU per iteration (is the loop issue-bound?)
    {
      uint32_t p0 = it, p1 = it + 1, p2 = it + 2, p3 = it + 3;
      asm volatile(
          "v_add_u32 %0, %0, %4\n v_add_u32 %1, %1, %4\n v_add_u32 %2, %2, %4\n v_add_u32 %3, %3, %4\n"
          "v_add_u32 %0, %0, %4\n v_add_u32 %1, %1, %4\n v_add_u32 %2, %2, %4\n v_add_u32 %3, %3, %4\n"
          "v_add_u32 %0, %0, %4\n v_add_u32 %1, %1, %4\n v_add_u32 %2, %2, %4\n v_add_u32 %3, %3, %4\n"
          : "+v"(p0), "+v"(p1), "+v"(p2), "+v"(p3) : "v"(relb));
    }
#endif
#if FC_DEC_ABL & 32  // diagnostics: 12 extra SALU per iteration
    {
      uint32_t s0 = __builtin_amdgcn_readfirstlane(it), s1 = s0 + 1;
      asm volatile(
          "s_add_u32 %0, %0, 3\n s_add_u32 %1, %1, 5\n s_add_u32 %0, %0, 3\n s_add_u32 %1, %1, 5\n"
          "s_add_u32 %0, %0, 3\n s_add_u32 %1, %1, 5\n s_add_u32 %0, %0, 3\n s_add_u32 %1, %1, 5\n"
          "s_add_u32 %0, %0, 3\n s_add_u32 %1, %1, 5\n s_add_u32 %0, %0, 3\n s_add_u32 %1, %1, 5\n"
          : "+s"(s0), "+s"(s1) :: "scc");
    }
#endif
    uint32_t moved = 0;
#pragma unroll
    for (int st = 0; st < (LONG ? 0 : 2); ++st) {  // table steps (the window holds >= 33 bits when they start)
      // the window is zero past the segment end (the client's next tile): no table
      // entry takes a code there
      const uint32_t ix = (uint32_t)(r.win >> (64 - kLutBits));
      const uint32_t e = lut[ix];
      uint32_t L;
      if (FC_DEC_TAB2) {
        L = llut[ix];
        relb += e & 0xFFu;
        acc_add_at<PLANE>(relb, ((int32_t)(e << 8)) >> 24, ptile, hib, err);
        relb += (e >> 8) & 0xFFu;
        acc_add_at<PLANE>(relb, ((int32_t)e) >> 24, ptile, hib, err);
      } else {
        relb += e & 0x7Fu;
        acc_add_at<PLANE>(relb, ((int32_t)(e << 12)) >> 26, ptile, hib, err);
        relb += (e >> 7) & 0x7Fu;
        acc_add_at<PLANE>(relb, ((int32_t)(e << 6)) >> 26, ptile, hib, err);
        L = e >> 26;
      }
      r.win <<= L;
      cons += (int32_t)L;
      if (st == 0) moved = L;  // a zero first step leaves the window as it was: so does the second
    }
    if (!LONG && STEP3) {
      // a third table step where the window still holds 13 or more valid bits (so
      // the refill below restores >= 33); otherwise an empty entry
      const bool ok3 = fill - cons >= kLutBits + 1;
      const uint32_t ix = (uint32_t)(r.win >> (64 - kLutBits));
      uint32_t e = lut[ix];
      e = ok3 ? e : 0u;
      uint32_t L;
      if (FC_DEC_TAB2) {
        L = ok3 ? (uint32_t)llut[ix] : 0u;
        relb += e & 0xFFu;
        acc_add_at<PLANE>(relb, ((int32_t)(e << 8)) >> 24, ptile, hib, err);
        relb += (e >> 8) & 0xFFu;
        acc_add_at<PLANE>(relb, ((int32_t)e) >> 24, ptile, hib, err);
      } else {
        relb += e & 0x7Fu;
        acc_add_at<PLANE>(relb, ((int32_t)(e << 12)) >> 26, ptile, hib, err);
        relb += (e >> 7) & 0x7Fu;
        acc_add_at<PLANE>(relb, ((int32_t)(e << 6)) >> 26, ptile, hib, err);
        L = e >> 26;
      }
      r.win <<= L;
      cons += (int32_t)L;
    }
    // A lane whose table steps took nothing (a code longer than 12 bits) decodes one
    // code arithmetically -- only on every kDecLong-th iteration, so the wave runs
    // that block rarely instead of whenever any of its 64 lanes needs it; the lane
    // idles meanwhile.  (Or at once when a quarter of the wave is waiting: streams
    // of long codes, e.g. 8-bit steps, would otherwise decode one code every
    // kDecLong iterations.)
    // LONG (a wave whose segments all average kDecLongBits or more per element, e.g.
    // 8-bit steps): no table steps, one code decoded arithmetically every iteration
    const bool idle = LONG || moved == 0;
    bool stop = false;
    // R1: one refill per iteration, after its last code. The first code starts with
    // >= 33 window bits; a later one is taken from the table only when it ends before
    // the window's last valid bit (the bits past it are zero, so a code that needs
    // them parses longer than the bits left), arithmetically only with >= 33 bits, and
    // otherwise waits for the next iteration. Every code leaves >= 1 valid bit, so the
    // refill restores >= 33.
    constexpr bool R1 = LONG && GEN && FC_DEC_LONG_R1;
    constexpr int NU = LONG ? (R1 ? kDecLongR1Codes : kDecLongUnroll) : 1;
#pragma unroll
    for (int u = 0; u < NU; ++u) {  // LONG: codes per iteration
    if (u > 0 && cons >= total) break;
    bool tdone = false;
    if (GEN && LONG) {
      // right after a refill (>= 33 window bits, every resolvable code <= 21): one
      // code from the single-code table; the run is at most 31 elements, so the
      // accumulator position is bounded by the segment-end check like the table steps'
      const uint32_t top = (uint32_t)(r.win >> 32);
      const uint32_t e = glut[top >> (32 - kLutBits)];
      const uint32_t L = e & 31u;
      if (L != 0u && (!R1 || u == 0 || (int32_t)L < fill - cons)) {
        const uint32_t m = __builtin_amdgcn_ubfe(top, 32u - L, e >> 5);
        const int32_t s = __builtin_amdgcn_sbfe((int32_t)e, 10, 1);  // -1: negative
        relb += (e >> 11) << 2;
        acc_add_at<PLANE>(relb, (int32_t)(m ^ (uint32_t)s) - s, ptile, hib, err);
        r.win <<= L;
        cons += (int32_t)L;
        tdone = true;
      }
    }
    if (!tdone && idle && (!R1 || u == 0 || fill - cons > 32) &&
        (LONG || (UNR ? K == kDecLong - 1 : (it & (kDecLong - 1)) == 0) ||
         (FC_DEC_LONG_LANES <= 64 && __popcll(__ballot(idle)) >= FC_DEC_LONG_LANES))) {
      // right after a refill (>= 33 window bits): one code decoded arithmetically
      const uint32_t top = (uint32_t)(r.win >> 32);
      const uint32_t z1 = (uint32_t)__clz(top);
      const uint32_t sa = 30u - 2u * z1;        // sign-bit position
      const uint32_t rest = top << (32u - sa);  // bits after the sign bit
      const uint32_t z2 = (uint32_t)__clz(rest);
      uint32_t L = 2u * (z1 + z2) + 3u;
      uint32_t d = top >> (sa + 1u);
      const uint32_t m = rest >> (31u - 2u * z2);
      int32_t v = ((top >> sa) & 1u) ? (int32_t)m : -(int32_t)m;
      if (L <= 32u) {
        r.win <<= L;
      } else {  // a code longer than 32 bits (or a malformed one)
        // land any batch-point load first: the registers it writes are free to the
        // compiler from here on (r.init below issues a new load into them), and
        // slow_code is a call whose temporaries may be those registers
        r.wait_nxt();
        const uint64_t pos = b0 + (uint64_t)cons;
        const CodeVal cv = slow_code(base, cap, pos);
        if (cv.L == 0) {
          bad = 1;
          stop = true;
          break;
        }
        L = cv.L;
        d = cv.d;
        v = cv.v;
        r.init(base, cap, pos + L, total - cons - (int32_t)L);
        fill = cons + (int32_t)L + r.nwin;
      }
      // the run may come from far before the tile: bound it before scaling to bytes
      const int32_t rel_now = ((int32_t)(relb - my_addr)) >> 2;
      uint32_t rel_new = (uint32_t)(rel_now + (int32_t)d);
      // a segment's first nonzero after a run of >= 2^27 zeros: the index's previous
      // nonzero is known modulo 2^28 only (FC_MAX_ELEMS), and so is the sum.  Only the
      // segment's first code (nothing consumed yet: its run starts at the index's
      // nonzero) is reduced; a later code's run starts inside the tile, so one that
      // leaves it is malformed (it used to be wrapped back in, unflagged)
      if (rel_new >= span && cons == 0) rel_new &= kIdxLastMask;
      bad |= rel_new >= span ? 1u : 0u;
      relb = my_addr + 4u * min(rel_new, span - 1);
      acc_add_at<PLANE>(relb, v, ptile, hib, err);
      cons += (int32_t)L;
    }
    if ((!R1 || u == NU - 1) && fill - cons <= 32) {  // (the blocks are zero past the segment end)
      const uint32_t w = r.pop32();
      r.win |= (uint64_t)w << (32 - (fill - cons));
      fill += 32;
    }
    }
    return stop;
  };
  if (FC_DEC_UNROLL) {
    static_assert(!FC_DEC_UNROLL || (kDecBatch == 4 && kDecLong == 4), "unrolled by four");
    while (cons < total) {
      if (iter(std::integral_constant<int, 0>{}) || !(cons < total)) break;
      if (iter(std::integral_constant<int, 1>{}) || !(cons < total)) break;
      if (iter(std::integral_constant<int, 2>{}) || !(cons < total)) break;
      if (iter(std::integral_constant<int, 3>{})) break;
    }
  } else {
    while (cons < total)
      if (iter(std::integral_constant<int, -1>{})) break;
  }
  // the reader's last batch-point load may still be in flight into its register
  // tuple: land it before the tuple dies (the registers are reused after the segment)
  r.wait_nxt();
  // every decoded value must have landed inside this tile's accumulator
  bad |= (relb < lo_addr || relb >= hi_addr) ? 1u : 0u;
  if (bad || cons != total) atomicOr(err, 1);
#ifdef FC_STAMPS
  atomicAdd(&g_stamps[14], (unsigned long long)it);  // diagnostics: lane iterations
#endif
}

// Persistent: each workgroup builds the decode table once, then walks tiles
// (tiles_per_wg at a time) with one lane per client segment, accumulating the
// clients' values in LDS and writing the tile's sum / dequantised values -- or
// (PLANE) storing each client's values into its q row (zeroed beforehand), for
// k_sum_planes to add in client order.  QTR: the lane segments are quarter tiles
// (256 elements, entries from the quarter index): four times the segments in
// flight for few clients with dense codes (config 2: 128 clients, ~10 bits per
// element -- each lane's serial chain, not memory, bounds the decode).
template <int PLANE, int SPAN_ = 1, bool QTR = false, bool VIRT = false>
#ifndef FC_DEC_WPE
#define FC_DEC_WPE 5  // waves per SIMD the register budget is held to
#endif
#ifndef FC_DEC_QTR_WPE
#define FC_DEC_QTR_WPE 5  // the same for quarter-tile segments (measured: 5 and 6 even, 8 spills: +12 %)
#endif
__global__ __launch_bounds__(kDecThreads) __attribute__((amdgpu_waves_per_eu(QTR ? FC_DEC_QTR_WPE : FC_DEC_WPE))) void k_decode(DecodeArgs a) {
  __shared__ __attribute__((aligned(16))) uint32_t lut[kLutSize];  // static: table reads fold its base into the offset
  // the single-code table for dense streams: quarter-tile segments (few clients,
  // where 8-bit steps occur); the other variants keep their LDS for occupancy
  constexpr bool GEN = FC_DEC_GEN && QTR && !PLANE;
  __shared__ __attribute__((aligned(16))) uint16_t glut[GEN ? kLutSize : 8];
  __shared__ __attribute__((aligned(16))) uint8_t llut[FC_DEC_TAB2 ? kLutSize : 16];
  extern __shared__ int32_t acc[];     // [units_per_wg][UE] sums
  // a lane's segment: SPAN consecutive units of one client (the accumulator path)
  constexpr int SPAN = PLANE ? 1 : SPAN_;
  constexpr int UE = QTR ? kTE / 4 : kTE;  // elements per unit (tile or quarter tile)
  constexpr int UPT = kTE / UE;            // units per tile
  const int tid = threadIdx.x;
  const int units_per_wg = kDecThreads / a.lanes_per_tile * SPAN;
  for (int i = tid; i < kLutSize / 4; i += kDecThreads)
    ((uint4*)lut)[i] = ((const uint4*)(FC_DEC_TAB2 ? g_dec_tabs.dlut : g_dec_tabs.lut))[i];
  if (FC_DEC_TAB2)
    for (int i = tid; i < kLutSize / 16; i += kDecThreads) ((uint4*)llut)[i] = ((const uint4*)g_dec_tabs.llut)[i];
  if (GEN)
    for (int i = tid; i < kLutSize / 8; i += kDecThreads) ((uint4*)glut)[i] = ((const uint4*)g_dec_tabs.glut)[i];
  const int sub = tid / a.lanes_per_tile;
  const int l = tid - sub * a.lanes_per_tile;
  // REPL accumulator copies (lane l picks copy l mod REPL, the copies one bank apart):
  // fewer same-bank atomics from lanes at the same tile position
  constexpr int REPL = PLANE ? 1 : QTR ? FC_DEC_QTR_REPL : FC_DEC_REPL;
  static_assert(REPL == 1 || REPL == 2 || REPL == 4, "accumulator copies: 1, 2 or 4");
  const int rstride = units_per_wg * UE + 1;  // words between copies
  const uint32_t my_addr =
      PLANE ? 0u : (uint32_t)(uintptr_t)(lds_iptr)(acc + sub * SPAN * UE + (REPL > 1 ? (l & (REPL - 1)) * rstride : 0));
  const int64_t e_end = min(a.P, (int64_t)a.t_end * kTE);  // elements this launch writes
  const int64_t u_begin = (int64_t)a.t_begin * UPT;
  const int64_t u_end = (e_end + UE - 1) / UE;  // units holding elements of the range
  const int64_t ngroups = (u_end - u_begin + units_per_wg - 1) / units_per_wg;
  if (PLANE) __syncthreads();  // the table (the accumulator path's first barrier covers it otherwise)
  for (int64_t grp = blockIdx.x; grp < ngroups; grp += gridDim.x) {
    const int64_t u0 = u_begin + grp * units_per_wg;
    if (!PLANE) {
      for (int i = tid; i < (REPL > 1 ? REPL * rstride : units_per_wg * UE); i += kDecThreads) acc[i] = 0;
      __syncthreads();
    }
    const int64_t u = u0 + sub * SPAN;
    if (u < u_end) {
      const int64_t t = u / UPT;
      const int qs = (int)(u - t * UPT);  // QTR: quarter of the tile
      const int64_t uEnd = min<int64_t>(u + SPAN, u_end);  // lane segment end unit
      // VIRT: a lane segment that straddles an encoder segment's end (a tile range
      // starting at an odd tile) is decoded as two pieces, one per encoder segment
      int64_t uA = uEnd;
      if (VIRT) {
        const int32_t tm = a.vK * a.vTv;
        const int32_t k0 = (int32_t)t < tm ? (int32_t)t / a.vTv : a.vK;
        if (k0 < a.vK) uA = min<int64_t>(uEnd, (int64_t)(k0 + 1) * a.vTv);
      }
      for (int piece = 0; piece < (VIRT ? 2 : 1); ++piece) {
      const int64_t pu = piece ? uA : u;          // the piece's first unit
      const int64_t uE = piece ? uEnd : uA;       // and end unit
      if (pu >= uE) break;
      const int64_t unit_base = pu * UE;
      const uint32_t span = (uint32_t)(uE - pu) * UE;
      const uint32_t paddr = my_addr + 4u * (uint32_t)((pu - u) * UE);  // the piece's accumulator
      int32_t vk = 0, vj = 0;  // VIRT: the encoder segment holding the piece (vK: the remainder), its tile there
      if (VIRT) {
        const int32_t tm = a.vK * a.vTv;
        vk = (int32_t)pu < tm ? (int32_t)pu / a.vTv : a.vK;
        vj = (int32_t)pu - vk * a.vTv;
      }
      for (int c = l; c < a.nclients; c += a.lanes_per_tile) {
#if FC_DEC_ABL & 8  // diagnostics: 8 clients' streams and indexes for every lane (cache-resident reads)
        const int cc = c & 7;
#else
        const int cc = c;
#endif
        const int64_t ib = (int64_t)cc * (a.T + 1) + t;
        uint64_t e0, e1;
        int64_t vc = cc;       // stream row (VIRT: the virtual client)
        int64_t rel_base = unit_base;  // the index's element coordinate of the unit (VIRT: segment-local)
        if (VIRT) {
          const uint64_t* vi;
          if (vk < a.vK) {
            vc = (int64_t)cc * a.vK + vk;
            vi = a.vidx_main + vc * (a.vTv + 1);
          } else {
            vc = (int64_t)a.nclients * a.vK + cc;
            vi = a.vidx_rem + (int64_t)cc * (a.vTr + 1);
          }
          e0 = vi[vj];
          e1 = vi[vj + (uE - pu)];
          rel_base = (int64_t)vj * kTE;
        } else if (QTR) {
          const uint64_t* q = a.idxq + 3 * ((int64_t)cc * a.T + t);
          e0 = qs == 0 ? a.idx[ib] : q[qs - 1];
          e1 = qs == 3 ? a.idx[ib + 1] : q[qs];
        } else {
          e0 = a.idx[ib];
          e1 = a.idx[ib + (uE - u)];
        }
        const int64_t soff = a.stream_off[vc], scap = a.stream_cap[vc];
        const uint64_t bstart = e0 & kMask36, bend = e1 & kMask36;
        if (bend <= bstart) continue;
        // last nonzero, unit-relative: the index holds 1 + it modulo 2^28, so this is exact
        // within 2^27 of the unit; a farther one is reached only by a run code longer than
        // 32 bits, which the slow path reduces modulo 2^28 (decode_segment)
        const int32_t rel = sext28((uint32_t)((int64_t)(e0 >> 36) - 1 - rel_base));
        int32_t* ptile = PLANE == 2 ? (int32_t*)((int8_t*)a.plane + (int64_t)c * a.plane_stride + unit_base)
                       : PLANE    ? a.plane + (int64_t)c * a.plane_stride + unit_base
                                  : nullptr;
        const uint32_t hib = PLANE ? 4u * (uint32_t)min<int64_t>(kTE, a.P - unit_base) : 0u;
        // a wave whose segments are all long-code streams skips the table steps
        if (kDecLongBits > 0 && __ballot(bend - bstart < (uint64_t)kDecLongBits * span) == 0)
          decode_segment<PLANE, true, false, GEN>(a.stream_buf + soff, scap, bstart, bend, rel, paddr, lut, a.err,
                                                  ptile, hib, span, glut, llut);
        else if (kDecStep3Bits16 > 0 && __ballot(bend - bstart >= (uint64_t)kDecStep3Bits16 * (span / 16)) == 0)
          decode_segment<PLANE, false, true>(a.stream_buf + soff, scap, bstart, bend, rel, paddr, lut, a.err, ptile,
                                             hib, span, nullptr, llut);
        else
          decode_segment<PLANE>(a.stream_buf + soff, scap, bstart, bend, rel, paddr, lut, a.err, ptile, hib, span,
                                nullptr, llut);
      }
      }  // pieces
    }
    if (PLANE) continue;
    __syncthreads();
    for (int i = tid; i < units_per_wg * UE; i += kDecThreads) {
      const int64_t e = u0 * UE + i;
      if (e >= e_end) break;
      int32_t v = acc[i];
#pragma unroll
      for (int k = 1; k < REPL; ++k) v = (int32_t)((uint32_t)v + (uint32_t)acc[i + k * rstride]);
      if (a.sum_in) v = (int32_t)((uint32_t)v + (uint32_t)a.sum_in[e]);
      if (a.sum_out) a.sum_out[e] = v;
      if (a.out) {
        float f = (float)v;
        if (a.noise_sum) f = f + a.noise_sum[e];
        a.out[e] = f * a.step;
      }
    }
    __syncthreads();
  }
}

// ---------------------------------------------------------------------------
// Decoder index from bare codes.  The reference decodes a client's message with
// tfc.run_length_gamma_decode(code, shape) -- the byte string alone
// (elias_gamma_encode.py:69-73, message at :97-109) -- so a server that receives
// stock TFC strings has no encoder index.  fc_build_index rebuilds it (and the
// quarter index) from the bytes, bit for bit what the encoder writes:
//   entry u = stream bit where the first code whose nonzero lies at or after
//   element G u starts | (1 + the last nonzero before it) << 36
// (G = 1024, or 256 with the quarter index), entry T = the bit where the trailing
// zero-run code starts (or the stream's end).
//
// A prefix code is parsed serially, so each lane parses its own chunk (a.chunk bits)
// of a client's code from a GUESSED start -- the chunk's first bit taken as a
// code start -- and records where its parse leaves the chunk (the first code
// start at or after the chunk's end) and the zero runs it summed.  Run-length
// gamma parses resynchronise fast: from a random bit they reach a true code start
// within 25 bits on average, 120 bits at the 99th percentile and 630 at most
// (measured on the oracle's codes: 3.8-bit, 10.3-bit, 2.7-bit, 1-bit and 0.2-bit
// streams), so the guessed parse almost always ends where the true one does.
//   k_idx_spec   every lane: the guessed parse of its chunk (exit bit, sum of runs)
//   k_idx_sync   lane j re-parses from lane j-1's exit and from its guessed start
//                in lockstep until both reach one code start (a few codes), and
//                corrects its run sum; no meeting inside the chunk: a full parse
//   k_idx_fix    a wave per client walks the chunks in order and redoes (serially,
//                rarely) any chunk whose true start differs from the one used
//   k_idx_scan   a wave per client: exclusive sums of the runs = the last nonzero
//                before each chunk's first code
//   k_idx_emit   every lane: the true parse of its chunk, writing the entries of
//                the units its codes enter; the chunk holding the end checks the
//                trailing run, the bit count and the byte length
//   k_idx_check  a client whose code never ended is malformed
// ---------------------------------------------------------------------------
// bits per chunk lane, chosen per launch (idx_chunk_bits): 2048, 4096 or 8192 (<= 8192:
// 13-bit checkpoint positions)
constexpr int kIdxChunkMax = 8192;
constexpr int64_t kIdxFail = -1;  // "the parse failed" (a guessed start, or past the stream's end)
// Checkpoints of the guessed parse: at the first code start at or after every
// a.ckb bits of the chunk, (bits from the chunk start [12:0], runs so far
// [63:13]).  A checkpoint at or after the point where the true parse meets the
// guessed one is a true code start, and its last nonzero follows from the chunk's
// true runs, so k_idx_emit parses from the checkpoint before each unit boundary
// instead of the whole chunk.
// per chunk: nck = min(FC_IDX_NCK_MAX, chunk / 256 - 1) checkpoints, chunk / (nck + 1) bits apart
#ifndef FC_IDX_NCK_MAX
#define FC_IDX_NCK_MAX 31  // checkpoints per chunk at most (15: the headline's rebuild +0.5 ms, profiles/r06/diag_idx_emit.txt)
#endif
inline int32_t idx_nck(int32_t chunk) { return std::min(FC_IDX_NCK_MAX, chunk / 256 - 1); }
#ifndef FC_IDX_ASYNC
#define FC_IDX_ASYNC 0
#endif
#ifndef FC_IDX_UNIFORM
#define FC_IDX_UNIFORM 1  // the guessed parse's wave-uniform fast steps (A/B knob)
#endif
constexpr uint64_t kCkNone = ~0ull;

struct IdxArgs {
  const uint8_t* stream_buf;
  const int64_t* stream_off;
  const int64_t* nbytes;  // [nclients]: each client's byte string length
  int32_t nclients;
  int64_t P;
  int32_t T;
  int64_t nchunks;  // chunk lanes per client
  int64_t* x1;      // [C][nchunks]: guessed parse's exit bit (kIdxFail: failed)
  int64_t* n1;      //               its sum of runs
  int64_t* x2;      //               true exit bit
  int64_t* n2;      //               true sum of runs, then (k_idx_scan) the last nonzero before the chunk
  int64_t* xm;      //               where the true parse meets the guessed one (kIdxFail: it does not)
  uint64_t* ck;     // [nck][C * nchunks]: the guessed parse's checkpoints (kCkNone: none)
  int32_t chunk;    // bits per chunk lane
  int32_t nck;      // checkpoints per chunk (idx_nck)
  int32_t ckb;      // their spacing: chunk / (nck + 1) bits
  int32_t* ended;   // [nclients]
  uint64_t* idx;
  uint64_t* idxq;   // nullable
  int64_t* total_bits;
  int32_t* err;
};

// MSB-first reader of one client's code: a 64-bit window of nv valid bits (the
// bits past the code's end read as zeros and are not counted).
struct IdxReader {
  const uint32_t* w;
  int64_t nbits;
  int64_t wpos;  // stream bit of the next word to load
  uint64_t win;
  int32_t nv;
  int64_t pos;   // stream bit at the window's MSB
  __device__ __forceinline__ void refill() {
    if (nv <= 32 && wpos < nbits) {
      uint32_t v = bswap32(w[wpos >> 5]);
      const int64_t vb = nbits - wpos;
      if (vb < 32) v &= ~0u << (32 - (int32_t)vb);
      win |= (uint64_t)v << (32 - nv);
      nv += vb < 32 ? (int32_t)vb : 32;
      wpos += 32;
    }
  }
  __device__ __forceinline__ void skip(uint32_t n) {
    win = n < 64 ? win << n : 0ull;
    nv -= (int32_t)n;
    pos += n;
  }
  __device__ __forceinline__ void init(const uint32_t* w_, int64_t nbits_, int64_t p) {
    w = w_;
    nbits = nbits_;
    pos = p;
    win = 0;
    nv = 0;
    wpos = p & ~31LL;
    refill();
    const int32_t s = (int32_t)(p & 31);
    win = s < 64 ? win << s : 0ull;
    nv = max(nv - s, 0);
    if (nv == 0) win = 0;
    refill();
  }
};

// Elias gamma value at the reader (advanced past it); 0 when malformed (more than
// 31 leading zeros) or cut by the stream's end.
__device__ __forceinline__ uint32_t idx_gamma(IdxReader& r) {
  r.refill();  // > 32 valid bits unless the stream ends
  const uint32_t z = r.win ? (uint32_t)__clzll(r.win) : 64u;
  if (z > 31u || (int32_t)z >= r.nv) return 0u;
  if ((int32_t)(2u * z + 1u) <= r.nv) {
    const uint32_t v = (uint32_t)((r.win << z) >> (63u - z));
    r.skip(2u * z + 1u);
    return v;
  }
  r.skip(z);
  r.refill();
  if ((int32_t)z + 1 > r.nv) return 0u;
  const uint32_t v = (uint32_t)(r.win >> (63u - z));
  r.skip(z + 1u);
  return v;
}

// One (run, sign, magnitude) code: returns the run (>= 1), 0 if it does not parse.
__device__ __forceinline__ uint32_t idx_code(IdxReader& r) {
  const uint32_t d = idx_gamma(r);
  if (!d) return 0u;
  r.refill();
  if (r.nv < 1) return 0u;
  r.skip(1);
  return idx_gamma(r) ? d : 0u;
}

struct IdxLock {
  int64_t x, n;
  int64_t m;  // (idx_lockstep) the meeting bit, kIdxFail if none
};

__device__ __forceinline__ const uint32_t* idx_words(const IdxArgs& a, int64_t c) {
  return (const uint32_t*)(a.stream_buf + a.stream_off[c]);
}

__device__ __forceinline__ void idx_put(const IdxArgs& a, int64_t c, int64_t u, uint64_t e) {
  if (!a.idxq) {
    a.idx[c * (a.T + 1) + u] = e;
    return;
  }
  const int64_t t = u >> 2;
  const int s = (int)(u & 3);
  if (s == 0) a.idx[c * (a.T + 1) + t] = e;
  else a.idxq[3 * (c * a.T + t) + s - 1] = e;
}

// Table-driven parse of one chunk's codes: every code starting in [start, stop),
// `start` a (true or guessed) code start.  The decoder's table (up to two complete
// codes per 12 window bits, their runs and length) takes the common codes; a code
// the table does not hold (longer than 12 bits, or the step would cross `stop` or,
// EMIT, the next unit boundary) is decoded from the window's top 32 bits, and a
// code longer than 32 bits -- or one that does not parse (the trailing zero-run
// code, a guessed start, a malformed code) -- by the IdxReader, after which the
// window restarts.
//   !EMIT: returns the exit (first code start >= stop, or kIdxFail) and the runs' sum.
//   EMIT: L = the last nonzero before `start` (true start); writes the entries of
//   the units (from unit u on) its codes enter and, at the code's end, the tail
//   entries, total_bits and `ended` (IdxEnd); bad on a malformed code.
struct IdxEnd {
  int64_t bend, total;  // bend >= 0: the code ended in this chunk
  bool bad;
};
// 4 x the runs of a table step's codes (ilut: one field; the decoder's table: two)
__device__ __forceinline__ int32_t idx_runs4(uint32_t e) {
  return FC_IDX_ILUT ? (int32_t)(e & 0xFFu) : (int32_t)((e & 0x7Fu) + ((e >> 7) & 0x7Fu));
}

template <bool EMIT>
__device__ __forceinline__ IdxLock idx_parse(const IdxArgs& a, int64_t c, const uint32_t* lut, int64_t start,
                                             int64_t stop, int64_t L, IdxEnd* end, uint64_t* ckp = nullptr,
                                             int64_t ckst = 0, int64_t u_stop = INT64_MAX) {
  const int64_t nbits = 8 * a.nbytes[c];
  const uint8_t* base = a.stream_buf + a.stream_off[c];
  const int64_t cap = (a.nbytes[c] + 15) & ~15LL;  // readable: the 16-byte block holding the end
  const uint32_t* w = (const uint32_t*)base;
  const int gs = a.idxq ? 8 : 10;                  // EMIT unit: quarter tile or tile
  const int64_t nu = a.idxq ? 4 * (int64_t)a.T : (int64_t)a.T;
  int64_t u = EMIT ? (L + ((int64_t)1 << gs)) >> gs : 0;  // the first unit starting after L
  // fast steps while the runs they add stay below `room4` (4 x elements to the next
  // unit boundary, or to P once every boundary is written: a code reaching element P
  // is the end's business)
  auto room_of = [&](int64_t Lc) -> int32_t {
    if (!EMIT) return 1 << 30;
    const int64_t nb = u < nu ? min<int64_t>(u << gs, a.P) : a.P;
    return (int32_t)min<int64_t>(4 * (nb - Lc), 1 << 30);
  };
  int64_t nsum = 0;  // !EMIT: the runs' sum outside the table steps
  int32_t acc4 = 0;  // the table steps' runs (x 4) since the last slow code
  int32_t room4 = room_of(L);
  const int32_t lim = (int32_t)(stop - start);
  // bits of the code from `start` on: a table / window code must end inside them (so
  // every path accepts exactly the codes the IdxReader does)
  const int32_t avail = (int32_t)min<int64_t>(nbits - start, (int64_t)lim + 8192);
  // (FC_IDX_ASYNC: the guessed parse on the decoder's untracked batch-point loads --
  // tools/audit_async_loads.py checks that no destination register is touched early)
  SegReaderT<!EMIT && FC_IDX_ASYNC> r;
  auto restart = [&](int32_t cons) {
    r.init(base, cap, (uint64_t)(start + cons), (int32_t)min<int64_t>(nbits - start - cons, lim - cons + 8192));
    return cons + r.nwin;
  };
  int32_t cons = 0;
  int32_t fill = restart(0);
  uint32_t it = 0;
  bool failed = false;
  int nk = 0;  // (!EMIT, ckp) checkpoints recorded
  int32_t ckt = ckp ? a.ckb : INT32_MAX;  // the next checkpoint's threshold (past the last: never)
  // one iteration (as decode_segment: FC_DEC_UNROLL places the batch points by position)
  auto iter = [&](auto kpos) -> bool {
    constexpr int K = decltype(kpos)::value;
    constexpr bool UNR = K >= 0;
    if (!EMIT && cons >= ckt) {  // a code start: checkpoint
      ckp[nk * ckst] = (uint64_t)cons | ((uint64_t)(nsum + (acc4 >> 2)) << 13);
      ++nk;
      ckt = nk < a.nck ? (nk + 1) * a.ckb : INT32_MAX;
    }
    if (!UNR) it = __builtin_amdgcn_readfirstlane(it + 1u);
    if (UNR ? K == kDecBatch - 1 : (it & (kDecBatch - 1)) == 0) r.batch();
    const uint32_t e = lut[(uint32_t)(r.win >> (64 - kLutBits))];
    const uint32_t Ls = e >> 26;
    const int32_t dd4 = idx_runs4(e);
    const int32_t lend = min(lim, avail);  // a table step's codes must end inside both
    bool stepped = false;
    if (!EMIT && FC_IDX_UNIFORM && __ballot(cons + 2 * kLutBits > lend) == 0) {
      // the guessed parse with every lane of the wave 24+ bits from its end: two table
      // steps with no per-lane checks and no divergent branch, as the decoder's (an entry
      // that takes nothing is all zero; the lane's code is decoded below)
      r.win <<= Ls;
      cons += (int32_t)Ls;
      acc4 += dd4;
      const uint32_t e2 = lut[(uint32_t)(r.win >> (64 - kLutBits))];
      const uint32_t L2 = e2 >> 26;
      r.win <<= L2;
      cons += (int32_t)L2;
      acc4 += idx_runs4(e2);
      stepped = Ls != 0u;
    } else if (Ls != 0u && cons + (int32_t)Ls <= lend && (!EMIT || acc4 + dd4 < room4)) {
      r.win <<= Ls;
      cons += (int32_t)Ls;
      acc4 += dd4;
      // a second table step (>= 21 valid window bits left); not taken, the next
      // iteration looks at the same bits again
      const uint32_t e2 = lut[(uint32_t)(r.win >> (64 - kLutBits))];
      const uint32_t L2 = e2 >> 26;
      const int32_t d24 = idx_runs4(e2);
      if (L2 != 0u && cons + (int32_t)L2 <= lend && (!EMIT || acc4 + d24 < room4)) {
        r.win <<= L2;
        cons += (int32_t)L2;
        acc4 += d24;
      }
      stepped = true;
    }
    if (!stepped) {
      // one code: from the window's top 32 bits if it fits there (>= 33 valid bits)
      const int64_t p = start + cons;
      if (EMIT) {
        L += acc4 >> 2;
        acc4 = 0;
      }
      const uint32_t top = (uint32_t)(r.win >> 32);
      const uint32_t z1 = (uint32_t)__clz(top);
      const uint32_t sa = 30u - 2u * z1;
      const uint32_t rest = top << (32u - sa);
      const uint32_t z2 = (uint32_t)__clz(rest);
      const uint32_t Lw = 2u * (z1 + z2) + 3u;
      uint32_t d = top >> (sa + 1u);
      bool took = false;
      if (EMIT && L == a.P - 1) {  // every element covered: the code ends here, no trailing run
        end->bend = end->total = p;
        return true;
      }
      if (z1 <= 15u && z2 <= 15u && Lw <= 32u && cons + (int32_t)Lw <= avail && (!EMIT || L + (int64_t)d < a.P)) {
        r.win <<= Lw;
        cons += (int32_t)Lw;
        took = true;
      } else {
        r.wait_nxt();  // (async) as in decode_segment's slow path: land the batch-point load first
        IdxReader ir;
        ir.init(w, nbits, p);
        d = idx_gamma(ir);
        if (EMIT) {
          if (!d || L + (int64_t)d > a.P) {
            end->bad = true;
            return true;
          }
          if (L + (int64_t)d == a.P) {  // the trailing zero run
            end->bend = p;
            end->total = ir.pos;
            return true;
          }
        }
        bool ok = d != 0u;
        if (ok) {
          ir.refill();
          ok = ir.nv >= 1;
          if (ok) {
            ir.skip(1);
            ok = idx_gamma(ir) != 0u;
          }
        }
        if (!ok) {
          if (EMIT) end->bad = true;
          failed = true;
          return true;
        }
        cons = (int32_t)(ir.pos - start);
        fill = restart(cons);
      }
      if (EMIT) {
        const int64_t nz = L + (int64_t)d;
        const uint64_t en = ((uint64_t)p & kMask36) | ((uint64_t)(L + 1) << 36);
        for (; u < nu && (u << gs) <= nz; ++u) idx_put(a, c, u, en);
        L = nz;
        room4 = room_of(L);
        if (u > u_stop) return true;  // the entries asked for are written
      } else {
        nsum += d;
      }
      if (!took) return false;  // the window restarted full
    }
    if (fill - cons <= 32) {  // (the blocks are zero past the code's end)
      const uint32_t wd = r.pop32();
      r.win |= (uint64_t)wd << (32 - (fill - cons));
      fill += 32;
    }
    return false;
  };
  if (FC_DEC_UNROLL) {
    while (cons < lim) {
      if (iter(std::integral_constant<int, 0>{}) || !(cons < lim)) break;
      if (iter(std::integral_constant<int, 1>{}) || !(cons < lim)) break;
      if (iter(std::integral_constant<int, 2>{}) || !(cons < lim)) break;
      if (iter(std::integral_constant<int, 3>{})) break;
    }
  } else {
    while (cons < lim)
      if (iter(std::integral_constant<int, -1>{})) break;
  }
  r.wait_nxt();  // (async) the last batch-point load lands before its registers are reused
  if (!EMIT && ckp)
    for (; nk < a.nck; ++nk) ckp[nk * ckst] = kCkNone;
  if (failed) return {kIdxFail, nsum};
  if (EMIT) {
    L += acc4 >> 2;
    // a code whose last element is nonzero and whose last code ends exactly on the
    // chunk's end leaves the loop with cons == lim before the in-loop end check
    if (!end->bad && end->bend < 0 && L == a.P - 1 && start + cons == nbits) end->bend = end->total = nbits;
    if (!end->bad && end->bend >= 0) {
      const uint64_t en = ((uint64_t)end->bend & kMask36) | ((uint64_t)(L + 1) << 36);
      for (; u < nu; ++u) idx_put(a, c, u, en);
      a.idx[c * (a.T + 1) + a.T] = en;
      a.total_bits[c] = end->total;
      a.ended[c] = 1;
    }
    return {start + cons, L};
  }
  return {start + cons, nsum + (acc4 >> 2)};
}

// The decode table in LDS for a workgroup of chunk lanes (persistent grids).
__device__ __forceinline__ void idx_load_lut(uint32_t* lut) {
  const uint4* src = (const uint4*)(FC_IDX_ILUT ? g_dec_tabs.ilut : g_dec_tabs.lut);
  for (int i = threadIdx.x; i < kLutSize / 4; i += blockDim.x) ((uint4*)lut)[i] = src[i];
  __syncthreads();
}

__global__ __launch_bounds__(kThreads) void k_idx_spec(IdxArgs a) {
  __shared__ __attribute__((aligned(16))) uint32_t lut[kLutSize];
  idx_load_lut(lut);
  const int64_t lanes = (int64_t)a.nclients * a.nchunks;
  for (int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; g < lanes; g += (int64_t)gridDim.x * blockDim.x) {
    const int64_t c = g / a.nchunks, j = g - c * a.nchunks;
    const int64_t cb = j * a.chunk;
    IdxLock r{kIdxFail, 0};
    if (cb < 8 * a.nbytes[c]) {
      r = idx_parse<false>(a, c, lut, cb, cb + a.chunk, 0, nullptr, a.ck + g, lanes);
    } else {
      for (int k = 0; k < a.nck; ++k) a.ck[k * lanes + g] = kCkNone;
    }
    a.x1[g] = r.x;
    a.n1[g] = r.n;
  }
}

// Chunk [cb, ce) from its true start s: the guessed parse A (from cb: exit x1, runs
// n1) replayed beside the true parse B until both stand on one code start, whence
// they coincide.  Returns the true exit and runs; `met` false when B left the chunk
// (or failed) without meeting A.
__device__ __noinline__ IdxLock idx_lockstep(const uint32_t* w, int64_t nbits, int64_t cb, int64_t ce, int64_t s,
                                             int64_t x1, int64_t n1) {
  IdxReader A, B;
  A.init(w, nbits, cb);
  B.init(w, nbits, s);
  int64_t pa = cb, pb = s, na = 0, nb = 0;
  bool adone = false;
  for (;;) {
    if (pa == pb) return {x1, n1 - na + nb, pa};
    if (pa < pb && !adone) {
      if (pa >= ce) {
        adone = true;  // A left the chunk at x1
        continue;
      }
      const uint32_t d = idx_code(A);
      if (!d) {
        adone = true;  // A failed at pa (x1 = fail)
      } else {
        na += d;
        pa = A.pos;
      }
      continue;
    }
    if (pb >= ce) return {pb, nb, kIdxFail};
    const uint32_t d = idx_code(B);
    if (!d) return {kIdxFail, nb, kIdxFail};
    nb += d;
    pb = B.pos;
  }
}

__global__ __launch_bounds__(kThreads) void k_idx_sync(IdxArgs a) {
  const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= (int64_t)a.nclients * a.nchunks) return;
  const int64_t c = g / a.nchunks, j = g - c * a.nchunks;
  const int64_t nbits = 8 * a.nbytes[c];
  const int64_t cb = j * a.chunk;
  IdxLock r{kIdxFail, 0, kIdxFail};
  if (j == 0) {
    r = {a.x1[g], a.n1[g], 0};  // chunk 0 starts at bit 0: its parse is the true one
  } else if (cb < nbits) {
    const int64_t s = a.x1[g - 1];
    if (s != kIdxFail) r = idx_lockstep(idx_words(a, c), nbits, cb, cb + a.chunk, s, a.x1[g], a.n1[g]);
  }
  a.x2[g] = r.x;
  a.n2[g] = r.n;
  a.xm[g] = r.m;
}

__device__ __forceinline__ int64_t rfl64(int64_t v) {
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)((uint64_t)v >> 32));
  return (int64_t)(((uint64_t)hi << 32) | lo);
}

// One wave per client: chunk j's true start is chunk j-1's final true exit; k_idx_sync
// used chunk j-1's guessed exit, so a chunk whose predecessor's exit changed is
// redone from the right start (lane 0, in order: a redone exit can change the next).
__global__ __launch_bounds__(64) void k_idx_fix(IdxArgs a) {
  const int64_t c = blockIdx.x;
  const int lane = threadIdx.x;
  const int64_t nbits = 8 * a.nbytes[c];
  const int64_t nch = min<int64_t>(a.nchunks, (nbits + a.chunk - 1) / a.chunk);
  if (nch <= 1) return;
  const int64_t* x1 = a.x1 + c * a.nchunks;
  const int64_t* n1 = a.n1 + c * a.nchunks;
  int64_t* x2 = a.x2 + c * a.nchunks;
  int64_t* n2 = a.n2 + c * a.nchunks;
  const uint32_t* w = idx_words(a, c);
  int64_t carried = x2[0];  // the final true exit of chunk j0 - 1
  int64_t j0 = 1;
  while (j0 < nch) {
    const int64_t j = j0 + lane;
    bool mism = false;
    if (j < nch) mism = (lane == 0 ? carried : x2[j - 1]) != x1[j - 1];
    const uint64_t m = __ballot(mism);
    if (m == 0) {
      carried = x2[min<int64_t>(j0 + 63, nch - 1)];
      j0 += 64;
      continue;
    }
    const int k = __builtin_ctzll(m);
    const int64_t jk = j0 + k;
    const int64_t s = k == 0 ? carried : x2[jk - 1];
    IdxLock r{kIdxFail, 0, kIdxFail};
    if (lane == 0 && s != kIdxFail) {
      const int64_t cb = jk * a.chunk;
      r = idx_lockstep(w, nbits, cb, cb + a.chunk, s, x1[jk], n1[jk]);
    }
    if (lane == 0) {
      x2[jk] = r.x;
      n2[jk] = r.n;
      a.xm[c * a.nchunks + jk] = r.m;
    }
    carried = rfl64(r.x);
    j0 = jk + 1;
  }
}

// One wave per client: n2[j] <- the last nonzero before chunk j's first code
// (-1 + the runs of every code before it).
__global__ __launch_bounds__(64) void k_idx_scan(IdxArgs a) {
  const int64_t c = blockIdx.x;
  const int lane = threadIdx.x;
  const int64_t nbits = 8 * a.nbytes[c];
  const int64_t nch = min<int64_t>(a.nchunks, (nbits + a.chunk - 1) / a.chunk);
  int64_t* n2 = a.n2 + c * a.nchunks;
  int64_t run = -1;
  for (int64_t j0 = 0; j0 < nch; j0 += 64) {
    const int64_t j = j0 + lane;
    const int64_t v = j < nch ? n2[j] : 0;
    int64_t incl = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int64_t u = __shfl_up(incl, o, 64);
      if (lane >= o) incl += u;
    }
    if (j < nch) n2[j] = run + incl - v;
    run += __shfl(incl, 63, 64);
  }
}

#ifndef FC_IDX_EMIT_WPE
#define FC_IDX_EMIT_WPE 4  // 6 or 8 (64-80 VGPRs) spill in the parse: 56 / 50 ms vs 38.5 at the headline
#endif
#ifndef FC_IDX_CK_CARRY
#define FC_IDX_CK_CARRY 1  // the emit's checkpoint scan carried over a lane's units (0: rescanned per unit)
#endif
#ifndef FC_IDX_CKW
#define FC_IDX_CKW 4  // checkpoint loads in flight per scan step
#endif
__global__ __launch_bounds__(kThreads) __attribute__((amdgpu_waves_per_eu(FC_IDX_EMIT_WPE))) void k_idx_emit(IdxArgs a) {
  __shared__ __attribute__((aligned(16))) uint32_t lut[kLutSize];
  idx_load_lut(lut);
  const int64_t lanes = (int64_t)a.nclients * a.nchunks;
  const int gs = a.idxq ? 8 : 10;  // unit: quarter tile or tile
  for (int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; g < lanes; g += (int64_t)gridDim.x * blockDim.x) {
    const int64_t c = g / a.nchunks, j = g - c * a.nchunks;
    const int64_t nbits = 8 * a.nbytes[c];
    const int64_t cb = j * a.chunk, ce = cb + a.chunk;
    if (cb >= nbits) continue;  // (an empty code never ends: k_idx_check)
    const int64_t s = j == 0 ? 0 : a.x2[g - 1];
    if (s == kIdxFail) continue;  // past the code's end
    const int64_t L = a.n2[g];    // the last nonzero before the chunk's first code
    if (L >= a.P) continue;       // (past the trailing run of a code with bytes after it)
    IdxEnd end{-1, -1, false};
    // checkpoints: a chunk two or more before the code's last, whose true parse met the
    // guessed one and whose codes stay short of the last element
    const int64_t m = a.xm[g];
    bool ckd = a.nck > 0 && j + 1 < (nbits - 1) / a.chunk && a.x2[g] != kIdxFail && m != kIdxFail;
    const int64_t Lnext = ckd ? a.n2[g + 1] : 0;  // the last nonzero of the chunk's last code
    ckd = ckd && Lnext >= L && Lnext < a.P - 1;
    // !ckd: the whole chunk, ends and all (one parse).  ckd: the units whose first element
    // lies in (L, Lnext], each by a parse from the latest true code start before it -- the
    // last parse's end, or a checkpoint past the meeting.  One parse call site either way.
    const int64_t adj = Lnext - a.n1[g];  // checkpoint runs (guessed parse) -> last nonzero
    int64_t u = (L + ((int64_t)1 << gs)) >> gs;
    const int64_t ulast = ckd ? Lnext >> gs : u;
    int64_t cp = s, cl = L;
    bool bad = false;
#if FC_IDX_CK_CARRY
    // the checkpoints rise in position and runs, and so do the unit bounds: the scan
    // carries over the lane's units (each checkpoint read once), FC_IDX_CKW loads in
    // flight; the latest one before the bound is the parse start if past the meeting
    int kc = ckd ? 0 : a.nck;       // checkpoints [0, kc) lie before an earlier bound
    int64_t kpos = -1, klk = 0;     // the latest of them (-1: none)
#endif
    while (u <= ulast) {
      const int64_t bound = u << gs;
      int64_t ps = cp, pl = cl;
#if FC_IDX_CK_CARRY
      while (kc < a.nck) {
        uint64_t e[FC_IDX_CKW];
#pragma unroll
        for (int i = 0; i < FC_IDX_CKW; ++i) e[i] = a.ck[(int64_t)min(kc + i, a.nck - 1) * lanes + g];
        int n = 0;
        bool stop = false;
#pragma unroll
        for (int i = 0; i < FC_IDX_CKW; ++i) {
          if (stop || kc + i >= a.nck) {
            stop = true;
          } else if (e[i] == kCkNone) {
            n = a.nck - kc;  // none after it either
            stop = true;
          } else {
            const int64_t lk = adj + (int64_t)(e[i] >> 13);
            if (lk >= bound) {
              stop = true;
            } else {
              kpos = cb + (int64_t)(e[i] & 0x1FFFu);
              klk = lk;
              n = i + 1;
            }
          }
        }
        kc += n;
        if (stop) break;
      }
      if (kpos >= m && kpos > ps) {
        ps = kpos;
        pl = klk;
      }
#else
      for (int k = 0; ckd && k < a.nck; ++k) {
        const uint64_t e = a.ck[k * lanes + g];
        if (e == kCkNone) break;
        const int64_t pos = cb + (int64_t)(e & 0x1FFFu);
        const int64_t lk = adj + (int64_t)(e >> 13);
        if (lk >= bound) break;
        if (pos >= m && pos > ps) {
          ps = pos;
          pl = lk;
        }
      }
#endif
      const IdxLock r = idx_parse<true>(a, c, lut, ps, ce, pl, &end, nullptr, 0, ckd ? u : INT64_MAX);
      if (!ckd) {
        if (end.bad) {
          bad = true;
        } else if (end.bend >= 0) {
          bad = (end.total + 7) / 8 != a.nbytes[c];  // bytes after the code, or a short final byte
        } else {
          bad = ce >= nbits;  // the code ends before its elements do
        }
        break;
      }
      if (end.bad || end.bend >= 0 || r.n < bound) {  // (a chunk before the last holds no end)
        bad = true;
        break;
      }
      cp = r.x;
      cl = r.n;
      u = (cl + ((int64_t)1 << gs)) >> gs;
    }
    if (bad) atomicOr(a.err, 1);
  }
}

__global__ void k_idx_check(IdxArgs a) {
  const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (c < a.nclients && !a.ended[c]) atomicOr(a.err, 1);
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

// QSGD server sum (qsgd.py:88-100): acc = in (or 0), then acc = acc + f32(q_c) *
// scale[c] for the clients of the plane rows in client order, float32 with no
// contraction -- the reference's sequential client-order sum, bit for bit.  One
// thread per 4 elements (rows padded to a multiple of 4 elements).
// QT int8_t: rows of bytes (4 per 32-bit load, sign-extended).
template <typename QT>
__global__ __launch_bounds__(256) void k_sum_planes(const QT* __restrict__ planes, int64_t stride, int32_t n,
                                                    int64_t P, const float* __restrict__ scale,
                                                    const float* in, float* out) {
  const int64_t e0 = 4 * ((int64_t)blockIdx.x * blockDim.x + threadIdx.x);
  if (e0 >= P) return;
  float acc[4] = {0.f, 0.f, 0.f, 0.f};
  const int m = (int)min<int64_t>(4, P - e0);
  if (in)
    for (int k = 0; k < m; ++k) acc[k] = in[e0 + k];
  for (int c = 0; c < n; ++c) {
    int4 q;
    if constexpr (sizeof(QT) == 1) {
      const uint32_t w = *(const uint32_t*)(planes + (int64_t)c * stride + e0);
      q = make_int4((int8_t)(w & 0xFFu), (int8_t)((w >> 8) & 0xFFu), (int8_t)((w >> 16) & 0xFFu), (int8_t)(w >> 24));
    } else {
      q = *(const int4*)(planes + (int64_t)c * stride + e0);
    }
    const float sc = scale[c];
    acc[0] = acc[0] + (float)q.x * sc;
    acc[1] = acc[1] + (float)q.y * sc;
    acc[2] = acc[2] + (float)q.z * sc;
    acc[3] = acc[3] + (float)q.w * sc;
  }
  for (int k = 0; k < m; ++k) out[e0 + k] = acc[k];
}

// noise_sum[i] = sum over clients, in client order, of TF's dither noise
// u01 - 0.5 for element i.  Each workgroup scrambles a chunk of 256 clients'
// seeds into Philox keys once (LDS); every thread then draws one Philox group
// (4 elements) per client with the key uniform across the wave (round keys on
// the scalar unit, as in the encoder).
__global__ __launch_bounds__(256) void k_noise_sum(const int64_t* __restrict__ seeds, int32_t n, int64_t P,
                                                   float* __restrict__ out) {
  __shared__ Key4 keys[256];
  const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t e0 = g * 4;
  float s[4] = {0.f, 0.f, 0.f, 0.f};
  for (int c0 = 0; c0 < n; c0 += 256) {
    __syncthreads();
    if (c0 + (int)threadIdx.x < n)
      keys[threadIdx.x] = tf_seed_scramble(seeds[2 * (c0 + threadIdx.x)], seeds[2 * (c0 + threadIdx.x) + 1]);
    __syncthreads();
    const int cn = min(256, n - c0);
    for (int j = 0; j < cn; ++j) {
      Key4 key = keys[j];
      key.k0 = __builtin_amdgcn_readfirstlane(key.k0);
      key.k1 = __builtin_amdgcn_readfirstlane(key.k1);
      key.c2 = __builtin_amdgcn_readfirstlane(key.c2);
      key.c3 = __builtin_amdgcn_readfirstlane(key.c3);
      const uint4 rb = philox_group_u(key, (uint32_t)g);
      s[0] = s[0] + (u01(rb.x) - 0.5f);
      s[1] = s[1] + (u01(rb.y) - 0.5f);
      s[2] = s[2] + (u01(rb.z) - 0.5f);
      s[3] = s[3] + (u01(rb.w) - 0.5f);
    }
  }
  if (e0 >= P) return;
#pragma unroll
  for (int k = 0; k < 4; ++k)
    if (e0 + k < P) out[e0 + k] = s[k];
}

// Per-client norm: one workgroup per client, float64 accumulation, fixed order.
__device__ __forceinline__ double shfl_xor_f64(double v, int m) {
  return __hiloint2double(__shfl_xor(__double2hiint(v), m), __shfl_xor(__double2loint(v), m));
}
__device__ __forceinline__ double wave_sum_f64(double v) {
#pragma unroll
  for (int m = 32; m > 0; m >>= 1) v += shfl_xor_f64(v, m);
  return v;
}

// Per-client normaliser / norm: one 1024-thread workgroup per client (enough
// waves per CU even for a few hundred clients); each wave reads 2048-element
// tiles with coalesced 4-byte loads, 8 in flight.  Max is exact in float32;
// sums accumulate every term in float64 (|x| and x^2 of a float32 are exact in
// float64), reduced in a fixed order: the float32 result is the correctly
// rounded norm but in astronomically rare ties.  The pass stays HBM-bound.
// Inputs pass through `+ 0.0f` (DAZ as TF-CPU).
// prescale (nullable [2C]): the norm of (x * prescale[2c]) * prescale[2c+1],
// element by element as the encoder quantises it (the value QuantizeEncode's
// normalize_fn sees behind the TFF clipping and mean wrappers).
// FC_NORM_L2_LINF: one pass for both wrapper norms, norms[c] = ||x||_2 and
// norms[C + c] = max |x| (builder.py:100-117: clipping and zeroing).
constexpr int kNormThreads = 1024;
// Row reads of the streaming reducers (k_client_norms, k_mask_encode): each byte is
// read once, FC_ROW_NT 1 issues them non-temporal.
#ifndef FC_ROW_NT
#define FC_ROW_NT 1  // one-bit 128 x 25 M encode -8 %, client norms -2 %, 1024 x 25 one-bit within noise (profiles/r05/diag_row_nt_ab.txt)
#endif
typedef float f4row_t __attribute__((ext_vector_type(4)));
__device__ __forceinline__ f4row_t ld_row4(const __attribute__((address_space(1))) f4row_t* p) {
  if (FC_ROW_NT) return __builtin_nontemporal_load(p);
  return *p;
}
// Client split (few clients per GPU): a client's row is summed in REDUCTION BLOCKS
// of kRedTiles 2048-element tiles, and each block's float64 partial is formed in an
// order fixed by the block alone (wave w takes tiles w, w + waves, ... of the block;
// lanes by a shuffle tree, then waves in order).  The part count S (gridDim.x:
// workgroups per client, chosen for occupancy) only decides which workgroup forms
// which blocks -- part s takes blocks [s nblk / S, (s + 1) nblk / S) -- and the
// finalize kernels add a client's blocks in block order, so every sum (norms,
// one-bit / DRIVE means, distortion) depends on P alone: the same bits for any
// client count per GPU (tests/test_gpu_aggregators.py::
// test_client_split_is_deterministic).
constexpr int kRedTiles = 64;
__host__ __device__ __forceinline__ int64_t red_blocks(int64_t P) { return ((P + 2047) / 2048 + kRedTiles - 1) / kRedTiles; }
__device__ __forceinline__ void part_range(int64_t n, int s, int S, int64_t& lo, int64_t& hi) {
  lo = n * s / S;
  hi = n * (s + 1) / S;
}
// ACC: 0 sum |x|, 1 sum x^2, 2 none (max only).  max |x| is always taken.
template <int ACC, bool PRE>
__global__ __launch_bounds__(kNormThreads) void k_client_norms(const float* const* xs, int64_t P,
                                                               const float* prescale, double* part) {
  const int c = blockIdx.y;
  const float* __restrict__ x = xs[c];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const float s0 = PRE ? prescale[2 * c] : 1.0f, s1 = PRE ? prescale[2 * c + 1] : 1.0f;
  const bool aligned = ((uintptr_t)x & 15u) == 0;
  const int64_t ntile = (P + 2047) / 2048, nblk = red_blocks(P);
  int64_t blo, bhi;
  part_range(nblk, (int)blockIdx.x, (int)gridDim.x, blo, bhi);
  // global (not flat) loads of the client's row
  typedef float f4v __attribute__((ext_vector_type(4)));
  typedef const __attribute__((address_space(1))) float* gfptr;
  typedef const __attribute__((address_space(1))) f4v* gf4ptr;
  const gfptr xg = (gfptr)x;
  for (int64_t b = blo; b < bhi; ++b) {
    // one float64 accumulator per float4 component: independent chains, summed in a
    // fixed order
    double acc4[4] = {0.0, 0.0, 0.0, 0.0};
    float mx = 0.0f;
    const int64_t te = min(ntile, (b + 1) * kRedTiles);
    for (int64_t tile = b * kRedTiles + wv; tile < te; tile += kNormThreads / 64) {
      const int64_t base = tile * 2048;
      const bool full = base + 2048 <= P && aligned;
      f4v raw[8];
      if (full) {
#pragma unroll
        for (int k = 0; k < 8; ++k) raw[k] = ld_row4((gf4ptr)(xg + base + 256 * k + 4 * lane));
      } else {
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const int64_t e = base + 256 * k + 4 * lane;
          raw[k].x = e < P ? xg[e] : 0.0f;
          raw[k].y = e + 1 < P ? xg[e + 1] : 0.0f;
          raw[k].z = e + 2 < P ? xg[e + 2] : 0.0f;
          raw[k].w = e + 3 < P ? xg[e + 3] : 0.0f;
        }
      }
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const float v4[4] = {raw[k].x, raw[k].y, raw[k].z, raw[k].w};
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          float v = v4[i] + 0.0f;  // DAZ as TF-CPU (zero padding past P adds nothing)
          if (PRE) v = (v * s0) * s1;
          const float a = fabsf(v);
          mx = fmaxf(mx, a);
          const double ad = (double)a;
          if (ACC == 0) acc4[i] += ad;
          if (ACC == 1) acc4[i] = fma(ad, ad, acc4[i]);
        }
      }
    }
    double r = (acc4[0] + acc4[1]) + (acc4[2] + acc4[3]);
    float m = mx;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      r += shfl_xor_f64(r, o);
      m = fmaxf(m, __shfl_xor(m, o));
    }
    if (lane == 0) {  // (block, wave) partial: no workgroup barrier in the loop
      double* pp = part + 2 * (((int64_t)c * nblk + b) * (kNormThreads / 64) + wv);
      pp[0] = r;
      pp[1] = (double)m;
    }
  }
}

// The norms from each client's (block, wave) partials: one wave per client, lane l
// adds blocks l, l + 64, ... in order (a block's waves in order), then a fixed
// shuffle tree over the lanes -- an order set by P alone.
__global__ __launch_bounds__(64) void k_norms_finalize(const double* part, int32_t nclients, int32_t nblk, int64_t P,
                                                       int kind, float* norms) {
  const int c = blockIdx.x;
  const int lane = threadIdx.x;
  constexpr int W = kNormThreads / 64;
  double t = 0.0;
  float tm = 0.0f;
  for (int64_t b = lane; b < nblk; b += 64) {
    const double* pp = part + 2 * ((int64_t)c * nblk + b) * W;
    double tb = pp[0];
    float mb = (float)pp[1];
    for (int w = 1; w < W; ++w) {
      tb += pp[2 * w];
      mb = fmaxf(mb, (float)pp[2 * w + 1]);
    }
    t += tb;
    tm = fmaxf(tm, mb);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    t += shfl_xor_f64(t, o);
    tm = fmaxf(tm, __shfl_xor(tm, o));
  }
  if (lane != 0) return;
  float out = tm;  // FC_NORM_MAX_MAGNITUDE / FC_NORM_LINF
  if (kind == FC_NORM_MEAN_MAGNITUDE) out = (float)(t / (double)P);
  if (kind == FC_NORM_DIMENSIONLESS) out = (float)sqrt(t / (double)P);
  if (kind == FC_NORM_L2 || kind == FC_NORM_L2_LINF) out = (float)sqrt(t);
  norms[c] = out;
  if (kind == FC_NORM_L2_LINF) norms[nclients + c] = tm;
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

// One-bit SGD (one_bit_sgd.py:56-81) and DRIVE (drive.py:58-76): ONE read
// pass per client.  One 256-thread workgroup per client; each wave walks
// 2048-element tiles with 16-byte loads, 8 in flight (lane l of load k: elements
// 256 k + 4 l .. +3).  A lane's four comparison bits form a nibble; three DPP
// rounds gather 8 lanes' nibbles into TF's mask word (bit i of word w = element
// 32 w + i), and the tile's 64 words go out through LDS as one coalesced 256-B
// store.  The means need the per-side sums and the distortion
// sum (x - decoded)^2 needs the means, so instead of a second pass the
// distortion is expanded per side:
//   sum_side (x - m)^2 = S2 - 2 m S1 + n m^2,  S1 = sum x, S2 = sum x^2,
// with every term accumulated in float64 (x^2 of a float32 is exact in float64;
// the expansion then cancels at the 1e-16 level, well inside the tolerance on
// TF's own float32 reduction).  Reductions are in a fixed order (deterministic).
// Inputs pass through `+ 0.0f` so denormals flush as on TF-CPU before the
// comparison.  KIND 0: one-bit SGD (threshold thr, class means).  KIND 1: DRIVE
// (mask = !(x < 0), scale from sum |x| and sum x^2, means -scale / +scale).
#ifndef FC_OB_THREADS
#define FC_OB_THREADS 256
#endif
constexpr int kObThreads = FC_OB_THREADS;
constexpr int kObWaves = kObThreads / 64;
// distortion / sum x^2 below which the one-pass expansion is recomputed term by
// term (float64 sums of x and x^2: relative error <= ~1e-11 of sum x^2)
constexpr double kObCancel = 1.0 / (1 << 20);

__device__ __forceinline__ uint32_t dpp_row_shl(uint32_t x, int n) {
  // lane l reads lane l + n of its 16-lane row (0 past the row end)
  return n == 1 ? __builtin_amdgcn_update_dpp(0u, x, 0x101, 0xf, 0xf, false)
       : n == 2 ? __builtin_amdgcn_update_dpp(0u, x, 0x102, 0xf, 0xf, false)
                : __builtin_amdgcn_update_dpp(0u, x, 0x104, 0xf, 0xf, false);
}

// Client split as k_client_norms: grid (S, C), part s of client c codes reduction
// blocks [s nblk / S, (s + 1) nblk / S) of the client's rotated block order (wave w:
// tiles w, w + 4, ... of each block) and writes block b's sums to part[c][b] = {S1,
// S2, A1, A2, count}; k_mask_finalize adds the blocks in block order and forms the
// means and the distortion (sums fixed by P alone).
constexpr int kObPart = 5;  // doubles per part
#ifndef FC_OB_F32X
#define FC_OB_F32X 0  // sums of x (and of x over the mask) in float32 tile partials (A/B knob; 0: float64)
#endif
#ifndef FC_OB_WPE
#define FC_OB_WPE 0  // waves per SIMD the mask encoder's registers are held to (0: the compiler's choice)
#endif
template <int KIND>
__global__ __launch_bounds__(kObThreads)
#if FC_OB_WPE
__attribute__((amdgpu_waves_per_eu(FC_OB_WPE)))
#endif
void k_mask_encode(const float* const* xs, int64_t P, float thr,
                                                            uint32_t* masks, double* part) {
  __shared__ uint32_t wordbuf[kObWaves][64];
  const int c = blockIdx.y;
  const float* __restrict__ x = xs[c];
  const int64_t nw = (P + 31) / 32;
  uint32_t* __restrict__ m = masks + (int64_t)c * nw;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int64_t ntile = (P + 2047) / 2048, nblk = red_blocks(P);
  int64_t blo, bhi;  // this part's reduction blocks, in rotated order
  part_range(nblk, (int)blockIdx.x, (int)gridDim.x, blo, bhi);
  const bool aligned = ((uintptr_t)x & 15u) == 0;
  // KIND 0: s1 = sum x, s2 = sum x^2, a1 / a2 = the same over x >= thr;
  // KIND 1: s1 = sum |x|, s2 = sum x^2.  Sums of x in float64 (FC_OB_F32X: float32
  // partials over a tile's 32 elements per lane, float64 across tiles); sums of
  // squares in float64 throughout (x^2 exact: the distortion below subtracts nearly
  // equal terms).  Fixed order everywhere.
  double s1 = 0.0, s2 = 0.0, a1 = 0.0, a2 = 0.0;
  uint32_t na = 0;
  // clients start at different tiles: rows share their alignment, and reading
  // every client's same offset at once would load the same HBM channels
#ifndef FC_OB_ROTATE
#define FC_OB_ROTATE 1
#endif
  const int64_t b0 = FC_OB_ROTATE ? ((int64_t)c * 977) % nblk : 0;
  // the wave's k-th tile of this part: block blo + k / kPerWave (rotated), tile
  // wv + kObWaves (k mod kPerWave) of it; -1 past the client's last tile (its last
  // block may be partial)
  constexpr int kPerWave = kRedTiles / kObWaves;
  auto tile_of = [&](int64_t k) -> int64_t {
    int64_t b = blo + k / kPerWave + b0;
    if (b >= nblk) b -= nblk;
    const int64_t t = b * kRedTiles + wv + kObWaves * (k % kPerWave);
    return t < ntile ? t : -1;
  };
  // global (not flat) loads: a flat load also counts in lgkmcnt, so every LDS
  // wait of the word assembly would wait for the in-flight tile too
  typedef float f4v __attribute__((ext_vector_type(4)));
  typedef const __attribute__((address_space(1))) float* gfptr;
  typedef const __attribute__((address_space(1))) f4v* gf4ptr;
  const gfptr xg = (gfptr)x;
  auto load_tile = [&](int64_t tile, f4v (&raw)[8]) {
    const int64_t base = tile * 2048;
    if (base + 2048 <= P && aligned) {  // wave-uniform: 8 float4 loads, no branches
#pragma unroll
      for (int k = 0; k < 8; ++k) raw[k] = ld_row4((gf4ptr)(xg + base + 256 * k + 4 * lane));
    } else {
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const int64_t e = base + 256 * k + 4 * lane;
        raw[k].x = e < P ? xg[e] : 0.0f;
        raw[k].y = e + 1 < P ? xg[e + 1] : 0.0f;
        raw[k].z = e + 2 < P ? xg[e + 2] : 0.0f;
        raw[k].w = e + 3 < P ? xg[e + 3] : 0.0f;
      }
    }
  };
  auto do_tile = [&](int64_t tile, const f4v (&raw)[8]) {
    const int64_t base = tile * 2048;
    const bool full = base + 2048 <= P;
    typedef __typeof__(FC_OB_F32X ? 0.0f : 0.0) xsum_t;  // the sums of x per tile
    xsum_t p1[2] = {0, 0}, q1[2] = {0, 0};  // two chains each
    double p2[2] = {0.0, 0.0}, q2[2] = {0.0, 0.0};
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int64_t e = base + 256 * k + 4 * lane;
      const float v4[4] = {raw[k].x + 0.0f, raw[k].y + 0.0f, raw[k].z + 0.0f, raw[k].w + 0.0f};
      uint32_t nib = 0;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        // zero padding past P (v = 0) adds nothing to the sums; only the mask bit
        // and the count need the bound
        const float v = v4[i];
        const bool ab = (full || e + i < P) && !(v < thr);
        nib |= ab ? (1u << i) : 0u;
        const double vd = (double)v;
        if (KIND == 0) {
          if (FC_OB_F32X) {
            const float tf = ab ? v : 0.0f;
            p1[k & 1] += v;
            q1[k & 1] += tf;
            const double td = (double)tf;
            p2[k & 1] = fma(vd, vd, p2[k & 1]);
            q2[k & 1] = fma(td, td, q2[k & 1]);
          } else {
            p1[k & 1] += vd;
            p2[k & 1] = fma(vd, vd, p2[k & 1]);
            const double td = ab ? vd : 0.0;
            q1[k & 1] += td;
            q2[k & 1] = fma(td, td, q2[k & 1]);
          }
        } else {
          if (FC_OB_F32X) p1[k & 1] += fabsf(v);
          else p1[k & 1] += fabs(vd);
          p2[k & 1] = fma(vd, vd, p2[k & 1]);
        }
      }
      na += (uint32_t)__popc(nib);
      // 8 lanes' nibbles -> one mask word in lane 8j (word 8k + j of the tile)
      uint32_t wd = nib | (dpp_row_shl(nib, 1) << 4);
      wd |= dpp_row_shl(wd, 2) << 8;
      wd |= dpp_row_shl(wd, 4) << 16;
      if ((lane & 7) == 0) wordbuf[wv][8 * k + (lane >> 3)] = wd;
    }
    s1 += (double)(p1[0] + p1[1]);
    s2 += p2[0] + p2[1];
    if (KIND == 0) {
      a1 += (double)(q1[0] + q1[1]);
      a2 += q2[0] + q2[1];
    }
    __builtin_amdgcn_wave_barrier();  // one wave's LDS accesses execute in order
    const uint32_t word = wordbuf[wv][lane];
    if (tile * 64 + lane < nw) m[tile * 64 + lane] = word;
  };
  // a block's sums of this wave, lanes reduced by a fixed shuffle tree, to its
  // (block, wave) slot: no workgroup barrier in the loop (k_mask_finalize adds the
  // waves and blocks in a fixed order)
  auto flush = [&](int64_t k) {
    const double S1w = wave_sum_f64(s1), S2w = wave_sum_f64(s2), A1w = wave_sum_f64(a1), A2w = wave_sum_f64(a2);
    const uint32_t nsum = (uint32_t)wave_sum_i((int32_t)na);
    s1 = s2 = a1 = a2 = 0.0;
    na = 0;
    if (lane == 0) {
      int64_t b = blo + k / kPerWave + b0;
      if (b >= nblk) b -= nblk;
      double* pp = part + kObPart * (((int64_t)c * nblk + b) * kObWaves + wv);
      pp[0] = S1w;
      pp[1] = S2w;
      pp[2] = A1w;
      pp[3] = A2w;
      pp[4] = (double)nsum;
    }
  };
  // software-pipelined: the wave's next tile's loads are in flight while a tile
  // computes (across block ends too); every wave walks kPerWave slots per block, so
  // all reach each block's reduction together
  const int64_t K = kPerWave * (bhi - blo);
  f4v ra[8], rb[8];
  int64_t ta = K > 0 ? tile_of(0) : -1;
  if (ta >= 0) load_tile(ta, ra);
  for (int64_t k = 0; k < K; k += 2) {  // K is even (kPerWave is)
    const int64_t tb = tile_of(k + 1);
    if (tb >= 0) load_tile(tb, rb);
    if (ta >= 0) do_tile(ta, ra);
    ta = k + 2 < K ? tile_of(k + 2) : -1;
    if (ta >= 0) load_tile(ta, ra);
    if (tb >= 0) do_tile(tb, rb);
    if ((k + 2) % kPerWave == 0) flush(k);
  }
}

// Means and distortion of each client from its (block, wave) partials: one wave
// per client, lane l adds blocks l, l + 64, ... in order (a block's waves in
// order), then a fixed shuffle tree -- an order set by P alone.
template <int KIND>
__global__ __launch_bounds__(64) void k_mask_finalize(const double* part, int32_t nclients, int32_t nblk, int64_t P,
                                                      int min_distortion, float* means, double* dist) {
  const int c = blockIdx.x;
  const int lane = threadIdx.x;
  double S1 = 0.0, S2 = 0.0, A1 = 0.0, A2 = 0.0;
  uint64_t n_ = 0;
  for (int64_t b = lane; b < nblk; b += 64) {
    const double* pp = part + kObPart * ((int64_t)c * nblk + b) * kObWaves;
    double b1 = pp[0], b2 = pp[1], c1 = pp[2], c2 = pp[3];
    n_ += (uint64_t)pp[4];
    for (int w = 1; w < kObWaves; ++w) {
      const double* q = pp + kObPart * w;
      b1 += q[0];
      b2 += q[1];
      c1 += q[2];
      c2 += q[3];
      n_ += (uint64_t)q[4];
    }
    S1 += b1;
    S2 += b2;
    A1 += c1;
    A2 += c2;
  }
  S1 = wave_sum_f64(S1);
  S2 = wave_sum_f64(S2);
  A1 = wave_sum_f64(A1);
  A2 = wave_sum_f64(A2);
  n_ = (uint64_t)wave_sum_i((int32_t)n_);
  if (lane != 0) return;
  {
    float mb, ma;
    double d_;
    if (KIND == 0) {
      const double B1 = S1 - A1, B2 = S2 - A2;
      const double nb = (double)(P - (int64_t)n_), nab = (double)n_;
      mb = (float)B1 / fmaxf((float)(P - (int64_t)n_), 1.0f);
      ma = (float)A1 / fmaxf((float)n_, 1.0f);
      const double mad = ma, mbd = mb;
      d_ = (A2 - 2.0 * mad * A1 + nab * mad * mad) + (B2 - 2.0 * mbd * B1 + nb * mbd * mbd);
    } else {
      const float norm1 = (float)S1;
      float scale;
      if (min_distortion) {
        scale = norm1 / (float)P;  // drive.py:61-62
      } else {
        const float norm2 = (float)sqrt(S2);
        const float n2sq = norm2 * norm2;
        scale = norm1 == 0.0f ? 0.0f : n2sq / norm1;  // drive.py:63-65 (divide_no_nan)
      }
      mb = -scale;
      ma = scale;
      const double sd = scale;
      // sum over x >= 0 of (x - s)^2 plus over x < 0 of (x + s)^2 = sum (|x| - s)^2
      d_ = S2 - 2.0 * sd * S1 + (double)P * sd * sd;
    }
    means[2 * c] = mb;
    means[2 * c + 1] = ma;
    // The expansion cancels when the spread is tiny next to the values (e.g. x =
    // 1000 +- 1e-3): its float64 rounding (~1e-16 S2 per add) is then no longer
    // small against the distortion.  Such a client is flagged (-1) and
    // k_mask_distortion recomputes sum (x - decoded)^2 term by term, as TF does.
    dist[c] = (d_ > kObCancel * S2) ? d_ : (S2 > 0.0 ? -1.0 : 0.0);
  }
}

// Exact distortion of the clients k_mask_encode flagged (dist[c] < 0): one
// workgroup per client, every term (x - decoded)^2 from the float32 difference
// (one_bit_sgd.py:76-78 / drive.py:69-70), float64 sums in a fixed order.
// Unflagged clients exit at once.
template <int KIND>
__global__ __launch_bounds__(kObThreads) void k_mask_distortion(const float* const* xs, int64_t P, float thr,
                                                                const float* means, double* dist) {
  __shared__ double red[kObWaves];
  const int c = blockIdx.x;
  if (!(dist[c] < 0.0)) return;
  const float* __restrict__ x = xs[c];
  const float mb = means[2 * c], ma = means[2 * c + 1];
  double s = 0.0;
  for (int64_t e = threadIdx.x; e < P; e += kObThreads) {
    const float v = x[e] + 0.0f;
    const float dec = KIND == 0 ? (!(v < thr) ? ma : mb) : (v < 0.0f ? mb : ma);
    const double d = (double)(v - dec);
    s = fma(d, d, s);
  }
  s = wave_sum_f64(s);
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  if (lane == 0) red[wv] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    double t = 0.0;
    for (int w = 0; w < kObWaves; ++w) t += red[w];
    dist[c] = t;
  }
}

// Server sum (one_bit_sgd.py:87-112): one thread per mask word (32 elements);
// clients in order, each decoded value exactly mask ? mean_above : mean_below
// (TF's mask * ma + (1 - mask) * mb), summed in float32 as the reference's
// accumulator.  The select is one bitop3 on the float bits.
__global__ __launch_bounds__(256) void k_onebit_decode_sum(const uint32_t* masks, const float* means, int32_t n,
                                                           int64_t P, int64_t w_begin, int64_t w_end, float* out) {
  const int64_t w = w_begin + (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t nw = (P + 31) / 32;
  if (w >= w_end) return;
  float s[32];
#pragma unroll
  for (int k = 0; k < 32; ++k) s[k] = 0.0f;
  for (int c = 0; c < n; ++c) {
    const uint32_t bits = masks[(int64_t)c * nw + w];
    const uint32_t mb = __float_as_uint(means[2 * c]), ma = __float_as_uint(means[2 * c + 1]);
    const uint32_t dx = ma ^ mb;
#pragma unroll
    for (int k = 0; k < 32; ++k) {
      const uint32_t sel = (uint32_t)(((int32_t)(bits << (31 - k))) >> 31);  // all ones if bit k
      s[k] = s[k] + __uint_as_float(mb ^ (dx & sel));
    }
  }
  const int64_t e0 = w * 32;
#pragma unroll
  for (int k = 0; k < 32; ++k)
    if (e0 + k < P) out[e0 + k] = s[k];
}


// ---------------------------------------------------------------------------
// Step-size vote (quantize_encode_client_lambda.py:105-130): for every client
// and every step option, the distortion and the exact run-length-gamma code
// length of its quantisation -- lengths only, nothing is packed.  The TF
// stateless stream is drawn once per element and shared by all options (the
// reference re-draws the same stream with the same seed for each option).
// Pass 1 (k_vote_tiles): one wave per (client, 1024-element tile) computes, per
// option, the tile's body bits (every code after its first nonzero's run code),
// first / last nonzero and distortion.  Pass 2 (k_vote_finalize): one
// workgroup per (client, option) stitches the tiles (run code of each tile's
// first nonzero from the last nonzero before it, trailing zero run).
// ---------------------------------------------------------------------------
struct VoteRec {
  uint32_t body;
  int32_t first, last;
  float dist;
};

struct VoteArgs {
  const float* const* xs;
  int32_t nclients;
  int64_t P;
  int32_t T;
  int32_t K;
  const float* steps;  // [K]
  const int64_t* seeds;  // [2 * nclients]
  VoteRec* rec;          // [nclients][K][T]
  int64_t* bits;         // [nclients * K]
  double* dist;          // [nclients * K]
};

template <int MODE>
__global__ __launch_bounds__(64) void k_vote_tiles(VoteArgs a) {
  const int lane = threadIdx.x;
  const int64_t total = (int64_t)a.nclients * a.T;
  for (int64_t tk = blockIdx.x; tk < total; tk += gridDim.x) {
    const int32_t c = (int32_t)(tk / a.T);
    const int32_t t = (int32_t)(tk - (int64_t)c * a.T);
    const int64_t tile_base = (int64_t)t * kTE;
    const float* x = a.xs[c];
    float xv[16];
    uint32_t rb[16];
    if (tile_base + kTE <= a.P && ((uintptr_t)x & 15u) == 0) {  // full, aligned tile: 4 x 16 B per lane
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const float4 v = *(const float4*)(x + tile_base + 16 * lane + 4 * g);
        xv[4 * g] = v.x; xv[4 * g + 1] = v.y; xv[4 * g + 2] = v.z; xv[4 * g + 3] = v.w;
      }
    } else {
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int64_t e = tile_base + 16 * lane + i;
        xv[i] = e < a.P ? x[e] : 0.0f;
      }
    }
    Key4 key{0, 0, 0, 0};
    if (MODE != FC_UNIFORM) {
      key = tf_seed_scramble(a.seeds[2 * c], a.seeds[2 * c + 1]);
      key.k0 = __builtin_amdgcn_readfirstlane(key.k0);  // wave-uniform: scalar-unit round keys
      key.k1 = __builtin_amdgcn_readfirstlane(key.k1);
      key.c2 = __builtin_amdgcn_readfirstlane(key.c2);
      key.c3 = __builtin_amdgcn_readfirstlane(key.c3);
    }
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      uint4 r = make_uint4(0, 0, 0, 0);
      if (MODE != FC_UNIFORM) r = philox_group_u(key, (uint32_t)((tile_base + 16 * lane + 4 * g) >> 2));
      rb[4 * g] = r.x; rb[4 * g + 1] = r.y; rb[4 * g + 2] = r.z; rb[4 * g + 3] = r.w;
    }
    for (int k = 0; k < a.K; ++k) {
      const float step = a.steps[k];
      float dist = 0.0f;
      int32_t lfirst = -1, prev = -1;
      uint32_t len = 0;
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int32_t rel = 16 * lane + i;
        const bool valid = tile_base + rel < a.P;
        float deq, noise;
        int32_t q = quantize_one<MODE>(xv[i], step, 0.0f, rb[i], deq, noise);
        const float dd = xv[i] - deq;
        dist = valid ? dist + dd * dd : dist;
        q = valid ? q : 0;
        if (q != 0) {
          uint32_t L = 1u + glen(mag_u32(q));
          if (prev >= 0) L += glen((uint32_t)(rel - prev));
          else lfirst = rel;
          len += L;
          prev = rel;
        }
      }
      const int32_t im = dpp_incl_max(prev);
      const int32_t lprev = dpp_shr1(im, -1);
      const uint32_t R = (lfirst >= 0 && lane > 0 && lprev >= 0) ? glen((uint32_t)(lfirst - lprev)) : 0u;
      const uint32_t body = (uint32_t)wave_sum_i((int32_t)(len + R));
      const float d = wave_sum_f(dist);
      const uint64_t fm = __ballot(lfirst >= 0);
      const int32_t tfirst = __builtin_amdgcn_readlane(lfirst, fm ? (int)__builtin_ctzll(fm) : 0);
      const int32_t tlast = lane63(im);
      if (lane == 0) {
        VoteRec r;
        r.body = body;
        r.first = fm ? tfirst : -1;
        r.last = tlast;
        r.dist = d;
        a.rec[((int64_t)c * a.K + k) * a.T + t] = r;
      }
    }
  }
}

__global__ __launch_bounds__(256) void k_vote_finalize(VoteArgs a) {
  __shared__ int64_t carry[256];
  __shared__ unsigned long long rbits[256];
  __shared__ double rdist[256];
  const int tid = threadIdx.x;
  const int64_t ck = blockIdx.x;
  const VoteRec* rec = a.rec + ck * a.T;
  const int32_t chunk = (a.T + 255) / 256;
  const int32_t t0 = min(a.T, tid * chunk), t1 = min(a.T, t0 + chunk);
  int64_t mylast = -1;
  for (int32_t t = t0; t < t1; ++t)
    if (rec[t].last >= 0) mylast = (int64_t)t * kTE + rec[t].last;
  carry[tid] = mylast;
  __syncthreads();
  if (tid == 0) {  // exclusive prefix max over threads (tiles are in thread order)
    int64_t m = -1;
    for (int i = 0; i < 256; ++i) {
      const int64_t v = carry[i];
      carry[i] = m;
      m = v > m ? v : m;
    }
  }
  __syncthreads();
  int64_t prevlast = carry[tid];
  unsigned long long b = 0;
  double dd = 0.0;
  for (int32_t t = t0; t < t1; ++t) {
    const VoteRec r = rec[t];
    b += r.body;
    dd += (double)r.dist;
    if (r.first >= 0) {
      b += glen((uint32_t)((int64_t)t * kTE + r.first - prevlast));
      prevlast = (int64_t)t * kTE + r.last;
    }
  }
  rbits[tid] = b;
  rdist[tid] = dd;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (tid < o) {
      rbits[tid] += rbits[tid + o];
      rdist[tid] += rdist[tid + o];
    }
    __syncthreads();
  }
  if (tid == 0) {
    unsigned long long total = rbits[0];
    int64_t L = -1;  // the overall last nonzero
    for (int32_t t = a.T - 1; t >= 0; --t)
      if (rec[t].last >= 0) { L = (int64_t)t * kTE + rec[t].last; break; }
    if (a.P - 1 - L > 0) total += glen((uint32_t)(a.P - L));  // trailing zero run
    a.bits[ck] = (int64_t)total;
    a.dist[ck] = rdist[0];
  }
}

// ---------------------------------------------------------------------------
// Randomized Hadamard rotation (the TFF HadamardTransformFactory wrapper that
// builder.py:68-71 puts around a codec): y = H D x / sqrt(n) on zero-padded
// length n = 2^k, D = Rademacher signs drawn from Philox4x32-10 of the round
// seed (element i: bit 31 of output word i % 4 of counter i / 4); the inverse
// is x = D H y / sqrt(n).  One pass does up to 12 butterfly levels of a 4096-
// element group in LDS: pass 0 covers levels 0..11 of contiguous blocks, later
// passes levels L0..L0+k-1 of groups of C = 4096 / 2^k consecutive columns by
// 2^k rows at stride 2^L0 (rows are C * 4 bytes contiguous).
// ---------------------------------------------------------------------------
__device__ __forceinline__ float rademacher(const Key4& key, int64_t i) {
  const uint4 r = philox_group(key, (uint32_t)(i >> 2));
  const uint32_t w = (i & 3) == 0 ? r.x : (i & 3) == 1 ? r.y : (i & 3) == 2 ? r.z : r.w;
  return (w >> 31) ? -1.0f : 1.0f;
}

__device__ __forceinline__ float sign_of(uint32_t w) { return (w >> 31) ? -1.0f : 1.0f; }

__global__ __launch_bounds__(256) void k_fwht_pass(float* const* rows, int64_t n, int L0, int k, int sign_in,
                                                   int sign_out, float scale, int64_t seed0, int64_t seed1) {
  __shared__ __attribute__((aligned(16))) float buf[4096];
  // every size is a power of two: index arithmetic by shifts and masks
  const int lg = L0 == 0 ? k : 12;                 // log2 group size
  const int lC = lg - k;                           // log2 consecutive columns per group
  const int64_t gsize = (int64_t)1 << lg;
  const int64_t C = (int64_t)1 << lC;
  const int lrow = 63 - __clzll((unsigned long long)(n >> lg));  // log2 groups per client row
  const int64_t c = (int64_t)blockIdx.x >> lrow;
  const int64_t g = (int64_t)blockIdx.x & (((int64_t)1 << lrow) - 1);
  const int lnblk = L0 - lC;                       // log2 column blocks below the levels (pass > 0)
  const int64_t hi = L0 == 0 ? g : g >> lnblk, cb = L0 == 0 ? 0 : g & (((int64_t)1 << lnblk) - 1);
  const int64_t base = L0 == 0 ? g << lg : (hi << (L0 + k)) + (cb << lC);
  float* x = rows[c];
  const Key4 key = tf_seed_scramble(seed0, seed1);
  // element of group index t: row t >> lC at stride 2^L0, column t & (C - 1)
  if (gsize >= 1024) {  // 4 consecutive elements per thread (C >= 4): float4 and one Philox group
    for (int64_t t = 4 * threadIdx.x; t < gsize; t += 1024) {
      const int64_t e = base + ((t >> lC) << L0) + (t & (C - 1));
      float4 v = *(const float4*)(x + e);
      if (sign_in) {
        const uint4 r = philox_group(key, (uint32_t)(e >> 2));
        v.x *= sign_of(r.x); v.y *= sign_of(r.y); v.z *= sign_of(r.z); v.w *= sign_of(r.w);
      }
      *(float4*)(buf + t) = v;
    }
  } else {
    for (int64_t t = threadIdx.x; t < gsize; t += 256) {
      const int64_t e = base + ((t >> lC) << L0) + (t & (C - 1));
      float v = x[e];
      if (sign_in) v *= rademacher(key, e);
      buf[t] = v;
    }
  }
  __syncthreads();
  for (int j = 0; j < k; ++j) {
    const int lh = lC + j;  // partner distance 2^lh in buf
    const int64_t h = (int64_t)1 << lh;
    for (int64_t b2 = threadIdx.x; b2 < gsize / 2; b2 += 256) {
      const int64_t lo = ((b2 >> lh) << (lh + 1)) + (b2 & (h - 1));
      const float u = buf[lo], w = buf[lo + h];
      buf[lo] = u + w;
      buf[lo + h] = u - w;
    }
    __syncthreads();
  }
  if (gsize >= 1024) {
    for (int64_t t = 4 * threadIdx.x; t < gsize; t += 1024) {
      const int64_t e = base + ((t >> lC) << L0) + (t & (C - 1));
      float4 v = *(const float4*)(buf + t);
      v.x *= scale; v.y *= scale; v.z *= scale; v.w *= scale;
      if (sign_out) {
        const uint4 r = philox_group(key, (uint32_t)(e >> 2));
        v.x *= sign_of(r.x); v.y *= sign_of(r.y); v.z *= sign_of(r.z); v.w *= sign_of(r.w);
      }
      *(float4*)(x + e) = v;
    }
  } else {
    for (int64_t t = threadIdx.x; t < gsize; t += 256) {
      const int64_t e = base + ((t >> lC) << L0) + (t & (C - 1));
      float v = buf[t] * scale;
      if (sign_out) v *= rademacher(key, e);
      x[e] = v;
    }
  }
}

// Measurement utility (bench.py): a 16-byte-per-lane grid-stride copy, the
// achievable HBM streaming rate the codec kernels are compared with.  Each lane
// keeps FC_COPY_U 16-B loads in flight (all issued before the stores); FC_COPY_NT
// makes the loads and stores non-temporal.
#ifndef FC_COPY_U
#define FC_COPY_U 8  // profiles/r05/copy_*.json: 4 / 8 loads in flight, plain / nt: 4.97 / 5.19 / 5.23 / 5.35 TB/s
#endif
#ifndef FC_COPY_NT
#define FC_COPY_NT 1
#endif
__global__ __launch_bounds__(256) void k_copy_f4(uint4* __restrict__ dst_, const uint4* __restrict__ src_, int64_t n) {
  typedef uint32_t v4u __attribute__((ext_vector_type(4)));
  v4u* __restrict__ dst = (v4u*)dst_;
  const v4u* __restrict__ src = (const v4u*)src_;
  constexpr int U = FC_COPY_U;
  const int64_t stride = (int64_t)gridDim.x * 256 * U;
  int64_t i = (int64_t)blockIdx.x * 256 * U + threadIdx.x;
  for (; i + 256 * (U - 1) < n; i += stride) {
    v4u v[U];
#pragma unroll
    for (int k = 0; k < U; ++k) v[k] = FC_COPY_NT ? __builtin_nontemporal_load(src + i + 256 * k) : src[i + 256 * k];
#pragma unroll
    for (int k = 0; k < U; ++k) {
      if (FC_COPY_NT) __builtin_nontemporal_store(v[k], dst + i + 256 * k);
      else dst[i + 256 * k] = v[k];
    }
  }
  for (; i < n; i += 256) dst[i] = src[i];
}

// Test utility (tests/test_gpu_progress.py): a workgroup holding a whole CU (all
// 160 KiB of LDS) for `ticks` of the 100 MHz real-time clock when its XCD's bit is
// set in xcd_mask (HW_REG_XCC_ID; the others exit at once) -- another kernel then
// cannot place a workgroup on the masked XCDs until it ends.  Bounded: every wave
// leaves after `ticks`.  `held` (nullable) counts the workgroups that held a CU.
__global__ __launch_bounds__(64) void k_occupy(uint32_t xcd_mask, uint64_t ticks, int32_t* held) {
  __shared__ uint32_t pin[40960];  // 160 KiB: one workgroup per CU
  uint32_t xcc;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
  if (!((xcd_mask >> (xcc & 7u)) & 1u)) return;
  pin[threadIdx.x] = threadIdx.x;
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(127);
  __syncthreads();
  if (threadIdx.x == 0 && held && pin[63] == 63u) atomicAdd(held, 1);
}

// Rademacher sign flip (the DFT rotation's D, the same stream as k_fwht_pass's):
// rows[c][i] *= sign of bit 31 of Philox output word i % 4 of counter i / 4.
__global__ __launch_bounds__(256) void k_sign_flip(float* const* rows, int64_t n, Key4 key) {
  float* x = rows[blockIdx.y];
  const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;  // 4-element group
  if (4 * g >= n) return;
  const uint4 r = philox_group(key, (uint32_t)g);
  const uint32_t w[4] = {r.x, r.y, r.z, r.w};
#pragma unroll
  for (int k = 0; k < 4; ++k)
    if (4 * g + k < n) x[4 * g + k] *= sign_of(w[k]);
}

// ---------------------------------------------------------------------------
// DFT rotation (tff.aggregators.DiscreteFourierTransformFactory, builder.py:70-71):
// the unitary DFT of the m = n / 2 complex numbers z_k = x[k] + i x[k + m], written
// back as (real, imaginary) halves.  Power-of-two lengths run a Stockham FFT
// directly; any other length goes through Bluestein's chirp-z identity
//   Z_j = c_j sum_k (z_k c_k) conj(c_{j-k}),  c_k = exp(-i pi k^2 / m),
// a circular convolution of length L = 2^ceil(log2(2m - 1)) done by two forward
// FFTs and one inverse.  The FFT is a sequence of out-of-place Stockham passes
// of radix 16 (a last pass of radix 2, 4 or 8): thread j reads the 16 elements
// j + r N / 16 (coalesced across threads), twiddles them by exp(-+2 pi i k r /
// (Ns 16)), k = j mod Ns, transforms them in registers and writes them to
// (j - k) 16 + k + r Ns -- natural order after the last pass, no bit reversal.
// The chirps reduce k^2 modulo 2m in integer arithmetic before the sine.
// ---------------------------------------------------------------------------
__device__ __forceinline__ float2 cmul(float2 a, float2 b) {
  return make_float2(a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x);
}

// In-register radix-2 DIT DFT of R points (R a power of two <= 16), direction sign
// (-1 forward, +1 inverse); the twiddles are compile-time constants.
template <int R>
__device__ __forceinline__ void dft_reg(float2 (&v)[R], float sign) {
  constexpr int LG = R == 2 ? 1 : R == 4 ? 2 : R == 8 ? 3 : 4;
#pragma unroll
  for (int i = 0; i < R; ++i) {
    int rv = 0;
#pragma unroll
    for (int b = 0; b < LG; ++b) rv |= ((i >> b) & 1) << (LG - 1 - b);
    if (i < rv) {
      const float2 t = v[i];
      v[i] = v[rv];
      v[rv] = t;
    }
  }
  // cos / sin of 2 pi j / 16, j = 0..15
  constexpr float kc[16] = {1.0f, 0.92387953251128674f, 0.70710678118654752f, 0.38268343236508977f,
                            0.0f, -0.38268343236508977f, -0.70710678118654752f, -0.92387953251128674f,
                            -1.0f, -0.92387953251128674f, -0.70710678118654752f, -0.38268343236508977f,
                            0.0f, 0.38268343236508977f, 0.70710678118654752f, 0.92387953251128674f};
  constexpr float ks[16] = {0.0f, 0.38268343236508977f, 0.70710678118654752f, 0.92387953251128674f,
                            1.0f, 0.92387953251128674f, 0.70710678118654752f, 0.38268343236508977f,
                            0.0f, -0.38268343236508977f, -0.70710678118654752f, -0.92387953251128674f,
                            -1.0f, -0.92387953251128674f, -0.70710678118654752f, -0.38268343236508977f};
#pragma unroll
  for (int len = 2; len <= R; len <<= 1) {
#pragma unroll
    for (int i = 0; i < R; i += len) {
#pragma unroll
      for (int k = 0; k < len / 2; ++k) {
        const int t = k * (16 / len);  // exp(sign 2 pi i k / len) = table entry k * 16 / len
        const float2 w = make_float2(kc[t], sign * ks[t]);
        const float2 a = v[i + k];
        const float2 b = k == 0 ? v[i + k + len / 2] : cmul(v[i + k + len / 2], w);
        v[i + k] = make_float2(a.x + b.x, a.y + b.y);
        v[i + k + len / 2] = make_float2(a.x - b.x, a.y - b.y);
      }
    }
  }
}

// One Stockham pass of radix R over N points (N / R threads), sub-transforms of Ns.
template <int R>
__global__ __launch_bounds__(256) void k_fft_pass(const float2* __restrict__ src, float2* __restrict__ dst, int64_t N,
                                                  int64_t Ns, float sign) {
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t q = N / R;
  if (j >= q) return;
  const int64_t k = j & (Ns - 1);
  float2 v[R];
#pragma unroll
  for (int r = 0; r < R; ++r) v[r] = src[j + r * q];
  if (Ns > 1) {
    // exp(sign 2 pi i k / (Ns R)), its powers by complex multiplies
    float sn, cs;
    sincospif(2.0f * (float)((double)k / (double)(Ns * R)), &sn, &cs);
    const float2 w1 = make_float2(cs, sign * sn);
    float2 w = w1;
#pragma unroll
    for (int r = 1; r < R; ++r) {
      v[r] = cmul(v[r], w);
      w = cmul(w, w1);
    }
  }
  dft_reg<R>(v, sign);
  const int64_t o = (j - k) * R + k;
#pragma unroll
  for (int r = 0; r < R; ++r) dst[o + r * Ns] = v[r];
}

// c_k = exp(-i pi k^2 / m) (conjugated: +i), k^2 reduced modulo 2m exactly.
__device__ __forceinline__ float2 chirp(int64_t k, int64_t m, bool conj_) {
  const uint64_t q = (uint64_t)((unsigned __int128)(uint64_t)k * (uint64_t)k % (unsigned __int128)(2 * m));
  double sn, cs;
  sincospi((double)q / (double)m, &sn, &cs);
  return make_float2((float)cs, conj_ ? (float)sn : (float)-sn);
}

// a_k = z_k (c_k) for k < m (inverse: conj(z_k) first), zero up to L.
__global__ __launch_bounds__(256) void k_dft_pre(float* const* rows, int32_t c, int64_t m, int64_t L, int bluestein,
                                                 int conj_in, float2* __restrict__ a) {
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= L) return;
  const float* __restrict__ x = rows[c];
  float2 z = make_float2(0.0f, 0.0f);
  if (k < m) {
    z = make_float2(x[k], conj_in ? -x[k + m] : x[k + m]);
    if (bluestein) z = cmul(z, chirp(k, m, false));
  }
  a[k] = z;
}

// b_l = conj(c_l) on l in (-m, m) arranged circularly over L.
__global__ __launch_bounds__(256) void k_dft_bvec(int64_t m, int64_t L, float2* __restrict__ b) {
  const int64_t l = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (l >= L) return;
  float2 v = make_float2(0.0f, 0.0f);
  if (l < m) v = chirp(l, m, true);
  else if (l > L - m) v = chirp(L - l, m, true);
  b[l] = v;
}

__global__ __launch_bounds__(256) void k_cmul(float2* __restrict__ a, const float2* __restrict__ b, int64_t n) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) a[i] = cmul(a[i], b[i]);
}

// x[j] = Re(w_j), x[j + m] = Im(w_j), w_j = (c_j) conv_j scale (inverse: conjugated).
__global__ __launch_bounds__(256) void k_dft_post(const float2* __restrict__ conv, int64_t m, int bluestein,
                                                  float scale, int conj_out, float* const* rows, int32_t c) {
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= m) return;
  float* __restrict__ x = rows[c];
  float2 w = conv[j];
  if (bluestein) w = cmul(w, chirp(j, m, false));
  x[j] = w.x * scale;
  x[j + m] = (conj_out ? -w.y : w.y) * scale;
}

// k_sign_flip for one row given directly (the DFT rotation's per-row loop).
__global__ __launch_bounds__(256) void k_sign_flip_row(float* const* rows, int32_t c, int64_t n, Key4 key) {
  const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (4 * g >= n) return;
  float* x = rows[c];
  const uint4 r = philox_group(key, (uint32_t)g);
  const uint32_t w[4] = {r.x, r.y, r.z, r.w};
#pragma unroll
  for (int k = 0; k < 4; ++k)
    if (4 * g + k < n) x[4 * g + k] *= sign_of(w[k]);
}

// Measurement kernel (not a reference interface; fc_quantize_floor): the encoder's
// arithmetic floor -- read x, draw TF's Philox4x32-10 stream, the exact quantiser
// (pow2 step: x * (1 / step); floor, ceil, Uint32ToFloat, compare, select; rintf
// uniform) and the distortion FMA and nonzero count per 1024-element tile, with no
// code construction, scan, look-back, emission or stores beyond two words per tile.
// Persistent waves over tile-major tickets like the encoder's, keys per client
// precomputed (k_floor_keys), all four chunk loads of a tile in flight at once.
__global__ void k_floor_keys(const int64_t* seeds, int32_t C, uint4* keys) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  const Key4 k = tf_seed_scramble(seeds[2 * c], seeds[2 * c + 1]);
  keys[c] = make_uint4(k.k0, k.k1, k.c2, k.c3);
}

// Streaming form (round 5): one client per blockIdx.y, its tiles cut into
// gridDim.x parts (part_range); the client's row pointer and Philox key are
// loaded once per workgroup (scalar), each wave walks its part's tiles with the
// next tile's four float4 loads in flight while a tile computes (registers,
// double-buffered), and nothing but two words per tile is stored.
template <int MODE, int DEPTH>
__global__ __launch_bounds__(256) void k_quant_floor(const float* const* xs, int64_t P, int32_t T, float rcp,
                                                     const uint4* keys, float* dist_part, int32_t* nnz_part) {
  const int lane = threadIdx.x & 63;
  const int wv = (int)uniform(threadIdx.x >> 6);
  const int c = blockIdx.y;
  typedef float f4v __attribute__((ext_vector_type(4)));
  typedef const __attribute__((address_space(1))) f4v* gf4ptr;
  const gf4ptr x = (gf4ptr)xs[c];
  const uint4 kk = keys[c];
  const Key4 key{uniform(kk.x), uniform(kk.y), uniform(kk.z), uniform(kk.w)};
  int64_t tlo, thi;
  part_range(T, (int)blockIdx.x, (int)gridDim.x, tlo, thi);
  auto load = [&](int64_t t, f4v (&v)[4]) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int64_t e0 = t * kTE + 4 * (64 * j + lane);
      v[j] = e0 + 3 < P ? x[e0 >> 2] : f4v{0.f, 0.f, 0.f, 0.f};
    }
  };
  auto tile = [&](int64_t t, const f4v (&v)[4]) {
    float dist = 0.0f;
    uint32_t nnz = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const uint32_t g = (uint32_t)((t * kTE) >> 2) + 64 * j + lane;
      uint4 rb = make_uint4(0, 0, 0, 0);
      if (MODE != FC_UNIFORM) rb = philox_group_u(key, g);
      const float xv[4] = {v[j].x, v[j].y, v[j].z, v[j].w};
      const uint32_t rr[4] = {rb.x, rb.y, rb.z, rb.w};
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const float sc = xv[k] * rcp;
        float r;
        if (MODE == FC_UNIFORM) {
          r = rintf(sc);
        } else {
          const float fl = floorf(sc);
          r = (u01(rr[k]) <= sc - fl) ? ceilf(sc) : fl;
        }
        const float dd = sc - r;
        dist = fmaf(dd, dd, dist);
        nnz += (uint32_t)__popcll(__ballot(r != 0.0f));  // scalar unit
      }
    }
    const float d = wave_sum_f(dist);
    if (lane == 0) {
      dist_part[(int64_t)c * T + t] = d;
      nnz_part[(int64_t)c * T + t] = (int32_t)nnz;
    }
  };
  f4v va[4], vb[4], vc[4];
  const int nw = (int)(blockDim.x >> 6);
  int64_t t = tlo + wv;
  if (DEPTH == 2) {  // the next tile's loads in flight while a tile computes
    if (t < thi) load(t, va);
    for (; t < thi; t += 2 * nw) {
      const int64_t tn = t + nw;
      if (tn < thi) load(tn, vb);
      tile(t, va);
      if (tn >= thi) break;
      if (tn + nw < thi) load(tn + nw, va);
      tile(tn, vb);
    }
  } else {  // the next two tiles' loads in flight
    if (t < thi) load(t, va);
    if (t + nw < thi) load(t + nw, vb);
    for (; t < thi; t += 3 * nw) {
      if (t + 2 * nw < thi) load(t + 2 * nw, vc);
      tile(t, va);
      if (t + nw >= thi) break;
      if (t + 3 * nw < thi) load(t + 3 * nw, va);
      tile(t + nw, vb);
      if (t + 2 * nw >= thi) break;
      if (t + 4 * nw < thi) load(t + 4 * nw, vb);
      tile(t + 2 * nw, vc);
    }
  }
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

// Library-owned device scratch for small per-launch partials (the client-split
// reductions), one grow-only buffer per (device, stream): calls on one stream run
// in order, so a stream's buffer is never used by two launches at once.  Growing
// it allocates (and frees the old buffer after a sync of the stream), which a
// stream under graph capture does not allow: there the call fails unless the buffer
// is already large enough (warm it with one uncaptured call of the same size).
int scratch_for(hipStream_t s, size_t bytes, void** out) {
  static std::mutex mu;
  static std::map<std::pair<int, hipStream_t>, std::pair<void*, size_t>> bufs;
  *out = nullptr;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return fail(-10, "scratch: hipGetDevice");
  std::lock_guard<std::mutex> g(mu);
  std::pair<void*, size_t>& b = bufs[std::make_pair(dev, s)];
  if (b.second < bytes) {
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(s, &cs) != hipSuccess || cs != hipStreamCaptureStatusNone)
      return fail(-1, "client-split scratch must grow, which is not possible while the stream is captured: "
                      "run the call once uncaptured first");
    if (b.first) {
      (void)hipStreamSynchronize(s);  // the old buffer may still be read by this stream's last launch
      (void)hipFree(b.first);
      b.first = nullptr;
      b.second = 0;
    }
    const size_t want = std::max<size_t>(bytes, 64 << 10);
    if (hipMalloc(&b.first, want) != hipSuccess) {
      b.first = nullptr;
      return fail(-3, "scratch allocation failed");
    }
    b.second = want;
  }
  *out = b.first;
  return 0;
}

// Workgroups per client for the per-client streaming passes (k_client_norms,
// k_mask_encode): about `per_cu` workgroups per CU in all, each part at least 64
// tiles of 2048 elements.  1024 clients: one each (as before the split).
int client_parts(int32_t nclients, int64_t ntile, int per_cu) {
  int dev = 0, ncu = 256;
  (void)hipGetDevice(&dev);
  (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
  int mult = 1;
  if (const char* e = getenv("FEDCODEC_PARTS_MULT")) mult = std::max(1, atoi(e));  // test knob
  const int64_t want = ((int64_t)per_cu * mult * ncu + nclients - 1) / nclients;
  return (int)std::max<int64_t>(1, std::min<int64_t>(want, ntile / 64));
}

template <int KIND>
int launch_mask_encode(const float* const* xs, int32_t nclients, int64_t P, float thr, int min_distortion,
                       uint32_t* masks, float* means, double* dist, hipStream_t s) {
  // four times the co-resident workgroups (parts per client): the last ones finish
  // together instead of one long row each (1024 x 25 M -4.5 %, 128 clients -7 %,
  // profiles/r05/diag_parts_mult.txt)
  const int64_t nblk = red_blocks(P);
  int parts = client_parts(nclients, (P + 2047) / 2048, 16);
  if (const char* e = getenv("FEDCODEC_OB_PARTS")) parts = std::max(1, atoi(e));  // test knob
  parts = (int)std::min<int64_t>(parts, nblk);
  double* part = nullptr;
  if (const int rc = scratch_for(s, sizeof(double) * kObPart * kObWaves * (size_t)nclients * nblk, (void**)&part))
    return rc;
  hipLaunchKernelGGL(k_mask_encode<KIND>, dim3((unsigned)parts, (unsigned)nclients), dim3(kObThreads), 0, s, xs, P,
                     thr, masks, part);
  if (const int rc = check_launch("k_mask_encode")) return rc;
  hipLaunchKernelGGL(k_mask_finalize<KIND>, dim3((unsigned)nclients), dim3(64), 0, s, (const double*)part,
                     nclients, (int32_t)nblk, P, min_distortion, means, dist);
  return check_launch("k_mask_finalize");
}


// Workspace: [status n*T*16][header: ticket shards, spin_err, counter2,
// slow_count, start heads][slow_flag n*4] (all zeroed per launch) [slow_list n*4]
// [ClientParam n*64].
constexpr int kHdrWords = kShardStride * (kTicketShards + 3 + kStartHeads);
int64_t enc_status_bytes(int32_t n, int64_t P) { return (int64_t)n * tiles_for(P) * 16; }
int64_t enc_zeroed_bytes(int32_t n, int64_t P) {
  return enc_status_bytes(n, P) + 4 * kHdrWords + 4 * (int64_t)n;
}
int64_t enc_params_offset(int32_t n, int64_t P) {
  return (enc_zeroed_bytes(n, P) + 4 * (int64_t)n + 255) & ~255LL;
}
int64_t enc_workspace_bytes(int32_t n, int64_t P) {
  return enc_params_offset(n, P) + (int64_t)n * (int64_t)sizeof(ClientParam);
}

// Quarter-tile decoder entries: the encoder's tile-relative records (quarter_rel)
// rebased on the tile's own entry -- the stream bit where the tile's codes start and
// its predecessor nonzero -- after the tile's leading run code.  A quarter with no
// nonzero of the tile before it starts where the tile does.
__global__ void k_quarter_index(const uint64_t* __restrict__ idx, uint64_t* __restrict__ idxq, int32_t nclients,
                                int32_t T) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;  // c * T + t
  if (i >= (int64_t)nclients * T) return;
  const int64_t c = i / T, t = i - c * T;
  const uint64_t e = idx[c * (T + 1) + t];
  const uint64_t body = e & kMask36;
  const int64_t last = (int64_t)(e >> 36) - 1;
  const int64_t tile_base = t * kTE;
  for (int s = 0; s < 3; ++s) {
    const uint64_t r = idxq[3 * i + s];
    const int32_t prev = (int32_t)((r >> 24) & 0x7FFu) - 1;
    const int32_t first = (int32_t)((r >> 35) & 0x7FFu) - 1;
    uint64_t o = e;
    if (prev >= 0) {
      const uint32_t R0 = glen((uint32_t)(tile_base + first - last));
      o = ((body + R0 + (r & 0xFFFFFFu)) & kMask36) | ((uint64_t)(tile_base + prev + 1) << 36);
    }
    idxq[3 * i + s] = o;
  }
}

// The fast encoders' look-back spin limit (g_spin_limit): 2^24 polls, or the test knob
// FEDCODEC_SPIN_LIMIT; written to the device only when it changes (per device).
int set_spin_limit() {
  static std::mutex mu;
  static std::map<int, uint32_t> cur;
  uint32_t want = 1u << 24;
  if (const char* e = getenv("FEDCODEC_SPIN_LIMIT")) want = (uint32_t)std::max(1L, atol(e));  // test knob
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return fail(-10, "hipGetDevice");
  std::lock_guard<std::mutex> g(mu);
  auto it = cur.find(dev);
  if (it != cur.end() && it->second == want) return 0;
  if (hipMemcpyToSymbol(HIP_SYMBOL(g_spin_limit), &want, sizeof(want)) != hipSuccess)
    return fail(-10, "g_spin_limit");
  cur[dev] = want;
  return 0;
}

int encode_common(const void* const* xs, int32_t nclients, int64_t P, float step, const float* norms,
                  const float* prescale, const int64_t* seeds, int mode, bool int_in, uint8_t* stream_buf,
                  const int64_t* stream_off, const int64_t* stream_cap, uint64_t* idx,
                  int64_t* total_bits, float* dist_part, int32_t* nnz_part, int32_t* overflow,
                  void* workspace, int64_t workspace_bytes, void* stream, const int64_t* elem_off = nullptr,
                  int64_t max_cap = 0, uint64_t* idxq = nullptr) {
  if (nclients <= 0) return fail(-1, "nclients must be > 0");
  if (P <= 0 || P > FC_MAX_ROW_ELEMS)
    return fail(-1, "P must be in [1, 2^26 - 1] for one encoder row; longer tensors: fc_quantize_encode_segmented");
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
  EncodeArgs a;
  a.elem_off = elem_off;
  a.idxq = idxq;
  a.xs = xs;
  a.nclients = nclients;
  a.P = P;
  a.T = (int32_t)T;
  a.T2 = (int32_t)((T + 1) / 2);
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
  a.counter = (uint32_t*)((uint8_t*)workspace + sb);
  a.spin_err = a.counter + kShardStride * kTicketShards;
  a.counter2 = a.counter + kShardStride * (kTicketShards + 1);
  a.slow_count = a.counter + kShardStride * (kTicketShards + 2);
  a.started = a.counter + kShardStride * (kTicketShards + 3);
  a.slow_flag = (int32_t*)(a.counter + kHdrWords);
  if (const int rc = set_spin_limit()) return rc;
  a.by_block = 0;
  if (const char* e = getenv("FEDCODEC_TICKET_BLOCKIDX")) a.by_block = atoi(e) != 0;  // regression-test knob
  a.slow_list = a.slow_flag + nclients;
  a.cparams = (const uint8_t*)workspace + enc_params_offset(nclients, P);
  int dev = 0, ncu = 256;
  (void)hipGetDevice(&dev);
  (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
  const int64_t total = (int64_t)nclients * T;
  // few clients: cap the tiles in flight per client so look-back windows stay short
  // power-of-two step (no per-client normalisation): x / step == x * (1 / step)
  int ex = 0;
  // (step^2 normal too: the encoder's distortion partials are then step^2 times exact
  // sums of (x / step - r)^2)
  const bool pow2 = !int_in && !norms && std::frexp(step, &ex) == 0.5f && std::isnormal(1.0f / step) &&
                    std::isnormal(step * step) && std::isfinite(step * step);
  // a host-known step that is not a power of two: Markstein's correctly rounded
  // quotient from RN(1 / step) (not for an all-ones significand, where the
  // remainder x - q0 * step is not exact)
  uint32_t sbits = 0;
  std::memcpy(&sbits, &step, 4);
  const bool mark = !int_in && !norms && !pow2 && std::isnormal(step) && std::isnormal(1.0f / step) &&
                    (sbits & 0x7FFFFFu) != 0x7FFFFFu;
  a.rcp = (pow2 || mark) ? 1.0f / step : 0.0f;
  void (*kern)(EncodeArgs) = nullptr;
  void (*kern2)(EncodeArgs) = nullptr;
  void (*kern4)(EncodeArgs) = nullptr;
  void (*kern8)(EncodeArgs) = nullptr;
  void (*exact)(EncodeArgs) = nullptr;
  const bool pre = !int_in && prescale != nullptr;
#define FC_PICK(M, I, D, Q)                                                                       \
  (kern = k_encode<M, I, D, Q>, kern2 = k_encode2<M, I, D, Q, 2>, kern4 = k_encode2<M, I, D, Q, 4>, \
   kern8 = k_encode2<M, I, D, Q, 8>, exact = k_encode_exact<M, I, D == 1>)
#define FC_PICK2(M, D) (pre ? FC_PICK(M, false, D, true) : FC_PICK(M, false, D, false))
#define FC_PICK3(M) (pow2 ? FC_PICK2(M, 1) : mark ? FC_PICK2(M, 2) : FC_PICK2(M, 0))
  if (int_in) FC_PICK(FC_UNIFORM, true, 0, false);
  else if (mode == FC_UNIFORM) FC_PICK3(FC_UNIFORM);
  else if (mode == FC_STOCHASTIC) FC_PICK3(FC_STOCHASTIC);
  else FC_PICK3(FC_DITHERED);
#undef FC_PICK3
#undef FC_PICK2
#undef FC_PICK
  {  // ticket -> (tile, client) by multiply-high
    const uint32_t d = (uint32_t)nclients;
    uint32_t l = 0;
    while (l < 32 && (1ull << l) < d) ++l;
    a.div_l = l;
    a.div_m = l == 0 ? 0u : (uint32_t)((((1ull << 32) * ((1ull << l) - d)) / d) + 1);
  }
  if ((uint64_t)nclients * (uint64_t)T >= (1ull << 32)) return fail(-1, "too many tiles (nclients x tiles >= 2^32)");
  // Super-tiles (k_encode2) when few tiles of a client are in flight (many clients):
  // their look-back runs right after the super-tile's own aggregate, so with many
  // super-tiles of one client in flight it waits on predecessors still coding
  // (1024 x 25 M: 39.0 vs 40.8 ms; 512 x 25 M: 21.8 vs 21.2; 128 x 25 M: 10.4 vs 6.2)
  int per_cu0 = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu0, kern2, kEncThreads * kEnc2Waves, 0) != hipSuccess ||
      per_cu0 < 1)
    per_cu0 = 1;
  // four tiles per ticket (FEDCODEC_ENC_NT=4): the per-ticket work (ticket, status,
  // look-back, reductions, store set-up) paid once per 4096 elements; the window
  // (the same LDS) then holds about 7.4 bits per element before the exact path
  // by the caller's largest stream capacity (host-known): codes expected within
  // kNt4Bits bits per element (+ slack) take four-tile tickets; denser ones, or an
  // unknown capacity, two (a window overflow sends the client to the exact path)
  // (eight-tile tickets, FC_ENC2_WAVES 8: 1024 x 25 M stochastic 29.7 -> see DESIGN §5)
  const double hint_bits = max_cap > 0 ? (8.0 * (double)max_cap - 8.0 * 8192.0) / (double)P : 1e9;
  int nt = hint_bits <= kNt8Bits ? 8 : hint_bits <= kNt4Bits ? 4 : 2;
  if (const char* e = getenv("FEDCODEC_ENC_NT")) nt = atoi(e) == 8 && kNt8Bits > 0 ? 8 : atoi(e) == 4 ? 4 : 2;  // test knob
  // with four-tile tickets (and the chained pair table) from 512 clients on a full
  // chip: 512 x 25 M stochastic 22.1 (k_encode) -> 15.9 ms, uniform 19.6 -> 15.3
  // (profiles/r03/diag_enc512.txt); fewer clients are segmented (codec.auto_segments)
  const int64_t rows_per_wave = nt >= 4 ? 8 : 4;
  bool super = (int64_t)ncu * per_cu0 * kEnc2Waves <= rows_per_wave * nclients && T >= 2;
  if (const char* e = getenv("FEDCODEC_ENC2")) super = atoi(e) != 0;  // test knob
  if (idxq) super = false;  // quarter-tile entries come from the one-tile kernel (few clients)
  if (super) {
    kern = nt == 8 ? kern8 : nt == 4 ? kern4 : kern2;
    a.T2 = (int32_t)((T + nt - 1) / nt);
  }
  const int wpg = super ? kEnc2Waves : 1;  // waves per workgroup
  const int64_t tickets = super ? (int64_t)nclients * a.T2 : total;
  // Persistent grid no larger than what fits co-resident on an idle chip (progress
  // needs only kTicketShards started waves, ticket_stream); very few clients: cap the tiles in flight per client (about
  // 256) so a look-back walks at most a few 64-tile windows.
  int per_cu = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, kEncThreads * wpg, 0) != hipSuccess || per_cu < 1)
    per_cu = 1;
  int64_t max_grid = std::min<int64_t>((int64_t)ncu * per_cu * wpg, std::max<int64_t>(128, 128LL * nclients));
  if (const char* g = getenv("FEDCODEC_ENC_GRID")) max_grid = std::max(1L, atol(g));  // test knob
  const int grid = (int)std::min<int64_t>(tickets, max_grid);  // waves
  a.nshards = (uint32_t)std::min(kTicketShards, grid);
  {  // look-back prefetch window: 64 statuses when few tiles of a client are in flight,
     // 16 when many are (measured at 25 M: C = 128 -13 %, C = 1024 +2 % with 16)
    int win = kLookbackWin;
    if (win <= 0) win = 2 * (int64_t)grid / nclients <= 24 ? 64 : 16;
    if (const char* w = getenv("FEDCODEC_LB_WIN")) win = atoi(w);  // test knob
    a.lb_lane0 = 64 - std::max(1, std::min(64, win));
  }
  {  // prologue: the zeroed workspace prefix (statuses, counters, slow flags; rounded up to
     // 16 bytes, below the client parameters) and the client parameters
    const int64_t nzero16 = (enc_zeroed_bytes(nclients, P) + 15) / 16;
    const int64_t blocks = std::max<int64_t>((nclients + 255) / 256,
                                             std::min<int64_t>((nzero16 + 255) / 256, (int64_t)ncu * 8));
    hipLaunchKernelGGL(k_client_params, dim3((unsigned)blocks), dim3(256), 0, s, a, (ClientParam*)a.cparams,
                       (int)(!int_in && mode != FC_UNIFORM), (uint4*)workspace, nzero16);
  }
  if (hipGetLastError() != hipSuccess) return fail(-10, "k_client_params launch");
  hipLaunchKernelGGL(kern, dim3((grid + wpg - 1) / wpg), dim3(kEncThreads * wpg), 0, s, a);
  if (const int rc_ = check_launch("k_encode")) return rc_;
  // clients with a tile beyond the fast path: exact re-encode (no-ops otherwise)
  hipLaunchKernelGGL(k_zero_slow, dim3(256), dim3(256), 0, s, a);
  hipLaunchKernelGGL(exact, dim3(grid), dim3(kEncThreads), 0, s, a);
  if (idxq) {
    if (const int rc_ = check_launch("k_encode_exact")) return rc_;
    hipLaunchKernelGGL(k_quarter_index, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, idx, idxq,
                       nclients, (int32_t)T);
    return check_launch("k_quarter_index");
  }
  return check_launch("k_encode_exact");
}

// ---------------------------------------------------------------------------
// Segmented encode (few clients per GPU).  The super-tile encoder needs about a
// thousand clients in flight to keep its look-back off the critical path; with
// fewer (the 8-GPU share of the headline: 128 clients) each client is cut into K
// element segments (seg_elems, a multiple of 2048, plus a remainder) that are
// encoded as independent "virtual clients" -- each continuing its client's
// Philox stream at its element offset -- and then stitched into the client's
// canonical stream:
//   * a segment's first code carries the run from virtual position -1; it is
//     replaced by the run from the client's last nonzero before the segment;
//   * every segment's trailing zero-run code is dropped; the client's own
//     trailing code (from its last nonzero) is appended at the end;
//   * the bits in between move to their final offset (a funnel-shift copy),
//     the decoder index entries are rebased, the distortion / nonzero partials
//     copied to the client's tile slots.
// The result is bit-identical to encoding the client in one piece.
// ---------------------------------------------------------------------------
struct SegPlan {       // one per segment, plus the client's trailing code (entry nseg)
  int64_t O;           // output bit where the segment's (new) first code starts
  int64_t len;         // output bits: new first run code + body (tail entry: tlen)
  const uint8_t* src;  // the segment's virtual stream (nullptr for the tail entry)
  int64_t gprev;       // the client's last nonzero before the segment (-1: none); tail: last overall
  uint32_t newR;       // bits of the new first run code (tail entry: trailing code bits)
  uint32_t dnew;       // its value (tail entry: the trailing code's value)
  uint32_t srcbit;     // source bit where the body starts (after the old first run code)
  uint32_t pad;
};

struct SegArgs {
  const void* const* xs;
  int32_t nclients, K, nseg;  // nseg = K (+1 with a remainder segment)
  int64_t P, seg_elems, rem_elems;
  int32_t Tv, Tr;             // tiles per main / remainder segment
  const float* norms;
  const float* prescale;
  const int64_t* seeds;
  // virtual clients: main v = c * K + k (k < K), remainder v = C * K + c
  const float** vptr;
  int64_t* voff;
  int64_t* vseeds;
  float* vnorms;
  float* vpre;
  int64_t* vstream_off;
  int64_t* vstream_cap;
  uint8_t* vstream;
  int64_t vcap_main, vcap_rem;
  uint64_t* vidx_main;        // [C * K][Tv + 1]
  uint64_t* vidx_rem;         // [C][Tr + 1]
  int64_t* vbits;             // [C * K + C]
  float* vdist_main;          // [C * K][Tv]
  float* vdist_rem;           // [C][Tr]
  int32_t* vnnz_main;
  int32_t* vnnz_rem;
  int32_t* vovf;              // [C * K + C]
  SegPlan* plan;              // [C][nseg + 1]
  // the client batch
  uint8_t* stream_buf;
  const int64_t* stream_off;
  const int64_t* stream_cap;
  uint64_t* idx;
  int64_t* total_bits;
  float* dist_part;
  int32_t* nnz_part;
  int32_t* overflow;
};

__global__ void k_seg_setup(SegArgs a) {
  const int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t nv = (int64_t)a.nclients * a.K + (a.rem_elems > 0 ? a.nclients : 0);
  if (v >= nv) return;
  const int64_t nmain = (int64_t)a.nclients * a.K;
  const bool main = v < nmain;
  const int32_t c = (int32_t)(main ? v / a.K : v - nmain);
  const int32_t k = (int32_t)(main ? v - (int64_t)c * a.K : a.K);
  const int64_t off = (int64_t)k * a.seg_elems;
  a.vptr[v] = (const float*)a.xs[c] + off;
  a.voff[v] = off;
  if (a.seeds) {
    a.vseeds[2 * v] = a.seeds[2 * c];
    a.vseeds[2 * v + 1] = a.seeds[2 * c + 1];
  }
  if (a.norms) a.vnorms[v] = a.norms[c];
  if (a.prescale) {
    a.vpre[2 * v] = a.prescale[2 * c];
    a.vpre[2 * v + 1] = a.prescale[2 * c + 1];
  }
  a.vstream_off[v] = main ? v * a.vcap_main : nmain * a.vcap_main + (int64_t)c * a.vcap_rem;
  a.vstream_cap[v] = main ? a.vcap_main : a.vcap_rem;
  if (main && k == 0) {  // a client's first segment codes in place: its bits do not move
    a.vstream_off[v] = (int64_t)((a.stream_buf + a.stream_off[c]) - a.vstream);
    a.vstream_cap[v] = a.stream_cap[c];
  }
}

__device__ __forceinline__ uint32_t glen64(uint64_t d) { return 2u * (63u - (uint32_t)__clzll(d)) + 1u; }

// One wave per client, lane k = segment k: each segment's first / last nonzero
// and old first / trailing codes, then the client's new first run codes (from the
// exclusive max-scan of the segments' last nonzeros), output offsets and the
// trailing code.
__global__ __launch_bounds__(64) void k_seg_plan(SegArgs a) {
  __shared__ int64_t lens[64];
  __shared__ int64_t gls[64];
  const int c = blockIdx.x;
  const int k = threadIdx.x;
  const bool live = k < a.nseg;
  const bool main = k < a.K;
  const int64_t v = main ? (int64_t)c * a.K + k : (int64_t)a.nclients * a.K + c;
  const int64_t Pk = main ? a.seg_elems : a.rem_elems;
  const int32_t Tk = main ? a.Tv : a.Tr;
  const int64_t sk = (int64_t)k * a.seg_elems;
  int64_t last = -1, len = 0, body = 0, gl = -1, f = -1;
  uint32_t oldR = 0, ovf = 0;
  const uint8_t* src = nullptr;
  if (live) {
    const uint64_t* vi = main ? a.vidx_main + v * (a.Tv + 1) : a.vidx_rem + (int64_t)c * (a.Tr + 1);
    last = (int64_t)(vi[Tk] >> 36) - 1;
    const int64_t nb = a.vbits[v];
    src = a.vstream + a.vstream_off[v];
    ovf = (uint32_t)a.vovf[v];
    if (last >= 0) {
      // the segment's first code is gamma(f + 1): z zeros, then z + 1 value bits
      // (its first words are stored even when the segment overflowed its staging)
      const uint32_t* s32 = (const uint32_t*)src;
      const uint64_t top = ((uint64_t)bswap32(s32[0]) << 32) | bswap32(s32[1]);
      const uint32_t z = (uint32_t)__clzll(top);
      const uint64_t d0 = (top << z) >> (63 - z);
      f = (int64_t)d0 - 1;
      oldR = 2 * z + 1;
      const int64_t trail = last < Pk - 1 ? (int64_t)glen64((uint64_t)(Pk - last)) : 0;
      body = nb - oldR - trail;
      gl = sk + last;
      // a segment code that contradicts its own index (it cannot happen for a code the
      // encoder completed) is never stitched: the client is re-encoded (capacity flag)
      if (body < 0 || f < 0 || f > last) ovf |= FC_OVERFLOW_CAPACITY;
    }
  }
  gls[k] = gl;
  __syncthreads();
  int64_t gprev = -1;
  for (int j = 0; j < k && j < a.nseg; ++j) gprev = max(gprev, gls[j]);
  uint32_t newR = 0, dnew = 0;
  if (live && last >= 0) {
    dnew = (uint32_t)(sk + f - gprev);
    newR = glen64(dnew);
    len = newR + body;
  }
  lens[k] = live ? len : 0;
  const uint64_t bad = __ballot(live && (ovf & FC_OVERFLOW_CAPACITY) != 0);
  const uint64_t stall = __ballot(live && (ovf & FC_OVERFLOW_STALL) != 0);
  __syncthreads();
  SegPlan* pl = a.plan + (int64_t)c * (a.nseg + 1);
  int64_t O = 0;
  for (int j = 0; j < k; ++j) O += lens[j];
  if (live) {
    SegPlan e;
    e.O = O;
    e.len = len;
    e.src = src;
    e.gprev = gprev;
    e.newR = newR;
    e.dnew = dnew;
    e.srcbit = oldR;
    e.pad = 0;
    pl[k] = e;
  }
  if (k == 0) {
    int64_t sum = 0, L = -1;
    for (int j = 0; j < a.nseg; ++j) {
      sum += lens[j];
      L = max(L, gls[j]);
    }
    SegPlan t;
    t.O = sum;
    t.src = nullptr;
    t.gprev = L;
    t.srcbit = 0;
    t.pad = 0;
    t.newR = 0;
    t.dnew = 0;
    if (L < a.P - 1) {
      t.dnew = (uint32_t)(a.P - L);
      t.newR = glen64((uint64_t)(a.P - L));
    }
    t.len = t.newR;
    pl[a.nseg] = t;
    const int64_t total = sum + t.newR;
    a.total_bits[c] = total;
    a.overflow[c] = ((bad != 0 || total < 0 || (total + 31) / 32 * 4 > a.stream_cap[c]) ? FC_OVERFLOW_CAPACITY : 0) |
                    (stall != 0 ? FC_OVERFLOW_STALL : 0);
  }
}

// bits [rel, rel + n) of an MSB-first code of `len` bits, right-aligned
__device__ __forceinline__ uint32_t code_bits(uint32_t code, uint32_t len, uint32_t rel, uint32_t n) {
  return (uint32_t)(((uint64_t)code >> (len - rel - n)) & ((1ull << n) - 1));
}

// The stitched words.  Persistent workgroups walk (client, block of 1024 words)
// items; a thread takes 4 consecutive words: inside one segment's moved body (the
// common case) they are a funnel shift of 5 source words and one 16-byte store;
// otherwise each word is gathered from the (usually one or two) pieces it spans.
// Bits past the client's last bit are zero, as the encoder's owner-written last word.
#ifndef FC_SEG_NT
#define FC_SEG_NT 0  // the stitch's segment reads and stream stores non-temporal (A/B knob)
#endif
constexpr int kSegGroups = 4;                      // 16-byte groups per thread per item
constexpr int kSegWordsPerBlock = 1024 * kSegGroups;  // words per (client, item)
__device__ __forceinline__ uint32_t seg_word(const SegPlan* pl, int nseg, int64_t total, int64_t w, int& k) {
  int64_t pos = 32 * w;
  const int64_t end = min(pos + 32, total);
  uint32_t acc = 0;
  while (pos < end) {
    while (k < nseg && pos >= pl[k + 1].O) ++k;
    while (k > 0 && pos < pl[k].O) --k;
    const SegPlan& e = pl[k];
    const int64_t rel = pos - e.O;
    uint32_t n, bits;
    if (k == nseg || rel < (int64_t)e.newR) {  // a new run code, or the trailing code
      n = (uint32_t)min<int64_t>(end - pos, (int64_t)e.newR - rel);
      bits = code_bits(e.dnew, e.newR, (uint32_t)rel, n);
    } else {  // body bits, moved
      n = (uint32_t)min<int64_t>(end - pos, e.len - rel);
      const uint64_t sb = (uint64_t)e.srcbit + (uint64_t)(rel - e.newR);
      const uint32_t* s32 = (const uint32_t*)e.src + (sb >> 5);
      const uint32_t o = (uint32_t)(sb & 31);
      uint32_t x = bswap32(s32[0]) << o;
      if (o + n > 32) x |= bswap32(s32[1]) >> (32 - o);
      bits = x >> (32 - n);
    }
    acc |= bits << (32 - (uint32_t)(pos - 32 * w) - n);
    pos += n;
  }
  return acc;
}

__global__ __launch_bounds__(256) void k_seg_copy(SegArgs a, int64_t blocks_per_client) {
  __shared__ SegPlan pl[65];
  __shared__ int64_t sh_total;
  const int64_t items = blocks_per_client * a.nclients;
  int cur = -1;
  for (int64_t it = blockIdx.x; it < items; it += gridDim.x) {
    const int c = (int)(it / blocks_per_client);
    const int64_t w0 = (it - (int64_t)c * blocks_per_client) * kSegWordsPerBlock;
    if (c != cur) {  // uniform across the workgroup
      __syncthreads();
      const SegPlan* src_pl = a.plan + (int64_t)c * (a.nseg + 1);
      for (int i = threadIdx.x; i <= a.nseg; i += blockDim.x) pl[i] = src_pl[i];
      if (threadIdx.x == 0) sh_total = (a.overflow[c] & FC_OVERFLOW_CAPACITY) ? 0 : src_pl[a.nseg].O + src_pl[a.nseg].len;
      __syncthreads();
      cur = c;
    }
    const int64_t total = sh_total;
    const int64_t nwords = (total + 31) / 32;
    // the first segment was coded in place: words before the one holding the second
    // segment's first bit are final already (that word is read and rewritten by
    // one thread: its first-segment bits come from the output itself)
    const int64_t wstart = pl[1].O / 32;
    if (w0 >= nwords || w0 + kSegWordsPerBlock <= wstart) continue;
    uint32_t* out32 = (uint32_t*)(a.stream_buf + a.stream_off[c]);
    const int64_t cap = a.stream_cap[c];
    // kSegGroups groups of 4 words per thread, each group a coalesced 4-KiB block
    // of the workgroup; every group's source loads are issued before any store
    uint32_t x[kSegGroups][5];
    uint32_t sh[kSegGroups];
    uint32_t fast = 0;
    int k = 0;
#pragma unroll
    for (int g = 0; g < kSegGroups; ++g) {
      const int64_t w = w0 + 4 * threadIdx.x + 1024 * g;
      if (w >= nwords || w + 4 <= wstart) continue;
      while (k < a.nseg && 32 * w >= pl[k + 1].O) ++k;
      const SegPlan& e = pl[k];
      if (w >= wstart && k < a.nseg && 32 * w >= e.O + e.newR && 32 * (w + 4) <= e.O + e.len && (w + 4) * 4 <= cap) {
        const uint64_t sb = (uint64_t)e.srcbit + (uint64_t)(32 * w - e.O - e.newR);
        const uint32_t* s32 = (const uint32_t*)e.src + (sb >> 5);
        sh[g] = (uint32_t)(sb & 31);
#pragma unroll
        for (int j = 0; j < 5; ++j) x[g][j] = FC_SEG_NT ? __builtin_nontemporal_load(s32 + j) : s32[j];
        fast |= 1u << g;
      }
    }
    k = 0;
#pragma unroll
    for (int g = 0; g < kSegGroups; ++g) {
      const int64_t w = w0 + 4 * threadIdx.x + 1024 * g;
      if (w >= nwords || w + 4 <= wstart) continue;
      if (fast & (1u << g)) {
        const uint32_t o = sh[g];
        uint32_t y[5];
#pragma unroll
        for (int j = 0; j < 5; ++j) y[j] = bswap32(x[g][j]);
        uint4 v;
        v.x = bswap32(o ? (y[0] << o) | (y[1] >> (32 - o)) : y[0]);
        v.y = bswap32(o ? (y[1] << o) | (y[2] >> (32 - o)) : y[1]);
        v.z = bswap32(o ? (y[2] << o) | (y[3] >> (32 - o)) : y[2]);
        v.w = bswap32(o ? (y[3] << o) | (y[4] >> (32 - o)) : y[3]);
        if (FC_SEG_NT) {
          typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
          __builtin_nontemporal_store(u32x4{v.x, v.y, v.z, v.w}, (u32x4*)(out32 + w));
        } else {
          *(uint4*)(out32 + w) = v;
        }
      } else {
        for (int64_t ww = max(w, wstart); ww < min(nwords, w + 4); ++ww) {
          const uint32_t v = seg_word(pl, a.nseg, total, ww, k);
          if ((ww + 1) * 4 <= cap) out32[ww] = bswap32(v);
        }
      }
    }
  }
}

// The client's decoder index and per-tile measurement partials from its segments'.
__global__ __launch_bounds__(256) void k_seg_index(SegArgs a) {
  const int64_t T = (int64_t)a.K * a.Tv + (a.rem_elems > 0 ? a.Tr : 0);
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (int64_t)a.nclients * (T + 1)) return;
  const int c = (int)(i / (T + 1));
  const int64_t t = i - (int64_t)c * (T + 1);
  const SegPlan* pl = a.plan + (int64_t)c * (a.nseg + 1);
  if (t == T) {
    a.idx[i] = ((uint64_t)pl[a.nseg].O & kMask36) | ((uint64_t)(pl[a.nseg].gprev + 1) << 36);
    return;
  }
  const bool main = t < (int64_t)a.K * a.Tv;
  const int k = main ? (int)(t / a.Tv) : a.K;
  const int64_t j = main ? t - (int64_t)k * a.Tv : t - (int64_t)a.K * a.Tv;
  const int64_t vrow = main ? ((int64_t)c * a.K + k) : c;
  const uint64_t e = main ? a.vidx_main[vrow * (a.Tv + 1) + j] : a.vidx_rem[vrow * (a.Tr + 1) + j];
  const int64_t vb = (int64_t)(e & kMask36), vl = (int64_t)(e >> 36) - 1;
  const SegPlan& s = pl[k];
  int64_t bits, last;
  if (vl >= 0) {
    bits = s.O + s.newR + (vb - (int64_t)s.srcbit);
    last = (int64_t)k * a.seg_elems + vl;
  } else {
    bits = s.O;
    last = s.gprev;
  }
  a.idx[i] = ((uint64_t)bits & kMask36) | ((uint64_t)(last + 1) << 36);
  const int64_t d = (int64_t)c * T + t;
  if (a.dist_part) a.dist_part[d] = main ? a.vdist_main[vrow * a.Tv + j] : a.vdist_rem[vrow * a.Tr + j];
  if (a.nnz_part) a.nnz_part[d] = main ? a.vnnz_main[vrow * a.Tv + j] : a.vnnz_rem[vrow * a.Tr + j];
}

struct SegLayout {
  int64_t seg_elems, rem_elems, nv, vcap_main, vcap_rem;
  int32_t Tv, Tr, nseg;
  int64_t o_ws_main, o_ws_rem, o_vptr, o_voff, o_vseeds, o_vnorms, o_vpre, o_vsoff, o_vscap, o_vidx_main,
      o_vidx_rem, o_vbits, o_vdist_main, o_vdist_rem, o_vnnz_main, o_vnnz_rem, o_vovf, o_plan, o_vstream, total;
};

// Workspace layout of fc_quantize_encode_segmented (every piece 256-B aligned).
// Returns false if the segmentation is not possible (segments below 2048 elements).
bool seg_layout(int32_t C, int64_t P, int32_t K, int64_t max_cap, SegLayout& L) {
  if (C <= 0 || K < 1 || K > 63 || P <= 0 || max_cap <= 0) return false;
  L.seg_elems = P / K / 2048 * 2048;
  if (L.seg_elems < 2048 || P > FC_MAX_ELEMS) return false;
  L.rem_elems = P - (int64_t)K * L.seg_elems;
  // every segment is one encoder row (26-bit look-back positions)
  if (L.seg_elems > FC_MAX_ROW_ELEMS || L.rem_elems > FC_MAX_ROW_ELEMS) return false;
  L.Tv = (int32_t)tiles_for(L.seg_elems);
  L.Tr = L.rem_elems > 0 ? (int32_t)tiles_for(L.rem_elems) : 0;
  L.nseg = K + (L.rem_elems > 0 ? 1 : 0);
  const int64_t nmain = (int64_t)C * K, nrem = L.rem_elems > 0 ? C : 0;
  L.nv = nmain + nrem;
  // a segment's staging holds the client's whole capacity (bounded by the
  // segment's worst case, 65 bits per element): a client whose nonzeros sit in
  // one segment (model deltas are uneven across layers) fits whenever its code
  // fits its own capacity -- a proportional share would overflow that segment and
  // re-encode the client.  Plus slack for the first run code and the trailing code.
  auto seg_cap = [&](int64_t n) {
    return (std::min(max_cap, (65 * n + 64) / 8 + 64) + 8192 + 255) / 256 * 256;
  };
  L.vcap_main = seg_cap(L.seg_elems);
  L.vcap_rem = nrem ? seg_cap(L.rem_elems) : 0;
  int64_t o = 0;
  auto take = [&](int64_t bytes) {
    const int64_t r = o;
    o += (bytes + 255) / 256 * 256;
    return r;
  };
  L.o_ws_main = take(enc_workspace_bytes((int32_t)nmain, L.seg_elems));
  L.o_ws_rem = take(nrem ? enc_workspace_bytes(C, L.rem_elems) : 0);
  L.o_vptr = take(8 * L.nv);
  L.o_voff = take(8 * L.nv);
  L.o_vseeds = take(16 * L.nv);
  L.o_vnorms = take(4 * L.nv);
  L.o_vpre = take(8 * L.nv);
  L.o_vsoff = take(8 * L.nv);
  L.o_vscap = take(8 * L.nv);
  L.o_vidx_main = take(8 * nmain * (L.Tv + 1));
  L.o_vidx_rem = take(8 * nrem * (L.Tr + 1));
  L.o_vbits = take(8 * L.nv);
  L.o_vdist_main = take(4 * nmain * L.Tv);
  L.o_vdist_rem = take(4 * nrem * L.Tr);
  L.o_vnnz_main = take(4 * nmain * L.Tv);
  L.o_vnnz_rem = take(4 * nrem * L.Tr);
  L.o_vovf = take(4 * L.nv);
  L.o_plan = take((int64_t)sizeof(SegPlan) * C * (L.nseg + 1));
  L.o_vstream = take(nmain * L.vcap_main + nrem * L.vcap_rem + 64);
  L.total = o;
  return true;
}

int encode_segmented(const float* const* xs, int32_t nclients, int64_t P, float step, const float* norms,
                     const float* prescale, const int64_t* seeds, int mode, int32_t K, int64_t max_cap,
                     uint8_t* stream_buf, const int64_t* stream_off, const int64_t* stream_cap, uint64_t* idx,
                     int64_t* total_bits, float* dist_part, int32_t* nnz_part, int32_t* overflow, void* workspace,
                     int64_t workspace_bytes, void* stream, void* stitch_stream = nullptr, bool int_in = false) {
  SegLayout L;
  if (!seg_layout(nclients, P, K, max_cap, L))
    return fail(-1, "segmented encode: segments must hold 2048 .. 2^26 - 1 elements (P <= FC_MAX_ELEMS, K <= 63)");
  if (!xs || !stream_buf || !stream_off || !stream_cap || !idx || !total_bits || !overflow)
    return fail(-1, "null required pointer");
  if (!workspace || workspace_bytes < L.total || ((uintptr_t)workspace & 255))
    return fail(-1, "segmented workspace too small or not 256-byte aligned");
  uint8_t* w = (uint8_t*)workspace;
  SegArgs a;
  a.xs = (const void* const*)xs;
  a.nclients = nclients;
  a.K = K;
  a.nseg = L.nseg;
  a.P = P;
  a.seg_elems = L.seg_elems;
  a.rem_elems = L.rem_elems;
  a.Tv = L.Tv;
  a.Tr = L.Tr;
  a.norms = norms;
  a.prescale = prescale;
  a.seeds = seeds;
  a.vptr = (const float**)(w + L.o_vptr);
  a.voff = (int64_t*)(w + L.o_voff);
  a.vseeds = (int64_t*)(w + L.o_vseeds);
  a.vnorms = (float*)(w + L.o_vnorms);
  a.vpre = (float*)(w + L.o_vpre);
  a.vstream_off = (int64_t*)(w + L.o_vsoff);
  a.vstream_cap = (int64_t*)(w + L.o_vscap);
  a.vstream = w + L.o_vstream;
  a.vcap_main = L.vcap_main;
  a.vcap_rem = L.vcap_rem;
  a.vidx_main = (uint64_t*)(w + L.o_vidx_main);
  a.vidx_rem = (uint64_t*)(w + L.o_vidx_rem);
  a.vbits = (int64_t*)(w + L.o_vbits);
  a.vdist_main = (float*)(w + L.o_vdist_main);
  a.vdist_rem = (float*)(w + L.o_vdist_rem);
  a.vnnz_main = (int32_t*)(w + L.o_vnnz_main);
  a.vnnz_rem = (int32_t*)(w + L.o_vnnz_rem);
  a.vovf = (int32_t*)(w + L.o_vovf);
  a.plan = (SegPlan*)(w + L.o_plan);
  a.stream_buf = stream_buf;
  a.stream_off = stream_off;
  a.stream_cap = stream_cap;
  a.idx = idx;
  a.total_bits = total_bits;
  a.dist_part = dist_part;
  a.nnz_part = nnz_part;
  a.overflow = overflow;
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(k_seg_setup, dim3((unsigned)((L.nv + 255) / 256)), dim3(256), 0, s, a);
  if (const int rc = check_launch("k_seg_setup")) return rc;
  const int32_t nmain = nclients * K;
  int rc = encode_common((const void* const*)a.vptr, nmain, L.seg_elems, step, norms ? a.vnorms : nullptr,
                         prescale ? a.vpre : nullptr, seeds ? a.vseeds : nullptr, mode, int_in, a.vstream,
                         a.vstream_off, a.vstream_cap, a.vidx_main, a.vbits, a.vdist_main, a.vnnz_main, a.vovf,
                         w + L.o_ws_main, L.o_ws_rem - L.o_ws_main, stream, a.voff,
                         std::min(L.vcap_main, max_cap * L.seg_elems / P + 8192));
  if (rc) return rc;
  if (L.rem_elems > 0) {
    rc = encode_common((const void* const*)(a.vptr + nmain), nclients, L.rem_elems, step,
                       norms ? a.vnorms + nmain : nullptr, prescale ? a.vpre + 2 * (int64_t)nmain : nullptr,
                       seeds ? a.vseeds + 2 * (int64_t)nmain : nullptr, mode, int_in, a.vstream, a.vstream_off + nmain,
                       a.vstream_cap + nmain, a.vidx_rem, a.vbits + nmain, a.vdist_rem, a.vnnz_rem, a.vovf + nmain,
                       w + L.o_ws_rem, L.o_vptr - L.o_ws_rem, stream, a.voff + nmain,
                       max_cap * L.rem_elems / P + 8192);
    if (rc) return rc;
  }
  hipLaunchKernelGGL(k_seg_plan, dim3(nclients), dim3(64), 0, s, a);
  if (const int rc2 = check_launch("k_seg_plan")) return rc2;
  // the stitch (bit moves, canonical index, partials) may run on a second stream,
  // beside a decode of the unstitched segments (fc_decode_accumulate_segmented)
  const bool split = stitch_stream && stitch_stream != stream;
  if (split) {
    hipEvent_t ev;
    if (hipEventCreateWithFlags(&ev, hipEventDisableTiming) != hipSuccess) return fail(-10, "event create");
    const bool ok = hipEventRecord(ev, s) == hipSuccess && hipStreamWaitEvent((hipStream_t)stitch_stream, ev, 0) == hipSuccess;
    (void)hipEventDestroy(ev);
    if (!ok) return fail(-10, "stitch stream ordering");
    s = (hipStream_t)stitch_stream;
  }
  const int64_t bpc = (max_cap / 4 + kSegWordsPerBlock - 1) / kSegWordsPerBlock;
  int dev = 0, ncu = 256;
  (void)hipGetDevice(&dev);
  (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
  // beside a decode (split stitch) the copy takes a few workgroups per CU, so the
  // decoder's workgroups stay resident
  int64_t per_cu = split ? 2 : 16;
  if (const char* e = getenv("FEDCODEC_SPLIT_COPY_WG")) if (split) per_cu = std::max(1, atoi(e));  // test knob
  const int64_t cgrid = std::min<int64_t>(bpc * nclients, (int64_t)ncu * per_cu);
  hipLaunchKernelGGL(k_seg_copy, dim3((unsigned)cgrid), dim3(256), 0, s, a, bpc);
  if (const int rc3 = check_launch("k_seg_copy")) return rc3;
  const int64_t T = tiles_for(P);
  hipLaunchKernelGGL(k_seg_index, dim3((unsigned)(((int64_t)nclients * (T + 1) + 255) / 256)), dim3(256), 0, s, a);
  return check_launch("k_seg_index");
}

// QSGD decode: client q rows per group at most this many bytes (fc_decode_scaled_workspace_bytes).

constexpr int64_t kScaledPlaneBudget = 1LL << 30;

// Shared launcher of k_decode (int32 client sum, or the q rows of a client group).
int decode_common(DecodeArgs a, const uint8_t* stream_buf, const int64_t* stream_off, const int64_t* stream_cap,
                  const uint64_t* idx, int32_t nclients, int64_t P, int32_t* err, void* stream,
                  int64_t tile_begin = 0, int64_t tile_end = -1, bool reset_err = true) {
  if (nclients <= 0) return fail(-1, "nclients must be > 0");
  if (P <= 0 || P > FC_MAX_ELEMS) return fail(-1, "P must be in [1, FC_MAX_ELEMS = 2^30 - 2^26]");
  if (!stream_buf || !stream_off || !stream_cap || !idx || !err) return fail(-1, "null required pointer");
  a.stream_buf = stream_buf;
  a.stream_off = stream_off;
  a.stream_cap = stream_cap;
  a.idx = idx;
  a.nclients = nclients;
  a.P = P;
  a.T = (int32_t)tiles_for(P);
  a.err = err;
  if (tile_end < 0) tile_end = a.T;
  if (tile_begin < 0 || tile_begin >= tile_end || tile_end > a.T) return fail(-1, "tile range must satisfy 0 <= begin < end <= tiles");
  a.t_begin = (int32_t)tile_begin;
  a.t_end = (int32_t)tile_end;
  // lanes per tile: 128 (two tiles per workgroup; measured 2-3 % faster than 256 at
  // 256 and 1024 clients, 64 is 20 % slower), fewer for few clients
  const bool plane = a.plane != nullptr;
  const bool virt = !plane && a.vidx_main != nullptr;  // an unstitched segmented batch
  const bool qtr = !plane && !virt && a.idxq != nullptr;  // quarter-tile lane segments
  int span = (!plane && !qtr && nclients >= kDecSpan2Clients) ? 2 : 1;
  if (const char* e = getenv("FEDCODEC_DEC_SPAN")) {  // test knob: 1, 2 or 4 tiles per lane segment
    const int v = atoi(e);
    // (an unstitched segmented batch: at most two, so a lane segment straddles at most one
    // encoder segment's end)
    span = (plane || qtr) ? 1 : v == 4 ? (virt ? 2 : 4) : v == 2 ? 2 : 1;
  }
  int lpt = span >= 2 ? 256 : 128;
  while (lpt > 64 && lpt / 2 >= nclients) lpt /= 2;
  if (const char* l = getenv("FEDCODEC_DEC_LPT")) {  // test knob: lanes per tile (64, 128 or 256)
    const int v = atoi(l);
    if (v == 64 || v == 128 || v == 256) lpt = v;
  }
  a.lanes_per_tile = lpt;
  void (*kern)(DecodeArgs) = plane  ? (a.plane8 ? k_decode<2> : k_decode<1>)
                             : qtr  ? k_decode<0, 1, true>
                             : virt ? (span == 2 ? k_decode<0, 2, false, true> : k_decode<0, 1, false, true>)
                             : span == 4 ? k_decode<0, 4> : span == 2 ? k_decode<0, 2> : k_decode<0, 1>;
  const int ue = qtr ? kTE / 4 : kTE;  // elements per unit
  const int tpw = kDecThreads / lpt * span;  // units per workgroup
  const int repl = qtr ? FC_DEC_QTR_REPL : FC_DEC_REPL;
  const size_t lds = plane ? 0 : (size_t)(repl > 1 ? repl * (tpw * ue + 1) : tpw * ue) * sizeof(int32_t);
  // (+ the static kLutSize-word table)
  int dev = 0, ncu = 256, per_cu = 0;
  (void)hipGetDevice(&dev);
  (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, kDecThreads, lds) != hipSuccess || per_cu < 1)
    per_cu = 1;
  const int64_t u_end = (std::min<int64_t>(P, (int64_t)a.t_end * kTE) + ue - 1) / ue;
  const int64_t ngroups = (u_end - (int64_t)a.t_begin * (kTE / ue) + tpw - 1) / tpw;
  // 5 workgroups/CU: more waves only add L2 line thrash (measured 4.2 ms at 5/CU vs 5.0 at 7/CU)
  // (quarter-tile segments: every co-resident workgroup -- short chains, few lines each)
  int64_t max_grid = (int64_t)ncu * std::min(per_cu, qtr ? 8 : 5);
  if (const char* g = getenv("FEDCODEC_DEC_GRID")) max_grid = std::max(1L, atol(g));  // test knob
  const dim3 grid((unsigned)std::min<int64_t>(ngroups, max_grid));
  hipStream_t s = (hipStream_t)stream;
  if (reset_err && hipMemsetAsync(err, 0, sizeof(int32_t), s) != hipSuccess) return fail(-10, "memset err");
  hipLaunchKernelGGL(kern, grid, dim3(kDecThreads), lds, s, a);
  return check_launch("k_decode");
}

// fc_build_index workspace: x1 | n1 | x2 | n2 | xm (int64 [nclients][nchunks] each) | ck (u64
// [nck][nclients * nchunks]) | ended (int32 [nclients]).
// Chunk size: the largest of 8192 / 4096 / 2048 bits that still gives about 600 K chunk
// lanes (a full chip's parse lanes about once over) -- longer chunks spend less per lane
// on the guess, the lockstep and the checkpoints, shorter ones fill the chip (measured:
// 1024 x 25 M 22.4 / 24.0 / 31.0 ms at 8192 / 4096 / 2048; config 2 1.22 / 0.93 / 0.91; config 3
// 1.14 / 1.01 / 1.20).
int32_t idx_chunk_bits(int32_t n, int64_t max_bytes) {
  int32_t cb = kIdxChunkMax;
  while (cb > 2048 && (int64_t)n * ((8 * max_bytes + cb - 1) / cb) < 600000) cb /= 2;
  if (const char* e = getenv("FEDCODEC_IDX_CHUNK")) {  // test knob
    const int v = atoi(e);
    if (v == 2048 || v == 4096 || v == 8192) cb = v;
  }
  return cb;
}
int64_t idx_nchunks(int32_t n, int64_t max_bytes) {
  const int64_t cb = idx_chunk_bits(n, max_bytes);
  return std::max<int64_t>(1, (8 * max_bytes + cb - 1) / cb);
}
int64_t idx_workspace_bytes(int32_t n, int64_t max_bytes) {
  const int64_t nck = idx_nck(idx_chunk_bits(n, max_bytes));
  return (5 + nck) * 8 * (int64_t)n * idx_nchunks(n, max_bytes) + ((4 * (int64_t)n + 255) & ~255LL);
}

int build_index(const uint8_t* stream_buf, const int64_t* stream_off, const int64_t* nbytes, int32_t nclients,
                int64_t P, int64_t max_bytes, uint64_t* idx, uint64_t* idxq, int64_t* total_bits, int32_t* err,
                void* workspace, int64_t workspace_bytes, void* stream) {
  if (nclients <= 0) return fail(-1, "nclients must be > 0");
  if (P <= 0 || P > FC_MAX_ELEMS) return fail(-1, "P must be in [1, FC_MAX_ELEMS = 2^30 - 2^26]");
  if (max_bytes < 0) return fail(-1, "max_bytes must be >= 0");
  if (!stream_buf || !stream_off || !nbytes || !idx || !total_bits || !err) return fail(-1, "null required pointer");
  if (!workspace || workspace_bytes < idx_workspace_bytes(nclients, max_bytes) || ((uintptr_t)workspace & 15))
    return fail(-1, "index workspace too small or not 16-byte aligned");
  IdxArgs a;
  a.stream_buf = stream_buf;
  a.stream_off = stream_off;
  a.nbytes = nbytes;
  a.nclients = nclients;
  a.P = P;
  a.T = (int32_t)tiles_for(P);
  a.chunk = idx_chunk_bits(nclients, max_bytes);
  a.nck = idx_nck(a.chunk);
  a.ckb = a.chunk / (a.nck + 1);
  a.nchunks = idx_nchunks(nclients, max_bytes);
  const int64_t lanes = (int64_t)nclients * a.nchunks;
  int64_t* w = (int64_t*)workspace;
  a.x1 = w;
  a.n1 = w + lanes;
  a.x2 = w + 2 * lanes;
  a.n2 = w + 3 * lanes;
  a.xm = w + 4 * lanes;
  a.ck = (uint64_t*)(w + 5 * lanes);
  a.ended = (int32_t*)(w + (5 + (int64_t)a.nck) * lanes);
  a.idx = idx;
  a.idxq = idxq;
  a.total_bits = total_bits;
  a.err = err;
  hipStream_t s = (hipStream_t)stream;
  if (hipMemsetAsync(err, 0, sizeof(int32_t), s) != hipSuccess ||
      hipMemsetAsync(a.ended, 0, 4 * (size_t)nclients, s) != hipSuccess)
    return fail(-10, "memset");
  const dim3 lgrid((unsigned)((lanes + kThreads - 1) / kThreads));
  int dev = 0, ncu = 256;
  (void)hipGetDevice(&dev);
  (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
  // the table-driven parses: persistent workgroups (one table copy each)
  const dim3 pgrid((unsigned)std::min<int64_t>((lanes + kThreads - 1) / kThreads, (int64_t)ncu * 8));
  hipLaunchKernelGGL(k_idx_spec, pgrid, dim3(kThreads), 0, s, a);
  if (const int rc = check_launch("k_idx_spec")) return rc;
  hipLaunchKernelGGL(k_idx_sync, lgrid, dim3(kThreads), 0, s, a);
  if (const int rc = check_launch("k_idx_sync")) return rc;
  hipLaunchKernelGGL(k_idx_fix, dim3(nclients), dim3(64), 0, s, a);
  if (const int rc = check_launch("k_idx_fix")) return rc;
  hipLaunchKernelGGL(k_idx_scan, dim3(nclients), dim3(64), 0, s, a);
  if (const int rc = check_launch("k_idx_scan")) return rc;
  hipLaunchKernelGGL(k_idx_emit, pgrid, dim3(kThreads), 0, s, a);
  if (const int rc = check_launch("k_idx_emit")) return rc;
  hipLaunchKernelGGL(k_idx_check, dim3((unsigned)((nclients + 255) / 256)), dim3(256), 0, s, a);
  return check_launch("k_idx_check");
}

// FFT of N = 2^k points from buf[0] (ping-pong with buf[1]); returns the buffer
// holding the result.
int fft_pow2(float2* b0, float2* b1, int64_t N, float sign, hipStream_t s, float2** res) {
  float2* src = b0;
  float2* dst = b1;
  int64_t Ns = 1;
  while (Ns < N) {
    const int64_t rem = N / Ns;
    const int R = rem >= 16 ? 16 : (int)rem;
    const int64_t q = N / R;
    const dim3 grid((unsigned)((q + 255) / 256));
    if (R == 16) hipLaunchKernelGGL(k_fft_pass<16>, grid, dim3(256), 0, s, src, dst, N, Ns, sign);
    else if (R == 8) hipLaunchKernelGGL(k_fft_pass<8>, grid, dim3(256), 0, s, src, dst, N, Ns, sign);
    else if (R == 4) hipLaunchKernelGGL(k_fft_pass<4>, grid, dim3(256), 0, s, src, dst, N, Ns, sign);
    else hipLaunchKernelGGL(k_fft_pass<2>, grid, dim3(256), 0, s, src, dst, N, Ns, sign);
    if (const int rc = check_launch("k_fft_pass")) return rc;
    Ns *= R;
    std::swap(src, dst);
  }
  *res = src;
  return 0;
}

int64_t dft_len(int64_t m) {  // FFT length: m itself (power of two) or the Bluestein length
  if ((m & (m - 1)) == 0) return m;
  int64_t L = 1;
  while (L < 2 * m - 1) L <<= 1;
  return L;
}

}  // namespace

extern "C" {

const char* fc_last_error(void) { return g_err.c_str(); }
const char* fc_version(void) { return "fedcodec 0.1 gfx950"; }
#ifdef FC_STAMPS
int fc_debug_stamps(unsigned long long* host8, int reset) {
  if (hipMemcpyFromSymbol(host8, HIP_SYMBOL(g_stamps), sizeof(unsigned long long) * 16) != hipSuccess) return -1;
  if (reset) {
    unsigned long long z[16] = {0};
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_stamps), z, sizeof(z)) != hipSuccess) return -1;
  }
  return 0;
}
#endif
int64_t fc_num_tiles(int64_t P) { return P <= 0 ? 0 : tiles_for(P); }
int32_t fc_decode_tables(uint32_t* lut, uint16_t* glut, int32_t n) {
  static constexpr DecTabs kHostTabs = make_dec_tabs();  // the same constant expression as g_dec_tabs
  if (n < kLutSize || !lut || !glut) return fail(-1, "table buffers must hold 4096 entries");
  std::memcpy(lut, kHostTabs.lut, sizeof(kHostTabs.lut));
  std::memcpy(glut, kHostTabs.glut, sizeof(kHostTabs.glut));
  return kLutSize;
}
int64_t fc_encode_workspace_bytes(int32_t nclients, int64_t P) {
  if (nclients <= 0 || P <= 0) return 256;
  return enc_workspace_bytes(nclients, P);
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

int64_t fc_segmented_workspace_bytes(int32_t nclients, int64_t P, int32_t nseg, int64_t max_cap) {
  SegLayout L;
  if (!seg_layout(nclients, P, nseg, max_cap, L)) return -1;
  return L.total;
}

int fc_quantize_encode_segmented(const float* const* xs, int32_t nclients, int64_t P, float step,
                                 const float* norms, const float* prescale, const int64_t* seeds, int mode,
                                 int32_t nseg, int64_t max_cap, uint8_t* stream_buf, const int64_t* stream_off,
                                 const int64_t* stream_cap, uint64_t* idx, int64_t* total_bits, float* dist_part,
                                 int32_t* nnz_part, int32_t* overflow, void* workspace, int64_t workspace_bytes,
                                 void* stream) {
  if (mode < 0 || mode > 2) return fail(-1, "mode must be 0 (uniform), 1 (stochastic) or 2 (dithered)");
  return encode_segmented(xs, nclients, P, step, norms, prescale, seeds, mode, nseg, max_cap, stream_buf, stream_off,
                          stream_cap, idx, total_bits, dist_part, nnz_part, overflow, workspace, workspace_bytes,
                          stream);
}

int fc_quantize_encode_segmented_split(const float* const* xs, int32_t nclients, int64_t P, float step,
                                       const float* norms, const float* prescale, const int64_t* seeds, int mode,
                                       int32_t nseg, int64_t max_cap, uint8_t* stream_buf,
                                       const int64_t* stream_off, const int64_t* stream_cap, uint64_t* idx,
                                       int64_t* total_bits, float* dist_part, int32_t* nnz_part, int32_t* overflow,
                                       void* workspace, int64_t workspace_bytes, void* stream,
                                       void* stitch_stream) {
  if (mode < 0 || mode > 2) return fail(-1, "mode must be 0 (uniform), 1 (stochastic) or 2 (dithered)");
  return encode_segmented(xs, nclients, P, step, norms, prescale, seeds, mode, nseg, max_cap, stream_buf, stream_off,
                          stream_cap, idx, total_bits, dist_part, nnz_part, overflow, workspace, workspace_bytes,
                          stream, stitch_stream);
}

int fc_decode_accumulate_segmented(const void* workspace, int64_t workspace_bytes, int32_t nclients, int64_t P,
                                   int32_t nseg, int64_t max_cap, int32_t tile_begin, int32_t tile_end,
                                   const int32_t* sum_in, int32_t* sum_out, float* out, float step,
                                   const float* noise_sum, int32_t* err, void* stream) {
  if (!sum_out && !out) return fail(-1, "one of sum_out / out required");
  SegLayout L;
  if (!seg_layout(nclients, P, nseg, max_cap, L)) return fail(-1, "segmented decode: segments below 2048 elements");
  if (!workspace || workspace_bytes < L.total || ((uintptr_t)workspace & 255))
    return fail(-1, "segmented workspace too small or not 256-byte aligned");
  const uint8_t* w = (const uint8_t*)workspace;
  DecodeArgs a{};
  a.sum_in = sum_in;
  a.sum_out = sum_out;
  a.out = out;
  a.step = step;
  a.noise_sum = noise_sum;
  a.vidx_main = (const uint64_t*)(w + L.o_vidx_main);
  a.vidx_rem = (const uint64_t*)(w + L.o_vidx_rem);
  a.vK = nseg;
  a.vTv = L.Tv;
  a.vTr = L.Tr;
  return decode_common(a, w + L.o_vstream, (const int64_t*)(w + L.o_vsoff), (const int64_t*)(w + L.o_vscap),
                       a.vidx_main, nclients, P, err, stream, tile_begin, tile_end, false);
}

int fc_quantize_encode_hinted(const float* const* xs, int32_t nclients, int64_t P, float step,
                              const float* norms, const float* prescale, const int64_t* seeds, int mode,
                              uint8_t* stream_buf, const int64_t* stream_off, const int64_t* stream_cap,
                              uint64_t* idx, int64_t* total_bits, float* dist_part, int32_t* nnz_part,
                              int32_t* overflow, void* workspace, int64_t workspace_bytes, int64_t max_cap,
                              void* stream) {
  return encode_common((const void* const*)xs, nclients, P, step, norms, prescale, seeds, mode, false, stream_buf,
                       stream_off, stream_cap, idx, total_bits, dist_part, nnz_part, overflow, workspace,
                       workspace_bytes, stream, nullptr, max_cap);
}

int fc_quantize_encode_quarters(const float* const* xs, int32_t nclients, int64_t P, float step,
                                const float* norms, const float* prescale, const int64_t* seeds, int mode,
                                uint8_t* stream_buf, const int64_t* stream_off, const int64_t* stream_cap,
                                uint64_t* idx, uint64_t* idxq, int64_t* total_bits, float* dist_part,
                                int32_t* nnz_part, int32_t* overflow, void* workspace, int64_t workspace_bytes,
                                void* stream) {
  if (!idxq) return fail(-1, "null required pointer");
  return encode_common((const void* const*)xs, nclients, P, step, norms, prescale, seeds, mode, false, stream_buf,
                       stream_off, stream_cap, idx, total_bits, dist_part, nnz_part, overflow, workspace,
                       workspace_bytes, stream, nullptr, 0, idxq);
}

int fc_rlgamma_encode(const int32_t* const* qs, int32_t nclients, int64_t P, uint8_t* stream_buf,
                      const int64_t* stream_off, const int64_t* stream_cap, uint64_t* idx,
                      int64_t* total_bits, int32_t* overflow, void* workspace, int64_t workspace_bytes,
                      void* stream) {
  return encode_common((const void* const*)qs, nclients, P, 1.0f, nullptr, nullptr, nullptr, FC_UNIFORM, true,
                       stream_buf, stream_off, stream_cap, idx, total_bits, nullptr, nullptr, overflow,
                       workspace, workspace_bytes, stream);
}

int fc_rlgamma_encode_segmented(const int32_t* const* qs, int32_t nclients, int64_t P, int32_t nseg, int64_t max_cap,
                                uint8_t* stream_buf, const int64_t* stream_off, const int64_t* stream_cap, uint64_t* idx,
                                int64_t* total_bits, int32_t* overflow, void* workspace, int64_t workspace_bytes,
                                void* stream) {
  return encode_segmented((const float* const*)qs, nclients, P, 1.0f, nullptr, nullptr, nullptr, FC_UNIFORM, nseg,
                          max_cap, stream_buf, stream_off, stream_cap, idx, total_bits, nullptr, nullptr, overflow,
                          workspace, workspace_bytes, stream, nullptr, true);
}

int64_t fc_index_workspace_bytes(int32_t nclients, int64_t max_bytes) {
  return nclients > 0 && max_bytes >= 0 ? idx_workspace_bytes(nclients, max_bytes) : -1;
}

int fc_build_index(const uint8_t* stream_buf, const int64_t* stream_off, const int64_t* nbytes, int32_t nclients,
                   int64_t P, int64_t max_bytes, uint64_t* idx, uint64_t* idxq, int64_t* total_bits, int32_t* err,
                   void* workspace, int64_t workspace_bytes, void* stream) {
  return build_index(stream_buf, stream_off, nbytes, nclients, P, max_bytes, idx, idxq, total_bits, err, workspace,
                     workspace_bytes, stream);
}

int fc_decode_accumulate(const uint8_t* stream_buf, const int64_t* stream_off, const int64_t* stream_cap,
                         const uint64_t* idx, int32_t nclients, int64_t P, const int32_t* sum_in,
                         int32_t* sum_out, float* out, float step, const float* noise_sum, int32_t* err,
                         void* stream) {
  if (!sum_out && !out) return fail(-1, "one of sum_out / out required");
  DecodeArgs a{};
  a.sum_in = sum_in;
  a.sum_out = sum_out;
  a.out = out;
  a.step = step;
  a.noise_sum = noise_sum;
  return decode_common(a, stream_buf, stream_off, stream_cap, idx, nclients, P, err, stream);
}

int fc_decode_accumulate_tiles(const uint8_t* stream_buf, const int64_t* stream_off,
                               const int64_t* stream_cap, const uint64_t* idx, int32_t nclients, int64_t P,
                               int32_t tile_begin, int32_t tile_end, const int32_t* sum_in, int32_t* sum_out,
                               float* out, float step, const float* noise_sum, int32_t* err, void* stream) {
  if (!sum_out && !out) return fail(-1, "one of sum_out / out required");
  DecodeArgs a{};
  a.sum_in = sum_in;
  a.sum_out = sum_out;
  a.out = out;
  a.step = step;
  a.noise_sum = noise_sum;
  return decode_common(a, stream_buf, stream_off, stream_cap, idx, nclients, P, err, stream, tile_begin,
                       tile_end, false);
}

int fc_decode_accumulate_quarters(const uint8_t* stream_buf, const int64_t* stream_off,
                                  const int64_t* stream_cap, const uint64_t* idx, const uint64_t* idxq,
                                  int32_t nclients, int64_t P, int32_t tile_begin, int32_t tile_end,
                                  const int32_t* sum_in, int32_t* sum_out, float* out, float step,
                                  const float* noise_sum, int32_t* err, void* stream) {
  if (!sum_out && !out) return fail(-1, "one of sum_out / out required");
  if (!idxq) return fail(-1, "null required pointer");
  DecodeArgs a{};
  a.sum_in = sum_in;
  a.sum_out = sum_out;
  a.out = out;
  a.step = step;
  a.noise_sum = noise_sum;
  a.idxq = idxq;
  return decode_common(a, stream_buf, stream_off, stream_cap, idx, nclients, P, err, stream, tile_begin,
                       tile_end, false);
}

int64_t fc_decode_scaled_workspace_bytes(int32_t nclients, int64_t P) {
  if (nclients <= 0 || P <= 0) return 256;
  const int64_t row = 4 * ((P + 3) & ~(int64_t)3);
  const int64_t group = std::max<int64_t>(1, std::min<int64_t>(nclients, kScaledPlaneBudget / row));
  return group * row;
}

int fc_decode_accumulate_scaled_bounded(const uint8_t* stream_buf, const int64_t* stream_off,
                                        const int64_t* stream_cap, const uint64_t* idx, int32_t nclients, int64_t P,
                                        const float* client_scale, const float* fsum_in, float* out, int32_t* err,
                                        int32_t qmax, void* workspace, int64_t workspace_bytes, void* stream) {
  if (!out || !client_scale || !workspace) return fail(-1, "null required pointer");
  if (nclients <= 0) return fail(-1, "nclients must be > 0");
  if (P <= 0 || P > FC_MAX_ELEMS) return fail(-1, "P must be in [1, FC_MAX_ELEMS = 2^30 - 2^26]");
  if ((uintptr_t)workspace & 15u) return fail(-1, "workspace must be 16-byte aligned");
  // |q| <= 127 declared: int8 rows (a quarter of the rows' memset / write / read traffic)
  const bool q8 = qmax > 0 && qmax <= 127;
  const int64_t eb = q8 ? 1 : 4;
  const int64_t stride = q8 ? (P + 15) & ~(int64_t)15 : (P + 3) & ~(int64_t)3;
  const int64_t group = std::min<int64_t>(nclients, workspace_bytes / (eb * stride));
  if (group < 1) return fail(-1, "workspace smaller than one client row (fc_decode_scaled_workspace_bytes)");
  const int64_t T = tiles_for(P);
  hipStream_t s = (hipStream_t)stream;
  // client groups in order: decode each group's q rows, then add them to the running
  // float32 sum in client order (the first group starts from fsum_in, or zero)
  for (int64_t c0 = 0; c0 < nclients; c0 += group) {
    const int32_t n = (int32_t)std::min<int64_t>(group, nclients - c0);
    if (hipMemsetAsync(workspace, 0, (size_t)(n * eb * stride), s) != hipSuccess) return fail(-10, "memset planes");
    DecodeArgs a{};
    a.plane = (int32_t*)workspace;
    a.plane_stride = stride;
    a.plane8 = q8 ? 1 : 0;
    const int rc = decode_common(a, stream_buf, stream_off + c0, stream_cap + c0, idx + c0 * (T + 1), n, P, err,
                                 stream, 0, -1, c0 == 0);
    if (rc) return rc;
    const int64_t thr = (P + 3) / 4;
    if (q8)
      hipLaunchKernelGGL(k_sum_planes<int8_t>, dim3((unsigned)((thr + 255) / 256)), dim3(256), 0, s,
                         (const int8_t*)workspace, stride, n, P, client_scale + c0, c0 == 0 ? fsum_in : out, out);
    else
      hipLaunchKernelGGL(k_sum_planes<int32_t>, dim3((unsigned)((thr + 255) / 256)), dim3(256), 0, s,
                         (const int32_t*)workspace, stride, n, P, client_scale + c0, c0 == 0 ? fsum_in : out, out);
    const int rs = check_launch("k_sum_planes");
    if (rs) return rs;
  }
  return 0;
}

int fc_decode_accumulate_scaled(const uint8_t* stream_buf, const int64_t* stream_off,
                                const int64_t* stream_cap, const uint64_t* idx, int32_t nclients, int64_t P,
                                const float* client_scale, const float* fsum_in, float* out, int32_t* err,
                                void* workspace, int64_t workspace_bytes, void* stream) {
  return fc_decode_accumulate_scaled_bounded(stream_buf, stream_off, stream_cap, idx, nclients, P, client_scale,
                                             fsum_in, out, err, 0, workspace, workspace_bytes, stream);
}

int64_t fc_vote_workspace_bytes(int32_t nclients, int64_t P, int32_t K) {
  if (nclients <= 0 || P <= 0 || K <= 0) return 256;
  return (int64_t)nclients * K * tiles_for(P) * (int64_t)sizeof(VoteRec);
}

int fc_vote_lengths(const float* const* xs, int32_t nclients, int64_t P, const float* steps, int32_t K,
                    const int64_t* seeds, int mode, int64_t* bits, double* dist, void* workspace,
                    int64_t workspace_bytes, void* stream) {
  if (nclients <= 0 || K <= 0) return fail(-1, "nclients and K must be > 0");
  if (P <= 0 || P > FC_MAX_ELEMS) return fail(-1, "P must be in [1, FC_MAX_ELEMS = 2^30 - 2^26]");
  if (mode < 0 || mode > 2) return fail(-1, "mode must be 0 (uniform), 1 (stochastic) or 2 (dithered)");
  if (!xs || !steps || !bits || !dist || (mode != FC_UNIFORM && !seeds)) return fail(-1, "null required pointer");
  if (!workspace || workspace_bytes < fc_vote_workspace_bytes(nclients, P, K) || ((uintptr_t)workspace & 15))
    return fail(-1, "workspace too small or misaligned");
  VoteArgs a;
  a.xs = xs;
  a.nclients = nclients;
  a.P = P;
  a.T = (int32_t)tiles_for(P);
  a.K = K;
  a.steps = steps;
  a.seeds = seeds;
  a.rec = (VoteRec*)workspace;
  a.bits = bits;
  a.dist = dist;
  int dev = 0, ncu = 256;
  (void)hipGetDevice(&dev);
  (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
  const int64_t total = (int64_t)nclients * a.T;
  const dim3 grid((unsigned)std::min<int64_t>(total, (int64_t)ncu * 16));
  hipStream_t s = (hipStream_t)stream;
  if (mode == FC_UNIFORM) hipLaunchKernelGGL(k_vote_tiles<FC_UNIFORM>, grid, dim3(64), 0, s, a);
  else if (mode == FC_STOCHASTIC) hipLaunchKernelGGL(k_vote_tiles<FC_STOCHASTIC>, grid, dim3(64), 0, s, a);
  else hipLaunchKernelGGL(k_vote_tiles<FC_DITHERED>, grid, dim3(64), 0, s, a);
  if (const int rc_ = check_launch("k_vote_tiles")) return rc_;
  hipLaunchKernelGGL(k_vote_finalize, dim3((unsigned)((int64_t)nclients * K)), dim3(256), 0, s, a);
  return check_launch("k_vote_finalize");
}

int fc_drive_encode(const float* const* xs, int32_t nclients, int64_t P, int min_distortion, uint32_t* masks,
                    float* means, double* dist, void* stream) {
  if (nclients <= 0 || nclients > 65535 || P <= 0) return fail(-1, "bad sizes");
  if (!xs || !masks || !means || !dist) return fail(-1, "null pointer");
  if (const int rc = launch_mask_encode<1>(xs, nclients, P, 0.0f, min_distortion, masks, means, dist,
                                           (hipStream_t)stream))
    return rc;
  hipLaunchKernelGGL(k_mask_distortion<1>, dim3(nclients), dim3(kObThreads), 0, (hipStream_t)stream, xs, P, 0.0f,
                     (const float*)means, dist);
  return check_launch("k_mask_distortion<1>");
}

int64_t fc_dft_workspace_bytes(int64_t n) {
  if (n <= 0 || (n & 1)) return -1;
  const int64_t m = n / 2;
  return 3 * dft_len(m) * (int64_t)sizeof(float2);
}

int fc_dft_rotate(float* const* rows, int32_t nclients, int64_t n, int inverse, int64_t seed0, int64_t seed1,
                  void* workspace, int64_t workspace_bytes, void* stream) {
  if (nclients <= 0 || n <= 0 || (n & 1) || n > (1LL << 33)) return fail(-1, "n must be even and positive");
  if (!rows || !workspace) return fail(-1, "null pointer");
  if (workspace_bytes < fc_dft_workspace_bytes(n) || ((uintptr_t)workspace & 15))
    return fail(-1, "DFT workspace too small (fc_dft_workspace_bytes) or misaligned");
  hipStream_t s = (hipStream_t)stream;
  const int64_t m = n / 2, L = dft_len(m);
  const bool blue = L != m;
  float2* w0 = (float2*)workspace;
  float2* w1 = w0 + L;
  float2* bb = w1 + L;
  const dim3 gL((unsigned)((L + 255) / 256)), gm((unsigned)((m + 255) / 256));
  float2* B = nullptr;
  if (blue) {  // the chirp filter's spectrum, once per call
    hipLaunchKernelGGL(k_dft_bvec, gL, dim3(256), 0, s, m, L, w0);
    if (const int rc = check_launch("k_dft_bvec")) return rc;
    float2* r = nullptr;
    if (const int rc = fft_pow2(w0, w1, L, -1.0f, s, &r)) return rc;
    if (r != bb) {
      if (hipMemcpyAsync(bb, r, L * sizeof(float2), hipMemcpyDeviceToDevice, s) != hipSuccess)
        return fail(-10, "hipMemcpyAsync");
    }
    B = bb;
  }
  // one row at a time through the workspace (rows: device array of row pointers)
  for (int32_t c = 0; c < nclients; ++c) {
    if (!inverse) {
      const Key4 key = tf_seed_scramble(seed0, seed1);
      hipLaunchKernelGGL(k_sign_flip_row, dim3((unsigned)(((n + 3) / 4 + 255) / 256)), dim3(256), 0, s, rows, c, n, key);
      if (const int rc = check_launch("k_sign_flip_row")) return rc;
    }
    hipLaunchKernelGGL(k_dft_pre, gL, dim3(256), 0, s, rows, c, m, L, blue ? 1 : 0, inverse ? 1 : 0, w0);
    if (const int rc = check_launch("k_dft_pre")) return rc;
    float2* r = nullptr;
    if (const int rc = fft_pow2(w0, w1, L, -1.0f, s, &r)) return rc;
    float scale = (float)(1.0 / std::sqrt((double)m));
    if (blue) {
      hipLaunchKernelGGL(k_cmul, gL, dim3(256), 0, s, r, (const float2*)B, L);
      if (const int rc = check_launch("k_cmul")) return rc;
      float2* other = r == w0 ? w1 : w0;
      if (const int rc = fft_pow2(r, other, L, 1.0f, s, &r)) return rc;
      scale = (float)(1.0 / (std::sqrt((double)m) * (double)L));
    }
    hipLaunchKernelGGL(k_dft_post, gm, dim3(256), 0, s, (const float2*)r, m, blue ? 1 : 0, scale, inverse ? 1 : 0, rows,
                       c);
    if (const int rc = check_launch("k_dft_post")) return rc;
    if (inverse) {
      const Key4 key = tf_seed_scramble(seed0, seed1);
      hipLaunchKernelGGL(k_sign_flip_row, dim3((unsigned)(((n + 3) / 4 + 255) / 256)), dim3(256), 0, s, rows, c, n, key);
      if (const int rc = check_launch("k_sign_flip_row")) return rc;
    }
  }
  return 0;
}

int fc_sign_flip(float* const* rows, int32_t nclients, int64_t n, int64_t seed0, int64_t seed1, void* stream) {
  if (nclients <= 0 || nclients > 65535 || n <= 0 || n > (1LL << 34)) return fail(-1, "bad nclients / n");
  if (!rows) return fail(-1, "null pointer");
  const Key4 key = tf_seed_scramble(seed0, seed1);
  const dim3 grid((unsigned)(((n + 3) / 4 + 255) / 256), (unsigned)nclients);
  hipLaunchKernelGGL(k_sign_flip, grid, dim3(256), 0, (hipStream_t)stream, rows, n, key);
  return check_launch("k_sign_flip");
}

int fc_hadamard(float* const* rows, int32_t nclients, int64_t n, int inverse, int64_t seed0, int64_t seed1,
                void* stream) {
  if (nclients <= 0 || n <= 0 || (n & (n - 1)) || n > (1LL << 30)) return fail(-1, "n must be a power of two");
  if (!rows) return fail(-1, "null pointer");
  int levels = 0;
  while ((1LL << levels) < n) ++levels;
  const float scale = (float)(1.0 / std::sqrt((double)n));
  hipStream_t s = (hipStream_t)stream;
  int L0 = 0;
  while (L0 < levels || (levels == 0 && L0 == 0)) {
    const int k = L0 == 0 ? std::min(levels, 12) : std::min(levels - L0, 8);
    const bool first = L0 == 0, last = L0 + k >= levels;
    const int64_t gsize = (int64_t)1 << (L0 == 0 ? k : 12);
    const int64_t groups = (int64_t)nclients * (n / gsize);
    hipLaunchKernelGGL(k_fwht_pass, dim3((unsigned)groups), dim3(256), 0, s, rows, n, L0, k,
                       (int)(first && !inverse), (int)(last && inverse), last ? scale : 1.0f, seed0, seed1);
    if (const int rc_ = check_launch("k_fwht_pass")) return rc_;
    if (levels == 0) break;
    L0 += k;
  }
  return 0;
}

int fc_quantize_floor(const float* const* xs, int32_t nclients, int64_t P, float step, const int64_t* seeds, int mode,
                      float* dist_part, int32_t* nnz_part, void* workspace, int64_t workspace_bytes, void* stream) {
  if (nclients <= 0 || nclients > 65535 || P <= 0 || P > FC_MAX_ELEMS) return fail(-1, "bad nclients / P");
  if (mode != FC_UNIFORM && mode != FC_STOCHASTIC) return fail(-1, "floor kernel: uniform or stochastic");
  if (!xs || !seeds || !dist_part || !nnz_part || !workspace || workspace_bytes < 16LL * nclients)
    return fail(-1, "null pointer or workspace below 16 bytes per client");
  int e = 0;
  const float m = std::frexp(step, &e);
  if (!(step > 0.0f) || m != 0.5f) return fail(-1, "floor kernel: step must be a power of two");
  hipStream_t s = (hipStream_t)stream;
  uint4* keys = (uint4*)workspace;
  hipLaunchKernelGGL(k_floor_keys, dim3((nclients + 255) / 256), dim3(256), 0, s, seeds, nclients, keys);
  int dev = 0, ncu = 256;
  (void)hipGetDevice(&dev);
  (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
  const int32_t T = (int32_t)tiles_for(P);
  // about 8 workgroups (32 waves) per CU in all; each part >= 64 tiles
  const int parts = (int)std::max<int64_t>(1, std::min<int64_t>((8LL * ncu + nclients - 1) / nclients, T / 64));
  const dim3 grid((unsigned)parts, (unsigned)nclients);
  // FEDCODEC_FLOOR_LDS (diagnostics): bytes of unused LDS per workgroup, to hold the
  // floor kernel to the encoder's occupancy (40960: 4 workgroups = 4 waves per SIMD)
  const char* le = std::getenv("FEDCODEC_FLOOR_LDS");
  const unsigned lds = le ? (unsigned)std::atoi(le) : 0u;
  // FEDCODEC_FLOOR_DEPTH (diagnostics): tiles in flight per wave, 1 (default) or 2
  const char* de = std::getenv("FEDCODEC_FLOOR_DEPTH");
  const bool deep = de && std::atoi(de) >= 2;
  void (*kern)(const float* const*, int64_t, int32_t, float, const uint4*, float*, int32_t*) =
      mode == FC_UNIFORM ? (deep ? k_quant_floor<FC_UNIFORM, 3> : k_quant_floor<FC_UNIFORM, 2>)
                         : (deep ? k_quant_floor<FC_STOCHASTIC, 3> : k_quant_floor<FC_STOCHASTIC, 2>);
  hipLaunchKernelGGL(kern, grid, dim3(256), lds, s, xs, P, T, 1.0f / step, keys, dist_part, nnz_part);
  return check_launch("k_quant_floor");
}

int fc_copy(void* dst, const void* src, int64_t nbytes, void* stream) {
  if (nbytes < 0 || (nbytes & 15) || ((uintptr_t)dst & 15) || ((uintptr_t)src & 15))
    return fail(-1, "fc_copy: 16-byte aligned pointers and a multiple of 16 bytes required");
  if (nbytes == 0) return 0;
  int dev = 0, ncu = 256;
  (void)hipGetDevice(&dev);
  (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
  const int64_t n = nbytes / 16;
#ifndef FC_COPY_WG
#define FC_COPY_WG 8
#endif
  const dim3 grid((unsigned)std::min<int64_t>((n + 256 * FC_COPY_U - 1) / (256 * FC_COPY_U), (int64_t)ncu * FC_COPY_WG));
  hipLaunchKernelGGL(k_copy_f4, grid, dim3(256), 0, (hipStream_t)stream, (uint4*)dst, (const uint4*)src, n);
  return check_launch("k_copy_f4");
}

int fc_diag_occupy(uint32_t xcd_mask, int64_t microseconds, int32_t* held, void* stream) {
  if (microseconds < 0 || microseconds > 5000000) return fail(-1, "fc_diag_occupy: 0 .. 5,000,000 microseconds");
  int dev = 0, ncu = 256;
  (void)hipGetDevice(&dev);
  (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
  hipLaunchKernelGGL(k_occupy, dim3((unsigned)ncu), dim3(64), 0, (hipStream_t)stream, xcd_mask & 0xFFu,
                     (uint64_t)microseconds * 100u, held);
  return check_launch("k_occupy");
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
  return fc_client_norms_scaled(xs, nclients, P, kind, nullptr, norms, stream);
}

int fc_client_norms_scaled(const float* const* xs, int32_t nclients, int64_t P, int kind, const float* prescale,
                           float* norms, void* stream) {
  if (nclients <= 0 || nclients > 65535 || P <= 0) return fail(-1, "bad sizes");
  if (kind < 1 || kind > 6) return fail(-1, "bad norm kind");
  if (!xs || !norms) return fail(-1, "null pointer");
  const int acc = kind == FC_NORM_MEAN_MAGNITUDE ? 0 : (kind == FC_NORM_MAX_MAGNITUDE || kind == FC_NORM_LINF) ? 2 : 1;
  void (*kern)(const float* const*, int64_t, const float*, double*) =
      prescale ? (acc == 0 ? k_client_norms<0, true> : acc == 1 ? k_client_norms<1, true> : k_client_norms<2, true>)
               : (acc == 0 ? k_client_norms<0, false> : acc == 1 ? k_client_norms<1, false> : k_client_norms<2, false>);
  hipStream_t s = (hipStream_t)stream;
  const int64_t nblk = red_blocks(P);
  const int parts = (int)std::min<int64_t>(nblk, client_parts(nclients, (P + 2047) / 2048, 8));  // 4x the resident workgroups (-1 to -2 %)
  double* part = nullptr;
  if (const int rc = scratch_for(s, sizeof(double) * 2 * (kNormThreads / 64) * (size_t)nclients * nblk, (void**)&part))
    return rc;
  hipLaunchKernelGGL(kern, dim3((unsigned)parts, (unsigned)nclients), dim3(kNormThreads), 0, s, xs, P, prescale, part);
  if (const int rc = check_launch("k_client_norms")) return rc;
  hipLaunchKernelGGL(k_norms_finalize, dim3((unsigned)nclients), dim3(64), 0, s, (const double*)part, nclients,
                     (int32_t)nblk, P, kind, norms);
  return check_launch("k_norms_finalize");
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
  if (nclients <= 0 || nclients > 65535 || P <= 0) return fail(-1, "bad sizes");
  if (!xs || !masks || !means || !dist) return fail(-1, "null pointer");
  if (const int rc = launch_mask_encode<0>(xs, nclients, P, threshold, 0, masks, means, dist, (hipStream_t)stream))
    return rc;
  hipLaunchKernelGGL(k_mask_distortion<0>, dim3(nclients), dim3(kObThreads), 0, (hipStream_t)stream, xs, P,
                     threshold, (const float*)means, dist);
  return check_launch("k_mask_distortion<0>");
}

int fc_onebit_decode_sum_range(const uint32_t* masks, const float* means, int32_t nclients, int64_t P,
                               int64_t word_begin, int64_t word_end, float* out, void* stream) {
  if (nclients <= 0 || P <= 0) return fail(-1, "bad sizes");
  if (!masks || !means || !out) return fail(-1, "null pointer");
  const int64_t nw = (P + 31) / 32;
  if (word_begin < 0 || word_end > nw || word_begin > word_end) return fail(-1, "bad word range");
  if (word_begin == word_end) return 0;
  const int64_t n = word_end - word_begin;
  hipLaunchKernelGGL(k_onebit_decode_sum, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                     masks, means, nclients, P, word_begin, word_end, out);
  return check_launch("k_onebit_decode_sum");
}

int fc_onebit_decode_sum(const uint32_t* masks, const float* means, int32_t nclients, int64_t P, float* out,
                         void* stream) {
  return fc_onebit_decode_sum_range(masks, means, nclients, P, 0, (P + 31) / 32, out, stream);
}

}  // extern "C"
