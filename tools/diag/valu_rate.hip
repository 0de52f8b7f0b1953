// VALU issue-rate microbenchmark (diagnostics): wave64 throughput of the
// instruction kinds k_encode's inner loop is made of, measured as SIMD cycles
// per instruction with the chip full (8 waves per SIMD, 8 independent chains
// per wave, each op in inline asm so no extra moves are generated).  Build:
//   hipcc --offload-arch=gfx950 -O3 -o tools/diag/valu_rate tools/diag/valu_rate.hip
#include <hip/hip_runtime.h>
#include <cstdio>

#define ITERS 2048
#define R8(M) M(a0) M(a1) M(a2) M(a3) M(a4) M(a5) M(a6) M(a7)

// 32-bit accumulators
#define K32(name, ins)                                                                      \
  __global__ __launch_bounds__(256) void name(uint32_t* out, uint32_t seed) {               \
    uint32_t a0 = threadIdx.x ^ seed, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4,    \
             a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;                                          \
    const uint32_t b = seed * 2654435761u;                                                   \
    const uint64_t m = (uint64_t)seed * 0x9E3779B97F4A7C15ull;                               \
    for (int i = 0; i < ITERS; ++i) {                                                        \
      R8(ins) R8(ins)                                                                        \
    }                                                                                        \
    out[blockIdx.x * 256 + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;             \
    (void)b; (void)m;                                                                        \
  }
// 64-bit accumulators
#define K64(name, ins)                                                                      \
  __global__ __launch_bounds__(256) void name(uint32_t* out, uint32_t seed) {               \
    uint64_t a0 = threadIdx.x ^ seed, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4,    \
             a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;                                          \
    const uint32_t b = seed * 2654435761u;                                                   \
    for (int i = 0; i < ITERS; ++i) {                                                        \
      R8(ins) R8(ins)                                                                        \
    }                                                                                        \
    out[blockIdx.x * 256 + threadIdx.x] = (uint32_t)(a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7); \
    (void)b;                                                                                 \
  }

#define V2(ins) (r) asm volatile(ins " %0, %0, %1" : "+v"(r) : "v"(b));
#define OP_ADD(r) asm volatile("v_add_u32 %0, %0, %1" : "+v"(r) : "v"(b));
#define OP_XOR(r) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(r) : "v"(b));
#define OP_MULF(r) asm volatile("v_mul_f32 %0, %0, %1" : "+v"(r) : "v"(b));
#define OP_FMAC(r) asm volatile("v_fmac_f32 %0, %1, %1" : "+v"(r) : "v"(b));
#define OP_FMAAK(r) asm volatile("v_fmaak_f32 %0, 4.0, %0, 0x4b400000" : "+v"(r));
#define OP_AND_OR(r) asm volatile("v_and_or_b32 %0, %0, %1, 1.0" : "+v"(r) : "v"(b));
#define OP_BITOP3(r) asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(r) : "v"(b), "s"(b));
#define OP_LSHLOR(r) asm volatile("v_lshl_or_b32 %0, %0, 8, %1" : "+v"(r) : "v"(b));
#define OP_ADD3(r) asm volatile("v_add3_u32 %0, %0, %1, %1" : "+v"(r) : "v"(b));
#define OP_BFE(r) asm volatile("v_bfe_u32 %0, %0, 4, 13" : "+v"(r));
#define OP_ALIGN(r) asm volatile("v_alignbit_b32 %0, %0, %1, 3" : "+v"(r) : "v"(b));
#define OP_LSHR(r) asm volatile("v_lshrrev_b32 %0, 16, %0" : "+v"(r));
#define OP_MOV(r) asm volatile("v_mov_b32 %0, %1" : "+v"(r) : "v"(b));
#define OP_CND(r) asm volatile("v_cndmask_b32_e64 %0, %0, %1, %2" : "+v"(r) : "v"(b), "s"(m));
#define OP_CMP(r) { uint64_t s_; asm volatile("v_cmp_gt_u32 %0, %1, %2" : "=s"(s_) : "v"(r), "v"(b)); r ^= 0; asm volatile("" :: "s"(s_)); }
#define OP_FLOOR(r) asm volatile("v_floor_f32 %0, %0" : "+v"(r));
#define OP_FRACT(r) asm volatile("v_fract_f32 %0, %0" : "+v"(r));
#define OP_RNDNE(r) asm volatile("v_rndne_f32 %0, %0" : "+v"(r));
#define OP_MAX3(r) asm volatile("v_max3_f32 %0, |%0|, |%1|, |%1|" : "+v"(r) : "v"(b));
#define OP_FFBH(r) asm volatile("v_ffbh_u32 %0, %0" : "+v"(r));
#define OP_MULLO(r) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(r) : "v"(b));
#define OP_CVT(r) asm volatile("v_cvt_u32_f32 %0, %0" : "+v"(r));
#define OP_DPP(r) asm volatile("v_add_u32_dpp %0, %0, %0 row_shr:1 bound_ctrl:1" : "+v"(r));
#define OP_SDWA(r) asm volatile("v_add_u32_sdwa %0, %0, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_1" : "+v"(r) : "v"(b));
#define OP_LSH64(r) asm volatile("v_lshlrev_b64 %0, %1, %0" : "+v"(r) : "v"(b));
#define OP_MAD64(r) asm volatile("v_mad_u64_u32 %0, s[20:21], %1, %2, %0" : "+v"(r) : "v"(b), "s"(0xD2511F53u) : "s20", "s21");
#define OP_LSHLADD64(r) asm volatile("v_lshl_add_u64 %0, %0, 0, %1" : "+v"(r) : "v"((uint64_t)b));
#define OP_MOV64(r) asm volatile("v_mov_b64 %0, %1" : "+v"(r) : "v"((uint64_t)b));
#define OP_PKADD(r) asm volatile("v_pk_add_f32 %0, %0, %1" : "+v"(r) : "v"((uint64_t)b));
#define OP_PKFMA(r) asm volatile("v_pk_fma_f32 %0, %0, %1, %0" : "+v"(r) : "v"((uint64_t)b));


#define OP_CMPVCC(r) asm volatile("v_cmp_gt_u32_e32 vcc, %0, %1" :: "v"(r), "v"(b) : "vcc");
#define OP_CNDVCC(r) asm volatile("v_cndmask_b32_e32 %0, %0, %1, vcc" : "+v"(r) : "v"(b));
#define OP_AND(r) asm volatile("v_and_b32 %0, %0, %1" : "+v"(r) : "v"(b));
#define OP_OR(r) asm volatile("v_or_b32 %0, %0, %1" : "+v"(r) : "v"(b));
#define OP_LSHL(r) asm volatile("v_lshlrev_b32 %0, %1, %0" : "+v"(r) : "v"(b));
#define OP_SUBF(r) asm volatile("v_sub_f32 %0, %0, %1" : "+v"(r) : "v"(b));
#define OP_ADDF(r) asm volatile("v_add_f32 %0, %0, %1" : "+v"(r) : "v"(b));
#define OP_ADDFABS(r) asm volatile("v_add_f32_e64 %0, |%0|, %1" : "+v"(r) : "v"(b));
#define OP_SUBU(r) asm volatile("v_sub_u32 %0, %0, %1" : "+v"(r) : "v"(b));
#define OP_CEIL(r) asm volatile("v_ceil_f32 %0, %0" : "+v"(r));
#define OP_MAXF(r) asm volatile("v_max_f32 %0, %0, %1" : "+v"(r) : "v"(b));
#define OP_MAXI(r) asm volatile("v_max_i32 %0, %0, %1" : "+v"(r) : "v"(b));
#define OP_MINU(r) asm volatile("v_min_u32 %0, %0, %1" : "+v"(r) : "v"(b));
#define OP_FMAMK(r) asm volatile("v_fmamk_f32 %0, %0, 0x4b400000, %1" : "+v"(r) : "v"(b));
#define OP_CVTF(r) asm volatile("v_cvt_f32_u32 %0, %0" : "+v"(r));
#define OP_MUL24(r) asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(r) : "v"(b));
#define OP_BFI(r) asm volatile("v_bfi_b32 %0, %0, %1, %1" : "+v"(r) : "v"(b));
#define OP_PERM(r) asm volatile("v_perm_b32 %0, %0, %1, %2" : "+v"(r) : "v"(b), "v"(0x3020100u));
#define OP_MED3(r) asm volatile("v_med3_f32 %0, %0, %1, %1" : "+v"(r) : "v"(b));
#define OP_ADDNC(r) asm volatile("v_add_u32_e64 %0, %0, %1" : "+v"(r) : "v"(b));
#define OP_LSHL64C(r) asm volatile("v_lshlrev_b64 %0, 3, %0" : "+v"(r));
#define OP_MIX(r) asm volatile("v_floor_f32 %0, %0\n v_add_u32 %0, %0, %1" : "+v"(r) : "v"(b));
#define OP_MIX2(r) asm volatile("v_floor_f32 %0, %0\n v_ffbh_u32 %0, %0" : "+v"(r));
#define OP_XORMIX(r) asm volatile("v_xor_b32 %0, %0, %1\n v_add_u32 %0, %0, %1" : "+v"(r) : "v"(b));

K32(k_cmpvcc, OP_CMPVCC) K32(k_cndvcc, OP_CNDVCC) K32(k_and, OP_AND) K32(k_or, OP_OR) K32(k_lshl, OP_LSHL)
K32(k_subf, OP_SUBF) K32(k_addf, OP_ADDF) K32(k_addfabs, OP_ADDFABS) K32(k_subu, OP_SUBU) K32(k_ceil, OP_CEIL)
K32(k_maxf, OP_MAXF) K32(k_maxi, OP_MAXI) K32(k_minu, OP_MINU) K32(k_fmamk, OP_FMAMK) K32(k_cvtf, OP_CVTF)
K32(k_mul24, OP_MUL24) K32(k_bfi, OP_BFI) K32(k_perm, OP_PERM) K32(k_med3, OP_MED3) K32(k_addnc, OP_ADDNC)
K64(k_lsh64c, OP_LSHL64C) K32(k_mix, OP_MIX) K32(k_mix2, OP_MIX2) K32(k_xormix, OP_XORMIX)
K32(k_add, OP_ADD) K32(k_xor, OP_XOR) K32(k_mulf, OP_MULF) K32(k_fmac, OP_FMAC) K32(k_fmaak, OP_FMAAK)
K32(k_and_or, OP_AND_OR) K32(k_bitop3, OP_BITOP3) K32(k_lshlor, OP_LSHLOR) K32(k_add3, OP_ADD3)
K32(k_bfe, OP_BFE) K32(k_align, OP_ALIGN) K32(k_lshr, OP_LSHR) K32(k_mov, OP_MOV) K32(k_cnd, OP_CND)
K32(k_cmp, OP_CMP) K32(k_floor, OP_FLOOR) K32(k_fract, OP_FRACT) K32(k_rndne, OP_RNDNE)
K32(k_max3, OP_MAX3) K32(k_ffbh, OP_FFBH) K32(k_mullo, OP_MULLO) K32(k_cvt, OP_CVT) K32(k_dpp, OP_DPP)
K32(k_sdwa, OP_SDWA)
K64(k_lsh64, OP_LSH64) K64(k_mad64, OP_MAD64) K64(k_lshladd64, OP_LSHLADD64) K64(k_mov64, OP_MOV64)
K64(k_pkadd, OP_PKADD) K64(k_pkfma, OP_PKFMA)

typedef void (*KFn)(uint32_t*, uint32_t);

int main() {
  hipDeviceProp_t prop;
  (void)hipGetDeviceProperties(&prop, 0);
  const int cus = prop.multiProcessorCount;
  const double clk = prop.clockRate * 1e3;  // Hz
  const int blocks = cus * 8;               // 256-thread blocks (4 waves): 8 waves per SIMD
  uint32_t* out;
  (void)hipMalloc(&out, (size_t)blocks * 256 * 4);
  struct { const char* name; KFn fn; } ks[] = {
      {"v_cmp_gt_u32_e32(vcc)", k_cmpvcc}, {"v_cndmask_b32_e32(vcc)", k_cndvcc}, {"v_and_b32", k_and},
      {"v_or_b32", k_or}, {"v_lshlrev_b32", k_lshl}, {"v_sub_f32", k_subf}, {"v_add_f32", k_addf},
      {"v_add_f32_e64 |a|", k_addfabs}, {"v_sub_u32", k_subu}, {"v_ceil_f32", k_ceil}, {"v_max_f32", k_maxf},
      {"v_max_i32", k_maxi}, {"v_min_u32", k_minu}, {"v_fmamk_f32", k_fmamk}, {"v_cvt_f32_u32", k_cvtf},
      {"v_mul_u32_u24", k_mul24}, {"v_bfi_b32", k_bfi}, {"v_perm_b32", k_perm}, {"v_med3_f32", k_med3},
      {"v_add_u32_e64", k_addnc}, {"v_lshlrev_b64 const", k_lsh64c},
      {"floor+add (per pair/2)", k_mix}, {"floor+ffbh (per pair/2)", k_mix2}, {"xor+add (per pair/2)", k_xormix},
      {"v_add_u32", k_add}, {"v_xor_b32", k_xor}, {"v_mul_f32", k_mulf}, {"v_fmac_f32", k_fmac},
      {"v_fmaak_f32", k_fmaak}, {"v_and_or_b32", k_and_or}, {"v_bitop3_b32", k_bitop3},
      {"v_lshl_or_b32", k_lshlor}, {"v_add3_u32", k_add3}, {"v_bfe_u32", k_bfe},
      {"v_alignbit_b32", k_align}, {"v_lshrrev_b32", k_lshr}, {"v_mov_b32", k_mov},
      {"v_cndmask_b32(sgpr)", k_cnd}, {"v_cmp_gt_u32(->sgpr)", k_cmp}, {"v_floor_f32", k_floor},
      {"v_fract_f32", k_fract}, {"v_rndne_f32", k_rndne}, {"v_max3_f32", k_max3},
      {"v_ffbh_u32", k_ffbh}, {"v_mul_lo_u32", k_mullo}, {"v_cvt_u32_f32", k_cvt},
      {"v_add_u32_dpp", k_dpp}, {"v_add_u32_sdwa", k_sdwa}, {"v_lshlrev_b64", k_lsh64},
      {"v_mad_u64_u32", k_mad64}, {"v_lshl_add_u64", k_lshladd64}, {"v_mov_b64", k_mov64},
      {"v_pk_add_f32", k_pkadd}, {"v_pk_fma_f32", k_pkfma}};
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  printf("CUs %d clock %.0f MHz blocks %d (8 waves per SIMD)\n", cus, clk / 1e6, blocks);
  for (auto& k : ks) {
    hipLaunchKernelGGL(k.fn, dim3(blocks), dim3(256), 0, 0, out, 1u);
    (void)hipEventRecord(e0);
    for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(k.fn, dim3(blocks), dim3(256), 0, 0, out, 1u + r);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    const double instr = (double)ITERS * 16 * 8.0 * 5;  // per SIMD: 16 ops x 8 waves x 5 launches
    printf("%-28s %.3f ms  %.2f SIMD cycles / wave64 instr\n", k.name, ms / 5, (ms * 1e-3) * clk / instr);
  }
  return 0;
}
