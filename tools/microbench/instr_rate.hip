// Diagnostic: issue cost of single VALU instructions on gfx950 (cycles per
// wave64 instruction per SIMD, at several waves per SIMD).  Each lane runs 8
// independent chains of one instruction; time / (instructions per SIMD) gives
// the throughput cost.  Build: hipcc --offload-arch=gfx950 -O3 -o ir instr_rate.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

constexpr int kIters = 4096;

#define BODY8(ASM)                                                                            \
  _Pragma("unroll 1") for (int i = 0; i < kIters; ++i) {                                       \
    ASM(a0, b0) ASM(a1, b1) ASM(a2, b2) ASM(a3, b3) ASM(a4, b4) ASM(a5, b5) ASM(a6, b6) ASM(a7, b7) \
  }

#define K(NAME, ASM)                                                                          \
  __global__ void NAME(uint32_t* out, uint32_t seed) {                                        \
    uint32_t a0 = threadIdx.x ^ seed, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4,    \
             a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;                                           \
    uint32_t b0 = a0 * 3, b1 = a1 * 3, b2 = a2 * 3, b3 = a3 * 3, b4 = a4 * 3, b5 = a5 * 3,   \
             b6 = a6 * 3, b7 = a7 * 3;                                                        \
    BODY8(ASM)                                                                                \
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7 ^ b0 ^ b1 ^ b2 ^ b3 ^ b4 ^ b5 ^ b6 ^ b7; \
  }

// the constraint-based forms below keep register allocation with the compiler
#define A_MAD(x, y) { uint64_t r, cc; asm volatile("v_mad_u64_u32 %0, %1, %2, %3, 0" : "=v"(r), "=s"(cc) : "v"(x), "v"(y)); x = (uint32_t)r; y = (uint32_t)(r >> 32); }
#define A_MULHI(x, y) asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(x) : "v"(y));
#define A_MULLO(x, y) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(x) : "v"(y));
#define A_MUL24(x, y) asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(x) : "v"(y));
#define A_ADD(x, y) asm volatile("v_add_u32 %0, %0, %1" : "+v"(x) : "v"(y));
#define A_XOR3(x, y) asm volatile("v_bitop3_b32 %0, %0, %1, %0 bitop3:0x96" : "+v"(x) : "v"(y));
#define A_FMA(x, y) asm volatile("v_fma_f32 %0, %0, %1, %0" : "+v"(x) : "v"(y));
#define A_SHL64(x, y) { uint64_t r = ((uint64_t)y << 32) | x; asm volatile("v_lshlrev_b64 %0, 3, %0" : "+v"(r)); x = (uint32_t)r; y = (uint32_t)(r >> 32); }
#define A_CNDMASK(x, y) asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(x) : "v"(y));
#define A_CVT(x, y) asm volatile("v_cvt_f32_u32 %0, %0" : "+v"(x));
#define A_FLOOR(x, y) asm volatile("v_floor_f32 %0, %0" : "+v"(x));
#define A_DPP(x, y) asm volatile("v_add_u32_dpp %0, %0, %0 row_shr:1 row_mask:0xf bank_mask:0xf" : "+v"(x));
#define A_PKFMA(x, y) { uint64_t r = ((uint64_t)y << 32) | x; asm volatile("v_pk_fma_f32 %0, %0, %0, %0" : "+v"(r)); x = (uint32_t)r; y = (uint32_t)(r >> 32); }


#define A_CND64(x, y) asm volatile("v_cndmask_b32_e64 %0, %0, %1, s[4:5]" : "+v"(x) : "v"(y) : "s4", "s5");
#define A_CMP(x, y) asm volatile("v_cmp_lt_u32_e64 s[6:7], %0, %1" :: "v"(x), "v"(y) : "s6", "s7");
#define A_CMPCND(x, y) asm volatile("v_cmp_lt_u32_e64 s[6:7], %0, %1\n\tv_cndmask_b32_e64 %0, %0, %1, s[6:7]" : "+v"(x) : "v"(y) : "s6", "s7");
#define A_LSHLOR(x, y) asm volatile("v_lshl_or_b32 %0, %0, 3, %1" : "+v"(x) : "v"(y));
#define A_ALIGNBIT(x, y) asm volatile("v_alignbit_b32 %0, %0, %1, 7" : "+v"(x) : "v"(y));
#define A_BFE(x, y) asm volatile("v_bfe_u32 %0, %0, 3, 9" : "+v"(x));
#define A_FFBH(x, y) asm volatile("v_ffbh_u32 %0, %0" : "+v"(x));
#define A_MAX3(x, y) asm volatile("v_max3_f32 %0, |%0|, |%1|, %0" : "+v"(x) : "v"(y));
#define A_CVTI(x, y) asm volatile("v_cvt_i32_f32 %0, %0" : "+v"(x));
#define A_MULF(x, y) asm volatile("v_mul_f32 %0, %0, %1" : "+v"(x) : "v"(y));
#define A_ANDOR(x, y) asm volatile("v_and_or_b32 %0, %0, %1, %0" : "+v"(x) : "v"(y));
#define A_LSHLADD64(x, y) { uint64_t r = ((uint64_t)y << 32) | x; asm volatile("v_lshl_add_u64 %0, %0, 2, %0" : "+v"(r)); x = (uint32_t)r; y = (uint32_t)(r >> 32); }
#define A_MOV(x, y) asm volatile("v_mov_b32 %0, %1" : "=v"(x) : "v"(y));
#define A_MAXDPP(x, y) asm volatile("v_max_i32_dpp %0, %0, %0 row_shr:1 row_mask:0xf bank_mask:0xf" : "+v"(x));
#define A_CEIL(x, y) asm volatile("v_ceil_f32 %0, %0" : "+v"(x));
#define A_RNDNE(x, y) asm volatile("v_rndne_f32 %0, %0" : "+v"(x));
#define A_LSHL32(x, y) asm volatile("v_lshlrev_b32 %0, %1, %0" : "+v"(x) : "v"(y));
#define A_WRITELANE(x, y) asm volatile("v_writelane_b32 %0, s8, 5" : "+v"(x) :: "s8");
#define A_READLANE(x, y) asm volatile("v_readlane_b32 s9, %0, 5" :: "v"(x) : "s9");
#define A_MBCNT(x, y) asm volatile("v_mbcnt_lo_u32_b32 %0, -1, %0" : "+v"(x));
#define A_DSOR(x, y) asm volatile("ds_or_b32 %0, %1" :: "v"(x & 0xFFCu), "v"(y) : "memory");
#define A_DSREAD(x, y) asm volatile("ds_read_b32 %0, %1" : "=v"(x) : "v"(y & 0x3FCu) : "memory");

#define A_ADDSDWA(x, y) asm volatile("v_add_u32_sdwa %0, %0, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_1" : "+v"(x) : "v"(y));
#define A_MOVSDWA(x, y) asm volatile("v_mov_b32_sdwa %0, sext(%1) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_2" : "=v"(x) : "v"(y));
#define A_BFEI(x, y) asm volatile("v_bfe_i32 %0, %0, 16, 8" : "+v"(x));
#define A_ASHR(x, y) asm volatile("v_ashrrev_i32 %0, 24, %0" : "+v"(x));
#define A_AND(x, y) asm volatile("v_and_b32 %0, %0, %1" : "+v"(x) : "v"(y));
#define A_SUB(x, y) asm volatile("v_sub_u32 %0, %0, %1" : "+v"(x) : "v"(y));
#define A_MIN(x, y) asm volatile("v_min_u32 %0, %0, %1" : "+v"(x) : "v"(y));
#define A_LSHLADD(x, y) asm volatile("v_lshl_add_u32 %0, %0, 2, %1" : "+v"(x) : "v"(y));
#define A_ADD3(x, y) asm volatile("v_add3_u32 %0, %0, %1, %0" : "+v"(x) : "v"(y));
K(k_mad, A_MAD)
K(k_mulhi, A_MULHI)
K(k_mullo, A_MULLO)
K(k_mul24, A_MUL24)
K(k_add, A_ADD)
K(k_xor3, A_XOR3)
K(k_fma, A_FMA)
K(k_shl64, A_SHL64)
K(k_cndmask, A_CNDMASK)
K(k_cvt, A_CVT)
K(k_floor, A_FLOOR)
K(k_dpp, A_DPP)
K(k_pkfma, A_PKFMA)
K(k_addsdwa, A_ADDSDWA)
K(k_movsdwa, A_MOVSDWA)
K(k_bfei, A_BFEI)
K(k_ashr, A_ASHR)
K(k_and, A_AND)
K(k_sub, A_SUB)
K(k_min, A_MIN)
K(k_lshladd, A_LSHLADD)
K(k_add3, A_ADD3)
K(k_cnd64, A_CND64)
K(k_cmp, A_CMP)
K(k_cmpcnd, A_CMPCND)
K(k_lshlor, A_LSHLOR)
K(k_alignbit, A_ALIGNBIT)
K(k_bfe, A_BFE)
K(k_ffbh, A_FFBH)
K(k_max3, A_MAX3)
K(k_cvti, A_CVTI)
K(k_mulf, A_MULF)
K(k_andor, A_ANDOR)
K(k_lshladd64, A_LSHLADD64)
K(k_mov, A_MOV)
K(k_maxdpp, A_MAXDPP)
K(k_ceil, A_CEIL)
K(k_rndne, A_RNDNE)
K(k_lshl32, A_LSHL32)
K(k_writelane, A_WRITELANE)
K(k_readlane, A_READLANE)
K(k_mbcnt, A_MBCNT)

int main() {
  int ncu = 0;
  CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
  int clk_khz = 0;
  CK(hipDeviceGetAttribute(&clk_khz, hipDeviceAttributeClockRate, 0));
  uint32_t* out;
  CK(hipMalloc(&out, sizeof(uint32_t) * 256 * 1024 * 64));
  struct { const char* n; void (*k)(uint32_t*, uint32_t); } ks[] = {
      {"v_mad_u64_u32", k_mad}, {"v_mul_hi_u32", k_mulhi}, {"v_mul_lo_u32", k_mullo},
      {"v_mul_u32_u24", k_mul24}, {"v_add_u32", k_add}, {"v_bitop3_b32", k_xor3},
      {"v_fma_f32", k_fma}, {"v_lshlrev_b64", k_shl64}, {"v_cndmask_b32", k_cndmask},
      {"v_cvt_f32_u32", k_cvt}, {"v_floor_f32", k_floor}, {"v_add_u32_dpp", k_dpp},
      {"v_pk_fma_f32", k_pkfma}, {"ADDSDWA", k_addsdwa}, {"MOVSDWA", k_movsdwa}, {"BFEI", k_bfei}, {"ASHR", k_ashr}, {"AND", k_and}, {"SUB", k_sub}, {"MIN", k_min}, {"LSHLADD", k_lshladd}, {"ADD3", k_add3}, {"CND64", k_cnd64}, {"CMP", k_cmp}, {"CMPCND", k_cmpcnd}, {"LSHLOR", k_lshlor}, {"ALIGNBIT", k_alignbit}, {"BFE", k_bfe}, {"FFBH", k_ffbh}, {"MAX3", k_max3}, {"CVTI", k_cvti}, {"MULF", k_mulf}, {"ANDOR", k_andor}, {"LSHLADD64", k_lshladd64}, {"MOV", k_mov}, {"MAXDPP", k_maxdpp}, {"CEIL", k_ceil}, {"RNDNE", k_rndne}, {"LSHL32", k_lshl32}, {"WRITELANE", k_writelane}, {"READLANE", k_readlane}, {"MBCNT", k_mbcnt}};
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  printf("CUs %d, clock %d MHz (nominal)\n", ncu, clk_khz / 1000);
  for (int wps : {8}) {  // waves per SIMD
    const int blocks = ncu * 4 * wps;
    for (auto& k : ks) {
      hipLaunchKernelGGL(k.k, dim3(blocks), dim3(64), 0, 0, out, 1u);
      CK(hipDeviceSynchronize());
      CK(hipEventRecord(e0));
      hipLaunchKernelGGL(k.k, dim3(blocks), dim3(64), 0, 0, out, 2u);
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, e0, e1));
      const double insts_per_simd = (double)wps * kIters * 8;
      const double cyc = ms * 1e-3 * 2.1e9 / insts_per_simd;  // at an assumed 2.1 GHz
      printf("waves/SIMD %d  %-16s %8.3f ms  %6.2f cyc/instr (at 2.1 GHz)\n", wps, k.n, ms, cyc);
    }
  }
  return 0;
}
