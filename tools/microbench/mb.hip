// Microbenchmarks that size the codec design on MI355X (gfx950):
//  - HBM read / copy rate for float4 streams (the roofline the codec is priced against)
//  - Philox4x32-10 throughput (stochastic rounding RNG cost per element)
//  - fused read + Philox + stochastic rounding (is stochastic mode ALU- or HBM-bound?)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

__device__ __forceinline__ void philox_round(uint32_t& c0, uint32_t& c1, uint32_t& c2, uint32_t& c3,
                                             uint32_t k0, uint32_t k1) {
  uint64_t p0 = (uint64_t)0xD2511F53u * c0;
  uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
  uint32_t n0 = (uint32_t)(p1 >> 32) ^ c1 ^ k0;
  uint32_t n2 = (uint32_t)(p0 >> 32) ^ c3 ^ k1;
  c1 = (uint32_t)p1;
  c3 = (uint32_t)p0;
  c0 = n0;
  c2 = n2;
}

__device__ __forceinline__ uint4 philox10(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3,
                                          uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    philox_round(c0, c1, c2, c3, k0, k1);
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  return make_uint4(c0, c1, c2, c3);
}

__global__ void k_read(const float4* __restrict__ x, size_t n4, float* out) {
  float acc = 0.f;
  size_t stride = (size_t)gridDim.x * blockDim.x;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
    float4 v = x[i];
    acc += v.x + v.y + v.z + v.w;
  }
  if (acc == 1234.5f) out[0] = acc;
}

__global__ void k_read_unroll(const float4* __restrict__ x, size_t n4, float* out) {
  // each block handles contiguous 4096-float tiles, 4 float4 per thread (the codec tile shape)
  float acc = 0.f;
  size_t ntiles = n4 / 1024;
  for (size_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
    const float4* p = x + t * 1024 + threadIdx.x;
    float4 v0 = p[0], v1 = p[256], v2 = p[512], v3 = p[768];
    acc += v0.x + v0.y + v0.z + v0.w + v1.x + v1.y + v1.z + v1.w + v2.x + v2.y + v2.z + v2.w + v3.x + v3.y + v3.z + v3.w;
  }
  if (acc == 1234.5f) out[0] = acc;
}

__global__ void k_copy(const float4* __restrict__ x, float4* __restrict__ y, size_t n4) {
  size_t stride = (size_t)gridDim.x * blockDim.x;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) y[i] = x[i];
}

__global__ void k_philox(size_t ngroups, uint32_t k0, uint32_t k1, uint32_t* out) {
  uint32_t acc = 0;
  size_t stride = (size_t)gridDim.x * blockDim.x;
  for (size_t g = (size_t)blockIdx.x * blockDim.x + threadIdx.x; g < ngroups; g += stride) {
    uint4 r = philox10((uint32_t)g, 0, 0x1234u, 0x5678u, k0, k1);
    acc ^= r.x ^ r.y ^ r.z ^ r.w;
  }
  if (acc == 0xdeadbeefu) out[0] = acc;
}

__global__ void k_stoch(const float4* __restrict__ x, size_t n4, float step, uint32_t k0, uint32_t k1,
                        int* out) {
  int acc = 0;
  size_t stride = (size_t)gridDim.x * blockDim.x;
  for (size_t g = (size_t)blockIdx.x * blockDim.x + threadIdx.x; g < n4; g += stride) {
    float4 v = x[g];
    uint4 r = philox10((uint32_t)g, 0, 0x1234u, 0x5678u, k0, k1);
    float vv[4] = {v.x, v.y, v.z, v.w};
    uint32_t rr[4] = {r.x, r.y, r.z, r.w};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      float s = vv[k] / step;
      float fl = floorf(s);
      float p = s - fl;
      float u = __uint_as_float((rr[k] & 0x7fffffu) | 0x3f800000u) - 1.0f;
      float q = (u <= p) ? ceilf(s) : fl;
      acc += (int)q;
    }
  }
  if (acc == 0x7eadbeef) out[0] = acc;
}

int main() {
  int dev = 0;
  hipDeviceProp_t prop;
  CK(hipGetDeviceProperties(&prop, dev));
  printf("device %s CUs %d clock %d kHz\n", prop.gcnArchName, prop.multiProcessorCount, prop.clockRate);
  size_t nbytes = (size_t)2 << 30;  // 2 GiB: far beyond the 256 MiB Infinity Cache
  size_t n4 = nbytes / 16;
  float4 *x, *y;
  float* o;
  CK(hipMalloc(&x, nbytes));
  CK(hipMalloc(&y, nbytes));
  CK(hipMalloc(&o, 64));
  CK(hipMemset(x, 0x3c, nbytes));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  float ms;
  int grids[] = {1024, 2048, 4096, 8192};
  for (int gi = 0; gi < 4; ++gi) {
    int g = grids[gi];
    for (int it = 0; it < 2; ++it) {
      hipEventRecord(a);
      k_read<<<g, 256>>>(x, n4, o);
      hipEventRecord(b);
      hipEventSynchronize(b);
    }
    hipEventElapsedTime(&ms, a, b);
    printf("read   grid %5d: %.1f GB/s\n", g, nbytes / ms / 1e6);
    for (int it = 0; it < 2; ++it) {
      hipEventRecord(a);
      k_read_unroll<<<g, 256>>>(x, n4, o);
      hipEventRecord(b);
      hipEventSynchronize(b);
    }
    hipEventElapsedTime(&ms, a, b);
    printf("readU  grid %5d: %.1f GB/s\n", g, nbytes / ms / 1e6);
    for (int it = 0; it < 2; ++it) {
      hipEventRecord(a);
      k_copy<<<g, 256>>>(x, y, n4);
      hipEventRecord(b);
      hipEventSynchronize(b);
    }
    hipEventElapsedTime(&ms, a, b);
    printf("copy   grid %5d: %.1f GB/s (r+w)\n", g, 2.0 * nbytes / ms / 1e6);
  }
  size_t ng = (size_t)1 << 28;
  for (int it = 0; it < 2; ++it) {
    hipEventRecord(a);
    k_philox<<<8192, 256>>>(ng, 1, 2, (uint32_t*)o);
    hipEventRecord(b);
    hipEventSynchronize(b);
  }
  hipEventElapsedTime(&ms, a, b);
  printf("philox: %.1f G calls/s = %.1f G elem/s\n", ng / ms / 1e6, 4.0 * ng / ms / 1e6);
  for (int gi = 0; gi < 4; ++gi) {
    int g = grids[gi];
    for (int it = 0; it < 2; ++it) {
      hipEventRecord(a);
      k_stoch<<<g, 256>>>(x, n4, 0.37f, 1, 2, (int*)o);
      hipEventRecord(b);
      hipEventSynchronize(b);
    }
    hipEventElapsedTime(&ms, a, b);
    printf("stoch  grid %5d: %.1f GB/s read\n", g, nbytes / ms / 1e6);
  }
  return 0;
}
