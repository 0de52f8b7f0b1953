// Diagnostic: FETCH_SIZE calibration for the decoder's read pattern (MI355X_MICROARCH.md,
// HBM: "calibrate on a known byte count in your own access pattern").
//
// Every lane streams its own contiguous segment of S bytes in 16-byte loads, one load
// every D dependent VALU steps (the decoder takes a 16-byte block every few loop
// iterations); the 64 lanes of a wave read 64 segments that lie far apart (the
// decoder's lanes are clients).  Each byte is read exactly once, so FETCH_SIZE /
// bytes is the counter's multiplier for this pattern at that pace.  A coalesced
// variant (each wave reads 1 KiB contiguous per instruction) reproduces the guide's
// "1/2 of the bytes" for wide streaming reads as the reference point.
//
// Build: hipcc --offload-arch=gfx950 -O3 -o fetch_calib fetch_calib.hip
// Run:   rocprofv3 --pmc FETCH_SIZE --kernel-trace -- ./fetch_calib  (kernel per line: bytes read)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

// lane = one segment of seg_blocks 16-byte blocks; segments of one wave are
// `stride` segments apart in memory (different "clients")
template <int D>
__global__ __launch_bounds__(256) void k_lane_streams(const uint4* __restrict__ buf, int64_t nseg, int seg_blocks,
                                                      int64_t stride, uint32_t* out) {
  const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= nseg) return;
  // lane-major: lane l of wave w reads segment (l * stride + w) mod nseg
  const int64_t w = g >> 6, l = g & 63;
  const int64_t s = (l * stride + w) % nseg;
  const uint4* p = buf + s * seg_blocks;
  uint32_t acc = (uint32_t)g;
  for (int b = 0; b < seg_blocks; ++b) {
    const uint4 v = p[b];
    acc ^= v.x + v.y + v.z + v.w;
#pragma unroll
    for (int i = 0; i < D; ++i) acc = acc * 2654435761u + (uint32_t)i;  // the decoder's work between blocks
  }
  if (acc == 0x12345678u) out[0] = acc;  // keep the loads
}

__global__ __launch_bounds__(256) void k_coalesced(const uint4* __restrict__ buf, int64_t nblocks, uint32_t* out) {
  uint32_t acc = 0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nblocks; i += (int64_t)gridDim.x * blockDim.x) {
    const uint4 v = buf[i];
    acc ^= v.x + v.y + v.z + v.w;
  }
  if (acc == 0x12345678u) out[0] = acc;
}

int main() {
  const int seg_blocks = 64;             // 1 KiB per lane segment (the headline's two-tile segments: ~1 KB)
  const int64_t nseg = 4 << 20;          // 4 Mi segments: 4 GiB, far past the 256 MiB Infinity Cache
  const int64_t bytes = nseg * seg_blocks * 16;
  uint4* buf;
  uint32_t* out;
  CK(hipMalloc(&buf, bytes));
  CK(hipMalloc(&out, 4));
  CK(hipMemset(buf, 1, bytes));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int64_t stride = 65537;  // lanes of a wave 64 KiB x 1.00002 apart
  auto run = [&](const char* name, auto launch) -> int {
    launch();
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0));
    launch();
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    printf("%-34s %10lld bytes  %8.3f ms  %7.0f GB/s\n", name, (long long)bytes, ms, bytes / ms / 1e6);
    return 0;
  };
  const dim3 grid((unsigned)((nseg + 255) / 256));
  if (run("lane streams, D=0", [&] { hipLaunchKernelGGL(k_lane_streams<0>, grid, dim3(256), 0, 0, buf, nseg, seg_blocks, stride, out); }))
    return 1;
  if (run("lane streams, D=64", [&] { hipLaunchKernelGGL(k_lane_streams<64>, grid, dim3(256), 0, 0, buf, nseg, seg_blocks, stride, out); }))
    return 1;
  if (run("lane streams, D=256", [&] { hipLaunchKernelGGL(k_lane_streams<256>, grid, dim3(256), 0, 0, buf, nseg, seg_blocks, stride, out); }))
    return 1;
  if (run("coalesced 16 B/lane", [&] { hipLaunchKernelGGL(k_coalesced, dim3(4096), dim3(256), 0, 0, buf, bytes / 16, out); }))
    return 1;
  CK(hipFree(buf));
  CK(hipFree(out));
  return 0;
}
