// Diagnostic: WRITE_SIZE calibration for the encoder's store pattern (MI355X_MICROARCH.md,
// HBM: "calibrate on a known byte count in your own access pattern").
//
// The encoder's waves each store one ticket's code words (~1.9 KB at the headline's
// 3.8 bits per element) with 4-byte lane stores, 256 B per wave instruction, into the
// ticket's client stream; consecutive tickets of one client are C tickets apart in time
// (tile-major tickets), so the 128-B line at a ticket boundary is written partly by
// two waves microseconds apart.  Each byte is written exactly once, so WRITE_SIZE /
// bytes is the counter's multiplier (and the real write amplification) for:
//   coalesced   16 B per lane, grid-stride (the reference point)
//   regions R   R words per ticket, tile-major tickets over C client streams,
//               store instructions from the ticket's first word (unaligned)
//   aligned R   the same, store instructions from the 128-B line holding it
// R = 512 words (2 KiB: ticket boundaries on line boundaries) and R = 486 (1944 B).
//
// Build: hipcc --offload-arch=gfx950 -O3 -o write_calib write_calib.hip
// Run:   rocprofv3 --pmc WRITE_SIZE --kernel-trace -- ./write_calib
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

__global__ __launch_bounds__(256) void k_coalesced_store(uint4* __restrict__ buf, int64_t nblocks) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nblocks; i += (int64_t)gridDim.x * blockDim.x)
    buf[i] = make_uint4((uint32_t)i, 1u, 2u, 3u);
}

// one wave per ticket stream position: wave w codes tickets w, w + nwaves, ...;
// ticket k -> tile t = k / C, client c = k % C; its words at c * T * R + t * R
template <bool ALIGN>
__global__ __launch_bounds__(64) void k_regions(uint32_t* __restrict__ buf, int C, int T, int R) {
  const int lane = threadIdx.x;
  const int64_t total = (int64_t)C * T;
  for (int64_t k = blockIdx.x; k < total; k += gridDim.x) {
    const int64_t t = k / C, c = k - t * C;
    uint32_t* out = buf + (c * T + t) * (int64_t)R;
    const uint32_t lead = ALIGN ? (uint32_t)(((uintptr_t)out >> 2) & 31u) : 0u;
    for (uint32_t j = lane; j < (uint32_t)R + lead; j += 64) {
      if (j < lead) continue;
      out[j - lead] = (uint32_t)(k * 977 + j);
    }
  }
}

int main() {
  const int C = 1024, T = 1024;
  const int64_t max_words = (int64_t)C * T * 512;  // 2 GiB
  uint32_t* buf;
  CK(hipMalloc(&buf, max_words * 4));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto run = [&](const char* name, int64_t bytes, auto launch) -> int {
    launch();
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0));
    launch();
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    printf("%-28s %11lld bytes  %8.3f ms  %7.0f GB/s\n", name, (long long)bytes, ms, bytes / ms / 1e6);
    return 0;
  };
  const int64_t cb = max_words * 4;
  if (run("coalesced 16 B/lane", cb, [&] {
        hipLaunchKernelGGL(k_coalesced_store, dim3(4096), dim3(256), 0, 0, (uint4*)buf, cb / 16);
      }))
    return 1;
  const int Rs[2] = {512, 486};
  for (int i = 0; i < 2; ++i) {
    const int R = Rs[i];
    const int64_t b = (int64_t)C * T * R * 4;
    char n0[64], n1[64];
    snprintf(n0, sizeof n0, "regions R=%d", R);
    snprintf(n1, sizeof n1, "aligned R=%d", R);
    if (run(n0, b, [&] { hipLaunchKernelGGL(k_regions<false>, dim3(16384), dim3(64), 0, 0, buf, C, T, R); })) return 1;
    if (run(n1, b, [&] { hipLaunchKernelGGL(k_regions<true>, dim3(16384), dim3(64), 0, 0, buf, C, T, R); })) return 1;
  }
  CK(hipFree(buf));
  return 0;
}
