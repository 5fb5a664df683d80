// Microbenchmark: HBM write rate of store patterns (5 GiB buffer).
//  A<nt>: coalesced — each wave-instruction writes 1 KiB contiguous, 4 instructions in flight per lane
//  B<nt>: MFMA-epilogue pattern — each wave-instruction writes 32 pixels x 32 B (pixel stride 256 B);
//         8 consecutive instructions complete the 32 pixels' 256 B rows
//  copy : float4 copy of 2.5 GiB -> 2.5 GiB (reads + writes)
// Build: hipcc -O3 --offload-arch=gfx950 store_pattern.hip -o store_pattern
#include <hip/hip_runtime.h>
#include <cstdio>

template <bool NT>
__device__ __forceinline__ void st(uint4* p, uint4 v) {
  typedef unsigned u4 __attribute__((ext_vector_type(4)));
  u4 w = {v.x, v.y, v.z, v.w};
  if constexpr (NT) __builtin_nontemporal_store(w, (u4*)p);
  else *(u4*)p = w;
}

template <bool NT>
__global__ void pat_a(uint4* out, size_t n16) {
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += 4 * stride) {
#pragma unroll
    for (int u = 0; u < 4; ++u)
      if (i + u * stride < n16) st<NT>(out + i + u * stride, make_uint4(i, u, 2, 3));
  }
}
template <bool NT>
__global__ void pat_b(uint4* out, size_t npix) {
  const int lane = threadIdx.x & 63;
  const int l32 = lane & 31, lh = lane >> 5;
  const size_t wave = ((size_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const size_t nw = ((size_t)gridDim.x * blockDim.x) >> 6;
  for (size_t g = wave; g * 32 < npix; g += nw) {
    uint4* base = out + (g * 32 + l32) * 16;
#pragma unroll
    for (int q = 0; q < 8; ++q) st<NT>(base + 2 * q + lh, make_uint4(q, lane, 0, 1));
  }
}
__global__ void copy(const uint4* in, uint4* out, size_t n16) {
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += stride) out[i] = in[i];
}

int main() {
  const size_t bytes = 5ull << 30;
  uint4* buf;
  if (hipMalloc(&buf, bytes) != hipSuccess) return 1;
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  const char* names[] = {"A plain", "A nt", "B plain", "B nt", "copy"};
  for (int grid : {1024, 2048, 8192}) {
    for (int v = 0; v < 5; ++v) {
      float best = 1e9;
      for (int r = 0; r < 4; ++r) {
        (void)hipEventRecord(e0);
        switch (v) {
          case 0: hipLaunchKernelGGL(pat_a<false>, dim3(grid), dim3(256), 0, 0, buf, bytes / 16); break;
          case 1: hipLaunchKernelGGL(pat_a<true>, dim3(grid), dim3(256), 0, 0, buf, bytes / 16); break;
          case 2: hipLaunchKernelGGL(pat_b<false>, dim3(grid), dim3(256), 0, 0, buf, bytes / 256); break;
          case 3: hipLaunchKernelGGL(pat_b<true>, dim3(grid), dim3(256), 0, 0, buf, bytes / 256); break;
          case 4: hipLaunchKernelGGL(copy, dim3(grid), dim3(256), 0, 0, buf, buf + bytes / 32, bytes / 32); break;
        }
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        float ms;
        (void)hipEventElapsedTime(&ms, e0, e1);
        if (ms < best) best = ms;
      }
      printf("grid %5d %-8s: %.3f ms  %.2f TB/s (bytes moved)\n", grid, names[v], best, bytes / best / 1e9);
    }
  }
  return 0;
}
