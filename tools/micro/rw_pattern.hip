// Microbenchmark: read-modify-write streams over [npix][256 B] fp16 rows (the convt_add shape: read
// the skip row, write the output row), comparing lane -> byte mappings of each wave instruction:
//   P  (MFMA-epilogue pattern): lanes 0-31 = 32 pixels two rows apart, lanes 32-63 the +16 B half:
//      each instruction touches 32 pixels x 32 B; 8 instructions complete the 32 rows
//   C  (coalesced): 16 lanes per 256 B row, 4 consecutive rows per instruction
//   C2 (coalesced, rows two apart as the phase scatter writes them)
// Build: hipcc -O3 --offload-arch=gfx950 rw_pattern.hip -o /tmp/rw_pattern
#include <hip/hip_runtime.h>
#include <cstdio>

__device__ __forceinline__ uint4 ld(const uint4* p) { return *p; }
__device__ __forceinline__ void st(uint4* p, uint4 v) { *p = v; }

// rows of 16 uint4; a wave owns tiles of 32 rows; `stride2` = the tile's rows are 2 apart
template <int MODE, bool STRIDE2>
__global__ __launch_bounds__(256) void rw(const uint4* __restrict__ in, uint4* __restrict__ out, long ntiles) {
  const int lane = threadIdx.x & 63;
  const long wave = ((long)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const long nw = ((long)gridDim.x * blockDim.x) >> 6;
  for (long t = wave; t < ntiles; t += nw) {
    // tile t: 32 rows; STRIDE2: rows 2r + (t & 1) of a 64-row block t / 2
    auto row = [&](int r) -> long { return STRIDE2 ? (t >> 1) * 64 + 2 * r + (t & 1) : t * 32 + r; };
    uint4 v[8];
    if (MODE == 0) {  // P
      const int r = lane & 31, h = lane >> 5;
#pragma unroll
      for (int q = 0; q < 8; ++q) v[q] = ld(in + row(r) * 16 + 2 * q + h);
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        uint4 w = v[q];
        w.x += 1;
        st(out + row(r) * 16 + 2 * q + h, w);
      }
    } else {  // C
      const int c = lane & 15, r4 = lane >> 4;
#pragma unroll
      for (int q = 0; q < 8; ++q) v[q] = ld(in + row(4 * q + r4) * 16 + c);
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        uint4 w = v[q];
        w.x += 1;
        st(out + row(4 * q + r4) * 16 + c, w);
      }
    }
  }
}

int main() {
  const long rows = 32L * 120 * 160;  // one 32-frame 120x160 level (157 MB each way)
  const long ntiles = rows / 32;
  uint4 *in, *out;
  if (hipMalloc(&in, rows * 256) != hipSuccess || hipMalloc(&out, rows * 256) != hipSuccess) return 1;
  hipMemset(in, 1, rows * 256);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  const char* names[] = {"P", "C", "P stride2", "C stride2"};
  for (int grid : {1024, 2048, 4096}) {
    for (int v = 0; v < 4; ++v) {
      float best = 1e9;
      for (int r = 0; r < 5; ++r) {
        (void)hipEventRecord(e0);
        switch (v) {
          case 0: hipLaunchKernelGGL((rw<0, false>), dim3(grid), dim3(256), 0, 0, in, out, ntiles); break;
          case 1: hipLaunchKernelGGL((rw<1, false>), dim3(grid), dim3(256), 0, 0, in, out, ntiles); break;
          case 2: hipLaunchKernelGGL((rw<0, true>), dim3(grid), dim3(256), 0, 0, in, out, ntiles); break;
          case 3: hipLaunchKernelGGL((rw<1, true>), dim3(grid), dim3(256), 0, 0, in, out, ntiles); break;
        }
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        float ms;
        (void)hipEventElapsedTime(&ms, e0, e1);
        if (ms < best) best = ms;
      }
      printf("grid %5d %-10s: %.4f ms  %.2f TB/s (read + write)\n", grid, names[v], best, 2.0 * rows * 256 / best / 1e9);
    }
  }
  return 0;
}
