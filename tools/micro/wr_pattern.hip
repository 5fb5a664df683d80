// Microbenchmark: write-only and read-only streams over [npix][256 B] rows (the stem's output
// shape: 32 frames x 480 x 640 pixels x 128 fp16 channels = 2.5 GB per slice), with the lane ->
// byte mappings of rw_pattern.hip:
//   P  (MFMA-epilogue pattern): lanes 0-31 = 32 pixels, lanes 32-63 the +16 B half; 8 instructions
//      complete the 32 rows
//   C  (coalesced): 16 lanes per 256 B row, 4 consecutive rows per instruction
// It bounds what the stem (HBM-write-bound) and the ConvT up-steps can reach.
// Build: hipcc -O3 --offload-arch=gfx950 wr_pattern.hip -o /tmp/wr_pattern
#include <hip/hip_runtime.h>
#include <cstdio>

// MODE 0: P writes, 1: C writes, 2: P reads, 3: C reads (summed into one store per lane)
template <int MODE>
__global__ __launch_bounds__(256) void wr(uint4* __restrict__ buf, long ntiles, uint4* __restrict__ sink) {
  const int lane = threadIdx.x & 63;
  const long wave = ((long)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const long nw = ((long)gridDim.x * blockDim.x) >> 6;
  uint4 acc = make_uint4(0, 0, 0, 0);
  for (long t = wave; t < ntiles; t += nw) {
    const long r0 = t * 32;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      long off;
      if (MODE == 0 || MODE == 2) off = (r0 + (lane & 31)) * 16 + 2 * q + (lane >> 5);
      else off = (r0 + 4 * q + (lane >> 4)) * 16 + (lane & 15);
      if (MODE < 2) {
        buf[off] = make_uint4((unsigned)t, (unsigned)q, (unsigned)lane, 0u);
      } else {
        const uint4 v = buf[off];
        acc.x ^= v.x;
        acc.y ^= v.y;
        acc.z ^= v.z;
        acc.w ^= v.w;
      }
    }
  }
  if (MODE >= 2 && acc.x == 0x12345678u) sink[threadIdx.x] = acc;  // keeps the loads
}

int main() {
  const long rows = 32L * 480 * 640;  // 2.5 GB
  const long ntiles = rows / 32;
  uint4 *buf, *sink;
  if (hipMalloc(&buf, rows * 256) != hipSuccess || hipMalloc(&sink, 4096) != hipSuccess) return 1;
  (void)hipMemset(buf, 1, rows * 256);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  const char* names[] = {"P write", "C write", "P read", "C read"};
  for (int grid : {1024, 2048, 4096, 8192}) {
    for (int v = 0; v < 4; ++v) {
      float best = 1e9;
      for (int r = 0; r < 5; ++r) {
        (void)hipEventRecord(e0);
        switch (v) {
          case 0: hipLaunchKernelGGL(wr<0>, dim3(grid), dim3(256), 0, 0, buf, ntiles, sink); break;
          case 1: hipLaunchKernelGGL(wr<1>, dim3(grid), dim3(256), 0, 0, buf, ntiles, sink); break;
          case 2: hipLaunchKernelGGL(wr<2>, dim3(grid), dim3(256), 0, 0, buf, ntiles, sink); break;
          case 3: hipLaunchKernelGGL(wr<3>, dim3(grid), dim3(256), 0, 0, buf, ntiles, sink); break;
        }
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        float ms;
        (void)hipEventElapsedTime(&ms, e0, e1);
        if (ms < best) best = ms;
      }
      printf("grid %5d %-8s: %.4f ms  %.2f TB/s\n", grid, names[v], best, (double)rows * 256 / best / 1e9);
    }
  }
  return 0;
}
