// Microbenchmark / FETCH_SIZE calibration for the halo kernels' read pattern: a [npix][256 B] tensor
// (128 fp16 channels NHWC, one 32-frame 240x320 level: 629 MB, past the 256 MB Infinity Cache)
// read three ways, each launch summing into one word per workgroup (no other traffic):
//   full  : every pixel's 256 B in one pass (16 lanes per pixel, coalesced 1 KiB per instruction)
//   block : four passes over the tensor, pass cb reading bytes [64 cb, 64 cb + 64) of every pixel
//           (what four 32-channel k-step blocks read when their halos are far apart in time)
//   tile  : per 512-pixel tile, the four 64-B block passes back to back (the conv3x3 order: the
//           next channel block's halo a few microseconds after the previous one)
// Run under rocprofv3 --pmc FETCH_SIZE (and --kernel-trace for the times): algorithmic bytes are
// the same 629 MB in every mode; FETCH_SIZE x 2 (the gfx950 correction for 16 B/lane streams)
// against it says whether reading half lines costs whole-line fetches.
// Build: hipcc -O3 --offload-arch=gfx950 halo_fetch.hip -o halo_fetch
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr long NPIX = 32L * 240 * 320;

__global__ __launch_bounds__(256) void rd_full(const uint4* __restrict__ in, unsigned* __restrict__ out) {
  unsigned acc = 0;
  const long n16 = NPIX * 16;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n16; i += (long)gridDim.x * 256) acc += in[i].x;
  if (acc == 0x12345678u) out[blockIdx.x] = acc;
}

// 4 lanes per pixel per pass (64 B), 16 pixels per wave instruction, pixels 256 B apart
__global__ __launch_bounds__(256) void rd_block(const uint4* __restrict__ in, unsigned* __restrict__ out) {
  unsigned acc = 0;
  for (int cb = 0; cb < 4; ++cb)
    for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < NPIX * 4; i += (long)gridDim.x * 256)
      acc += in[(i >> 2) * 16 + cb * 4 + (i & 3)].x;
  if (acc == 0x12345678u) out[blockIdx.x] = acc;
}

__global__ __launch_bounds__(256) void rd_tile(const uint4* __restrict__ in, unsigned* __restrict__ out) {
  unsigned acc = 0;
  const long ntiles = NPIX / 512;
  for (long t = blockIdx.x; t < ntiles; t += gridDim.x)
    for (int cb = 0; cb < 4; ++cb)
      for (int j = threadIdx.x; j < 512 * 4; j += 256) {
        const long px = t * 512 + (j >> 2);
        acc += in[px * 16 + cb * 4 + (j & 3)].x;
      }
  if (acc == 0x12345678u) out[blockIdx.x] = acc;
}

int main() {
  uint4* in;
  unsigned* out;
  hipMalloc(&in, NPIX * 256);
  hipMalloc(&out, 4096 * 4);
  hipMemset(in, 1, NPIX * 256);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int rep = 0; rep < 2; ++rep) {
    for (int mode = 0; mode < 3; ++mode) {
      hipEventRecord(e0);
      if (mode == 0) rd_full<<<2048, 256>>>(in, out);
      else if (mode == 1) rd_block<<<2048, 256>>>(in, out);
      else rd_tile<<<1024, 256>>>(in, out);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      printf("%s %.3f ms %.2f TB/s of algorithmic reads\n", mode == 0 ? "full " : mode == 1 ? "block" : "tile ", ms,
             NPIX * 256 / (ms * 1e-3) / 1e12);
    }
  }
  hipFree(in);
  hipFree(out);
  return 0;
}
