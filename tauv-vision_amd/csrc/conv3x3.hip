// conv3x3.hip — weight repack, tile geometry and the dispatch of the persistent halo-tile 3x3
// kernel (conv3x3_kernel.h; instances in conv3x3_n2/n4/n8.hip).
#include "conv3x3_kernel.h"

namespace tv {
namespace c3 {

// [Npad][Kpad] (K = tap * 128 + channel) -> [ntile][k-step q][bnk rows][4 x 16 B] (channel tiles
// of bnk = 128 or 64 rows), q = cb*9 + tap (res: q = cb*10 + j, j = 9 the residual segment's
// channel block cb at K offset 9*128), slot s of row r holding chunk s ^ wswz(r) of the k-step
__global__ void repack_weights(const uint4* __restrict__ w, int kpad16, int ntiles, int res, int bnk, int ncb, int k16,
                               uint4* __restrict__ out) {
  const int sp = (9 + res) * ncb;
  const int n = ntiles * sp * BN * 4;  // ntiles of 128 rows
  for (int o = blockIdx.x * blockDim.x + threadIdx.x; o < n; o += gridDim.x * blockDim.x) {
    const int slot = o & 3, row = (o >> 2) % bnk, q = (o / (4 * bnk)) % sp, nt = (o / (4 * bnk)) / sp;
    const int chunk = slot ^ wswz(row, k16 != 0);  // the body's weight-row swizzle
    const int cb = q / (9 + res), tap = q - cb * (9 + res);
    const int k16 = (tap * CBK * ncb + cb * CBK) / 8 + chunk;  // 16-byte column (8 elements); tap 9 = residual
    // (residual blocks past a narrower residual segment: zero weights, past Kpad included)
    out[o] = k16 < kpad16 ? w[(size_t)(nt * bnk + row) * kpad16 + k16] : make_uint4(0, 0, 0, 0);
  }
}

}  // namespace c3

int conv3x3_tiles(int B, int H, int W, int tw, int nw) {
  const int th = 64 * nw / tw;
  return B * ((H + th - 1) / th) * ((W + tw - 1) / tw);
}

size_t conv3x3_weight_bytes(int ntiles, int res, int ncb) {
  return (size_t)ntiles * (9 + res) * ncb * c3::WSLOT;
}

int conv3x3_k16(int epi, int res, int ni, int nw) { return c3::M16 && !res && epi == 0 && ni == 4 && nw == 8; }

int conv3x3_repack(const void* w, int Kpad, int esz, int ntiles, int res, int ni, int ncb, int k16, void* out, hipStream_t s) {
  if ((Kpad * esz) % 16 || Kpad < (9 * ncb + res) * 32 || (ni != 4 && ni != 2) || (ncb != 2 && ncb != 4 && ncb != 8)) {
    set_error("conv3x3_repack: bad Kpad / ni / channel blocks");
    return 1;
  }
  hipLaunchKernelGGL(c3::repack_weights, dim3(256), dim3(256), 0, s, (const uint4*)w, Kpad * esz / 16, ntiles, res,
                     32 * ni, ncb, k16, (uint4*)out);
  TV_HIP(hipGetLastError());
  return 0;
}

int launch_conv3x3(const ConvParams& p, const ConvParams* dp, void* out, int dtype, int tw, int grid,
                   hipStream_t s, int epi, int res, int ni, int nw) {
  using namespace c3;
  if (p.act < 0 || p.act > 2 || (ni != 4 && ni != 2) || (ni == 2 && epi != 0)) {
    set_error("conv3x3: bad activation / channel tile");
    return 1;
  }
  const int ncb = p.seg[0].C / CBK;
  if (ncb != 2 && ncb != 4 && ncb != 8) {
    set_error("conv3x3: inputs of 64, 128 or 256 channels");
    return 1;
  }
  if (nw != 8 && (nw != 4 || epi || res)) {
    set_error("conv3x3: 8-wave workgroups, or 4-wave ones with the plain epilogue");
    return 1;
  }
  if (ncb == 2) return launch_ncb2(p, dp, out, dtype, tw, grid, s, epi, res, ni, nw);
  if (ncb == 8) return launch_ncb8(p, dp, out, dtype, tw, grid, s, epi, res, ni, nw);
  return launch_ncb4(p, dp, out, dtype, tw, grid, s, epi, res, ni, nw);
}

}  // namespace tv
