// conv3x3 instances for 128-channel inputs (NCB = 4): the "R18" DLA levels, RES and fused-heads variants
#include "conv3x3_kernel.h"

namespace tv {
namespace c3 {

int launch_ncb4(const ConvParams& p, const ConvParams* dp, void* out, int dtype, int tw, int grid, hipStream_t s, int epi,
                int res, int ni) {
  if (res) return launch_res<4>(p, dp, out, dtype, tw, grid, s, epi, ni);  // ResidualBlock conv2 + conv_residual
  if (epi == 1) {  // fused 1x1 heads: the stacked heads' LeakyReLU only
    if (p.act != 2 || p.ntiles > 16) {
      set_error("conv3x3: fused heads need LeakyReLU and <= 16 channel tiles");
      return 1;
    }
    if (dtype == F16) return tw == 32 ? launch_t<_Float16, 32, 2, 1>(p, dp, out, grid, s) : launch_t<_Float16, 16, 2, 1>(p, dp, out, grid, s);
    if (dtype == BF16) return tw == 32 ? launch_t<__bf16, 32, 2, 1>(p, dp, out, grid, s) : launch_t<__bf16, 16, 2, 1>(p, dp, out, grid, s);
    set_error("conv3x3: fp16/bf16 only");
    return 1;
  }
  static const Launch f16[2][2][3] = {
      {{launch_t<_Float16, 16, 0, 0, 0, 2>, launch_t<_Float16, 16, 1, 0, 0, 2>, launch_t<_Float16, 16, 2, 0, 0, 2>},
       {launch_t<_Float16, 32, 0, 0, 0, 2>, launch_t<_Float16, 32, 1, 0, 0, 2>, launch_t<_Float16, 32, 2, 0, 0, 2>}},
      {{launch_t<_Float16, 16, 0>, launch_t<_Float16, 16, 1>, launch_t<_Float16, 16, 2>},
       {launch_t<_Float16, 32, 0>, launch_t<_Float16, 32, 1>, launch_t<_Float16, 32, 2>}}};
  static const Launch b16[2][2][3] = {
      {{launch_t<__bf16, 16, 0, 0, 0, 2>, launch_t<__bf16, 16, 1, 0, 0, 2>, launch_t<__bf16, 16, 2, 0, 0, 2>},
       {launch_t<__bf16, 32, 0, 0, 0, 2>, launch_t<__bf16, 32, 1, 0, 0, 2>, launch_t<__bf16, 32, 2, 0, 0, 2>}},
      {{launch_t<__bf16, 16, 0>, launch_t<__bf16, 16, 1>, launch_t<__bf16, 16, 2>},
       {launch_t<__bf16, 32, 0>, launch_t<__bf16, 32, 1>, launch_t<__bf16, 32, 2>}}};
  if (dtype == F16) return f16[ni == 4][tw == 32][p.act](p, dp, out, grid, s);
  if (dtype == BF16) return b16[ni == 4][tw == 32][p.act](p, dp, out, grid, s);
  set_error("conv3x3: fp16/bf16 only");
  return 1;

}

}  // namespace c3
}  // namespace tv
