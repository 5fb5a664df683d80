// conv3x3 instances for 128-channel inputs (NCB = 4): the "R18" DLA levels, RES and fused-heads variants
#include "conv3x3_kernel.h"

namespace tv {
namespace c3 {

int launch_ncb4(const ConvParams& p, const ConvParams* dp, void* out, int dtype, int tw, int grid, hipStream_t s, int epi,
                int res, int ni, int nw) {
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
  if (nw == 4) return launch_plain<4, 4>(p, dp, out, dtype, tw, grid, s, ni);
  return launch_plain<4, 8>(p, dp, out, dtype, tw, grid, s, ni);

}

}  // namespace c3
}  // namespace tv
