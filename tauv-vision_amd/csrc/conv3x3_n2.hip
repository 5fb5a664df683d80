// conv3x3 instances for 64-channel inputs (NCB = 2): DLA-34 level 2, its up-path and the stacked heads
#include "conv3x3_kernel.h"

namespace tv {
namespace c3 {

int launch_ncb2(const ConvParams& p, const ConvParams* dp, void* out, int dtype, int tw, int grid, hipStream_t s, int epi,
                int res, int ni, int nw) {
  if (res) return launch_res<2>(p, dp, out, dtype, tw, grid, s, epi, ni);  // DLA-34 BasicBlock identity residual
  // 64-channel inputs (DLA-34 level 2 and its up-path, the stacked DLA-34 heads)
    if (epi == 1) {
      if (p.act < 1 || p.ntiles > 16) {
        set_error("conv3x3: fused 1x1 needs ReLU / LeakyReLU and <= 16 channel tiles");
        return 1;
      }
      static const Launch e2[2][2][2] = {
          {{launch_t<_Float16, 16, 1, 1, 0, 4, 2>, launch_t<_Float16, 16, 2, 1, 0, 4, 2>},
           {launch_t<_Float16, 32, 1, 1, 0, 4, 2>, launch_t<_Float16, 32, 2, 1, 0, 4, 2>}},
          {{launch_t<__bf16, 16, 1, 1, 0, 4, 2>, launch_t<__bf16, 16, 2, 1, 0, 4, 2>},
           {launch_t<__bf16, 32, 1, 1, 0, 4, 2>, launch_t<__bf16, 32, 2, 1, 0, 4, 2>}}};
      if (dtype != F16 && dtype != BF16) { set_error("conv3x3: fp16/bf16 only"); return 1; }
      return e2[dtype == BF16][tw == 32][p.act - 1](p, dp, out, grid, s);
    }
    if (nw != 8) {
    set_error("conv3x3: 4-wave workgroups for 128-channel inputs only");
    return 1;
  }
  return launch_plain<2, 8>(p, dp, out, dtype, tw, grid, s, ni);
  
}

}  // namespace c3
}  // namespace tv
