// conv3x3 instances for 256-channel inputs (NCB = 8): the YOLACT protonet, DLA-34 level 4
#include "conv3x3_kernel.h"

namespace tv {
namespace c3 {

int launch_ncb8(const ConvParams& p, const ConvParams* dp, void* out, int dtype, int tw, int grid, hipStream_t s, int epi,
                int res, int ni, int nw) {
  if (res) return launch_res<8>(p, dp, out, dtype, tw, grid, s, epi, ni);  // DLA-34 BasicBlock identity residual
  // 256-channel inputs (protonet, DLA-34 level 4)
    if (epi == 1) {
      if (p.act != 2 || p.ntiles > 16) {
        set_error("conv3x3: fused 1x1 needs LeakyReLU and <= 16 channel tiles");
        return 1;
      }
      if (dtype == F16) return tw == 32 ? launch_t<_Float16, 32, 2, 1, 0, 4, 8>(p, dp, out, grid, s) : launch_t<_Float16, 16, 2, 1, 0, 4, 8>(p, dp, out, grid, s);
      if (dtype == BF16) return tw == 32 ? launch_t<__bf16, 32, 2, 1, 0, 4, 8>(p, dp, out, grid, s) : launch_t<__bf16, 16, 2, 1, 0, 4, 8>(p, dp, out, grid, s);
      set_error("conv3x3: fp16/bf16 only");
      return 1;
    }
    if (nw != 8) {
    set_error("conv3x3: 4-wave workgroups for 128-channel inputs only");
    return 1;
  }
  return launch_plain<8, 8>(p, dp, out, dtype, tw, grid, s, ni);
  
}

}  // namespace c3
}  // namespace tv
