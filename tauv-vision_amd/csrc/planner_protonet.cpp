// Planner for the YOLACT protonet, reference Masknet (src/tauv_vision/yolact/model/masknet.py:8-55):
//  (1) parameter registration order = Masknet.state_dict() (:15-41): `_layers_1.0.0`,
//      `_upsample_layer_1`, `_layers_2.0.0`, `_upsample_layer_2`, `_layers_3.0.0`, `_output_layer`
//      (n_masknet_layers_pre/post_upsample are not read by the reference: one conv per stage);
//  (2) the forward pass (:44-55) lowered over NHWC tensors:
//        * fpn[0] fp32 NCHW -> NHWC compute dtype            -> OP_LAYOUT_IN
//        * Conv2d(F, F, 3, p=1) + LeakyReLU                   -> one GEMM (K = 9F)
//        * ConvTranspose2d(F, F, 3, s=2, p=1), output_size 2x (output_padding 1) + LeakyReLU
//          -> four phase GEMMs over the low-resolution grid, one per output parity (pi, pj):
//             out[2m + pi][2n + pj] = sum over the phase's (1 + pi) x (1 + pj) taps — exactly the
//             transposed conv's 9 taps per 2x2 output block (no zero-stuffing, no wasted MACs),
//             each written by the phase-scatter epilogue (up_s = 2, shift (pi, pj), no skip add)
//        * Conv2d(F, k, 1) + LeakyReLU                        -> one GEMM into the fp32 output, or
//          (fp16 / bf16) fused into the preceding 3x3 conv's epilogue: the F-channel activation
//          at 4x resolution never reaches HBM
#include "common.h"
#include "planner.h"

namespace tv {

int build_plan_protonet(const tv_model_desc& d, Plan* plan) {
  const int F = d.channels[0], k = d.head_channels[0];
  const int vec = 16 / dtype_size(d.compute_dtype);
  if (d.n_heads != 1 || F < 1 || F % vec || k < 1 || d.in_h < 1 || d.in_w < 1 || d.compute_dtype < 0 ||
      d.compute_dtype > 2) {
    set_error("protonet desc: need channels[0] = feature_depth (multiple of " + std::to_string(vec) +
              "), one head of n_prototype_masks channels, in_h/in_w = fpn[0] size");
    return TV_EINVAL;
  }
  *plan = Plan();
  Plan& P = *plan;
  auto add = [&](const std::string& n, std::vector<int64_t> s) { P.params.push_back({n, std::move(s)}); };
  for (int i = 1; i <= 3; ++i) {
    add("_layers_" + std::to_string(i) + ".0.0.weight", {F, F, 3, 3});
    add("_layers_" + std::to_string(i) + ".0.0.bias", {F});
    if (i < 3) {
      add("_upsample_layer_" + std::to_string(i) + ".weight", {F, F, 3, 3});
      add("_upsample_layer_" + std::to_string(i) + ".bias", {F});
    }
  }
  add("_output_layer.weight", {k, F, 1, 1});
  add("_output_layer.bias", {k});
  for (const ParamInfo& p : P.params) P.names.insert(p.name);

  auto tensor = [&](int H, int W, int C) {
    P.tensors.push_back({H, W, C});
    return (int)P.tensors.size() - 1;
  };
  P.in_channels = F;
  int x = tensor(d.in_h, d.in_w, F);
  {
    OpSpec op;
    op.kind = OP_LAYOUT_IN;
    op.label = "fpn[0] NCHW fp32 -> NHWC";
    op.out = x;
    op.N = F;
    P.ops.push_back(op);
  }
  auto conv3 = [&](const std::string& name, int src) {
    const TensorSpec t = P.tensors[src];
    OpSpec op;
    op.kind = OP_CONV;
    op.label = name + " + LeakyReLU";
    op.segs = {SegSpec{src, name, "", 0, F, 3, 3, 1, 1}};
    op.N = F;
    op.act = 2;
    op.flops = 2.0 * t.H * t.W * F * 9.0 * F;
    op.out = tensor(t.H, t.W, F);
    P.ops.push_back(op);
    return op.out;
  };
  auto up = [&](const std::string& name, int src) {
    const TensorSpec t = P.tensors[src];
    const int out = tensor(2 * t.H, 2 * t.W, F);
    for (int ph = 0; ph < 4; ++ph) {
      const int pi = ph >> 1, pj = ph & 1;
      OpSpec op;
      op.kind = OP_CONV;
      op.label = name + " phase (" + std::to_string(pi) + "," + std::to_string(pj) + ") + LeakyReLU";
      SegSpec sg{src, name, "", 0, F, 1 + pi, 1 + pj, 1, 0};
      sg.convt_phase = ph;
      op.segs = {sg};
      op.N = F;
      op.act = 2;
      op.up_s = 2;
      op.sy = pi;
      op.sx = pj;
      op.gh = t.H;
      op.gw = t.W;
      op.cov_y1 = 2 * t.H;
      op.cov_x1 = 2 * t.W;
      op.flops = 2.0 * t.H * t.W * F * (double)((1 + pi) * (1 + pj)) * F;
      op.out = out;
      P.ops.push_back(op);
    }
    return out;
  };
  x = conv3("_layers_1.0.0", x);
  x = up("_upsample_layer_1", x);
  x = conv3("_layers_2.0.0", x);
  x = up("_upsample_layer_2", x);
  x = conv3("_layers_3.0.0", x);
  const TensorSpec t = P.tensors[x];
  OpSpec o;
  o.kind = OP_CONV;
  o.label = "_output_layer + LeakyReLU -> fp32 NHWC";
  o.segs = {SegSpec{x, "", "", 0, F, 1, 1, 1, 0}};
  // as a one-head "block-diagonal" 1x1 so the engine can fuse it into the 3x3 conv's epilogue
  // (conv3x3 EPI 1: MFMA on the rounded 3x3 output, fp32 partial sums of the 128-channel tiles
  // added into the output, LeakyReLU applied by a pass over the k output channels afterwards)
  o.stack_w = {"_output_layer"};
  o.stack_n = {k};
  o.diag_in_off = {0};
  o.diag_out_off = {0};
  P.out_c = k;
  P.out_cpad = (k + 3) / 4 * 4;
  P.out_h = t.H;
  P.out_w = t.W;
  o.N = P.out_cpad;
  o.act = 2;
  o.flops = 2.0 * t.H * t.W * k * (double)F;
  o.out = -1;
  P.ops.push_back(o);
  for (auto& op : P.ops) P.flops_per_frame += op.flops;
  return TV_OK;
}

}  // namespace tv
