// Network planner for the reference "R18" CenterNet (Centernet + DLABackbone):
// enumerates the reference state_dict layout and lowers the forward pass to a list of
// fused GEMM launches over NHWC tensors.
#pragma once
#include <cstdint>
#include <set>
#include <string>
#include <vector>

#include "../../include/tauv_vision_amd.h"

namespace tv {

struct ParamInfo {
  std::string name;
  std::vector<int64_t> shape;
};

// One K-segment of a fused conv: input channels [ci0, ci0 + cin) of a PyTorch conv weight,
// applied to tensor `src` (whose stored channel count may be padded beyond cin).
struct SegSpec {
  int src;               // tensor id
  std::string wname;     // "<prefix>.weight" of the Conv2d
  std::string bn;        // BatchNorm2d prefix folded into this conv ("" = none)
  int ci0, cin;          // slice of the weight's input channels
  int kh, kw, stride, pad;
  int pad_w = -1;        // width padding when it differs from `pad` (row-expanded stem input)
  int row_expand = 0;    // k > 0: `src` holds the k horizontal taps of a k x k conv per pixel
                         // (DCN columns: k = 9 taps of a 3x3 weight per pixel, kh = kw = 1)
  bool identity = false; // residual added as-is (BasicBlock residual = x): an identity 1x1 weight
  // >= 0: one output phase (pi * 2 + pj) of a ConvTranspose2d(3, stride 2, padding 1) weight
  // [cin][cout][3][3] (masknet.py:21,33): the phase's taps as a kh x kw (= 1 + pi, 1 + pj) conv
  // with no padding over the low-resolution input (tap dy reads row oy + dy: ky = 1 for pi = 0,
  // ky = 2 - 2 dy for pi = 1; the same along x)
  int convt_phase = -1;
};

enum OpKind {
  OP_PREP = 0,
  OP_CONV = 1,
  OP_CONVT_ADD = 2,
  // CenterpointDLA34 (centerpoint_dla.py): elementwise / gather ops on HBM bandwidth
  OP_MAXPOOL = 3,    // MaxPool2d(2, 2, ceil_mode=True) of `src` (Tree.downsample, :199-200)
  OP_DCN = 4,        // DCNv2 sampling: columns [9 taps][C] per pixel of `src` at the offsets /
                     // sigmoid(mask logits) in tensor `add` (18 offsets, 9 logits; :386-392)
  OP_DWCONVT_ADD = 5, // depthwise ConvTranspose2d(2f, f, f//2) of `src` + pad_to_match + `add`
                      // (IDAUp, :446-451); up_s = f, (sy, sx) = (pad_above, pad_left)
  OP_LAYOUT_IN = 6    // fp32 NCHW input with N channels -> NHWC compute dtype (protonet fpn[0] input)
};

struct OpSpec {
  int kind;
  std::string label;          // human-readable (reference module path)
  std::vector<SegSpec> segs;  // OP_CONV
  int out;                    // tensor id (-1 = the caller's fp32 output buffer)
  int N;                      // output channels (GEMM columns before phase expansion)
  int act;                    // 0 none, 1 relu, 2 leaky
  // head fusion: weights of several convs stacked along N (names in order, N each)
  std::vector<std::string> stack_w;
  std::vector<int> stack_n;
  // final block-diagonal 1x1 heads: weight j feeds output channels [out_off[j], +n) from
  // input channels [in_off[j], +cin)
  std::vector<int> diag_in_off, diag_out_off;
  // OP_CONVT_ADD (and OP_CONV: `add` >= 0 = tensor added before the activation)
  int src = -1, add = -1, up_s = 0, sy = 0, sx = 0;
  std::string up_w;           // ConvTranspose2d prefix
  int cov_y0 = 0, cov_y1 = 0, cov_x0 = 0, cov_x1 = 0;  // covered target rectangle
  double flops = 0;           // algorithmic FLOPs per frame (2*MAC)
  // OP_CONV with up_s > 0: a phase-scatter GEMM over the (gh, gw) grid of its input whose output
  // pixel (oy, ox) lands at (oy * up_s + sy, ox * up_s + sx) of `out` (no skip tensor when add < 0)
  int gh = 0, gw = 0;
  // a second output tensor (the fused stem + block0.conv1 launch also writes the stem at the even
  // pixels, the block's residual input): placed and kept live like `out`
  int out2 = -1;
};

struct TensorSpec {
  int H, W, C;  // per frame, stored channels (ldc == C)
};

struct Plan {
  std::vector<ParamInfo> params;     // reference state_dict order
  std::vector<TensorSpec> tensors;
  std::vector<OpSpec> ops;
  int out_h = 0, out_w = 0, out_c = 0, out_cpad = 0;
  int in_cpad = 0;
  int in_channels = 3;               // channels of one input frame (fp32 NCHW path)
  double flops_per_frame = 0;
  std::set<std::string> names;       // every key of `params`
};

// Returns 0 or a TV_E* code (with tv_last_error set).
int build_plan(const tv_model_desc& d, Plan* plan);
int build_plan_dla34(const tv_model_desc& d, Plan* plan);  // planner_dla34.cpp
int build_plan_protonet(const tv_model_desc& d, Plan* plan);  // planner_protonet.cpp

}  // namespace tv
