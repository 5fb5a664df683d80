// Planner: the reference module tree, walked twice —
//  (1) parameter registration order, which is the reference state_dict layout
//      (dla.py:8-416, centernet.py:32-61), so reference checkpoints load by key;
//  (2) the forward pass (dla.py:39-52,71-76,123-135,182-192,265-284,340-357,377-390,409-416;
//      centernet.py:65-92) lowered to fused GEMMs over NHWC tensors:
//        * conv + BatchNorm(eval) + ReLU           -> one GEMM, BN folded, ReLU epilogue
//        * ResidualBlock conv2 + 1x1 residual + add -> one GEMM with two K-segments
//        * Root 1x1 over torch.cat(children)       -> one GEMM, one K-segment per child
//        * ConvTranspose2d(k=s) + pad_to_match + add -> one phase-scatter GEMM (+ margin copy)
//        * all heads' 3x3 convs                    -> one GEMM (N = heads * 2C), LeakyReLU
//        * all heads' 1x1 convs                    -> one block-diagonal GEMM, fp32 output
#include "planner.h"

#include <algorithm>
#include <functional>

#include "common.h"

namespace tv {
namespace {


struct Walker {
  const tv_model_desc& d;
  Plan& P;
  explicit Walker(const tv_model_desc& desc, Plan& plan) : d(desc), P(plan) {}
  bool backbone_only() const { return d.arch == TV_ARCH_CENTERNET_BACKBONE; }

  // ---------------- (1) parameters ----------------
  void add(const std::string& n, std::vector<int64_t> s) { P.params.push_back({n, std::move(s)}); }
  void conv_p(const std::string& p, int cout, int cin, int k) {
    add(p + ".weight", {cout, cin, k, k});
    add(p + ".bias", {cout});
  }
  void bn_p(const std::string& p, int c) {
    add(p + ".weight", {c});
    add(p + ".bias", {c});
    add(p + ".running_mean", {c});
    add(p + ".running_var", {c});
    add(p + ".num_batches_tracked", {});
  }
  void block_p(const std::string& p, int cin, int cout) {
    conv_p(p + ".conv1", cout, cin, 3);
    bn_p(p + ".bn1", cout);
    conv_p(p + ".conv2", cout, cout, 3);
    bn_p(p + ".bn2", cout);
    conv_p(p + ".conv_residual", cout, cin, 1);
    bn_p(p + ".bn_residual", cout);
  }
  void tree_p(const std::string& p, int cin, int cout, int h, int root_ch) {
    if (root_ch < 0) root_ch = 2 * cout;
    if (h == 1) {
      block_p(p + ".tree_l", cin, cout);
      block_p(p + ".tree_r", cout, cout);
      conv_p(p + ".root.conv", cout, root_ch, 1);
      bn_p(p + ".root.bn", cout);
    } else {
      tree_p(p + ".tree_l", cin, cout, h - 1, -1);
      tree_p(p + ".tree_r", cout, cout, h - 1, root_ch + cout);
    }
  }
  void ida_p(const std::string& p, const std::vector<int>& fc, const std::vector<int>& scales, bool reverse) {
    const int n = (int)fc.size() - 1;
    for (int j = 0; j < n; ++j) {
      int c = reverse ? fc[0] : fc[j];
      conv_p(p + ".projection_layers." + std::to_string(j) + ".0", c, fc[j + 1], 3);
      bn_p(p + ".projection_layers." + std::to_string(j) + ".1", c);
    }
    for (int j = 0; j < n; ++j) {
      int c = reverse ? fc[0] : fc[j];
      conv_p(p + ".output_layers." + std::to_string(j) + ".0", c, c, 3);
      bn_p(p + ".output_layers." + std::to_string(j) + ".1", c);
    }
    for (int j = 0; j < n; ++j) {
      int c = reverse ? fc[0] : fc[j];
      std::string u = p + ".upsample_layers." + std::to_string(j);
      add(u + ".weight", {c, c, scales[j], scales[j]});
      add(u + ".bias", {c});
    }
  }
  void params() {
    const int L = d.n_levels;
    std::vector<int> ch(d.channels, d.channels + L + 1);
    const std::string dd = "backbone.dla_down";
    conv_p(dd + ".projection_layer.0", ch[0], 3, 7);
    bn_p(dd + ".projection_layer.1", ch[0]);
    for (int i = 0; i < d.downsamples; ++i) block_p(dd + ".block_layers." + std::to_string(i), ch[0], ch[0]);
    for (int i = 0; i < L; ++i)
      tree_p(dd + ".tree_layers." + std::to_string(i), ch[i], ch[i + 1], d.heights[i], -1);
    for (int i = 0; i < L; ++i) {
      std::vector<int> fc(ch.begin(), ch.begin() + (L + 1 - i));
      ida_p("backbone.multi_ida_up.ida_up_layers." + std::to_string(i), fc, std::vector<int>(fc.size() - 1, 2),
            false);
    }
    std::vector<int> fc(ch.begin(), ch.begin() + L);
    std::vector<int> sc;
    for (int i = 1; i < L; ++i) sc.push_back(1 << i);
    ida_p("backbone.ida_up_reverse", fc, sc, true);
    for (int h = 0; h < (backbone_only() ? 0 : d.n_heads); ++h) {
      conv_p("heads." + std::to_string(h) + ".0", 2 * ch[0], ch[0], 3);
      conv_p("heads." + std::to_string(h) + ".2", d.head_channels[h], 2 * ch[0], 1);
    }
  }

  // ---------------- (2) forward lowering ----------------
  int tensor(int H, int W, int C) {
    P.tensors.push_back({H, W, C});
    return (int)P.tensors.size() - 1;
  }
  static int out_dim(int x, int k, int s, int pad) { return (x + 2 * pad - k) / s + 1; }

  int conv(const std::string& label, std::vector<SegSpec> segs, int N, int act) {
    const TensorSpec& s0 = P.tensors[segs[0].src];
    int Ho = out_dim(s0.H, segs[0].kh, segs[0].stride, segs[0].pad);
    int Wo = out_dim(s0.W, segs[0].kw, segs[0].stride, segs[0].pad_w >= 0 ? segs[0].pad_w : segs[0].pad);
    OpSpec op;
    op.kind = OP_CONV;
    op.label = label;
    op.N = N;
    op.act = act;
    for (auto& sg : segs) {
      const TensorSpec& t = P.tensors[sg.src];
      op.flops += 2.0 * Ho * Wo * N * (double)(sg.kh * (sg.row_expand ? sg.row_expand : sg.kw) * sg.cin);
      (void)t;
    }
    op.segs = std::move(segs);
    op.out = tensor(Ho, Wo, N);
    P.ops.push_back(op);
    return op.out;
  }
  SegSpec seg(int src, const std::string& conv_prefix, const std::string& bn, int ci0, int cin, int k, int stride,
              int pad) {
    return SegSpec{src, conv_prefix, bn, ci0, cin, k, k, stride, pad};
  }
  int conv_bn_relu(const std::string& conv_p, const std::string& bn, int x, int cin, int cout, int k, int stride,
                   int pad) {
    return conv(conv_p, {seg(x, conv_p, bn, 0, cin, k, stride, pad)}, cout, 1);
  }
  int block(const std::string& p, int x, int cin, int cout, int stride) {
    int t = conv_bn_relu(p + ".conv1", p + ".bn1", x, cin, cout, 3, stride, 1);
    return conv(p + ".conv2+conv_residual",
                {seg(t, p + ".conv2", p + ".bn2", 0, cout, 3, 1, 1),
                 seg(x, p + ".conv_residual", p + ".bn_residual", 0, cin, 1, stride, 0)},
                cout, 1);
  }
  int root(const std::string& p, const std::vector<int>& kids, int cout) {
    std::vector<SegSpec> segs;
    int off = 0;
    for (int k : kids) {
      int c = P.tensors[k].C;
      segs.push_back(seg(k, p + ".conv", p + ".bn", off, c, 1, 1, 0));
      off += c;
    }
    return conv(p + ".conv", segs, cout, 1);
  }
  int tree(const std::string& p, int x, int cin, int cout, int h, int stride, std::vector<int> kids) {
    if (h == 1) {
      int l = block(p + ".tree_l", x, cin, cout, stride);
      int r = block(p + ".tree_r", l, cout, cout, 1);
      kids.push_back(l);
      kids.push_back(r);
      return root(p + ".root", kids, cout);
    }
    int left = tree(p + ".tree_l", x, cin, cout, h - 1, stride, {});
    kids.push_back(left);
    return tree(p + ".tree_r", left, cout, cout, h - 1, 1, kids);
  }
  // up(project(x)) added to feature f with pad_to_match (dla.py:195-209)
  int up_add(const std::string& p, int j, int x, int f, int s) {
    const std::string js = std::to_string(j);
    const int c = P.tensors[f].C;
    int pr = conv_bn_relu(p + ".projection_layers." + js + ".0", p + ".projection_layers." + js + ".1", x,
                          P.tensors[x].C, c, 3, 1, 1);
    const TensorSpec src = P.tensors[pr];
    const TensorSpec tgt = P.tensors[f];
    const int hu = src.H * s, wu = src.W * s;
    OpSpec op;
    op.kind = OP_CONVT_ADD;
    op.label = p + ".upsample_layers." + js + "+pad_to_match+add";
    op.src = pr;
    op.add = f;
    op.up_s = s;
    op.up_w = p + ".upsample_layers." + js;
    op.N = c;
    if (hu != tgt.H || wu != tgt.W) {
      // F.pad(t, (above, below, left, right)) pads W by (above, below) and H by (left, right)
      int above = std::max(0, (hu - tgt.H) / 2), below = std::max(0, tgt.H - hu - above);
      int left = std::max(0, (wu - tgt.W) / 2), right = std::max(0, tgt.W - wu - left);
      if (hu + left + right < tgt.H || wu + above + below < tgt.W) {
        set_error("pad_to_match would yield a smaller tensor than its target; the reference fails here too");
        return -1;
      }
      op.sy = left;
      op.sx = above;
    }
    op.cov_y0 = op.sy;
    op.cov_y1 = std::min(tgt.H, op.sy + hu);
    op.cov_x0 = op.sx;
    op.cov_x1 = std::min(tgt.W, op.sx + wu);
    op.flops = 2.0 * src.H * src.W * (double)(s * s * c) * c;
    op.out = tensor(tgt.H, tgt.W, c);
    P.ops.push_back(op);
    const int u = op.out;
    return conv_bn_relu(p + ".output_layers." + js + ".0", p + ".output_layers." + js + ".1", u, c, c, 3, 1, 1);
  }
  std::vector<int> ida_up(const std::string& p, const std::vector<int>& feats) {
    const int n = (int)feats.size() - 1;
    std::vector<int> outs(n);
    int cur = feats.back();
    for (int i = n - 1; i >= 0; --i) {
      cur = up_add(p, i, cur, feats[i], 2);
      if (cur < 0) return {};
      outs[i] = cur;
    }
    return outs;
  }
  int forward() {
    const int L = d.n_levels;
    std::vector<int> ch(d.channels, d.channels + L + 1);
    // input staged row-expanded for the 7x7 stem: pixel (y, x) holds the 7 horizontal taps
    // x-3..x+3 of its 3 channels (21 values, zero-padded to a whole 16-byte chunk), so the
    // stem is a 7x1 conv with K = 7 * 24 instead of 49 taps of a padded pixel
    const int vec = 16 / dtype_size(d.compute_dtype);
    const int cpad = (7 * 3 + vec - 1) / vec * vec;
    P.in_cpad = cpad;
    int img = tensor(d.in_h, d.in_w, cpad);
    {
      OpSpec op;
      op.kind = OP_PREP;
      op.label = "input staging (NCHW fp32 / u8 frames -> NHWC)";
      op.out = img;
      op.N = cpad;
      P.ops.push_back(op);
    }
    const std::string dd = "backbone.dla_down";
    SegSpec stem = seg(img, dd + ".projection_layer.0", dd + ".projection_layer.1", 0, 3, 7, 1, 3);
    stem.kw = 1;
    stem.pad_w = 0;
    stem.row_expand = 7;
    int x = conv(dd + ".projection_layer.0", {stem}, ch[0], 1);
    for (int i = 0; i < d.downsamples; ++i) x = block(dd + ".block_layers." + std::to_string(i), x, ch[0], ch[0], 2);
    std::vector<int> feats{x};
    for (int i = 0; i < L; ++i) {
      x = tree(dd + ".tree_layers." + std::to_string(i), x, ch[i], ch[i + 1], d.heights[i], 2, {});
      feats.push_back(x);
    }
    std::vector<int> collected;
    for (int i = 0; i < L; ++i) {
      feats = ida_up("backbone.multi_ida_up.ida_up_layers." + std::to_string(i), feats);
      if (feats.empty()) return 2;
      collected.push_back(feats.back());
    }
    std::reverse(collected.begin(), collected.end());
    int cur = collected[0];
    for (int i = 0; i + 1 < (int)collected.size(); ++i) {
      cur = up_add("backbone.ida_up_reverse", i, collected[i + 1], cur, 1 << (i + 1));
      if (cur < 0) return 2;
    }
    const int C = ch[0];
    if (backbone_only()) {
      // DLABackbone.forward's result (dla.py:409-416) into the caller's fp32 NHWC buffer: an
      // identity 1x1 GEMM (exact: one product per output, fp32 accumulation)
      const TensorSpec ft = P.tensors[cur];
      OpSpec o;
      o.kind = OP_CONV;
      o.label = "backbone output -> fp32 NHWC";
      SegSpec sg{cur, "", "", 0, C, 1, 1, 1, 0};
      sg.identity = true;
      o.segs = {sg};
      o.N = C;
      o.act = 0;
      o.out = -1;
      P.out_c = C;
      P.out_cpad = C;
      P.out_h = ft.H;
      P.out_w = ft.W;
      P.ops.push_back(o);
      for (auto& op : P.ops) P.flops_per_frame += op.flops;
      return 0;
    }
    // heads: stacked 3x3 (C -> 2C each) + LeakyReLU, then block-diagonal 1x1 to fp32 output
    OpSpec h1;
    h1.kind = OP_CONV;
    h1.label = "heads.*.0 (stacked) + LeakyReLU";
    h1.segs = {SegSpec{cur, "", "", 0, C, 3, 3, 1, 1}};
    h1.N = 2 * C * d.n_heads;
    h1.act = 2;
    for (int h = 0; h < d.n_heads; ++h) {
      h1.stack_w.push_back("heads." + std::to_string(h) + ".0");
      h1.stack_n.push_back(2 * C);
    }
    const TensorSpec ft = P.tensors[cur];
    h1.flops = 2.0 * ft.H * ft.W * h1.N * 9.0 * C;
    h1.out = tensor(ft.H, ft.W, h1.N);
    P.ops.push_back(h1);
    OpSpec h2;
    h2.kind = OP_CONV;
    h2.label = "heads.*.2 (block-diagonal) -> fp32 NHWC";
    h2.segs = {SegSpec{h1.out, "", "", 0, h1.N, 1, 1, 1, 0}};
    int ctot = 0;
    for (int h = 0; h < d.n_heads; ++h) {
      h2.stack_w.push_back("heads." + std::to_string(h) + ".2");
      h2.stack_n.push_back(d.head_channels[h]);
      h2.diag_in_off.push_back(2 * C * h);
      h2.diag_out_off.push_back(ctot);
      h2.flops += 2.0 * ft.H * ft.W * d.head_channels[h] * 2.0 * C;
      ctot += d.head_channels[h];
    }
    P.out_c = ctot;
    P.out_cpad = (ctot + 3) / 4 * 4;
    P.out_h = ft.H;
    P.out_w = ft.W;
    h2.N = P.out_cpad;
    h2.act = 0;
    h2.out = -1;
    P.ops.push_back(h2);
    for (auto& op : P.ops) P.flops_per_frame += op.flops;
    return 0;
  }
};

}  // namespace

int build_plan(const tv_model_desc& d0, Plan* plan) {
  // TV_F32X3 plans as TV_F32 (fp32 storage; only the engine's GEMM kernel choice differs)
  tv_model_desc d = d0;
  if (d.compute_dtype == TV_F32X3) d.compute_dtype = TV_F32;
  if (d.arch == TV_ARCH_DLA34) return build_plan_dla34(d, plan);
  if (d.arch == TV_ARCH_PROTONET) return build_plan_protonet(d, plan);
  if (d.arch != TV_ARCH_CENTERNET && d.arch != TV_ARCH_CENTERNET_BACKBONE) {
    set_error("unknown model arch");
    return TV_EINVAL;
  }
  const bool heads = d.arch == TV_ARCH_CENTERNET;
  if (d.n_levels < 1 || d.n_levels > 8 || d.downsamples < 0 || d.downsamples > 6 || (heads && d.n_heads < 1) ||
      d.n_heads > 16 || d.in_h < 1 || d.in_w < 1 || d.compute_dtype < 0 || d.compute_dtype > 2) {
    set_error("model desc out of range");
    return TV_EINVAL;
  }
  const int vec = 16 / dtype_size(d.compute_dtype);
  for (int i = 0; i <= d.n_levels; ++i) {
    if (d.channels[i] < 1 || d.channels[i] % vec) {
      set_error("backbone_channels must be multiples of " + std::to_string(vec) + " for this dtype");
      return TV_ESHAPE;
    }
  }
  for (int i = 0; i < d.n_levels; ++i)
    if (d.heights[i] < 1 || d.heights[i] > 8) {
      set_error("backbone_heights out of range");
      return TV_EINVAL;
    }
  for (int h = 0; heads && h < d.n_heads; ++h)
    if (d.head_channels[h] < 1) {
      set_error("head channel counts must be positive");
      return TV_EINVAL;
    }
  *plan = Plan();
  Walker w(d, *plan);
  w.params();
  for (const ParamInfo& p : plan->params) plan->names.insert(p.name);
  int rc = w.forward();
  if (rc) return rc;
  for (auto& op : plan->ops)
    if (op.kind == OP_CONV && op.segs.size() > (size_t)kMaxSeg) {
      set_error("too many concatenated inputs for one Root (tree height too large)");
      return TV_ESHAPE;
    }
  return TV_OK;
}

}  // namespace tv
