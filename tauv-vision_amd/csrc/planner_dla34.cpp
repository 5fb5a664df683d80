// Planner for the reference's CenterpointDLA34 (src/tauv_vision/centernet/model/backbones/
// centerpoint_dla.py): the module tree walked twice, like planner.cpp does for Centernet —
//  (1) parameter registration order = the reference state_dict layout (keys `model.*`,
//      CenterpointDLA34 wraps DLASeg as `self.model`, :549-556), so checkpoints load by key;
//  (2) the forward pass (:30-59, 147-221, 224-306, 360-462, 476-525) lowered to fused GEMMs and
//      bandwidth kernels over NHWC tensors:
//        * conv(bias=False) + BN + ReLU                 -> one GEMM, BN folded
//        * BasicBlock conv2 + residual (+= , ReLU)      -> one GEMM; the residual is a second
//          K-segment: Tree.project's 1x1 + BN over the max-pooled bottom, or an identity 1x1
//        * Root 1x1 over torch.cat(children)            -> one GEMM, one K-segment per child
//        * Tree.downsample MaxPool2d(2, 2, ceil_mode)   -> OP_MAXPOOL
//        * DeformConv: offset + mask 3x3 convs          -> one GEMM (N = 18 + 9, padded to 32)
//                      DCNv2 bilinear sampling x mask   -> OP_DCN (9-tap column tensor)
//                      DeformConv2d + bias + BN + ReLU  -> one GEMM over the columns (K = 9 * C)
//        * IDAUp depthwise ConvTranspose2d + pad_to_match + add -> OP_DWCONVT_ADD
//        * heads: 3x3 (64 -> 256) + bias + ReLU, stacked -> one GEMM (N = 256 * heads);
//                 1x1 (256 -> n) + bias -> one block-diagonal GEMM into the fp32 output
// The outer Tree's `project` of a height-2 tree is computed by the reference but never read
// (its tree1 recomputes its own residual, :209-216): it is not lowered.
#include <algorithm>
#include <map>

#include "common.h"
#include "planner.h"

namespace tv {
namespace {

constexpr int kLevels[6] = {1, 1, 1, 2, 2, 1};       // dla34(), :309-315
constexpr int kChannels[6] = {16, 32, 64, 128, 256, 512};
constexpr int kHeadConv = 256;                       // get_pose_net head_conv, :534-541
constexpr int kFirstLevel = 2, kLastLevel = 5;       // down_ratio 4, last_level 5

struct DlaWalker {
  const tv_model_desc& d;
  Plan& P;
  std::map<int, int> pooled;  // tensor -> its max-pooled tensor (shared by tree1 and the Root)
  DlaWalker(const tv_model_desc& desc, Plan& plan) : d(desc), P(plan) {}

  // ---------------- (1) parameters ----------------
  void add(const std::string& n, std::vector<int64_t> s) { P.params.push_back({n, std::move(s)}); }
  void conv_w(const std::string& p, int cout, int cin, int k) { add(p + ".weight", {cout, cin, k, k}); }
  void conv_wb(const std::string& p, int cout, int cin, int k) {
    conv_w(p, cout, cin, k);
    add(p + ".bias", {cout});
  }
  void bn_p(const std::string& p, int c) {
    add(p + ".weight", {c});
    add(p + ".bias", {c});
    add(p + ".running_mean", {c});
    add(p + ".running_var", {c});
    add(p + ".num_batches_tracked", {});
  }
  void basic_p(const std::string& p, int cin, int cout) {
    conv_w(p + ".conv1", cout, cin, 3);
    bn_p(p + ".bn1", cout);
    conv_w(p + ".conv2", cout, cout, 3);
    bn_p(p + ".bn2", cout);
  }
  // Tree.__init__ (:168-200): tree1, tree2, [root], [project]
  void tree_p(const std::string& p, int levels, int cin, int cout, bool level_root, int root_dim) {
    if (root_dim == 0) root_dim = 2 * cout;
    if (level_root) root_dim += cin;
    if (levels == 1) {
      basic_p(p + ".tree1", cin, cout);
      basic_p(p + ".tree2", cout, cout);
    } else {
      tree_p(p + ".tree1", levels - 1, cin, cout, false, 0);
      tree_p(p + ".tree2", levels - 1, cout, cout, false, root_dim + cout);
    }
    if (levels == 1) {
      conv_w(p + ".root.conv", cout, root_dim, 1);
      bn_p(p + ".root.bn", cout);
    }
    if (cin != cout) {
      conv_w(p + ".project.0", cout, cin, 1);
      bn_p(p + ".project.1", cout);
    }
  }
  void deform_p(const std::string& p, int chi, int cho) {  // DeformConv (:360-384)
    bn_p(p + ".actf.0", cho);
    conv_wb(p + ".offset", 18, chi, 3);
    conv_wb(p + ".mask", 9, chi, 3);
    conv_wb(p + ".conv", cho, chi, 3);
  }
  // IDAUp.__init__ (:411-428): per i: proj_i, up_i, node_i
  void ida_p(const std::string& p, int o, const std::vector<int>& ch, const std::vector<int>& up_f) {
    for (size_t i = 1; i < ch.size(); ++i) {
      const int f = up_f[i];
      deform_p(p + ".proj_" + std::to_string(i), ch[i], o);
      add(p + ".up_" + std::to_string(i) + ".weight", {o, 1, 2 * f, 2 * f});
      deform_p(p + ".node_" + std::to_string(i), o, o);
    }
  }
  // DLAUp.__init__ (:435-449): the IDAUps and their channel / scale bookkeeping (in_channels
  // aliases `channels` and is rewritten as the loop goes)
  struct IdaDef { int o; std::vector<int> ch, up_f; };
  std::vector<IdaDef> dla_up_defs() const {
    std::vector<int> channels(kChannels + kFirstLevel, kChannels + 6), in_ch = channels;
    std::vector<int> scales;
    for (size_t i = 0; i < channels.size(); ++i) scales.push_back(1 << i);
    std::vector<IdaDef> defs;
    const int n = (int)channels.size();
    for (int i = 0; i < n - 1; ++i) {
      const int j = n - i - 2;
      IdaDef def{channels[j], std::vector<int>(in_ch.begin() + j, in_ch.end()), {}};
      for (int k = j; k < n; ++k) def.up_f.push_back(scales[k] / scales[j]);
      defs.push_back(def);
      for (int k = j + 1; k < n; ++k) {
        scales[k] = scales[j];
        in_ch[k] = channels[j];
      }
    }
    return defs;
  }
  IdaDef ida_up_def() const {  // DLASeg.ida_up (:491-492)
    IdaDef def{kChannels[kFirstLevel], {}, {}};
    for (int l = kFirstLevel; l < kLastLevel; ++l) {
      def.ch.push_back(kChannels[l]);
      def.up_f.push_back(1 << (l - kFirstLevel));
    }
    return def;
  }
  void params() {
    const std::string b = "model.base";
    conv_w(b + ".base_layer.0", kChannels[0], 3, 7);
    bn_p(b + ".base_layer.1", kChannels[0]);
    int cin = kChannels[0];
    for (int l = 0; l < 2; ++l)
      for (int c = 0; c < kLevels[l]; ++c) {
        conv_w(b + ".level" + std::to_string(l) + "." + std::to_string(3 * c), kChannels[l], cin, 3);
        bn_p(b + ".level" + std::to_string(l) + "." + std::to_string(3 * c + 1), kChannels[l]);
        cin = kChannels[l];
      }
    for (int l = 2; l < 6; ++l)
      tree_p(b + ".level" + std::to_string(l), kLevels[l], kChannels[l - 1], kChannels[l], l >= 3, 0);
    const auto defs = dla_up_defs();
    for (size_t i = 0; i < defs.size(); ++i) ida_p("model.dla_up.ida_" + std::to_string(i), defs[i].o, defs[i].ch, defs[i].up_f);
    const IdaDef iu = ida_up_def();
    ida_p("model.ida_up", iu.o, iu.ch, iu.up_f);
    for (int h = 0; h < d.n_heads; ++h) {
      conv_wb("model." + std::to_string(h) + ".0", kHeadConv, kChannels[kFirstLevel], 3);
      conv_wb("model." + std::to_string(h) + ".2", d.head_channels[h], kHeadConv, 1);
    }
  }

  // ---------------- (2) forward lowering ----------------
  int tensor(int H, int W, int C) {
    P.tensors.push_back({H, W, C});
    return (int)P.tensors.size() - 1;
  }
  static int out_dim(int x, int k, int s, int pad) { return (x + 2 * pad - k) / s + 1; }
  static SegSpec seg(int src, const std::string& w, const std::string& bn, int ci0, int cin, int k, int stride,
                     int pad) {
    return SegSpec{src, w, bn, ci0, cin, k, k, stride, pad};
  }
  int conv(const std::string& label, std::vector<SegSpec> segs, int N, int act) {
    const TensorSpec s0 = P.tensors[segs[0].src];
    const int Ho = out_dim(s0.H, segs[0].kh, segs[0].stride, segs[0].pad);
    const int Wo = out_dim(s0.W, segs[0].kw, segs[0].stride, segs[0].pad_w >= 0 ? segs[0].pad_w : segs[0].pad);
    OpSpec op;
    op.kind = OP_CONV;
    op.label = label;
    op.N = N;
    op.act = act;
    for (auto& sg : segs)
      if (!sg.identity) op.flops += 2.0 * Ho * Wo * N * (double)(sg.kh * (sg.row_expand ? sg.row_expand : sg.kw) * sg.cin);
    op.segs = std::move(segs);
    op.out = tensor(Ho, Wo, N);
    P.ops.push_back(op);
    return op.out;
  }
  int maxpool(int x) {
    auto it = pooled.find(x);
    if (it != pooled.end()) return it->second;
    const TensorSpec t = P.tensors[x];
    OpSpec op;
    op.kind = OP_MAXPOOL;
    op.label = "MaxPool2d(2, 2, ceil_mode=True)";
    op.src = x;
    op.N = t.C;
    op.out = tensor((t.H + 1) / 2, (t.W + 1) / 2, t.C);
    P.ops.push_back(op);
    pooled[x] = op.out;
    return op.out;
  }
  // BasicBlock (:30-59) with its residual as the second K-segment of conv2
  int basic(const std::string& p, int x, int cin, int cout, int stride, SegSpec res) {
    int t = conv(p + ".conv1", {seg(x, p + ".conv1", p + ".bn1", 0, cin, 3, stride, 1)}, cout, 1);
    const TensorSpec to = P.tensors[t], tr = P.tensors[res.src];
    if (tr.H != to.H || tr.W != to.W) {  // pad_to_match never fires for stride-2 ceil pooling
      set_error("DLA34 BasicBlock residual shape mismatch");
      return -1;
    }
    return conv(p + ".conv2+residual", {seg(t, p + ".conv2", p + ".bn2", 0, cout, 3, 1, 1), res}, cout, 1);
  }
  static SegSpec identity(int x, int c) {
    SegSpec s = seg(x, "", "", 0, c, 1, 1, 0);
    s.identity = true;
    return s;
  }
  int root(const std::string& p, const std::vector<int>& kids, int cout) {
    std::vector<SegSpec> segs;
    int off = 0;
    for (int k : kids) {
      const int c = P.tensors[k].C;
      segs.push_back(seg(k, p + ".conv", p + ".bn", off, c, 1, 1, 0));
      off += c;
    }
    return conv(p + ".conv", segs, cout, 1);
  }
  // Tree.forward (:202-221)
  int tree(const std::string& p, int x, int levels, int stride, int cin, int cout, bool level_root,
           std::vector<int> children) {
    const int bottom = stride > 1 ? maxpool(x) : x;
    if (level_root) children.push_back(bottom);
    if (levels == 1) {
      const SegSpec res = cin != cout ? seg(bottom, p + ".project.0", p + ".project.1", 0, cin, 1, 1, 0)
                                      : identity(bottom, cin);
      const int x1 = basic(p + ".tree1", x, cin, cout, stride, res);
      if (x1 < 0) return -1;
      const int x2 = basic(p + ".tree2", x1, cout, cout, 1, identity(x1, cout));
      if (x2 < 0) return -1;
      std::vector<int> kids{x2, x1};
      kids.insert(kids.end(), children.begin(), children.end());
      return root(p + ".root", kids, cout);
    }
    const int x1 = tree(p + ".tree1", x, levels - 1, stride, cin, cout, false, {});
    if (x1 < 0) return -1;
    children.push_back(x1);
    return tree(p + ".tree2", x1, levels - 1, 1, cout, cout, false, children);
  }
  // DeformConv.forward (:386-392)
  int deform(const std::string& p, int x, int cho) {
    const TensorSpec t = P.tensors[x];
    OpSpec om;
    om.kind = OP_CONV;
    om.label = p + ".offset+mask";
    om.segs = {seg(x, "", "", 0, t.C, 3, 1, 1)};
    om.N = 32;  // 18 offsets (dy, dx per tap) + 9 mask logits + 5 zero columns
    om.act = 0;
    om.stack_w = {p + ".offset", p + ".mask"};
    om.stack_n = {18, 9};
    om.flops = 2.0 * t.H * t.W * 27 * 9.0 * t.C;
    om.out = tensor(t.H, t.W, 32);
    P.ops.push_back(om);
    OpSpec dc;
    dc.kind = OP_DCN;
    dc.label = p + ".conv (DCNv2 sampling)";
    dc.src = x;
    dc.add = om.out;
    dc.N = 9 * t.C;
    dc.out = tensor(t.H, t.W, 9 * t.C);
    P.ops.push_back(dc);
    SegSpec cs = seg(dc.out, p + ".conv", p + ".actf.0", 0, t.C, 1, 1, 0);
    cs.row_expand = 9;
    return conv(p + ".conv+actf", {cs}, cho, 1);
  }
  // IDAUp.forward (:453-460): layers[i] = node(pad_to_match(up(proj(layers[i]))) + layers[i-1])
  int ida(const std::string& p, std::vector<int>& layers, int startp, int endp, int o) {
    for (int i = startp + 1; i < endp; ++i) {
      const std::string js = std::to_string(i - startp);
      const int pr = deform(p + ".proj_" + js, layers[i], o);
      const TensorSpec src = P.tensors[pr], tgt = P.tensors[layers[i - 1]];
      const std::string uw = p + ".up_" + js;
      int f = 0;
      for (const ParamInfo& pi : P.params)
        if (pi.name == uw + ".weight") f = (int)pi.shape[2] / 2;
      if (f < 1) {
        set_error("DLA34 planner: missing " + uw);
        return -1;
      }
      const int hu = (src.H - 1) * f - 2 * (f / 2) + 2 * f, wu = (src.W - 1) * f - 2 * (f / 2) + 2 * f;
      OpSpec op;
      op.kind = OP_DWCONVT_ADD;
      op.label = uw + "+pad_to_match+add";
      op.src = pr;
      op.add = layers[i - 1];
      op.up_s = f;
      op.up_w = uw;
      op.N = o;
      op.sy = std::max(0, (hu - tgt.H) / 2);  // pad_to_match (:394-407), (W, H) order correct here
      op.sx = std::max(0, (wu - tgt.W) / 2);
      op.flops = 2.0 * src.H * src.W * o * 4.0 * f * f;
      op.out = tensor(tgt.H, tgt.W, o);
      P.ops.push_back(op);
      layers[i] = deform(p + ".node_" + js, op.out, o);
    }
    return 0;
  }
  int forward() {
    const int vec = 16 / dtype_size(d.compute_dtype);
    const int cpad = (7 * 3 + vec - 1) / vec * vec;  // row-expanded 7x7 stem input (planner.cpp)
    P.in_cpad = cpad;
    const int img = tensor(d.in_h, d.in_w, cpad);
    {
      OpSpec op;
      op.kind = OP_PREP;
      op.label = "input staging (NCHW fp32 / u8 frames -> NHWC)";
      op.out = img;
      op.N = cpad;
      P.ops.push_back(op);
    }
    const std::string b = "model.base";
    SegSpec stem = seg(img, b + ".base_layer.0", b + ".base_layer.1", 0, 3, 7, 1, 3);
    stem.kw = 1;
    stem.pad_w = 0;
    stem.row_expand = 7;
    int x = conv(b + ".base_layer.0", {stem}, kChannels[0], 1);
    std::vector<int> layers;
    int cin = kChannels[0];
    for (int l = 0; l < 2; ++l) {  // _make_conv_level (:288-297)
      for (int c = 0; c < kLevels[l]; ++c) {
        const std::string q = b + ".level" + std::to_string(l) + ".";
        x = conv(q + std::to_string(3 * c), {seg(x, q + std::to_string(3 * c), q + std::to_string(3 * c + 1), 0, cin, 3,
                                                 c == 0 ? (l == 1 ? 2 : 1) : 1, 1)},
                 kChannels[l], 1);
        cin = kChannels[l];
      }
      layers.push_back(x);
    }
    for (int l = 2; l < 6; ++l) {
      x = tree(b + ".level" + std::to_string(l), x, kLevels[l], 2, kChannels[l - 1], kChannels[l], l >= 3, {});
      if (x < 0) return TV_ESHAPE;
      layers.push_back(x);
    }
    // DLAUp.forward (:451-457)
    const auto defs = dla_up_defs();
    std::vector<int> out{layers.back()};
    const int n = (int)layers.size();
    for (int i = 0; i < n - kFirstLevel - 1; ++i) {
      if (ida("model.dla_up.ida_" + std::to_string(i), layers, n - i - 2, n, defs[i].o)) return TV_ESHAPE;
      out.insert(out.begin(), layers.back());
    }
    // DLASeg.forward (:515-525)
    std::vector<int> y(out.begin(), out.begin() + (kLastLevel - kFirstLevel));
    if (ida("model.ida_up", y, 0, (int)y.size(), ida_up_def().o)) return TV_ESHAPE;
    const int cur = y.back();
    const TensorSpec ft = P.tensors[cur];
    const int C = ft.C;
    OpSpec h1;
    h1.kind = OP_CONV;
    h1.label = "model.*.0 (stacked heads) + ReLU";
    h1.segs = {SegSpec{cur, "", "", 0, C, 3, 3, 1, 1}};
    h1.N = kHeadConv * d.n_heads;
    h1.act = 1;
    for (int h = 0; h < d.n_heads; ++h) {
      h1.stack_w.push_back("model." + std::to_string(h) + ".0");
      h1.stack_n.push_back(kHeadConv);
    }
    h1.flops = 2.0 * ft.H * ft.W * h1.N * 9.0 * C;
    h1.out = tensor(ft.H, ft.W, h1.N);
    P.ops.push_back(h1);
    OpSpec h2;
    h2.kind = OP_CONV;
    h2.label = "model.*.2 (block-diagonal) -> fp32 NHWC";
    h2.segs = {SegSpec{h1.out, "", "", 0, h1.N, 1, 1, 1, 0}};
    int ctot = 0;
    for (int h = 0; h < d.n_heads; ++h) {
      h2.stack_w.push_back("model." + std::to_string(h) + ".2");
      h2.stack_n.push_back(d.head_channels[h]);
      h2.diag_in_off.push_back(kHeadConv * h);
      h2.diag_out_off.push_back(ctot);
      h2.flops += 2.0 * ft.H * ft.W * d.head_channels[h] * (double)kHeadConv;
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

int build_plan_dla34(const tv_model_desc& d, Plan* plan) {
  if (d.n_heads < 1 || d.n_heads > 16 || d.in_h < 1 || d.in_w < 1 || d.compute_dtype < 0 || d.compute_dtype > 2) {
    set_error("model desc out of range");
    return TV_EINVAL;
  }
  for (int h = 0; h < d.n_heads; ++h)
    if (d.head_channels[h] < 1) {
      set_error("head channel counts must be positive");
      return TV_EINVAL;
    }
  if (d.in_h < 32 || d.in_w < 32) {
    set_error("CenterpointDLA34 needs frames of at least 32x32 (five stride-2 levels)");
    return TV_ESHAPE;
  }
  *plan = Plan();
  DlaWalker w(d, *plan);
  w.params();
  for (const ParamInfo& p : plan->params) plan->names.insert(p.name);
  return w.forward();
}

}  // namespace tv
