// Engine: BN folding + weight packing at create, liveness-planned HBM workspace per
// (stream, batch), and the launch sequence of one forward. C ABI in capi.cpp.
#include "engine.h"

#include <algorithm>
#include <cmath>
#include <cstring>
#include <cstdlib>
#include <set>

namespace tv {

namespace {

constexpr int kTile = 128;

uint16_t f32_to_bf16(float f) {
  uint32_t u;
  std::memcpy(&u, &f, 4);
  if ((u & 0x7F800000u) == 0x7F800000u && (u & 0x7FFFFFu)) return (uint16_t)((u >> 16) | 0x40);  // NaN
  u += 0x7FFFu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}

void store_elem(void* base, size_t i, float v, int dtype) {
  if (dtype == F32) {
    reinterpret_cast<float*>(base)[i] = v;
  } else if (dtype == F16) {
    reinterpret_cast<_Float16*>(base)[i] = (_Float16)v;
  } else {
    reinterpret_cast<uint16_t*>(base)[i] = f32_to_bf16(v);
  }
}

size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

}  // namespace

const float* Engine::weight(const std::string& name, int64_t numel) {
  auto it = host_w.find(name);
  if (it == host_w.end()) {
    set_error("missing state_dict key: " + name);
    return nullptr;
  }
  if (it->second.second != numel) {
    set_error("state_dict key " + name + ": expected " + std::to_string(numel) + " elements, got " +
              std::to_string(it->second.second));
    return nullptr;
  }
  return it->second.first;
}

// Folded BN affine for a conv `p` (+ BatchNorm `bn`): scale, shift per output channel.
int Engine::fold(const std::string& conv, const std::string& bn, int cout, std::vector<double>& scale,
                 std::vector<double>& shift) {
  scale.assign(cout, 1.0);
  shift.assign(cout, 0.0);
  // bias=False convs (DLA34, centerpoint_dla.py:24-27) have no `.bias` key in the layout
  std::vector<float> zeros;
  const float* b = nullptr;
  if (plan.names.count(conv + ".bias")) {
    b = weight(conv + ".bias", cout);
    if (!b) return TV_ENOTFOUND;
  } else {
    zeros.assign(cout, 0.f);
    b = zeros.data();
  }
  for (int i = 0; i < cout; ++i) shift[i] = b[i];
  if (bn.empty()) return TV_OK;
  const float* g = weight(bn + ".weight", cout);
  const float* be = weight(bn + ".bias", cout);
  const float* mu = weight(bn + ".running_mean", cout);
  const float* var = weight(bn + ".running_var", cout);
  if (!g || !be || !mu || !var) return TV_ENOTFOUND;
  for (int i = 0; i < cout; ++i) {
    double s = (double)g[i] / std::sqrt((double)var[i] + 1e-5);
    scale[i] = s;
    shift[i] = ((double)b[i] - (double)mu[i]) * s + (double)be[i];
  }
  return TV_OK;
}

int Engine::pack_op(size_t oi) {
  const OpSpec& op = plan.ops[oi];
  Packed& pk = packed[oi];
  const int esz = dtype_size(dtype);
  const int BK = 128 / esz;
  if (op.kind == OP_PREP || op.kind == OP_MAXPOOL || op.kind == OP_DCN || op.kind == OP_LAYOUT_IN) return TV_OK;
  if (op.kind == OP_DWCONVT_ADD) {  // depthwise ConvTranspose2d weight [C][1][2f][2f] -> fp32 [2f][2f][C]
    const int c = op.N, k = 2 * op.up_s;
    const float* w = weight(op.up_w + ".weight", (int64_t)c * k * k);
    if (!w) return TV_ENOTFOUND;
    std::vector<float> t((size_t)k * k * c);
    for (int co = 0; co < c; ++co)
      for (int tap = 0; tap < k * k; ++tap) t[(size_t)tap * c + co] = w[(size_t)co * k * k + tap];
    TV_HIP(hipMalloc(&pk.w, t.size() * sizeof(float)));
    TV_HIP(hipMemcpy(pk.w, t.data(), t.size() * sizeof(float), hipMemcpyHostToDevice));
    weight_bytes += t.size() * sizeof(float);
    return TV_OK;
  }

  std::vector<float> hw;    // [Npad][Kpad] fp32 staging
  std::vector<float> bias;  // [Npad]
  if (op.kind == OP_CONVT_ADD) {
    const TensorSpec& src = plan.tensors[op.src];
    const int c = op.N, s = op.up_s, cin = src.C;
    const int N = s * s * c;
    pk.Npad = (int)align_up(N, kTile);
    pk.seg_ksteps = {(cin + BK - 1) / BK};
    pk.Kpad = pk.seg_ksteps[0] * BK;
    hw.assign((size_t)pk.Npad * pk.Kpad, 0.f);
    bias.assign(pk.Npad, 0.f);
    const float* w = weight(op.up_w + ".weight", (int64_t)cin * c * s * s);
    const float* b = weight(op.up_w + ".bias", c);
    if (!w || !b) return TV_ENOTFOUND;
    for (int i = 0; i < s; ++i)
      for (int j = 0; j < s; ++j)
        for (int co = 0; co < c; ++co) {
          const int n = (i * s + j) * c + co;
          bias[n] = b[co];
          for (int ci = 0; ci < cin; ++ci) hw[(size_t)n * pk.Kpad + ci] = w[(((size_t)ci * c + co) * s + i) * s + j];
        }
  } else {
    const int N = op.N;
    // rows of the PyTorch weight: a plain conv into the caller's fp32 output stores out_cpad
    // columns of an out_c-channel conv (protonet _output_layer)
    const int wN = (op.out < 0 && op.stack_w.empty()) ? plan.out_c : N;
    pk.Npad = (int)align_up(N, kTile);
    int kbase = 0;
    pk.seg_ksteps.clear();
    for (const SegSpec& sg : op.segs) {
      const int cs = plan.tensors[sg.src].C;
      const int ks = (sg.kh * sg.kw * cs + BK - 1) / BK;
      pk.seg_ksteps.push_back(ks);
      kbase += ks;
    }
    pk.Kpad = kbase * BK;
    hw.assign((size_t)pk.Npad * pk.Kpad, 0.f);
    bias.assign(pk.Npad, 0.f);
    if (!op.stack_w.empty()) {
      // stacked heads (3x3, single segment) or block-diagonal 1x1 heads
      const SegSpec& sg = op.segs[0];
      const int cs = plan.tensors[sg.src].C;
      const bool diag = !op.diag_in_off.empty();
      int row = 0;
      for (size_t h = 0; h < op.stack_w.size(); ++h) {
        const int n = op.stack_n[h];
        const int cin = diag ? plan.tensors[sg.src].C / (int)op.stack_w.size() : sg.cin;
        const int k = sg.kh;
        const float* w = weight(op.stack_w[h] + ".weight", (int64_t)n * cin * k * k);
        const float* b = weight(op.stack_w[h] + ".bias", n);
        if (!w || !b) return TV_ENOTFOUND;
        const int r0 = diag ? op.diag_out_off[h] : row;
        const int c0 = diag ? op.diag_in_off[h] : 0;
        for (int co = 0; co < n; ++co) {
          bias[r0 + co] = b[co];
          for (int ci = 0; ci < cin; ++ci)
            for (int t = 0; t < k * k; ++t)
              hw[(size_t)(r0 + co) * pk.Kpad + t * cs + c0 + ci] = w[((size_t)co * cin + ci) * k * k + t];
        }
        row += n;
      }
    } else {
      // BN-folded segments; bias = sum over the distinct convs feeding this GEMM
      std::set<std::string> seen;
      int kb = 0;
      for (size_t si = 0; si < op.segs.size(); ++si) {
        const SegSpec& sg = op.segs[si];
        const int cs = plan.tensors[sg.src].C;
        if (sg.identity) {  // residual added as-is: identity 1x1 (exact in every compute dtype)
          for (int co = 0; co < std::min(N, sg.cin); ++co) hw[(size_t)co * pk.Kpad + (size_t)kb * BK + co] = 1.f;
          kb += pk.seg_ksteps[si];
          continue;
        }
        // total input channels of the PyTorch weight = max over segments sharing it
        int wcin = 0;
        for (const SegSpec& o : op.segs)
          if (o.wname == sg.wname) wcin = std::max(wcin, o.ci0 + o.cin);
        const int re = sg.row_expand;  // row-expanded input: K index = ky * cs + kx * cin + c
        const int kk = re ? sg.kh * re : sg.kh * sg.kw;
        if (sg.convt_phase >= 0) {
          // ConvTranspose2d(3, s2, p1) weight [cin][cout][3][3], one output parity (pi, pj): tap
          // (dy, dx) of the phase conv reads input (m + dy, n + dx) and uses kernel element
          // ky = 1 (pi = 0) or 2 - 2 dy (pi = 1) — out[2m + pi] += x[m + dy] W[ky] with
          // 2m + pi = 2(m + dy) - 1 + ky — and kx likewise
          const float* w = weight(sg.wname + ".weight", (int64_t)wcin * wN * 9);
          if (!w) return TV_ENOTFOUND;
          std::vector<double> scale, shift;
          int rc = fold(sg.wname, "", wN, scale, shift);
          if (rc) return rc;
          for (int co = 0; co < wN; ++co) bias[co] += (float)shift[co];
          const int pi = sg.convt_phase >> 1, pj = sg.convt_phase & 1;
          for (int dy = 0; dy < sg.kh; ++dy)
            for (int dx = 0; dx < sg.kw; ++dx) {
              const int ky = pi == 0 ? 1 : 2 - 2 * dy, kx = pj == 0 ? 1 : 2 - 2 * dx;
              const int t = dy * sg.kw + dx;
              for (int co = 0; co < wN; ++co)
                for (int ci = 0; ci < sg.cin; ++ci)
                  hw[(size_t)co * pk.Kpad + (size_t)kb * BK + (size_t)t * cs + ci] =
                      w[(((size_t)(sg.ci0 + ci) * wN + co) * 3 + ky) * 3 + kx];
            }
          // all four phases in one launch (convt3.hip): the phase-(0,0) op carries the whole
          // ConvTranspose2d's weight in that kernel's fragment order (knob TV_CT3=0: off)
          if (ct3_mode && dtype != F32 && sg.convt_phase == 0 && op.segs.size() == 1 && sg.ci0 == 0 &&
              sg.cin == cs && wcin == cs && convt3_supported(cs, wN, cs, wN, 1, 1, esz)) {
            std::vector<uint8_t> frag(convt3_weight_bytes(cs, wN));
            convt3_pack(w, cs, wN, dtype, frag.data());
            TV_HIP(hipMalloc(&pk.w_ct3, frag.size()));
            TV_HIP(hipMemcpy(pk.w_ct3, frag.data(), frag.size(), hipMemcpyHostToDevice));
            weight_bytes += frag.size();
          }
          kb += pk.seg_ksteps[si];
          continue;
        }
        const float* w = weight(sg.wname + ".weight", (int64_t)wN * wcin * kk);
        if (!w) return TV_ENOTFOUND;
        std::vector<double> scale, shift;
        int rc = fold(sg.wname, sg.bn, wN, scale, shift);
        if (rc) return rc;
        if (seen.insert(sg.wname).second)
          for (int co = 0; co < wN; ++co) bias[co] += (float)shift[co];
        for (int co = 0; co < wN; ++co)
          for (int ci = 0; ci < sg.cin; ++ci)
            for (int t = 0; t < kk; ++t) {
              const size_t k = re ? (size_t)(t / re) * cs + (t % re) * sg.cin + ci : (size_t)t * cs + ci;
              hw[(size_t)co * pk.Kpad + (size_t)kb * BK + k] =
                  (float)((double)w[((size_t)co * wcin + sg.ci0 + ci) * kk + t] * scale[co]);
            }
        kb += pk.seg_ksteps[si];
      }
    }
  }
  // fused 1x1 heads (conv3x3 EPI 1): per 128-channel tile nt of the hidden (stacked 3x3) output,
  // fragment (k-step j, lane l) = 8 weights W2[row0 + l%32][128nt + 16j + 8(l/32) + e]
  if (dtype != F32 && !op.diag_in_off.empty() && op.segs.size() == 1) {
    const int K = plan.tensors[op.segs[0].src].C;  // hidden channels
    const int nts = K / 128;
    const int hid = K / (int)op.stack_w.size();    // hidden channels per head
    bool ok = K % 128 == 0 && nts <= 16 && hid % 128 == 0;
    for (size_t h = 0; h < op.stack_n.size(); ++h) ok = ok && op.stack_n[h] <= 32;
    if (ok) {
      std::vector<uint8_t> frag((size_t)nts * 8 * 64 * 16, 0);
      std::vector<float> hb((size_t)nts * 32, 0.f);
      for (int nt = 0; nt < nts; ++nt) {
        const int h = nt * 128 / hid;
        const int row0 = op.diag_out_off[h], nr = op.stack_n[h];
        pk.head_row0[nt] = row0;
        pk.head_nrows[nt] = nr;
        if (nt * 128 == op.diag_in_off[h])
          for (int r = 0; r < nr; ++r) hb[nt * 32 + r] = bias[row0 + r];
        for (int j = 0; j < 8; ++j)
          for (int l = 0; l < 64; ++l)
            for (int e = 0; e < 8; ++e) {
              const int r = l & 31, k = nt * 128 + 16 * j + 8 * (l >> 5) + e;
              const float v = r < nr ? hw[(size_t)(row0 + r) * pk.Kpad + k] : 0.f;
              store_elem(frag.data(), ((size_t)(nt * 8 + j) * 64 + l) * 8 + e, v, dtype);
            }
      }
      TV_HIP(hipMalloc(&pk.head_w, frag.size()));
      TV_HIP(hipMemcpy(pk.head_w, frag.data(), frag.size(), hipMemcpyHostToDevice));
      TV_HIP(hipMalloc((void**)&pk.head_b, hb.size() * sizeof(float)));
      TV_HIP(hipMemcpy(pk.head_b, hb.data(), hb.size() * sizeof(float), hipMemcpyHostToDevice));
      pk.head_ok = 1;
    }
  }
  // device copies
  std::vector<uint8_t> hbuf((size_t)pk.Npad * pk.Kpad * esz);
  for (size_t i = 0; i < hw.size(); ++i) store_elem(hbuf.data(), i, hw[i], dtype);
  if ((int)oi == stem_op) {  // stem.hip streams its weights in MFMA B-fragment order
    std::vector<uint8_t> frag(stem_weight_bytes());
    stem_fragment_order(reinterpret_cast<const uint16_t*>(hbuf.data()), pk.Npad, pk.Kpad,
                        reinterpret_cast<uint16_t*>(frag.data()));
    hbuf.swap(frag);
  }
  TV_HIP(hipMalloc(&pk.w, hbuf.size()));
  TV_HIP(hipMemcpy(pk.w, hbuf.data(), hbuf.size(), hipMemcpyHostToDevice));
  TV_HIP(hipMalloc((void**)&pk.bias, bias.size() * sizeof(float)));
  TV_HIP(hipMemcpy(pk.bias, bias.data(), bias.size() * sizeof(float), hipMemcpyHostToDevice));
  weight_bytes += hbuf.size() + bias.size() * 4;
  return TV_OK;
}

int Engine::create(const tv_model_desc& d, const tv_weight_view* w, int n, int dev,
                   const std::vector<std::pair<std::string, std::string>>& knobs) {
  desc = d;
  device = dev;
  if (desc.compute_dtype == TV_F32X3) {  // fp32 storage; the pipelined GEMMs' products as three fp16 MFMAs
    desc.compute_dtype = TV_F32;
    f32x3 = 1;
  }
  dtype = desc.compute_dtype;
  int rc = build_plan(desc, &plan);
  if (rc) return rc;
  for (int i = 0; i < n; ++i) {
    if (!w[i].name || (!w[i].data && w[i].numel)) {
      set_error("null weight view");
      return TV_EINVAL;
    }
    host_w[w[i].name] = {w[i].data, w[i].numel};
  }
  TV_HIP(hipSetDevice(device));
  TV_HIP(hipMalloc(&zero_page, 256));
  TV_HIP(hipMemset(zero_page, 0, 256));
  {
    int ncu = 0;
    if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && ncu > 0)
      cu_count = ncu;
  }
  // diagnostics only (tv_engine_create_diag): kernel-choice overrides for A/B experiments; the
  // product entry point (tv_engine_create) passes none and reads no environment
  for (const auto& kv : knobs) {
    const std::string& k = kv.first;
    const char* env = kv.second.c_str();
    const int v = std::atoi(env);
    if (k == "TV_CONV_PIPE") pipe_mode = v;
    else if (k == "TV_CONV3") conv3_mode = v;
    else if (k == "TV_C3_TW") c3_tw_force = v == 16 ? 16 : v == 32 ? 32 : 0;
    else if (k == "TV_CUS") cu_count = std::max(8, std::min(cu_count, v));
    else if (k == "TV_STEM") stem_mode = v;
    else if (k == "TV_STEMFUSE") stemfuse_mode = v;
    else if (k == "TV_LAT") lat_mode = v;
    else if (k == "TV_LAT_UNITS") lat_units = v;
    else if (k == "TV_LAT_SPLIT") lat_split_max = std::max(1, std::min(8, v));
    else if (k == "TV_LAT_SPLIT_MIN") lat_split_min_nks = std::max(0, v);
    else if (k == "TV_LAT_F32") lat_f32 = v ? 1 : 0;
    else if (k == "TV_LAT_SPLIT_F32") lat_split_max_f32 = std::max(1, std::min(16, v));
    else if (k == "TV_PIPE_SPLIT") pipe_split_mode = std::max(0, std::min(2, v));
    else if (k == "TV_PIPE_SPLIT_MAX") pipe_split_max = std::max(1, std::min(64, v));
    else if (k == "TV_PIPE_SPLIT_RED") pipe_split_red = std::max(0, v);
    else if (k == "TV_F32X3") f32x3 = v ? 1 : 0;
    else if (k == "TV_LATGROUP") lat_group = v ? 1 : 0;
    else if (k == "TV_CT3") ct3_mode = v ? 1 : 0;
    else if (k == "TV_BURST") burst_mode = std::max(0, std::min(2, v));
    else if (k == "TV_C1X1") c1x1_mode = std::max(0, std::min(2, v));
    else if (k == "TV_LATGROUP_B") lat_group_max_b = std::max(1, v);
    else if (k == "TV_DCN64") dcn64_mode = v;
    else if (k == "TV_DCN_SPLIT") dcn_split_max = std::max(0, std::min(9, v));
    else if (k == "TV_CONVT") convt_mode = v;
    else if (k == "TV_CONV3S2") s2_mode = v;
    else if (k == "TV_CONV3_MINPIX") conv3_min_pix = v;
    else if (k == "TV_HEADFUSE") headfuse_mode = v;
    else if (k == "TV_S2_MINTILES") s2_min_tiles = v;
    else if (k == "TV_C3_NI") c3_ni_force = v == 2 ? 2 : v == 4 ? 4 : 0;
    else if (k == "TV_C3_NW") c3_nw_mode = v == 8 ? 8 : 0;
    else if (k == "TV_C3_HALF_COST") c3_half_cost = v;
    else if (k == "TV_CSM_HALO") csm_halo = std::max(0, std::min(2, v));
    else if (k == "TV_SLICES") slices = std::max(1, std::min(kMaxSlices, v));
    else if (k == "TV_SLICE_LAG") slice_lag = std::max(0, v);
    else if (k == "TV_C3_STAMPS") {  // "op:device pointer" (stamp builds of conv3x3 only)
#if defined(TV_C3_EXP) && TV_C3_EXP == 9
      stamp_op = v;
      const char* c = std::strchr(env, ':');
      stamp_buf = c ? reinterpret_cast<unsigned long long*>(std::strtoull(c + 1, nullptr, 0)) : nullptr;
      // the stamp kernel writes 8 counters per wave of every workgroup it may launch (<= one per
      // CU, 8 waves): the pointer must lie in a device allocation with that much room after it
      hipDeviceptr_t base = nullptr;
      size_t size = 0;
      const size_t need = (size_t)cu_count * 8 * 8 * sizeof(unsigned long long);
      if (!stamp_buf || hipMemGetAddressRange(&base, &size, stamp_buf) != hipSuccess ||
          (char*)stamp_buf + need > (char*)base + size) {
        (void)hipGetLastError();
        set_error("TV_C3_STAMPS: the pointer is not inside a device allocation of >= " + std::to_string(need) +
                  " bytes");
        return TV_EINVAL;
      }
#else
      set_error("TV_C3_STAMPS needs the stamp build of the library (EXTRA=-DTV_C3_EXP=9)");
      return TV_EINVAL;
#endif
    }
    else if (k == "TV_SLICE_SIZES") {
      for (const char* c = env; *c;) {
        slice_sizes_env.push_back(std::atoi(c));
        while (*c && *c != ',') ++c;
        if (*c == ',') ++c;
      }
    } else {
      set_error("unknown engine knob: " + k);
      return TV_EINVAL;
    }
  }
  // fused staging + stem (stem.hip): the row-expanded 7x7 conv right after the staging op
  if (stem_mode && dtype != F32)
    for (size_t i = 0; i + 1 < plan.ops.size(); ++i)
      if (plan.ops[i].kind == OP_PREP && plan.ops[i + 1].kind == OP_CONV && plan.ops[i + 1].segs.size() == 1 &&
          plan.ops[i + 1].segs[0].row_expand == 7 && plan.ops[i + 1].N <= 128 && plan.ops[i + 1].N % 8 == 0 &&
          plan.ops[i + 1].act == 1) {
        stem_op = (int)i + 1;
        break;
      }
  // stem + block0.conv1 in one launch (stem_s2.hip): the 128-channel stem feeds exactly the block's
  // stride-2 3x3 conv1 and its stride-2 1x1 conv_residual (dla.py:13-37, 182-186). The plan gets a
  // tensor R = stem(2y, 2x) [Ho, Wo, 128], written by the fused launch (conv1's second output) and
  // read by conv2's residual segment at stride 1; the stem output itself is never stored.
  if (stemfuse_mode && stem_op >= 0 && stem_op + 2 < (int)plan.ops.size()) {
    const OpSpec& st = plan.ops[stem_op];
    const OpSpec& c1 = plan.ops[stem_op + 1];
    const OpSpec& c2 = plan.ops[stem_op + 2];
    const int so = st.out;
    bool ok = st.N == 128 && so >= 0 && plan.tensors[so].C == 128 && c1.kind == OP_CONV && c1.segs.size() == 1 &&
              c1.segs[0].src == so && c1.segs[0].kh == 3 && c1.segs[0].kw == 3 && c1.segs[0].stride == 2 &&
              c1.segs[0].pad == 1 && (c1.segs[0].pad_w < 0 || c1.segs[0].pad_w == 1) && !c1.segs[0].row_expand &&
              c1.segs[0].ci0 == 0 && c1.segs[0].cin == 128 && c1.N == 128 && c1.act == 1 && c1.out >= 0 &&
              c1.add < 0 && !c1.up_s && c1.stack_w.empty() && plan.tensors[c1.out].C == 128 &&
              plan.tensors[c1.out].H == (desc.in_h + 1) / 2 && plan.tensors[c1.out].W == (desc.in_w + 1) / 2 &&
              c2.kind == OP_CONV && c2.segs.size() == 2 && c2.segs[0].src == c1.out && c2.segs[1].src == so &&
              c2.segs[1].kh == 1 && c2.segs[1].kw == 1 && c2.segs[1].stride == 2 && c2.segs[1].pad == 0 &&
              !c2.segs[1].identity && c2.segs[1].ci0 == 0 && c2.segs[1].cin == 128;
    for (size_t i = 0; ok && i < plan.ops.size(); ++i) {  // nothing else reads the stem output
      if ((int)i == stem_op + 1 || (int)i == stem_op + 2) continue;
      const OpSpec& o = plan.ops[i];
      ok = o.src != so && o.add != so;
      for (const SegSpec& sg : o.segs) ok = ok && sg.src != so;
    }
    if (ok) {
      const TensorSpec t1 = plan.tensors[c1.out];
      plan.tensors.push_back(TensorSpec{t1.H, t1.W, 128});
      const int r = (int)plan.tensors.size() - 1;
      plan.ops[stem_op + 1].out2 = r;
      plan.ops[stem_op + 2].segs[1].src = r;
      plan.ops[stem_op + 2].segs[1].stride = 1;
      ss2_op = stem_op + 1;
    }
  }
  packed.resize(plan.ops.size());
  for (size_t i = 0; i < plan.ops.size(); ++i) {
    rc = pack_op(i);
    if (rc) return rc;
  }
  host_w.clear();  // views are only valid during create
  return TV_OK;
}

Engine::~Engine() {
  if (zero_page) (void)hipFree(zero_page);
  for (auto& p : packed) {
    if (p.w) (void)hipFree(p.w);
    if (p.w_c3) (void)hipFree(p.w_c3);
    if (p.w_c3h) (void)hipFree(p.w_c3h);
    if (p.w_c3e) (void)hipFree(p.w_c3e);
    if (p.w_ss2) (void)hipFree(p.w_ss2);
    if (p.w_burst) (void)hipFree(p.w_burst);
    if (p.w_x3) (void)hipFree(p.w_x3);
    if (p.w_ct3) (void)hipFree(p.w_ct3);
    if (p.head_w) (void)hipFree(p.head_w);
    if (p.head_b) (void)hipFree(p.head_b);
    if (p.bias) (void)hipFree(p.bias);
  }
  for (auto& kv : workspaces) {
    if (kv.second->arena) (void)hipFree(kv.second->arena);
    if (kv.second->dparams) (void)hipFree(kv.second->dparams);
    if (kv.second->dks) (void)hipFree(kv.second->dks);
    if (kv.second->slab) (void)hipFree(kv.second->slab);
    for (hipEvent_t ev : kv.second->gev) (void)hipEventDestroy(ev);
    if (kv.second->pslab) (void)hipFree(kv.second->pslab);
    if (kv.second->pcnt) (void)hipFree(kv.second->pcnt);
    if (kv.second->dslab) (void)hipFree(kv.second->dslab);
    if (kv.second->dcnt) (void)hipFree(kv.second->dcnt);
    if (kv.second->cnt) (void)hipFree(kv.second->cnt);
    delete kv.second;
  }
  for (auto& kv : side) {
    if (kv.second.fork) (void)hipEventDestroy(kv.second.fork);
    for (hipEvent_t e : kv.second.join) (void)hipEventDestroy(e);
    for (hipStream_t t : kv.second.s) (void)hipStreamDestroy(t);
  }
}

// Liveness-planned arena: a tensor lives from its producing op to its last reader;
// first-fit placement of each new tensor into the gaps left by dead ones.
int Engine::make_workspace(int B, Workspace* ws) {
  const int esz = dtype_size(dtype);
  const size_t nt = plan.tensors.size();
  const size_t nops = plan.ops.size();
  // Dependency levels: a conv / ConvT + add op runs one level after the last producer of a tensor
  // it reads (the MultiIDAUp wavefront: IDAUp i+1's step at a level needs only IDAUp i's output
  // there and its own previous step, dla.py:265-284, 377-390; the IDAUpReverse projections need
  // only MultiIDAUp's outputs); every other op (staging, the fp32-output heads, DCN sampling,
  // pooling, depthwise up-sampling) is a barrier after everything before it. Ops then run by
  // level (plan order within one), and the arena's lifetimes are counted in levels, so that ops
  // of one level may run in one launch.
  // Only on the latency path (B <= lat_group_max_b frames per launch): at B = 32 per slice the
  // other slice fills the CUs these small layers leave idle, and the reordering measured 0.5%
  // slower there (profiles/r4y); at B = 1 it took 1.43 -> 1.35 ms.
  const bool grouping = lat_group && B <= lat_group_max_b;
  ws->level.assign(nops, 0);
  {
    std::vector<int> prod(nt, -1);
    int barrier = -1, maxlev = -1;
    for (size_t i = 0; i < nops; ++i) {
      const OpSpec& op = plan.ops[i];
      int lv;
      if (!grouping) {
        lv = (int)i;
      } else if ((op.kind == OP_CONV || op.kind == OP_CONVT_ADD) && op.out >= 0) {
        lv = barrier + 1;
        auto after = [&](int t) { if (t >= 0 && prod[t] >= 0) lv = std::max(lv, prod[t] + 1); };
        for (const SegSpec& sg : op.segs) after(sg.src);
        after(op.src);
        after(op.add);
      } else {
        lv = maxlev + 1;
        barrier = lv;
      }
      ws->level[i] = lv;
      maxlev = std::max(maxlev, lv);
      if (op.out >= 0) prod[op.out] = std::max(prod[op.out], lv);
      if (op.out2 >= 0) prod[op.out2] = std::max(prod[op.out2], lv);
    }
    ws->order.resize(nops);
    for (size_t i = 0; i < nops; ++i) ws->order[i] = (int)i;
    std::stable_sort(ws->order.begin(), ws->order.end(), [&](int a, int b) { return ws->level[a] < ws->level[b]; });
  }
  const std::vector<int>& lev = ws->level;
  std::vector<int> def(nt, -1), last(nt, -1);
  for (size_t i = 0; i < nops; ++i) {
    const OpSpec& op = plan.ops[i];
    const int t = lev[i];
    if (op.out >= 0) def[op.out] = t, last[op.out] = std::max(last[op.out], t);
    if (op.out2 >= 0) def[op.out2] = t, last[op.out2] = std::max(last[op.out2], t);
    for (const SegSpec& s : op.segs) last[s.src] = std::max(last[s.src], t);
    if (op.src >= 0) last[op.src] = std::max(last[op.src], t);
    if (op.add >= 0) last[op.add] = std::max(last[op.add], t);
    // the fused DCNv2 kernel (dcn.hip) samples x and reads the offset / mask tensor while it runs
    // the column GEMM (op i): both stay live through it
    if (op.kind == OP_CONV && i > 0 && plan.ops[i - 1].kind == OP_DCN && op.segs.size() == 1 &&
        op.segs[0].src == plan.ops[i - 1].out) {
      last[plan.ops[i - 1].src] = std::max(last[plan.ops[i - 1].src], t);
      last[plan.ops[i - 1].add] = std::max(last[plan.ops[i - 1].add], t);
    }
  }
  // DCNv2 sampling + its column GEMM that run as one fused kernel (dcn.hip): the column tensor
  // (B x H x W x 9C) is never materialised, so it gets no arena space
  auto dcn_fusable = [&](size_t i) {
    if (dtype == F32 || i + 1 >= plan.ops.size()) return false;
    const OpSpec& d = plan.ops[i];
    const OpSpec& g = plan.ops[i + 1];
    if (d.kind != OP_DCN || g.kind != OP_CONV || g.segs.size() != 1 || g.segs[0].src != d.out ||
        g.segs[0].row_expand != 9 || g.out < 0 || g.add >= 0)
      return false;
    const TensorSpec& xt = plan.tensors[d.src];
    return dcn_gemm_supported((long)B * xt.H * xt.W, xt.C, g.N, xt.C, plan.tensors[d.add].C, plan.tensors[g.out].C,
                              packed[i + 1].Kpad) &&
           g.segs[0].cin == xt.C;
  };
  std::vector<char> virt(nt, 0);
  for (size_t i = 0; i < plan.ops.size(); ++i)
    if (dcn_fusable(i)) virt[plan.ops[i].out] = 1;
  ws->off.assign(nt, 0);
  struct Live { size_t off, size; int last; };
  std::vector<Live> live;
  std::vector<char> placed(nt, 0);  // a tensor written by several ops (ConvT phases) is placed once
  size_t peak = 0;
  for (const int i : ws->order) {
    const OpSpec& op = plan.ops[i];
    live.erase(std::remove_if(live.begin(), live.end(), [&](const Live& l) { return l.last < lev[i]; }), live.end());
    if (op.out < 0 || (stem_op >= 0 && op.kind == OP_PREP)) continue;  // fused stem: no staged input
    if (ss2_op >= 0 && i == stem_op) continue;                           // stem fused into block0.conv1: never stored
    if (virt[op.out]) continue;                                          // fused DCN: no column tensor
    auto place = [&](int tid) {
      if (placed[tid]) return;
      placed[tid] = 1;
      const TensorSpec& t = plan.tensors[tid];
      size_t sz = align_up((size_t)B * t.H * t.W * t.C * esz, 256);
      std::sort(live.begin(), live.end(), [](const Live& a, const Live& b) { return a.off < b.off; });
      size_t pos = 0;
      for (const Live& l : live) {
        if (pos + sz <= l.off) break;
        pos = std::max(pos, l.off + l.size);
      }
      ws->off[tid] = pos;
      live.push_back({pos, sz, last[tid]});
      peak = std::max(peak, pos + sz);
    };
    place(op.out);
    if (op.out2 >= 0) place(op.out2);
  }
  ws->bytes = peak;
  ws->B = B;
  TV_HIP(hipSetDevice(device));
  TV_HIP(hipMalloc(&ws->arena, std::max<size_t>(peak, 256)));
  // launch parameters for every op
  ws->params.assign(plan.ops.size(), ConvParams{});
  char* base = (char*)ws->arena;
  for (size_t i = 0; i < plan.ops.size(); ++i) {
    const OpSpec& op = plan.ops[i];
    if (op.kind != OP_CONV && op.kind != OP_CONVT_ADD) continue;  // DLA34 bandwidth ops: no GEMM
    ConvParams& p = ws->params[i];
    const Packed& pk = packed[i];
    std::memset(&p, 0, sizeof(p));
    p.weight = pk.w;
    p.bias = pk.bias;
    p.Kpad = pk.Kpad;
    p.act = op.act;
    int kbase = 0;
    if (op.kind == OP_CONV) {
      p.nseg = (int)op.segs.size();
      for (size_t s = 0; s < op.segs.size(); ++s) {
        const SegSpec& sg = op.segs[s];
        const TensorSpec& t = plan.tensors[sg.src];
        p.seg[s] = ConvSegment{base + ws->off[sg.src], t.H, t.W, t.C, t.C, sg.kh, sg.kw, sg.stride, sg.pad,
                               sg.pad_w >= 0 ? sg.pad_w : sg.pad, pk.seg_ksteps[s], kbase};
        kbase += pk.seg_ksteps[s];
      }
      const int Ho = op.up_s ? op.gh : op.out >= 0 ? plan.tensors[op.out].H : plan.out_h;
      const int Wo = op.up_s ? op.gw : op.out >= 0 ? plan.tensors[op.out].W : plan.out_w;
      p.Ho = Ho;
      p.Wo = Wo;
      p.M = B * Ho * Wo;
      p.N = op.N;
      p.out = op.out >= 0 ? (void*)(base + ws->off[op.out]) : nullptr;  // patched per call
      p.out_ldc = op.out >= 0 ? plan.tensors[op.out].C : plan.out_cpad;
      p.out_coff = 0;
      p.mtiles = (p.M + kTile - 1) / kTile;
      p.ntiles = pk.Npad / kTile;
      if (op.up_s) {  // phase scatter into the high-resolution output (protonet ConvT phases)
        const TensorSpec& tgt = plan.tensors[op.out];
        p.up_s = op.up_s;
        p.up_cout = op.N;
        p.tH = tgt.H;
        p.tW = tgt.W;
        p.sy = op.sy;
        p.sx = op.sx;
        p.add = op.add >= 0 ? base + ws->off[op.add] : nullptr;
        p.add_ldc = op.add >= 0 ? plan.tensors[op.add].C : 0;
      }
    } else {
      const TensorSpec& src = plan.tensors[op.src];
      const TensorSpec& tgt = plan.tensors[op.out];
      p.nseg = 1;
      p.seg[0] = ConvSegment{base + ws->off[op.src], src.H, src.W, src.C, src.C, 1, 1, 1, 0, 0, pk.seg_ksteps[0], 0};
      p.Ho = src.H;
      p.Wo = src.W;
      p.M = B * src.H * src.W;
      p.N = op.up_s * op.up_s * op.N;
      p.out = base + ws->off[op.out];
      p.out_ldc = tgt.C;
      p.mtiles = (p.M + kTile - 1) / kTile;
      p.ntiles = (p.N + kTile - 1) / kTile;
      p.up_s = op.up_s;
      p.up_cout = op.N;
      p.tH = tgt.H;
      p.tW = tgt.W;
      p.sy = op.sy;
      p.sx = op.sx;
      p.add = base + ws->off[op.add];
      p.add_ldc = plan.tensors[op.add].C;
    }
  }
  // k-step descriptors for the pipelined kernel and the per-op kernel choice
  const int BK = 128 / esz;
  std::vector<KStep> all_ks;
  std::vector<size_t> ks_off(plan.ops.size(), 0);
  std::vector<std::vector<KStep>> op_ks(plan.ops.size());  // per op: its k-steps when all are mode 0
  ws->use_pipe.assign(plan.ops.size(), 0);
  ws->kname.assign(plan.ops.size(), std::string());
  ws->c3_tw.assign(plan.ops.size(), 0);
  ws->c3_grid.assign(plan.ops.size(), 0);
  ws->s2_grid.assign(plan.ops.size(), 0);
  ws->c3_res.assign(plan.ops.size(), 0);
  ws->c3_ni.assign(plan.ops.size(), 4);
  ws->c3_nw.assign(plan.ops.size(), 8);
  for (size_t i = 0; i < plan.ops.size(); ++i) {
    const OpSpec& op = plan.ops[i];
    if (op.kind != OP_CONV && op.kind != OP_CONVT_ADD) continue;
    ConvParams& p = ws->params[i];
    std::vector<KStep> ks;
    bool ok = true;
    for (int s = 0; s < p.nseg && ok; ++s) {
      const ConvSegment& sg = p.seg[s];
      for (int kk = 0; kk < sg.ksteps; ++kk) {
        KStep d{};
        d.src = sg.src;
        d.seg = s;
        d.H = sg.H; d.W = sg.W; d.ldc = sg.ldc; d.stride = sg.stride;
        d.pad_h = sg.pad; d.pad_w = sg.pad_w; d.kh = sg.kh; d.kw = sg.kw;
        d.kw_inv = 1.0f / (float)sg.kw;
        const int kel = kk * BK;
        const int vec = 16 / esz;
        if (sg.C % BK == 0 && sg.kh * sg.kw <= 32) {
          const int tap = kel / sg.C;
          d.mode = 0; d.tap = tap;
          d.off = ((long long)(tap / sg.kw) * sg.W + tap % sg.kw) * sg.ldc + kel % sg.C;
        } else if (sg.C < BK && sg.C % vec == 0 && (sg.kh * sg.kw + 8) * (sg.C / vec) < (1 << 16)) {
          d.mode = 1; d.q0 = kel / vec; d.cpt = sg.C / vec;
          d.cpt_inv = 1.0f / (float)d.cpt;
        } else {
          ok = false;
          break;
        }
        ks.push_back(d);
      }
    }
    if (ok && std::all_of(ks.begin(), ks.end(), [](const KStep& d) { return d.mode == 0; })) op_ks[i] = ks;
    const int mt = (p.M + kPipeTileM - 1) / kPipeTileM;
    const bool big = (long)mt * p.ntiles >= 256;
    ws->use_pipe[i] = ok && (pipe_mode == 1 || (pipe_mode < 0 && big));
    if (ws->use_pipe[i]) {
      ks_off[i] = all_ks.size();
      all_ks.insert(all_ks.end(), ks.begin(), ks.end());
      p.nks = (int)ks.size();
      p.mtiles = mt;
    }
    p.zero = zero_page;
    // persistent halo-tile 3x3 kernel (conv3x3.hip): 3x3 / stride 1 / pad 1, one input of 128
    // channels, fp16/bf16, 16-byte aligned channel slices, byte offsets within 2^31
    // A second segment is accepted when it is ResidualBlock's 1x1 conv_residual (128 channels,
    // stride 1 or 2, ReLU after the sum): one extra k-step per channel block (RES).
    // (or DLA-34 BasicBlock's identity residual: 64 / 128 / 256 channels, an identity 1x1)
    // (a residual narrower than the 3x3 input — DLA-34 Tree's `project` of the pooled bottom, C/2
    // channels — reads zeros with zero weights in its missing channel blocks)
    const bool res2 = op.segs.size() == 2 && op.segs[1].kh == 1 && op.segs[1].kw == 1 && op.segs[1].pad == 0 &&
                      p.seg[1].C <= p.seg[0].C && p.seg[1].C % 32 == 0 && p.seg[1].ldc % 8 == 0 && op.act == 1 &&
                      (size_t)p.seg[1].H * p.seg[1].W * p.seg[1].ldc * esz < (1ull << 31) &&
                      p.seg[1].H >= (p.Ho - 1) * p.seg[1].stride + 1 && p.seg[1].W >= (p.Wo - 1) * p.seg[1].stride + 1;
    if (conv3_mode && dtype != F32 && op.kind == OP_CONV && (op.segs.size() == 1 || res2) && op.out >= 0 &&
        op.add < 0 && (int)i != ss2_op) {
      const SegSpec& sg = op.segs[0];
      const ConvSegment& cs = p.seg[0];
      const int pw = sg.pad_w >= 0 ? sg.pad_w : sg.pad;
      const size_t src_bytes = (size_t)B * cs.H * cs.W * cs.ldc * esz;
      if (sg.kh == 3 && sg.kw == 3 && sg.stride == 1 && sg.pad == 1 && pw == 1 && !sg.row_expand &&
          (cs.C == 128 || cs.C == 256 || cs.C == 64) &&
          cs.ldc % 8 == 0 && p.out_ldc % 8 == 0 && p.out_coff % 8 == 0 && src_bytes < (1ull << 31) &&
          p.ntiles * 128 <= kConv3MaxN && p.act >= 0 && p.act <= 2 && cs.H * cs.W >= conv3_min_pix &&
          (size_t)cs.H * cs.W * p.out_ldc * esz < (1ull << 31)) {
        const int res = res2 ? 1 : 0;
        const bool heads = op.act >= 1 && !res && op.out >= 0 && i + 1 < plan.ops.size() &&
                           !plan.ops[i + 1].diag_in_off.empty();
        int nw = 8, tw = 0, mt = 0, ni = 4;
        long t4 = 0;
        auto geometry = [&](int nwv) {  // tile width, tiles and channel-tile choice for a workgroup size
          const int slots = nwv == 4 ? 2 * cu_count : cu_count;  // resident workgroups
          const int t16 = conv3x3_tiles(B, cs.H, cs.W, 16, nwv), t32 = conv3x3_tiles(B, cs.H, cs.W, 32, nwv);
          tw = c3_tw_force ? c3_tw_force : t32 <= t16 ? 32 : 16;
          mt = tw == 32 ? t32 : t16;
          // 64-channel half tiles when the last round of 128-channel tiles would leave most CUs
          // idle: a half tile costs ~c3_half_cost of a full one (two work units per tile)
          t4 = (long)mt * p.ntiles;
          const long r4 = (t4 + slots - 1) / slots, r2 = (2 * t4 + slots - 1) / slots;
          ni = c3_ni_force ? c3_ni_force : (c3_half_cost > 0 && c3_half_cost * r2 < 100 * r4) ? 2 : 4;
          if (p.N <= 64) ni = 2;  // one 64-channel half tile holds every output channel
          if (heads) ni = 4;      // the stacked heads (fused 1x1 epilogue) keep 128-channel tiles
        };
        geometry(8);
        // two 4-wave workgroups per CU (256-pixel tiles) for the plain 128-channel-input convs that
        // run 64-channel half tiles. Measured (profiles/r3c): the R18 60x80 layers 1.000 -> 0.916 ms
        // per slice; on the dominant 120x160 layer (128-channel tiles) 1.432 -> 1.506 ms, so those
        // keep one 8-wave workgroup per CU
        if (ni == 2 && c3_nw_mode != 8 && !res && !heads && cs.C == 128 && p.ntiles <= 2) {
          nw = 4;
          geometry(4);
          ni = 2;
        }
        const int slots = nw == 4 ? 2 * cu_count : cu_count;
        const long total = (ni == 2 && p.N <= 64) ? t4 : t4 * (4 / ni);
        int grid = (int)std::min<long>(total, slots);
        // XCD-aware contiguous ranges need a multiple of 8 workgroups; rounding down is only
        // worth it when every workgroup still gets several units (measured at B=1: 20 units on
        // 16 workgroups ran two rounds, 29 us instead of 18)
        if (grid >= 8 && total > 2L * slots) grid -= grid % 8;
        Packed& pk3 = packed[i];
        void*& wc = ni == 4 ? pk3.w_c3 : pk3.w_c3h;
        if (!wc) {
          TV_HIP(hipMalloc(&wc, conv3x3_weight_bytes(p.ntiles, res, cs.C / 32)));
          int rc = conv3x3_repack(pk3.w, pk3.Kpad, esz, p.ntiles, res, ni, cs.C / 32, conv3x3_k16(0, res, ni, nw), wc, nullptr);
          if (rc) return rc;
          TV_HIP(hipDeviceSynchronize());
        }
        p.weight = wc;
        ws->c3_tw[i] = tw;
        ws->c3_ni[i] = ni;
        ws->c3_nw[i] = nw;
        ws->c3_res[i] = res;
        ws->c3_grid[i] = grid;
        ws->use_pipe[i] = 0;
        p.mtiles = mt;
      }
    }
    // persistent stride-2 3x3 kernel (conv3x3s2.hip): 128 -> 128 channels, fp16/bf16, at least
    // one 512-pixel tile per CU (smaller layers stay on the pipelined implicit GEMM)
    if (s2_mode && dtype != F32 && op.kind == OP_CONV && op.segs.size() == 1 && op.out >= 0 && op.add < 0 &&
        (int)i != ss2_op) {
      const SegSpec& sg = op.segs[0];
      const ConvSegment& cs = p.seg[0];
      const int pw = sg.pad_w >= 0 ? sg.pad_w : sg.pad;
      const size_t frame_bytes = (size_t)cs.H * cs.W * cs.ldc * esz;
      const int mt = conv3x3s2_tiles(B, p.Ho, p.Wo);
      if (sg.kh == 3 && sg.kw == 3 && sg.stride == 2 && sg.pad == 1 && pw == 1 && !sg.row_expand && cs.C == 128 &&
          p.N == 128 && p.ntiles == 1 && cs.ldc % 8 == 0 && p.out_ldc % 8 == 0 && frame_bytes < (1ull << 31) &&
          mt >= (s2_min_tiles >= 0 ? s2_min_tiles : cu_count)) {
        Packed& pk3 = packed[i];
        if (!pk3.w_c3) {
          TV_HIP(hipMalloc(&pk3.w_c3, conv3x3s2_weight_bytes()));
          int rc = conv3x3s2_repack(pk3.w, pk3.Kpad, esz, pk3.w_c3, nullptr);
          if (rc) return rc;
          TV_HIP(hipDeviceSynchronize());
        }
        int grid = std::min(mt, cu_count);
        if (grid >= 8 && mt > 2 * cu_count) grid -= grid % 8;
        p.weight = pk3.w_c3;
        p.mtiles = mt;
        ws->s2_grid[i] = grid;
        ws->use_pipe[i] = 0;
      }
    }
  }
  // narrow-channel 3x3 convs (16 / 32 input channels) on conv_small.hip
  ws->small.assign(plan.ops.size(), 0);
  for (size_t i = 0; i < plan.ops.size(); ++i) {
    const OpSpec& op = plan.ops[i];
    if (dtype == F32 || op.kind != OP_CONV || op.segs.size() != 1 || op.out < 0 || op.add >= 0 || op.up_s ||
        ws->c3_tw[i] || ws->s2_grid[i] || (int)i == ss2_op)
      continue;
    const SegSpec& sg = op.segs[0];
    const ConvParams& p = ws->params[i];
    if (sg.kh == 3 && sg.kw == 3 && sg.pad == 1 && (sg.pad_w < 0 || sg.pad_w == 1) && !sg.row_expand &&
        conv_small_supported(p.seg[0].C, op.N, sg.stride, p.seg[0].ldc, p.out_ldc) && p.N == op.N) {
      ws->small[i] = 1;
      ws->use_pipe[i] = 0;
    }
  }
  // DCNv2 sampling + its column GEMM -> one fused kernel (dcn.hip)
  ws->dcn_skip.assign(plan.ops.size(), 0);
  ws->dcn.assign(plan.ops.size(), DcnParams{});
  for (size_t i = 0; i + 1 < plan.ops.size(); ++i) {
    if (!dcn_fusable(i)) continue;
    const OpSpec& d = plan.ops[i];
    const OpSpec& g = plan.ops[i + 1];
    const TensorSpec& xt = plan.tensors[d.src];
    const TensorSpec& omt = plan.tensors[d.add];
    const TensorSpec& ot = plan.tensors[g.out];
    DcnParams& q = ws->dcn[i + 1];
    q.x = base + ws->off[d.src];
    q.B = B;
    q.H = xt.H;
    q.W = xt.W;
    q.C = xt.C;
    q.ldx = xt.C;
    q.om = base + ws->off[d.add];
    q.om_ldc = omt.C;
    q.w = packed[i + 1].w;
    q.Kpad = packed[i + 1].Kpad;
    q.bias = packed[i + 1].bias;
    q.act = g.act;
    q.out = base + ws->off[g.out];
    q.out_ldc = ot.C;
    q.N = g.N;
    ws->dcn_skip[i] = 1;
    ws->use_pipe[i + 1] = 0;
  }
  // dcn_gemm64 split-K: a layer whose (pixel, channel) tiles fill at most half the CUs (DLA-34 at
  // B=1: a 30x40 256-channel layer is 38 tiles of 36 k-steps, each k-step a chain of corner gathers)
  // runs ksplit workgroups per tile over tap ranges; their fp32 partials meet in dslab
  if (dcn_split_max >= 2 && (dcn64_mode == 1 || dcn64_mode == 2)) {
    long slab_floats = 0, tickets = 0;
    for (size_t i = 0; i < plan.ops.size(); ++i) {
      DcnParams& q = ws->dcn[i];
      if (!q.x || q.C % 64) continue;
      int bn, px;
      dcn64_tile(q, dcn64_mode, &bn, &px);
      const long units = ((long)q.B * q.H * q.W + px - 1) / px * (q.N / bn);
      const int ks = (int)std::min<long>(dcn_split_max, cu_count / std::max(1L, units));
      if (ks < 2) continue;
      q.ksplit = ks;
      slab_floats = std::max(slab_floats, dcn_split_floats(q, dcn64_mode, ks));
      tickets = std::max(tickets, units);
    }
    if (tickets) {
      TV_HIP(hipMalloc((void**)&ws->dslab, (size_t)slab_floats * sizeof(float)));
      TV_HIP(hipMalloc((void**)&ws->dcnt, (size_t)tickets * sizeof(unsigned)));
      TV_HIP(hipMemset(ws->dcnt, 0, (size_t)tickets * sizeof(unsigned)));
      for (size_t i = 0; i < plan.ops.size(); ++i)
        if (ws->dcn[i].ksplit > 1) {
          ws->dcn[i].slab = ws->dslab;
          ws->dcn[i].cnt = ws->dcnt;
        }
    }
  }
  // stacked 3x3 heads on conv3x3 + block-diagonal 1x1 heads -> one launch (EPI 1)
  ws->head_fused.assign(plan.ops.size(), 0);
  ws->head_skip.assign(plan.ops.size(), 0);
  for (size_t i = 0; headfuse_mode && i + 1 < plan.ops.size(); ++i) {
    const OpSpec& h2 = plan.ops[i + 1];
    const Packed& pk2 = packed[i + 1];
    if (!ws->c3_tw[i] || ws->c3_ni[i] != 4 || ws->c3_nw[i] != 8 || h2.diag_in_off.empty() || !pk2.head_ok || h2.out >= 0 || h2.segs[0].src != plan.ops[i].out ||
        (plan.ops[i].act != 2 && !(plan.ops[i].act == 1 && plan.tensors[plan.ops[i].segs[0].src].C == 64)) ||
        ws->params[i].ntiles != plan.ops[i].N / 128)
      continue;
    ConvParams& p = ws->params[i];
    if (conv3x3_k16(1, 0, 4, 8) != conv3x3_k16(0, 0, 4, 8)) {  // the fused-heads body reads the other swizzle
      Packed& pk3 = packed[i];
      if (!pk3.w_c3e) {
        const int ncb = plan.tensors[plan.ops[i].segs[0].src].C / 32;
        TV_HIP(hipMalloc(&pk3.w_c3e, conv3x3_weight_bytes(p.ntiles, 0, ncb)));
        int rc = conv3x3_repack(pk3.w, pk3.Kpad, dtype_size(dtype), p.ntiles, 0, 4, ncb, conv3x3_k16(1, 0, 4, 8), pk3.w_c3e, nullptr);
        if (rc) return rc;
        TV_HIP(hipDeviceSynchronize());
      }
      p.weight = pk3.w_c3e;
    }
    p.head_w = pk2.head_w;
    p.head_b = pk2.head_b;
    p.head_ldc = plan.out_cpad;
    for (int t = 0; t < 16; ++t) {
      p.head_row0[t] = pk2.head_row0[t];
      p.head_nrows[t] = pk2.head_nrows[t];
    }
    // plain stores when the tiles' head rows tile the output columns exactly once (one 128-channel
    // hidden tile per head: a 64-channel backbone's 2C heads); otherwise (a head's 2C = 256 hidden
    // channels, centernet.py:45-50 on the 128-channel "R18" and DLA-34, span two tiles that meet in
    // the output) atomics onto a zeroed output
    {
      std::vector<int> cover(plan.out_cpad, 0);
      bool ok = true;
      for (int t = 0; t < p.ntiles && t < 16; ++t)
        for (int r = 0; r < p.head_nrows[t]; ++r) {
          const int c = p.head_row0[t] + r;
          if (c < 0 || c >= plan.out_cpad) ok = false;
          else ++cover[c];
        }
      for (int c : cover) ok = ok && c == 1;
      p.head_store = ok ? 1 : 0;
    }
    ws->head_fused[i] = 1;
    ws->head_skip[i + 1] = 1;
  }
  // ConvTranspose + pad_to_match + add on convt.hip (fp16/bf16, 128 -> 128 channels)
  ws->convt.assign(plan.ops.size(), 0);
  ws->tparams.assign(plan.ops.size(), ConvTParams{});
  for (size_t i = 0; i < plan.ops.size(); ++i) {
    const OpSpec& op = plan.ops[i];
    if (!convt_mode || dtype == F32 || op.kind != OP_CONVT_ADD) continue;
    const TensorSpec& src = plan.tensors[op.src];
    const TensorSpec& tgt = plan.tensors[op.out];
    const TensorSpec& add = plan.tensors[op.add];
    if (!convt_supported(src.C, op.N, src.C, add.C, tgt.C)) continue;
    ConvTParams& t = ws->tparams[i];
    t.src = base + ws->off[op.src];
    t.h = src.H;
    t.w = src.W;
    t.src_ldc = src.C;
    t.weight = packed[i].w;
    t.Kpad = packed[i].Kpad;
    t.bias = packed[i].bias;
    t.add = base + ws->off[op.add];
    t.add_ldc = add.C;
    t.out = base + ws->off[op.out];
    t.out_ldc = tgt.C;
    t.B = B;
    t.s = op.up_s;
    t.tH = tgt.H;
    t.tW = tgt.W;
    t.sy = op.sy;
    t.sx = op.sx;
    convt_schedule(t, cu_count);
    ws->convt[i] = 1;
    ws->use_pipe[i] = 0;
  }
  // ConvTranspose2d(3, s2, p1, op1) as its four consecutive phase ops (protonet): one convt3.hip
  // launch from the phase-(0,0) op over the shared input halo; the other three launch nothing
  ws->ct3.assign(plan.ops.size(), 0);
  ws->ct3p.assign(plan.ops.size(), ConvT3Params{});
  for (size_t i = 0; i + 3 < plan.ops.size(); ++i) {
    const OpSpec& op = plan.ops[i];
    if (!packed[i].w_ct3 || op.kind != OP_CONV || op.segs.size() != 1 || op.segs[0].convt_phase != 0 ||
        op.up_s != 2 || op.out < 0 || op.add >= 0)
      continue;
    bool ok = true;
    for (int ph = 1; ph < 4; ++ph) {
      const OpSpec& o = plan.ops[i + ph];
      ok = ok && o.kind == OP_CONV && o.segs.size() == 1 && o.segs[0].convt_phase == ph &&
           o.segs[0].src == op.segs[0].src && o.out == op.out && o.up_s == 2 && o.act == op.act && o.add < 0;
    }
    const TensorSpec& src = plan.tensors[op.segs[0].src];
    const TensorSpec& tgt = plan.tensors[op.out];
    ok = ok && tgt.H == 2 * src.H && tgt.W == 2 * src.W && op.N == tgt.C &&
         convt3_supported(src.C, op.N, src.C, tgt.C, src.H, src.W, esz);
    if (!ok) continue;
    ConvT3Params& t = ws->ct3p[i];
    t.src = base + ws->off[op.segs[0].src];
    t.B = B;
    t.H = src.H;
    t.W = src.W;
    t.C = src.C;
    t.ldc = src.C;
    t.w = packed[i].w_ct3;
    t.bias = packed[i].bias;
    t.act = op.act;
    t.out = base + ws->off[op.out];
    t.out_ldc = tgt.C;
    t.N = op.N;
    convt3_tile(t.H, t.W, &t.tw, &t.tr);
    ws->ct3[i] = 1;
    for (int ph = 0; ph < 4; ++ph) ws->use_pipe[i + ph] = 0;
    for (int ph = 1; ph < 4; ++ph) ws->ct3[i + ph] = 2;
  }
  // layers the chosen kernel spreads over fewer work units than the threshold (the deep pyramid
  // levels: a few 512-pixel tiles on 256 CUs) -> conv_lat.hip (small tiles, K split over waves)
  ws->lat.assign(plan.ops.size(), 0);
  const int lat_min = lat_units >= 0 ? lat_units : cu_count;
  for (size_t i = 0; lat_mode && (dtype != F32 || lat_f32) && i < plan.ops.size(); ++i) {
    const OpSpec& op = plan.ops[i];
    ConvParams& p = ws->params[i];
    if (op.kind != OP_CONV || op.up_s || op.out < 0 || op.add >= 0 || (int)i == stem_op || (int)i == ss2_op ||
        op_ks[i].empty() ||
        ws->small[i] || ws->dcn[i].x || ws->dcn_skip[i] || ws->head_fused[i] || ws->head_skip[i] || p.N % 8 ||
        p.out_ldc % 8 || p.out_coff % 8)
      continue;
    long units;
    if (ws->c3_tw[i]) units = (long)p.mtiles * p.ntiles * (ws->c3_ni[i] == 2 && p.N > 64 ? 2 : 1) / (ws->c3_nw[i] == 4 ? 2 : 1);
    else if (ws->s2_grid[i]) units = p.mtiles;
    else if (ws->use_pipe[i]) units = (long)p.mtiles * p.ntiles;
    else units = 0;  // conv_igemm corner case: always worse than conv_lat
    if (units >= lat_min) continue;
    const int nks = (int)op_ks[i].size();
    if (nks < 2) continue;
    // only when its 64 x 128 tiles fit one round of workgroups (one per CU): measured on MI355X, a
    // second round costs more than the halo kernels' under-filled grid (30x40 level at B=32:
    // 44-50 us vs 24 us), one round wins or ties (15x20 and below, Roots, DLA-34's 27-channel
    // offset / mask conv at 15x20: 43 vs 98 us)
    int lmt = 0, lnt = 0;
    if (lat_units < 0 && conv_lat_tiles(p.M, p.N, &lmt, &lnt) > cu_count) continue;
    p.weight = packed[i].w;  // [Npad][Kpad] (the halo kernels may have swapped in their own copy)
    conv_lat_tiles(p.M, p.N, &p.mtiles, &p.ntiles);
    p.nks = nks;
    if (!ws->use_pipe[i]) {
      ks_off[i] = all_ks.size();
      all_ks.insert(all_ks.end(), op_ks[i].begin(), op_ks[i].end());
    }
    ws->use_pipe[i] = 0;
    ws->c3_tw[i] = 0;
    ws->s2_grid[i] = 0;
    ws->lat[i] = 1;
  }
  // the conv_lat layers conv_burst.hip represents (every segment a 3x3 / stride 1 window or a 1x1
  // over 128-channel multiples, K <= 1280, the staged window within LDS) take the one-shot kernel:
  // no k-step chain, no split-K hand-off (knob TV_BURST=0 keeps them on conv_lat)
  ws->burst.assign(plan.ops.size(), 0);
  ws->bparams.assign(plan.ops.size(), BurstParams{});
  for (size_t i = 0; burst_mode && dtype != F32 && i < plan.ops.size(); ++i) {  // (fp16 / bf16 kernel)
    if (!ws->lat[i]) continue;
    BurstParams bp{};
    if (!conv_burst_plan(ws->params[i], B, &bp)) continue;
    // only where every tile is resident at once with a small window: measured (profiles/r5): a
    // second round of tiles, or one workgroup per CU for an 89 KiB 80-column window, loses to
    // conv_lat's split-K (60x80 at B=1: 25.6 vs 16.5 us per launch; 15x20 at B=32: 16.7 vs 17 us)
    const int per_cu = std::min(3, (160 * 1024) / std::max(1, bp.lds));
    if (burst_mode == 1 && (bp.lds > 64 * 1024 || conv_burst_workgroups(bp) > per_cu * cu_count)) continue;
    Packed& pk = packed[i];
    if (!pk.w_burst) {
      TV_HIP(hipMalloc(&pk.w_burst, conv_burst_weight_bytes(bp)));
      int rc = conv_burst_repack(pk.w, pk.Kpad, esz, bp, pk.w_burst, nullptr);
      if (rc) return rc;
      TV_HIP(hipDeviceSynchronize());
    }
    bp.w = pk.w_burst;
    ws->bparams[i] = bp;
    ws->burst[i] = 1;
    ws->lat[i] = 0;
  }
  // stride-1 1x1 convs over concatenated inputs (the Roots) that the pipelined GEMM would run: the
  // streaming kernel (conv1x1.hip) with the weights resident in LDS, 128 output channels per
  // workgroup (knob TV_C1X1=0: off, 2: only layers of at most 128 output channels)
  ws->c1x1.assign(plan.ops.size(), 0);
  for (size_t i = 0; i < plan.ops.size(); ++i) {
    const OpSpec& op = plan.ops[i];
    if (!c1x1_mode || dtype == F32 || op.kind != OP_CONV || op.up_s || op.add >= 0 || op.out < 0 || ws->lat[i] ||
        ws->burst[i] ||
        ws->small[i] || ws->c3_tw[i] || ws->s2_grid[i] || ws->head_fused[i] || ws->head_skip[i] || ws->dcn[i].x ||
        ws->dcn_skip[i] || (int)i == stem_op || (int)i == ss2_op || ws->convt[i])
      continue;
    bool one = !op.segs.empty();
    for (const SegSpec& sg : op.segs)
      one = one && sg.kh == 1 && sg.kw == 1 && sg.stride == 1 && sg.pad == 0 && !sg.row_expand && sg.convt_phase < 0;
    if (!one || !conv1x1_stream_supported(ws->params[i], esz) || (c1x1_mode == 2 && ws->params[i].N > 128)) continue;
    ws->c1x1[i] = 1;
    ws->use_pipe[i] = 0;
  }
  // conv_lat split-K over workgroups for the layers whose tiles leave most CUs idle (the latency
  // path: at B=1 every conv_lat layer is one k-step chain of ~9 latency-bound k-steps per K group):
  // up to lat_split_max workgroups per tile, each slice >= 2 k-steps (one per K group), the tiles x
  // slices within one round of CUs. Partial tiles meet in `slab`, tickets in `cnt` (conv_lat.hip).
  // The schedule: in execution order, consecutive conv_lat layers of one level share a launch
  // (up to kLatGroupMax, their workgroups within one round of CUs); slot k of a group has its own
  // split-K slab and tickets.
  std::vector<int> slot(nops, 0);
  {
    size_t slab_floats = 0, tickets = 0;
    for (size_t i = 0; i < nops; ++i) {
      if (!ws->lat[i]) continue;
      ConvParams& p = ws->params[i];
      const int tiles = p.mtiles * p.ntiles;
      // only layers with a long k-step chain: measured at B=1 (profiles/r5/b1_knobs.txt), the hand-off
      // (write-through partial tiles, ticket, sc1 loads) costs more than it saves on the 18-20 k-step
      // 128-channel layers (R18 1.295 -> 1.269 ms without it) and far less on DLA-34's 36-72 k-step
      // 256 / 512-channel ones (1.284 -> 1.398 ms without it)
      // (fp32: a k-step is a quarter of the fp16 one's MFMA rate at half its depth, so the chains are
      // twice as long and 2x slower per step: up to lat_split_max_f32 slices)
      const int smax = dtype == F32 ? lat_split_max_f32 : lat_split_max;
      int ks = p.nks >= lat_split_min_nks ? std::min(smax, p.nks / 2) : 1;
      ks = std::min(ks, cu_count / std::max(1, tiles));
      p.ksplit = ks > 1 ? ks : 0;
      if (!p.ksplit) continue;
      slab_floats = std::max(slab_floats, (size_t)tiles * ks * kLatSlabFloats);
      tickets = std::max(tickets, (size_t)tiles);
    }
    auto wgs = [&](int i) { const ConvParams& p = ws->params[i]; return p.mtiles * p.ntiles * std::max(1, p.ksplit); };
    // a ConvT + add on convt.hip that covers its whole target (no uncovered-margin copy after it)
    auto convt_groupable = [&](int i) {
      const OpSpec& op = plan.ops[i];
      if (!ws->convt[i] || op.out < 0) return false;
      const TensorSpec& tg = plan.tensors[op.out];
      return op.cov_y0 <= 0 && op.cov_x0 <= 0 && op.cov_y1 >= tg.H && op.cov_x1 >= tg.W;
    };
    ws->groups.clear();
    for (size_t k = 0; k < nops;) {
      const int i = ws->order[k++];
      std::vector<int> g{i};
      if (grouping && ws->burst[i]) {  // one-shot layers of one level: no CU budget (no tickets)
        while (k < nops && (int)g.size() < kBurstGroupMax) {
          const int j = ws->order[k];
          if (!ws->burst[j] || ws->level[j] != ws->level[i]) break;
          g.push_back(j);
          ++k;
        }
      } else if (grouping && ws->lat[i]) {
        int used = wgs(i);
        while (k < nops && (int)g.size() < kLatGroupMax) {
          const int j = ws->order[k];
          if (!ws->lat[j] || ws->level[j] != ws->level[i] || used + wgs(j) > cu_count) break;
          slot[j] = (int)g.size();
          used += wgs(j);
          g.push_back(j);
          ++k;
        }
      } else if (grouping && convt_groupable(i)) {  // up-steps of one level with the same phase grouping
        int used = convt_workgroups(ws->tparams[i]);
        while (k < nops && (int)g.size() < kConvTGroupMax) {
          const int j = ws->order[k];
          if (!convt_groupable(j) || ws->level[j] != ws->level[i] || ws->tparams[j].np != ws->tparams[i].np ||
              used + convt_workgroups(ws->tparams[j]) > cu_count)
            break;
          used += convt_workgroups(ws->tparams[j]);
          g.push_back(j);
          ++k;
        }
      }
      ws->groups.push_back(std::move(g));
    }
    if (tickets) {
      const int nslot = grouping ? kLatGroupMax : 1;
      ws->cnt_bytes = align_up(nslot * tickets * sizeof(unsigned), 16);
      TV_HIP(hipMalloc((void**)&ws->slab, nslot * slab_floats * sizeof(float)));
      TV_HIP(hipMalloc((void**)&ws->cnt, ws->cnt_bytes));
      TV_HIP(hipMemset(ws->cnt, 0, ws->cnt_bytes));
      for (size_t i = 0; i < nops; ++i)
        if (ws->lat[i] && ws->params[i].ksplit) {
          ws->params[i].slab = ws->slab + (size_t)slot[i] * slab_floats;
          ws->params[i].cnt = ws->cnt + (size_t)slot[i] * tickets;
        }
    }
  }
  if (stamp_op >= 0 && stamp_op < (int)plan.ops.size() && ws->c3_tw[stamp_op]) ws->params[stamp_op].dbg = stamp_buf;
  if (ss2_op >= 0) {  // block0.conv1 fused with the stem: its weights in stem_s2.hip's k-step order
    ws->use_pipe[ss2_op] = 0;
    Packed& pk = packed[ss2_op];
    if (!pk.w_ss2) {
      TV_HIP(hipMalloc(&pk.w_ss2, stem_s2_weight_bytes()));
      int rc = stem_s2_repack(pk.w, pk.Kpad, esz, pk.w_ss2, nullptr);
      if (rc) return rc;
      TV_HIP(hipDeviceSynchronize());
    }
  }
  // conv_pipe split-K for layers whose 256 x 128 tiles fill the CUs badly: the fp32 path's
  // deep levels at small batches (R18 at B=1: a 15x20 level is 2 tiles of 36 k-steps on 2 of 256
  // CUs) and its 300-tile 240x320 layers (two rounds, the second 17% full). ksplit workgroups per
  // tile, partial tiles meet in pslab, tickets in pcnt (knob TV_PIPE_SPLIT: 0 off, 1 fp32 only,
  // 2 every dtype; TV_PIPE_SPLIT_MAX slices per tile; TV_PIPE_SPLIT_RED hand-off cost)
  {
    size_t slab_floats = 0, tickets = 0;
    for (size_t i = 0; i < nops; ++i) {
      ConvParams& p = ws->params[i];
      if (!ws->use_pipe[i]) continue;  // (both epilogues: the ConvT phase scatter + add runs after the sum)
      if (!(pipe_split_mode == 2 || (pipe_split_mode == 1 && dtype == F32))) continue;
      // slices per tile by a cost model in tenths of a k-step: rounds of workgroups x k-steps per
      // slice, plus the hand-off (each slice's partial tile written, then read by the reducer:
      // pipe_split_red per slice); split only when it saves >= 10%
      const long tiles = (long)p.mtiles * p.ntiles;
      auto cost = [&](int k) {
        const long rounds = (tiles * k + cu_count - 1) / cu_count;
        return rounds * ((p.nks + k - 1) / k) * 10 + (k > 1 ? (long)pipe_split_red * (k + 1) : 0);
      };
      int ks = 1;
      for (int k = 2; k <= pipe_split_max && k <= p.nks / 2; ++k)
        if (cost(k) < cost(ks)) ks = k;
      if (cost(ks) * 10 > cost(1) * 9) ks = 1;
      p.ksplit = ks > 1 ? ks : 0;
      if (!p.ksplit) continue;
      slab_floats = std::max(slab_floats, (size_t)tiles * ks * kPipeTileM * 128);
      tickets = std::max(tickets, (size_t)tiles);
    }
    if (tickets) {
      TV_HIP(hipMalloc((void**)&ws->pslab, slab_floats * sizeof(float)));
      TV_HIP(hipMalloc((void**)&ws->pcnt, tickets * sizeof(unsigned)));
      TV_HIP(hipMemset(ws->pcnt, 0, tickets * sizeof(unsigned)));
      for (size_t i = 0; i < nops; ++i)
        if (ws->use_pipe[i] && ws->params[i].ksplit) {
          ws->params[i].slab = ws->pslab;
          ws->params[i].cnt = ws->pcnt;
        }
    }
  }
  // fp32 X3: the pipelined and conv_lat layers read the hi / lo fp16 copy of their weights
  if (dtype == F32 && f32x3) {
    for (size_t i = 0; i < nops; ++i) {
      if (!ws->use_pipe[i] && !ws->lat[i]) continue;
      Packed& pk = packed[i];
      if (!pk.w_x3) {
        TV_HIP(hipMalloc(&pk.w_x3, (size_t)pk.Npad * pk.Kpad * 4));
        int rc = conv_pipe_x3_repack(pk.w, pk.Npad, pk.Kpad, pk.w_x3, nullptr);
        if (rc) return rc;
        TV_HIP(hipDeviceSynchronize());
      }
      ws->params[i].weight = pk.w_x3;
    }
  }
  if (!all_ks.empty()) {
    TV_HIP(hipMalloc((void**)&ws->dks, all_ks.size() * sizeof(KStep)));
    TV_HIP(hipMemcpy(ws->dks, all_ks.data(), all_ks.size() * sizeof(KStep), hipMemcpyHostToDevice));
    for (size_t i = 0; i < plan.ops.size(); ++i)
      if (ws->use_pipe[i] || ws->lat[i]) ws->params[i].ks = ws->dks + ks_off[i];
  }
  TV_HIP(hipMalloc((void**)&ws->dparams, ws->params.size() * sizeof(ConvParams)));
  TV_HIP(hipMemcpy(ws->dparams, ws->params.data(), ws->params.size() * sizeof(ConvParams), hipMemcpyHostToDevice));
  return TV_OK;
}

int Engine::get_workspace(int B, hipStream_t stream, Workspace** out) {
  std::lock_guard<std::mutex> g(mu);
  auto key = std::make_pair((void*)stream, B);
  auto it = workspaces.find(key);
  if (it != workspaces.end()) {
    *out = it->second;
    return TV_OK;
  }
  Workspace* ws = new Workspace();
  int rc = make_workspace(B, ws);
  if (rc) {
    if (ws->arena) (void)hipFree(ws->arena);
    if (ws->dparams) (void)hipFree(ws->dparams);
    if (ws->dks) (void)hipFree(ws->dks);
    if (ws->slab) (void)hipFree(ws->slab);
    for (hipEvent_t ev : ws->gev) (void)hipEventDestroy(ev);
    if (ws->pslab) (void)hipFree(ws->pslab);
    if (ws->pcnt) (void)hipFree(ws->pcnt);
    if (ws->dslab) (void)hipFree(ws->dslab);
    if (ws->dcnt) (void)hipFree(ws->dcnt);
    if (ws->cnt) (void)hipFree(ws->cnt);
    delete ws;
    return rc;
  }
  workspaces[key] = ws;
  *out = ws;
  return TV_OK;
}

int Engine::trim() {
  std::lock_guard<std::mutex> g(mu);
  TV_HIP(hipSetDevice(device));
  TV_HIP(hipDeviceSynchronize());  // no queued launch still reads an arena
  for (auto& kv : workspaces) {
    if (kv.second->arena) (void)hipFree(kv.second->arena);
    if (kv.second->dparams) (void)hipFree(kv.second->dparams);
    if (kv.second->dks) (void)hipFree(kv.second->dks);
    if (kv.second->slab) (void)hipFree(kv.second->slab);
    for (hipEvent_t ev : kv.second->gev) (void)hipEventDestroy(ev);
    if (kv.second->pslab) (void)hipFree(kv.second->pslab);
    if (kv.second->pcnt) (void)hipFree(kv.second->pcnt);
    if (kv.second->dslab) (void)hipFree(kv.second->dslab);
    if (kv.second->dcnt) (void)hipFree(kv.second->dcnt);
    if (kv.second->cnt) (void)hipFree(kv.second->cnt);
    delete kv.second;
  }
  workspaces.clear();
  return TV_OK;
}

int Engine::run_op(size_t i, Workspace* ws, const void* input, int input_u8, float* out, hipStream_t s) {
  const OpSpec& op = plan.ops[i];
  char* base = (char*)ws->arena;
  if (stem_op >= 0 && op.kind == OP_PREP) return TV_OK;  // staging runs inside the stem kernel
  if (ss2_op >= 0 && (int)i == stem_op) return TV_OK;    // the stem runs inside block0.conv1's launch
  if ((int)i == ss2_op) {
    const OpSpec& st = plan.ops[stem_op];
    const TensorSpec& t1 = plan.tensors[op.out];
    StemS2Params sp{};
    sp.input = input;
    sp.u8 = input_u8;
    sp.B = ws->B;
    sp.H = desc.in_h;
    sp.W = desc.in_w;
    sp.Ho = t1.H;
    sp.Wo = t1.W;
    sp.stem_w = packed[stem_op].w;
    sp.stem_bias = packed[stem_op].bias;
    (void)st;
    sp.w1 = packed[i].w_ss2;
    sp.bias1 = packed[i].bias;
    sp.out = base + ws->off[op.out];
    sp.out_ldc = t1.C;
    sp.res = base + ws->off[op.out2];
    sp.res_ldc = plan.tensors[op.out2].C;
    if (stamp_op == (int)i) sp.dbg = stamp_buf;
    return launch_stem_s2(sp, dtype, cu_count, s);
  }
  if ((int)i == stem_op) {
    StemParams sp{};
    sp.input = input;
    sp.u8 = input_u8;
    sp.B = ws->B;
    sp.H = desc.in_h;
    sp.W = desc.in_w;
    sp.out = base + ws->off[op.out];
    sp.out_ldc = plan.tensors[op.out].C;
    sp.N = op.N;
    sp.weight = packed[i].w;
    sp.bias = packed[i].bias;
    return launch_stem(sp, dtype, cu_count, s);
  }
  if (op.kind == OP_LAYOUT_IN) {
    if (input_u8) {
      set_error("this model takes an fp32 NCHW feature map, not u8 frames");
      return TV_EINVAL;
    }
    return launch_nchw_to_nhwc((const float*)input, ws->B, op.N, desc.in_h, desc.in_w, base + ws->off[op.out],
                               plan.tensors[op.out].C, dtype, s);
  }
  if (op.kind == OP_PREP) {
    void* dst = base + ws->off[op.out];
    return input_u8 ? launch_prep_u8((const uint8_t*)input, ws->B, desc.in_h, desc.in_w, dst, plan.in_cpad, dtype, s)
                    : launch_prep_nchw((const float*)input, ws->B, desc.in_h, desc.in_w, dst, plan.in_cpad, dtype, s);
  }
  if (ws->dcn_skip[i]) return TV_OK;  // sampled inside the next op's fused DCNv2 kernel
  if (ws->dcn[i].x) return launch_dcn_gemm(ws->dcn[i], dtype, dcn64_mode, cu_count, s);
  if (op.kind == OP_MAXPOOL || op.kind == OP_DCN || op.kind == OP_DWCONVT_ADD) {
    const TensorSpec& src = plan.tensors[op.src];
    const TensorSpec& dst = plan.tensors[op.out];
    void* o = base + ws->off[op.out];
    const void* x = base + ws->off[op.src];
    if (op.kind == OP_MAXPOOL) return launch_maxpool2(x, ws->B, src.H, src.W, src.C, o, dst.H, dst.W, dtype, s);
    const TensorSpec& ad = plan.tensors[op.add];
    const void* a = base + ws->off[op.add];
    if (op.kind == OP_DCN) return launch_dcn_sample(x, ws->B, src.H, src.W, src.C, a, ad.C, o, dtype, s);
    return launch_dwconvt_add(x, ws->B, src.H, src.W, src.C, (const float*)packed[i].w, op.up_s, a, ad.C, o, dst.H,
                              dst.W, op.sy, op.sx, dtype, s);
  }
  if (ws->head_skip[i])  // fused into the 3x3 heads launch; an activation after the summed 1x1 runs here
    return op.act == 2 ? launch_leaky_inplace(out, (size_t)ws->B * plan.out_h * plan.out_w * plan.out_cpad, s)
                       : TV_OK;
  if (ws->head_fused[i]) {
    if (!ws->params[i].head_store) {
      int rc = launch_fill_zero(out, (size_t)ws->B * plan.out_h * plan.out_w * plan.out_cpad * sizeof(float), s);
      if (rc) return rc;
    }
    return launch_conv3x3(ws->params[i], ws->dparams + i, out, dtype, ws->c3_tw[i], ws->c3_grid[i], s, 1);
  }
  if (ws->convt[i]) {
    int rc = launch_convt(ws->tparams[i], dtype, s);
    if (rc) return rc;
    const TensorSpec& tgt = plan.tensors[op.out];
    const ConvTParams& t = ws->tparams[i];
    if (op.cov_y0 > 0 || op.cov_x0 > 0 || op.cov_y1 < tgt.H || op.cov_x1 < tgt.W)
      return launch_uncovered_copy(t.add, t.add_ldc, t.out, t.out_ldc, tgt.C, ws->B, tgt.H, tgt.W, op.cov_y0,
                                   op.cov_y1, op.cov_x0, op.cov_x1, dtype, s);
    return TV_OK;
  }
  if (ws->ct3[i] == 2) return TV_OK;  // a ConvTranspose2d phase done by the phase-(0,0) op's launch
  if (ws->ct3[i]) return launch_convt3(ws->ct3p[i], dtype, cu_count, s);
  ConvParams p = ws->params[i];
  if (op.out < 0) p.out = out;
  const bool out_f32 = op.out < 0;
  const int mode = op.kind == OP_CONVT_ADD || op.up_s ? 1 : 0;
  if (ws->small[i]) return launch_conv_small(p, ws->dparams + i, dtype, cu_count, csm_variant(p.seg[0].stride), s);
  if (ws->burst[i]) {
    const BurstParams* bp = &ws->bparams[i];
    return launch_conv_burst(&bp, 1, dtype, s);
  }
  if (ws->lat[i]) return launch_conv_lat(p, ws->dparams + i, dtype, s, dtype == F32 && f32x3);
  if (ws->c1x1[i]) return launch_conv1x1_stream(p, ws->dparams + i, dtype, cu_count, s);
  int rc = ws->s2_grid[i] ? launch_conv3x3s2(p, ws->dparams + i, p.out, dtype, ws->s2_grid[i], s)
           : ws->c3_tw[i] ? launch_conv3x3(p, ws->dparams + i, p.out, dtype, ws->c3_tw[i], ws->c3_grid[i], s, 0,
                                           ws->c3_res[i], ws->c3_ni[i], ws->c3_nw[i])
           : ws->use_pipe[i] ? launch_conv_pipe(p, ws->dparams + i, p.out, dtype, out_f32, mode, s, dtype == F32 && f32x3)
                             : launch_conv(p, ws->dparams + i, p.out, dtype, out_f32, mode, s);
  if (rc) return rc;
  if (op.kind == OP_CONVT_ADD) {
    const TensorSpec& tgt = plan.tensors[op.out];
    if (op.cov_y0 > 0 || op.cov_x0 > 0 || op.cov_y1 < tgt.H || op.cov_x1 < tgt.W)
      return launch_uncovered_copy(p.add, p.add_ldc, p.out, p.out_ldc, tgt.C, ws->B, tgt.H, tgt.W, op.cov_y0,
                                   op.cov_y1, op.cov_x0, op.cov_x1, dtype, s);
  }
  return TV_OK;
}

int Engine::get_side(hipStream_t s, int n, SideStreams** out) {
  std::lock_guard<std::mutex> g(mu);
  SideStreams& ss = side[(void*)s];
  if (!ss.fork) TV_HIP(hipEventCreateWithFlags(&ss.fork, hipEventDisableTiming));
  while ((int)ss.s.size() < n) {
    hipStream_t t;
    hipEvent_t e;
    TV_HIP(hipStreamCreateWithFlags(&t, hipStreamNonBlocking));
    TV_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    ss.s.push_back(t);
    ss.join.push_back(e);
  }
  *out = &ss;
  return TV_OK;
}

std::vector<int> Engine::slice_sizes(int B) const {
  if (!slice_sizes_env.empty()) {
    int sum = 0;
    for (int v : slice_sizes_env) sum += v > 0 ? v : 1 << 30;
    if (sum == B && (int)slice_sizes_env.size() <= kMaxSlices) return slice_sizes_env;
  }
  if (slices > 1 && B >= slices * slice_min) {
    std::vector<int> sz(slices);
    for (int k = 0; k < slices; ++k) sz[k] = B / slices + (k < B % slices ? 1 : 0);
    return sz;
  }
  return {B};
}

int Engine::run_all(const void* input, int input_u8, int B, float* out, hipStream_t s, size_t op0, size_t op1) {
  Workspace* ws = nullptr;
  int rc = get_workspace(B, s, &ws);
  if (rc) return rc;
  // conv_lat split-K tickets: zeroed when the workspace is made, and every tile's last-arriving
  // slice resets its own ticket, so each complete forward leaves them all at zero for the next
  // (no per-forward reset launch on the latency path; a memset node in a captured graph also broke
  // the replays after the first on this ROCm: aux.hip fill_zero16)
  const size_t nops = plan.ops.size();
  if (op0 == 0 && op1 >= nops) {  // the whole forward: the schedule's groups
    if (insitu && ws->gev.size() != ws->groups.size() + 1) {
      for (hipEvent_t e : ws->gev) (void)hipEventDestroy(e);
      ws->gev.assign(ws->groups.size() + 1, nullptr);
      for (hipEvent_t& e : ws->gev) TV_HIP(hipEventCreate(&e));
    }
    size_t gi = 0;
    for (const std::vector<int>& g : ws->groups) {
      if (insitu) TV_HIP(hipEventRecord(ws->gev[gi], s));
      ++gi;
      if (g.size() == 1) {
        rc = run_op((size_t)g[0], ws, input, input_u8, out, s);
      } else if (ws->burst[g[0]]) {
        const BurstParams* bp[kBurstGroupMax];
        for (size_t k = 0; k < g.size(); ++k) bp[k] = &ws->bparams[g[k]];
        rc = launch_conv_burst(bp, (int)g.size(), dtype, s);
      } else if (ws->convt[g[0]]) {
        const ConvTParams* tp[kConvTGroupMax];
        for (size_t k = 0; k < g.size(); ++k) tp[k] = &ws->tparams[g[k]];
        rc = launch_convt_group(tp, (int)g.size(), dtype, s);
      } else {
        const ConvParams* hp[kLatGroupMax];
        const ConvParams* dp[kLatGroupMax];
        for (size_t k = 0; k < g.size(); ++k) {
          hp[k] = &ws->params[g[k]];
          dp[k] = ws->dparams + g[k];
        }
        rc = launch_conv_lat_group(hp, dp, (int)g.size(), dtype, s, dtype == F32 && f32x3);
      }
      if (rc) return rc;
    }
    if (insitu) TV_HIP(hipEventRecord(ws->gev[gi], s));
    return TV_OK;
  }
  for (size_t k = op0; k < nops && k < op1; ++k) {  // positions op0 .. op1 - 1 of the execution order
    rc = run_op((size_t)ws->order[k], ws, input, input_u8, out, s);
    if (rc) return rc;
  }
  return TV_OK;
}

int Engine::prepare(int B, hipStream_t s) {
  TV_HIP(hipSetDevice(device));
  const std::vector<int> sz = slice_sizes(B);
  Workspace* ws = nullptr;
  if (sz.size() > 1) {
    SideStreams* ss = nullptr;
    int rc = get_side(s, (int)sz.size() - 1, &ss);
    if (rc) return rc;
    for (size_t k = 1; k < sz.size(); ++k) {
      rc = get_workspace(sz[k], ss->s[k - 1], &ws);
      if (rc) return rc;
    }
  }
  return get_workspace(sz[0], s, &ws);
}

int Engine::forward(const void* input, int input_u8, int B, float* out, hipStream_t s) {
  if (B < 1) {
    set_error("batch must be >= 1");
    return TV_EINVAL;
  }
  if (!input || !out) {
    set_error("null input/output pointer");
    return TV_EINVAL;
  }
  TV_HIP(hipSetDevice(device));
  const std::vector<int> sz = slice_sizes(B);
  if (sz.size() > 1) {
    // frames are independent (no cross-frame state): slice 0 on `s`, the others on side
    // streams forked from and joined back into `s` (graph-capture safe: event fork / join)
    SideStreams* ss = nullptr;
    int rc = get_side(s, (int)sz.size() - 1, &ss);
    if (rc) return rc;
    const size_t in_frame = input_u8 ? (size_t)desc.in_h * desc.in_w * 3
                                     : (size_t)plan.in_channels * desc.in_h * desc.in_w * 4;
    const size_t out_frame = (size_t)plan.out_h * plan.out_w * plan.out_cpad;
    // (diagnostic TV_SLICE_LAG = L: the other slices start once slice 0 has run its first L
    // ops, so that their heavy first layers meet slice 0's latency-bound deep levels — measured
    // slower: 4647 frames/s at L = 0, 4465 / 4338 / 4311 at L = 26 / 56 / 64, profiles/r4r)
    const size_t lag = std::min((size_t)slice_lag, plan.ops.size());
    if (lag) {
      rc = run_all(input, input_u8, sz[0], out, s, 0, lag);
      if (rc) return rc;
    }
    TV_HIP(hipEventRecord(ss->fork, s));
    size_t f0 = (size_t)sz[0];
    for (size_t k = 1; k < sz.size(); ++k) {
      TV_HIP(hipStreamWaitEvent(ss->s[k - 1], ss->fork, 0));
      rc = run_all((const char*)input + f0 * in_frame, input_u8, sz[k], out + f0 * out_frame, ss->s[k - 1]);
      if (rc) return rc;
      f0 += (size_t)sz[k];
    }
    rc = run_all(input, input_u8, sz[0], out, s, lag, plan.ops.size());
    if (rc) return rc;
    for (size_t k = 1; k < sz.size(); ++k) {
      TV_HIP(hipEventRecord(ss->join[k - 1], ss->s[k - 1]));
      TV_HIP(hipStreamWaitEvent(s, ss->join[k - 1], 0));
    }
    return TV_OK;
  }
  return run_all(input, input_u8, B, out, s);
}

int Engine::forward_insitu(const void* input, int input_u8, int B, float* out, hipStream_t s, float* ms, int cap,
                           int* n_slices) {
  if (slice_lag) {
    set_error("forward_insitu: not with a slice lag");
    return TV_EINVAL;
  }
  profiled_u8 = input_u8;
  const int prev = insitu;
  insitu = 1;
  int rc = forward(input, input_u8, B, out, s);
  insitu = prev;
  if (rc) return rc;
  TV_HIP(hipStreamSynchronize(s));  // (the side slices are joined into s)
  return insitu_read(B, s, ms, cap, n_slices);
}

int Engine::insitu_read(int B, hipStream_t s, float* ms, int cap, int* n_slices) {
  int rc = 0;
  const std::vector<int> sz = slice_sizes(B);
  SideStreams* ss = nullptr;
  if (sz.size() > 1) {
    rc = get_side(s, (int)sz.size() - 1, &ss);
    if (rc) return rc;
  }
  const size_t nops = plan.ops.size();
  for (size_t k = 0; k < sz.size(); ++k) {
    Workspace* ws = nullptr;
    rc = get_workspace(sz[k], k ? ss->s[k - 1] : s, &ws);
    if (rc) return rc;
    if (ws->gev.size() != ws->groups.size() + 1) {
      set_error("forward_insitu: no events recorded");
      return TV_EINVAL;
    }
    for (size_t i = 0; i < nops && (int)i < cap; ++i) ms[k * cap + i] = 0.f;
    for (size_t gi = 0; gi < ws->groups.size(); ++gi) {
      float t = 0;
      TV_HIP(hipEventElapsedTime(&t, ws->gev[gi], ws->gev[gi + 1]));
      const int i = ws->groups[gi][0];
      if (i < cap) ms[k * cap + i] = t;
    }
  }
  *n_slices = (int)sz.size();
  return TV_OK;
}

const char* Engine::op_kernel(int B, size_t i) {
  std::lock_guard<std::mutex> g(mu);
  for (const auto& kv : workspaces) {
    if (kv.first.second != B) continue;
    Workspace* ws = kv.second;
    // the kernel instance as rocprofv3 demangles it (template <T, OutT, MODE or TW>)
    static const char* tn[3] = {"float", "_Float16", "__bf16"};
    const OpSpec& op = plan.ops[i];
    if (op.kind == OP_PREP) return stem_op >= 0 ? "prep (fused into the stem)" : "prep";
    if (ss2_op >= 0 && (int)i == stem_op) return "(fused into block_layers.0.conv1: stem_s2)";
    if ((int)i == ss2_op) {
      std::string& name = ws->kname[i];  // (input kind of the last profile(): rebuilt per call)
      const int smode = profiled_u8 ? (desc.in_w % 4 == 0 ? 2 : 1) : 0;
      name = std::string("tv::ss2::stem_s2<") + tn[dtype] + ", " + std::to_string(smode) + ">";
      return name.c_str();
    }
    if ((int)i == stem_op) {
      std::string& name = ws->kname[i];  // (input kind of the last profile(): rebuilt per call)
      const int smode = profiled_u8 ? (desc.in_w % 4 == 0 ? 2 : 1) : 0;
      name = std::string("tv::stem::stem_conv<") + tn[dtype] + ", " + std::to_string(smode) + ", " +
             (plan.ops[i].N <= 32 ? "1" : "4") + ">";
      return name.c_str();
    }
    if (op.kind == OP_LAYOUT_IN) return dtype == F32 ? "tv::nchw_to_nhwc<float>" : dtype == F16 ? "tv::nchw_to_nhwc<_Float16>" : "tv::nchw_to_nhwc<__bf16>";
    const int mode = op.kind == OP_CONVT_ADD || op.up_s ? 1 : 0;
    const char* t = tn[dtype];
    const char* o = (op.out < 0) ? "float" : t;
    std::string& name = ws->kname[i];
    if (name.empty() && !ws->dcn_skip[i] && (op.kind == OP_MAXPOOL || op.kind == OP_DCN || op.kind == OP_DWCONVT_ADD))
      name = std::string(op.kind == OP_MAXPOOL ? "tv::dla::maxpool2_ceil<" : op.kind == OP_DCN ? "tv::dla::dcn_sample<"
                                                                                            : "tv::dla::dwconvt_add<") +
             t + ">";
    if (name.empty()) {
      if (ws->convt[i]) name = std::string("tv::convt::convt_add<") + t + ", " + std::to_string(ws->tparams[i].np) + ">";
      else if (ws->ct3[i] == 1) name = std::string("tv::ct3::convt3<") + t + ", " + std::to_string(ws->ct3p[i].act) + ">";
      else if (ws->ct3[i] == 2) name = "(fused into the phase (0,0) launch: convt3)";
      else if (ws->head_skip[i]) name = "(fused into the 3x3 heads)";
      else if (ws->dcn_skip[i]) name = "(sampled inside the fused DCNv2 kernel)";
      else if (ws->dcn[i].x) {
        const DcnParams& d = ws->dcn[i];
        const bool wide = d.N % 128 == 0;
        if ((dcn64_mode == 3 || dcn64_mode == 4) && dcn_win_supported(d)) {
          name = std::string("tv::dcn::dcn_win<") + t + ">";
        } else if (dcn64_mode == 5 && d.C % 64 == 0 && d.om_ldc % 2 == 0) {
          name = std::string("tv::dcn::dcn_gemm64d<") + t + (wide ? ", 128, 64>" : ", 64, 64>");
        } else if (dcn64_mode && d.C % 64 == 0) {  // dcn_gemm64<T, BN, PX>: the pixel tile as launch_dcn_gemm picks it
          const long tiles128 = ((long)d.B * d.H * d.W + 127) / 128 * (d.N / 128);
          const int px = !wide || dcn64_mode == 2 || tiles128 < 1024 ? 64 : 128;
          name = std::string("tv::dcn::dcn_gemm64<") + t + (wide ? ", 128, " : ", 64, ") + std::to_string(px) + ">";
          if (d.ksplit > 1) name += " split-K " + std::to_string(d.ksplit);
        } else {
          name = std::string("tv::dcn::dcn_gemm<") + t + (wide ? ", 128>" : ", 64>");
        }
      }
      else if (ws->small[i])
        name = std::string(csm_variant(op.segs[0].stride) ? "tv::csm::conv_small_halo<" : "tv::csm::conv_small<") + t + ", " + std::to_string(plan.tensors[op.segs[0].src].C) + ", " +
               std::to_string(op.N) + ", " + std::to_string(op.segs[0].stride) + ", " + std::to_string(op.act) + ">";
      else if (ws->lat[i])
        name = std::string("tv::lat::conv_lat<") + t + (dtype == F32 && f32x3 ? ", true>" : ">");
      else if (ws->burst[i]) {
        const int q = (ws->bparams[i].nk16 + 3) / 4;
        int kpw = 20;
        for (int v : {4, 6, 8, 12, 18, 20})
          if (q <= v) { kpw = v; break; }
        name = std::string("tv::burst::conv_burst<") + t + ", " + std::to_string(kpw) + ">";
      }
      else if (ws->c1x1[i])
        name = std::string("tv::c1x1::conv1x1_stream<") + t + (op.N > 64 ? ", 4>" : ", 2>");
      else if (ws->s2_grid[i]) name = std::string("tv::c3s2::conv3x3s2<") + t + ", " + std::to_string(op.act) + ">";
      else if (ws->c3_tw[i]) name = std::string("tv::c3::conv3x3<") + t + ", " + t + ", " + std::to_string(ws->c3_tw[i]) + ", " + std::to_string(op.act) + ", " + std::to_string(ws->head_fused[i]) + ", " + std::to_string(ws->c3_res[i]) + ", " + std::to_string(ws->c3_ni[i]) + ", " + std::to_string(plan.tensors[op.segs[0].src].C / 32) + ", " + std::to_string(ws->c3_nw[i]) + ">";
      else if (ws->use_pipe[i]) {
        name = std::string("tv::pipe::conv_pipe<") + t + ", " + o + ", " + std::to_string(mode) +
               (dtype == F32 && f32x3 ? ", true>" : ">");
        if (ws->params[i].ksplit > 1) name += " split-K " + std::to_string(ws->params[i].ksplit);
      }
      else name = std::string("tv::conv_igemm<") + t + ", " + o + ", " + std::to_string(mode) + ">";
    }
    return name.c_str();
  }
  return "";
}

int Engine::profile(const void* input, int input_u8, int B, float* out, hipStream_t s, float* ms, double* flops,
                    int cap, int* n_ops) {
  profiled_u8 = input_u8;
  TV_HIP(hipSetDevice(device));
  Workspace* ws = nullptr;
  int rc = get_workspace(B, s, &ws);
  if (rc) return rc;
  const size_t n = plan.ops.size();
  std::vector<hipEvent_t> ev(n + 1);
  for (auto& e : ev) TV_HIP(hipEventCreate(&e));
  // one op per launch, in execution order (each op's time between its neighbours' events)
  TV_HIP(hipEventRecord(ev[0], s));
  for (size_t k = 0; k < n; ++k) {
    rc = run_op((size_t)ws->order[k], ws, input, input_u8, out, s);
    if (rc) {  // name the op (with AMD_SERIALIZE_KERNEL=3 a faulting launch reports here)
      set_error("op " + std::to_string(ws->order[k]) + " (" + plan.ops[ws->order[k]].label + "): " + tv_last_error());
      break;
    }
    TV_HIP(hipEventRecord(ev[k + 1], s));
  }
  if (!rc) {
    TV_HIP(hipEventSynchronize(ev[n]));
    for (size_t k = 0; k < n; ++k) {
      const int i = ws->order[k];
      if (i >= cap) continue;
      float t = 0;
      TV_HIP(hipEventElapsedTime(&t, ev[k], ev[k + 1]));
      ms[i] = t;
      flops[i] = plan.ops[i].flops * B;
    }
    // an op fused into another launch does its FLOPs there: the stem inside stem_s2 (block0.conv1's
    // launch), the block-diagonal 1x1 heads inside the 3x3 heads' epilogue. Their own rows launch
    // nothing (or only an in-place activation) and report no FLOPs.
    for (size_t i = 0; i < n && (int)i < cap; ++i) {
      int host = -1;
      if (ss2_op >= 0 && (int)i == stem_op) host = ss2_op;
      else if (ws->head_skip[i] && i > 0 && ws->head_fused[i - 1]) host = (int)i - 1;
      else if (ws->ct3[i] == 2) host = (int)i - plan.ops[i].segs[0].convt_phase;
      if (host < 0 || host >= cap) continue;
      flops[host] += flops[i];
      flops[i] = 0.0;
    }
    *n_ops = (int)n;
  }
  for (auto& e : ev) (void)hipEventDestroy(e);
  return rc;
}

}  // namespace tv
