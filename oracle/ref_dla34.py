"""Oracle (test infrastructure): functional PyTorch-CPU restatement of the reference's
`CenterpointDLA34` forward (src/tauv_vision/centernet/model/backbones/centerpoint_dla.py).

Follows, op for op and in the reference's order:
  * BasicBlock        centerpoint_dla.py:30-59   (conv1/bn1/relu, conv2/bn2, += pad_to_match(residual), relu)
  * Root              centerpoint_dla.py:147-165 (1x1 over torch.cat(children), bn, [+children[0]], relu)
  * Tree              centerpoint_dla.py:168-221 (MaxPool2d(s, s, ceil_mode) bottom, 1x1+bn project,
                                                  level_root children, tree1 ignores the residual it is
                                                  handed and recomputes its own, :209-221)
  * DLA / dla34       centerpoint_dla.py:224-315 (base_layer 7x7, level0/1 conv levels, level2-5 Trees)
  * DeformConv        centerpoint_dla.py:360-392 (offset conv -> 18 ch, sigmoid(mask conv) -> 9 ch,
                                                  DeformConv2d(bias) -> BN -> ReLU)
  * pad_to_match      centerpoint_dla.py:394-407 (F.pad tuple in the correct (W, H) order here)
  * IDAUp / DLAUp     centerpoint_dla.py:410-462 (depthwise ConvTranspose2d(2f, f, f//2, groups=o))
  * DLASeg heads      centerpoint_dla.py:476-531 (3x3 + bias, ReLU, 1x1 + bias; heads '0'..'n-1')
  * CenterpointDLA34  centerpoint_dla.py:544-578 (Prediction pop order, same as centernet.py:77-90)

`deform_conv2d` restates torchvision 0.15.2's modulated deformable convolution
(requirements.txt:3; torchvision is absent here and not vendored): per output pixel and
tap k = i*3 + j, sample input(y, x) with y = oy*s - p + i + offset[2k], x = ox*s - p + j +
offset[2k+1] by bilinear interpolation (0 outside, a corner counts only inside the image,
the whole sample is 0 when y <= -1, y >= H, x <= -1 or x >= W), multiply by mask[k], then
contract the columns [Cin*9] with the weight and add the bias. PARITY UNPINNED for that
function: no reference test or fixture pins DCNv2 numerics; everything around it is pinned
by goldens made by the reference module with this function plugged in.
Weights are read from a reference-layout state_dict (keys of DLASeg, i.e. without the
`model.` prefix CenterpointDLA34 adds).
"""
import torch
import torch.nn.functional as F

from .ref_forward import PredictionRef


def deform_conv2d(x, offset, mask, weight, bias, stride=1, padding=1):
    """torchvision.ops.deform_conv2d restatement (offset_groups = 1, dilation 1)."""
    B, C, H, W = x.shape
    cout, _, kh, kw = weight.shape
    Ho = (H + 2 * padding - kh) // stride + 1
    Wo = (W + 2 * padding - kw) // stride + 1
    oy = (torch.arange(Ho, dtype=x.dtype) * stride - padding).view(1, Ho, 1)
    ox = (torch.arange(Wo, dtype=x.dtype) * stride - padding).view(1, 1, Wo)
    flat = x.reshape(B, C, H * W)
    cols = []
    for i in range(kh):
        for j in range(kw):
            k = i * kw + j
            y = oy + i + offset[:, 2 * k]          # [B, Ho, Wo]
            xx = ox + j + offset[:, 2 * k + 1]
            inside = (y > -1) & (y < H) & (xx > -1) & (xx < W)
            y0 = torch.floor(y)
            x0 = torch.floor(xx)
            ly, lx = y - y0, xx - x0
            hy, hx = 1 - ly, 1 - lx
            y0i, x0i = y0.long(), x0.long()
            val = torch.zeros(B, C, Ho, Wo, dtype=x.dtype)
            for dy, dx, wgt in ((0, 0, hy * hx), (0, 1, hy * lx), (1, 0, ly * hx), (1, 1, ly * lx)):
                yy, xq = y0i + dy, x0i + dx
                ok = inside & (yy >= 0) & (yy <= H - 1) & (xq >= 0) & (xq <= W - 1)
                idx = (yy.clamp(0, H - 1) * W + xq.clamp(0, W - 1)).view(B, 1, Ho * Wo).expand(B, C, Ho * Wo)
                v = torch.gather(flat, 2, idx).view(B, C, Ho, Wo)
                val = val + (wgt * ok.to(x.dtype)).unsqueeze(1) * v
            cols.append(mask[:, k].unsqueeze(1) * val)
    col = torch.stack(cols, 2).reshape(B, C * kh * kw, Ho * Wo)   # row index c*9 + k
    out = torch.matmul(weight.reshape(cout, C * kh * kw), col).view(B, cout, Ho, Wo)
    if bias is not None:
        out = out + bias.view(1, cout, 1, 1)
    return out


def _bn(sd, p, x):
    return F.batch_norm(x, sd[p + ".running_mean"], sd[p + ".running_var"],
                        sd[p + ".weight"], sd[p + ".bias"], False, 0.1, 1e-5)


def _conv(sd, p, x, stride=1, padding=0):
    return F.conv2d(x, sd[p + ".weight"], sd.get(p + ".bias"), stride, padding)


def pad_to_match(feature, shape):
    """centerpoint_dla.py:394-407."""
    if feature.shape == shape:
        return feature
    pa = max(0, (feature.shape[2] - shape[2]) // 2)
    pb = max(0, shape[2] - feature.shape[2] - pa)
    pl = max(0, (feature.shape[3] - shape[3]) // 2)
    pr = max(0, shape[3] - feature.shape[3] - pl)
    return F.pad(feature, (pl, pr, pa, pb))[:, :, :shape[2], :shape[3]]


def _basic(sd, p, x, stride, residual=None):
    residual = x if residual is None else residual
    out = F.relu(_bn(sd, p + ".bn1", _conv(sd, p + ".conv1", x, stride, 1)))
    out = _bn(sd, p + ".bn2", _conv(sd, p + ".conv2", out, 1, 1))
    out = out + pad_to_match(residual, out.shape)
    return F.relu(out)


def _root(sd, p, kids, residual=False):
    y = _bn(sd, p + ".bn", _conv(sd, p + ".conv", torch.cat(kids, 1)))
    if residual:
        y = y + kids[0]
    return F.relu(y)


def _tree(sd, p, x, levels, stride, cin, cout, level_root, children=None):
    children = [] if children is None else children
    bottom = F.max_pool2d(x, stride, stride, ceil_mode=True) if stride > 1 else x
    residual = _bn(sd, p + ".project.1", _conv(sd, p + ".project.0", bottom)) if cin != cout else bottom
    if level_root:
        children.append(bottom)
    if levels == 1:
        x1 = _basic(sd, p + ".tree1", x, stride, residual)
        x2 = _basic(sd, p + ".tree2", x1, 1)
        return _root(sd, p + ".root", [x2, x1] + children)
    x1 = _tree(sd, p + ".tree1", x, levels - 1, stride, cin, cout, False)   # ignores `residual`
    children.append(x1)
    return _tree(sd, p + ".tree2", x1, levels - 1, 1, cout, cout, False, children)


DLA34_LEVELS = [1, 1, 1, 2, 2, 1]
DLA34_CHANNELS = [16, 32, 64, 128, 256, 512]


def dla34_base(sd, img, p="base"):
    x = F.relu(_bn(sd, p + ".base_layer.1", _conv(sd, p + ".base_layer.0", img, 1, 3)))
    y = []
    # level0 / level1: _make_conv_level (conv3x3 + bn + relu per conv)
    for lvl, stride in ((0, 1), (1, 2)):
        for c in range(DLA34_LEVELS[lvl]):
            q = f"{p}.level{lvl}"
            x = F.relu(_bn(sd, f"{q}.{3 * c + 1}", _conv(sd, f"{q}.{3 * c}", x, stride if c == 0 else 1, 1)))
        y.append(x)
    for lvl in range(2, 6):
        x = _tree(sd, f"{p}.level{lvl}", x, DLA34_LEVELS[lvl], 2, DLA34_CHANNELS[lvl - 1], DLA34_CHANNELS[lvl],
                  lvl >= 3)
        y.append(x)
    return y


def _deform(sd, p, x):
    off = _conv(sd, p + ".offset", x, 1, 1)
    mask = torch.sigmoid(_conv(sd, p + ".mask", x, 1, 1))
    y = deform_conv2d(x, off, mask, sd[p + ".conv.weight"], sd.get(p + ".conv.bias"), 1, 1)
    return F.relu(_bn(sd, p + ".actf.0", y))


def _ida(sd, p, layers, startp, endp):
    for i in range(startp + 1, endp):
        j = i - startp
        w = sd[f"{p}.up_{j}.weight"]
        f = w.shape[2] // 2
        u = F.conv_transpose2d(_deform(sd, f"{p}.proj_{j}", layers[i]), w, None, stride=f, padding=f // 2,
                               groups=w.shape[0])
        layers[i] = _deform(sd, f"{p}.node_{j}", pad_to_match(u, layers[i - 1].shape) + layers[i - 1])


def dlaseg_forward(sd, img, n_heads, first_level=2, last_level=5):
    """DLASeg.forward (centerpoint_dla.py:515-525) -> list of head outputs (NCHW)."""
    layers = dla34_base(sd, img)
    out = [layers[-1]]
    for i in range(len(layers) - first_level - 1):
        _ida(sd, f"dla_up.ida_{i}", layers, len(layers) - i - 2, len(layers))
        out.insert(0, layers[-1])
    y = [out[i].clone() for i in range(last_level - first_level)]
    _ida(sd, "ida_up", y, 0, len(y))
    z = []
    for h in range(n_heads):
        t = F.relu(_conv(sd, f"{h}.0", y[-1], 1, 1))
        z.append(_conv(sd, f"{h}.2", t))
    return z


def centerpoint_dla34_forward(sd, img, flags, n_heads):
    """CenterpointDLA34.forward (centerpoint_dla.py:558-578); sd keyed like DLASeg."""
    outs = dlaseg_forward(sd, img, n_heads)

    def nhwc(t):
        return t.permute(0, 2, 3, 1)

    heat = outs.pop(0)
    kh = ka = None
    if flags.get("keypoints"):
        kh = outs.pop(0)
        t = outs.pop(0)
        ka = t.reshape(t.size(0), t.size(1) // 2, 2, t.size(2), t.size(3))
    size = nhwc(outs.pop(0))
    offset = nhwc(outs.pop(0))
    ang = {}
    for name in ("roll", "pitch", "yaw"):
        ang[name] = (nhwc(outs.pop(0)), nhwc(outs.pop(0))) if flags.get(name) else (None, None)
    depth = nhwc(outs.pop(0)) if flags.get("depth") else None
    return PredictionRef(heatmap=heat, keypoint_heatmap=kh, keypoint_affinity=ka, size=size,
                         offset=offset, roll_bin=ang["roll"][0], roll_offset=ang["roll"][1],
                         pitch_bin=ang["pitch"][0], pitch_offset=ang["pitch"][1],
                         yaw_bin=ang["yaw"][0], yaw_offset=ang["yaw"][1], depth=depth)
