"""Per-stage error budget of the fp16 / bf16 engine against the north star's 1e-4 bar (CPU).

The engine's reduced-precision numerics, restated op for op on the CPU (this file is measurement
infrastructure and imports the oracle; nothing in the product path uses it):
  * BatchNorm folded into the conv weights in double, the folded weights rounded to the compute
    dtype, the folded bias kept fp32 (engine.cpp pack_op);
  * activations stored in the compute dtype: the normalised input (stem LUT), every conv output
    after its activation, every ConvTranspose + pad_to_match + skip sum (convt.hip: one rounding
    of (acc + bias) + skip);
  * fp32 accumulation; ResidualBlock conv2 and its 1x1 residual in one accumulator; Root over the
    concatenated children in one accumulator;
  * the stacked 3x3 heads' LeakyReLU output fed to the fused 1x1 heads as hi + lo (= fp32 to ~2x
    the dtype's precision, conv3x3 EPI 1), the 1x1 head weights in the dtype, fp32 output.
Stage k of the forward (stem, block0, block1, tree0-4, IDAUp 0-4, IDAUpReverse 0-3, heads) can be
switched to fp32 arithmetic; the report gives, on the golden 480x640 frame of the bench's parity
leg (seeded weights, tests/golden/recipe.py), the two quantities of bench.py's parity leg:
heatmap drift (max |logit - reference|) and max box error at the reference's top-100 peaks
(max over |dy|/in_h, |dx|/in_w, |dh|, |dw| of decode's Detection fields, decode.py:205-212).

  python tools/precision_budget.py [--dtype fp16|bf16] [--out profiles/r4/precision_budget.json]

Rows: `all_low` (every stage in the dtype: the simulated engine), `only_<stage>` (that stage
alone in the dtype: its own contribution), `fp32_from_<stage>` (the stages before it in the
dtype: the error left if everything from there on ran in fp32 — the "mixed tail" candidates).
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch
import torch.nn.functional as F

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))

from oracle import ref_forward as R  # noqa: E402
from recipe import seeded_state_dict, normalize  # noqa: E402

HEIGHTS, CHANNELS, DOWNSAMPLES = [2] * 5, [128] * 6, 2
STAGES = (["stem", "block0", "block1"] + [f"tree{i}" for i in range(5)] + [f"idaup{i}" for i in range(5)] +
          [f"reverse{i}" for i in range(4)] + ["heads"])


class Numerics:
    def __init__(self, dtype, low, acts=True, weights=True):
        self.dt = dtype
        self.low = set(low)  # stages in the compute dtype
        self.stage = None
        self.acts, self.weights = acts, weights  # which of the two roundings the low stages apply

    def q(self, x):
        """an activation stored by a stage in the compute dtype"""
        return x.to(self.dt).float() if self.stage in self.low and self.acts else x

    def w(self, t):
        """a weight tensor in the compute dtype"""
        return t.to(self.dt).float() if self.weights else t.float()

    def lowp(self):
        return self.stage in self.low


def _fold(sd, conv, bn):
    w = sd[conv + ".weight"].double()
    b = sd[conv + ".bias"].double() if (conv + ".bias") in sd else torch.zeros(w.shape[0], dtype=torch.float64)
    if bn is None:
        return w, b
    s = sd[bn + ".weight"].double() / torch.sqrt(sd[bn + ".running_var"].double() + 1e-5)
    return w * s.view(-1, 1, 1, 1), (b - sd[bn + ".running_mean"].double()) * s + sd[bn + ".bias"].double()


def conv_bn(nm, sd, terms, act):
    """sum over (input, conv prefix, bn prefix, stride, padding) terms of conv+BN, one accumulator,
    then the activation; the low-precision form rounds the folded weights and the inputs."""
    if not nm.lowp():
        y = None
        for x, conv, bn, stride, pad in terms:
            t = R._conv(sd, conv, x, stride, pad)
            if bn is not None:
                t = R._bn(sd, bn, t)
            y = t if y is None else y + t
    else:
        y = None
        bias = None
        for x, conv, bn, stride, pad in terms:
            w, b = _fold(sd, conv, bn)
            t = F.conv2d(nm.q(x), nm.w(w.float()), None, stride, pad)
            y = t if y is None else y + t
            bias = b if bias is None else bias + b
        y = y + bias.float().view(1, -1, 1, 1)
    if act == "relu":
        y = F.relu(y)
    elif act == "leaky":
        y = F.leaky_relu(y)
    return nm.q(y)


def block(nm, sd, p, x, stride):
    a = conv_bn(nm, sd, [(x, p + ".conv1", p + ".bn1", stride, 1)], "relu")
    return conv_bn(nm, sd, [(a, p + ".conv2", p + ".bn2", 1, 1), (x, p + ".conv_residual", p + ".bn_residual", stride, 0)],
                   "relu")


def tree(nm, sd, p, x, height, stride, children=None):
    kids = [] if children is None else children
    if height == 1:
        left = block(nm, sd, p + ".tree_l", x, stride)
        right = block(nm, sd, p + ".tree_r", left, 1)
        cat = torch.cat(kids + [left, right], 1)
        return conv_bn(nm, sd, [(cat, p + ".root.conv", p + ".root.bn", 1, 0)], "relu")
    left = tree(nm, sd, p + ".tree_l", x, height - 1, stride)
    return tree(nm, sd, p + ".tree_r", left, height - 1, 1, kids + [left])


def up_add(nm, sd, p, i, src, skip):
    """projection + ConvTranspose(k = s) + pad_to_match + skip (convt.hip's one rounding)"""
    proj = conv_bn(nm, sd, [(src, f"{p}.projection_layers.{i}.0", f"{p}.projection_layers.{i}.1", 1, 1)], "relu")
    w = sd[f"{p}.upsample_layers.{i}.weight"]
    b = sd[f"{p}.upsample_layers.{i}.bias"]
    s = w.shape[2]
    if nm.lowp():
        u = F.conv_transpose2d(proj, nm.w(w), b, stride=s)
    else:
        u = F.conv_transpose2d(proj, w, b, stride=s)
    return nm.q(skip + R.pad_to_match(u, skip.shape))


def forward(nm, sd, img):
    p = "backbone.dla_down"
    nm.stage = "stem"
    x = nm.q(img)  # the stem LUT's normalised input in the dtype
    x = conv_bn(nm, sd, [(x, p + ".projection_layer.0", p + ".projection_layer.1", 1, 3)], "relu")
    for i in range(DOWNSAMPLES):
        nm.stage = f"block{i}"
        x = block(nm, sd, f"{p}.block_layers.{i}", x, 2)
    feats = [x]
    for i, h in enumerate(HEIGHTS):
        nm.stage = f"tree{i}"
        x = tree(nm, sd, f"{p}.tree_layers.{i}", x, h, 2)
        feats.append(x)
    collected = []
    for k in range(len(feats) - 1):
        nm.stage = f"idaup{k}"
        pp = f"backbone.multi_ida_up.ida_up_layers.{k}"
        n = len(feats) - 1
        cur = feats[-1]
        outs = []
        for i in reversed(range(n)):
            s = up_add(nm, sd, pp, i, cur, feats[i])
            cur = conv_bn(nm, sd, [(s, f"{pp}.output_layers.{i}.0", f"{pp}.output_layers.{i}.1", 1, 1)], "relu")
            outs.append(cur)
        feats = outs[::-1]
        collected.append(feats[-1])
    collected = collected[::-1]
    cur = collected[0]
    pp = "backbone.ida_up_reverse"
    for i in range(len(collected) - 1):
        nm.stage = f"reverse{i}"
        s = up_add(nm, sd, pp, i, collected[i + 1], cur)
        cur = conv_bn(nm, sd, [(s, f"{pp}.output_layers.{i}.0", f"{pp}.output_layers.{i}.1", 1, 1)], "relu")
    nm.stage = "heads"
    outs = []
    i = 0
    while f"heads.{i}.0.weight" in sd:
        if nm.lowp():
            h = F.leaky_relu(F.conv2d(nm.q(cur), nm.w(sd[f"heads.{i}.0.weight"]), sd[f"heads.{i}.0.bias"], 1, 1))
            # hidden fed as hi + lo (fp32 to ~2x the dtype's precision); 1x1 weights in the dtype
            outs.append(F.conv2d(h, nm.w(sd[f"heads.{i}.2.weight"]), sd[f"heads.{i}.2.bias"]))
        else:
            h = F.leaky_relu(F.conv2d(cur, sd[f"heads.{i}.0.weight"], sd[f"heads.{i}.0.bias"], 1, 1))
            outs.append(F.conv2d(h, sd[f"heads.{i}.2.weight"], sd[f"heads.{i}.2.bias"]))
        i += 1
    return outs[0], outs[1].permute(0, 2, 3, 1), outs[2].permute(0, 2, 3, 1)  # heatmap, size, offset


def metrics(out, ref, index, in_h=480, in_w=640):
    heat, size, off = out
    rh, rs, ro = ref
    drift = float((heat - rh).abs().max())
    W = rh.shape[3]
    hw = rh.shape[2] * W
    cells = index % hw
    ys, xs = cells // W, cells % W
    ds = (size[0, ys, xs] - rs[0, ys, xs]).abs()
    do = (off[0, ys, xs] - ro[0, ys, xs]).abs()
    box = max(float(ds.max()), float(do[:, 0].max()) / in_h, float(do[:, 1].max()) / in_w)
    return {"heatmap_drift": round(drift, 8), "max_box_err": round(box, 8),
            "max_size_err": round(float(ds.max()), 8)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dtype", default="fp16", choices=["fp16", "bf16"])
    ap.add_argument("--out", default=None)
    ap.add_argument("--rows", default="all", help="all | quick (all_low + fp32_from_* only)")
    a = ap.parse_args()
    dt = torch.float16 if a.dtype == "fp16" else torch.bfloat16
    sys.path.insert(0, os.path.join(ROOT, "tauv-vision_amd"))
    import bench
    # the bench's R18 state_dict keys (host-only: the model class is never run)
    import tauv_vision_amd as tv
    A = tv.AngleConfig
    oc = tv.ObjectConfigSet([tv.ObjectConfig(f"class{i}", A(False, None), A(False, None), A(False, None), False, False,
                                             None) for i in range(bench.N_LABELS)])
    keys = tv.Centernet(tv.DLABackbone(HEIGHTS, CHANNELS, DOWNSAMPLES), oc).state_dict()
    sd = seeded_state_dict([(k, tuple(v.shape)) for k, v in keys.items()])
    name, seed = bench.GOLDEN["r18"]
    g = np.load(os.path.join(ROOT, "tests", "golden", name + ".npz"))
    frame = torch.randint(0, 256, (1, 480, 640, 3), generator=torch.Generator().manual_seed(seed), dtype=torch.uint8)
    img = normalize(frame.permute(0, 3, 1, 2).float() / 255.0)
    index = torch.from_numpy(g["decode_k100_index"][0].astype(np.int64))
    torch.set_grad_enabled(False)
    t0 = time.time()
    ref = forward(Numerics(dt, []), sd, img)
    # the restatement in fp32 is the oracle: check it against the reference's stored heatmap
    ref_check = float(np.abs(ref[0].numpy() - g["heatmap"]).max())
    rows = {}

    def run(tag, low):
        rows[tag] = metrics(forward(Numerics(dt, low), sd, img), ref, index)
        print(tag, rows[tag], f"{time.time() - t0:.0f}s", flush=True)

    run("all_low", STAGES)
    rows["acts_only_low"] = metrics(forward(Numerics(dt, STAGES, weights=False), sd, img), ref, index)
    rows["weights_only_low"] = metrics(forward(Numerics(dt, STAGES, acts=False), sd, img), ref, index)
    print("acts_only_low", rows["acts_only_low"], "weights_only_low", rows["weights_only_low"], flush=True)
    if a.rows == "all":
        for s in STAGES:
            run(f"only_{s}", [s])
    for k in range(1, len(STAGES)):
        run(f"fp32_from_{STAGES[k]}", STAGES[:k])
    res = {"dtype": a.dtype, "frame": f"tests/golden/{name}.npz input (seed {seed}), 480x640, seeded R18 weights",
           "fp32_restatement_vs_reference_heatmap": ref_check, "stages": STAGES, "rows": rows,
           "method": "tools/precision_budget.py: CPU restatement of the engine's rounding points"}
    if a.out:
        os.makedirs(os.path.dirname(a.out), exist_ok=True)
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)
    print(json.dumps({k: v for k, v in res.items() if k != "rows"}))


if __name__ == "__main__":
    main()
