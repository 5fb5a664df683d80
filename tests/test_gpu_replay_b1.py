"""BASELINE config 2 (the latency path) as bench.py times it: the B=1 step — forward_u8 + device
decode + async D2H of the records — captured once as a hipGraph and replayed (bench.py
latency_b1). At B=1 the engine runs its latency-path schedule (engine.cpp make_workspace: ops by
dependency level, grouped conv_lat / convt_add launches, conv_lat split-K slabs whose tickets are
self-resetting: zeroed once when the workspace is made, and each tile's last-arriving slice zeroes
its own ticket, so every complete replay leaves them at zero for the next — no memset node, which
on this ROCm did not re-run correctly on replay). Checked here, for the R18 step in fp16 and bf16
and the DLA-34 step in fp16:

  * three replays, each after the heads, records and counts were clobbered (NaN / -1), reproduce
    the eager step bit for bit — a split-K ticket left non-zero between replays, or a grouped
    launch reading a tensor before its producer, would change the outputs, not the timing;
  * the replayed golden frame meets the low-precision parity bars of test_gpu_parity_lowp.py
    against the reference's own Prediction tensors and decode(K=100) records (tests/golden).
"""
import numpy as np
import pytest
import torch

import bench
from detcmp import peak_parity
from helpers import golden
from test_gpu_capture import _same
from test_gpu_parity_lowp import FIELDS, TOL

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("arch,precision", [("r18", "fp16"), ("r18", "bf16"), ("dla34", "fp16")])
def test_b1_graph_replay_matches_eager_and_reference(arch, precision):
    dev = torch.device("cuda", 0)
    model, oc, _ = bench.build_model(precision, dev, arch)
    H, W, K = 480, 640, 100
    mc = bench.tv.ModelConfig(bench.HEIGHTS, bench.CHANNELS, H, W, bench.DOWNSAMPLES, 1.0)
    name, seed = bench.GOLDEN[arch]
    g = golden(name)
    frame = torch.randint(0, 256, (1, H, W, 3), generator=torch.Generator().manual_seed(seed),
                          dtype=torch.uint8).to(dev)
    # exactly bench.latency_b1's sequence: workspaces keyed to the capture stream by eager steps
    s = torch.cuda.Stream(dev)
    s.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(s):
        pipe = bench.Pipeline(model, oc, mc, 1, K, 0.0, dev)
        assert pipe.eng.slices(1) == [1]
        for _ in range(3):
            pipe.step(frame)
        s.synchronize()
        heads = pipe.out.clone()
        rec = pipe.host.clone()
        cnt = pipe.host_counts.clone()
    torch.cuda.current_stream(dev).wait_stream(s)
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph, stream=s):
        pipe.step(frame)
    for r in range(3):
        pipe.out.fill_(float("nan"))
        pipe.host.fill_(-1.0)
        pipe.host_counts.fill_(-1)
        graph.replay()
        torch.cuda.synchronize()
        assert torch.equal(pipe.out, heads), f"replay {r}: heads differ from the eager step"
        _same(pipe.host, pipe.host_counts, rec, cnt, f"replay {r}")
    assert int(cnt[0]) == K

    # the replayed outputs against the reference (test_gpu_parity_lowp.py's bars)
    tol = TOL[(arch, precision)]
    for f in FIELDS:
        if f not in g.files or getattr(pipe.pred, f) is None:
            continue
        ref = g[f][0]
        got = getattr(pipe.pred, f)[0].detach().float().cpu().numpy()
        rel = float(np.abs(got - ref).max()) / max(1.0, float(np.abs(ref).max()))
        assert rel <= tol, f"{arch} {precision} {f}: {rel:.3e} > {tol}"
    hm_err = float(np.abs(pipe.pred.heatmap[0].float().cpu().numpy() - g["heatmap"][0]).max())
    pp = peak_parity(pipe.host.numpy()[:1], g["heatmap"][:1], g["decode_k100_index"][:1], g["decode_k100"][:1],
                     max(hm_err, 1e-6))
    assert pp["determined_found"] == pp["determined"], pp
    assert pp["extra_ok"], pp
    assert pp["max_score_err"] <= hm_err / 4 + 1e-6, pp
    assert pp["max_box_err"] <= tol * max(1.0, float(np.abs(g["size"]).max())), pp
