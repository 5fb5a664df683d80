"""hipGraph capture of the batched product step: forward_u8 of 64 frames (launched as two
concurrent 32-frame slices: the second on an engine side stream forked from and joined back
into the capturing stream with events, engine.cpp Engine::forward) + device decode + the
async D2H copy of the records. The replayed graph must reproduce the eager step bit for bit.
"""
import pytest
import torch

import bench

pytestmark = pytest.mark.gpu


def _same(host, host_counts, rec, cnt, what):
    """Records [B, K, 10] / counts [B]: rows past a frame's count are not part of the result."""
    assert torch.equal(host_counts, cnt), f"{what}: counts differ {host_counts.tolist()} vs {cnt.tolist()}"
    for b in range(rec.shape[0]):
        n = int(cnt[b])
        a, e = host[b, :n].view(torch.int32), rec[b, :n].view(torch.int32)  # bitwise (absent fields are NaN)
        if not torch.equal(a, e):
            bad = (a != e).nonzero()[:5].tolist()
            raise AssertionError(f"{what}: frame {b} (count {n}) records differ at {bad}: "
                                 f"{host[b, bad[0][0]].tolist()} vs {rec[b, bad[0][0]].tolist()}")


def test_capture_b64_two_slices_bit_identical():
    dev = torch.device("cuda", 0)
    model, oc, sd = bench.build_model("fp16", dev, "r18")
    mc = bench.tv.ModelConfig(bench.HEIGHTS, bench.CHANNELS, 480, 640, bench.DOWNSAMPLES, 1.0)
    B, K = 64, 100
    s = torch.cuda.Stream(dev)
    s.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(s):
        pipe = bench.Pipeline(model, oc, mc, B, K, 0.3, dev)  # workspaces + side streams keyed by s
        assert len(pipe.eng.slices(B)) == 2, "the batched path under test runs two concurrent slices"
        g = torch.Generator(device=dev).manual_seed(5)
        frames = torch.randint(0, 256, (B, 480, 640, 3), generator=g, device=dev, dtype=torch.uint8)
        pipe.step(frames)
        s.synchronize()
        heads = pipe.out.clone()
        rec = pipe.host.clone()
        cnt = pipe.host_counts.clone()
        pipe.out.fill_(float("nan"))
        pipe.host.fill_(-1.0)
        pipe.step(frames)  # the eager step again after the clobber: deterministic
        s.synchronize()
        assert torch.equal(pipe.out, heads), "eager heads differ between two runs"
        _same(pipe.host, pipe.host_counts, rec, cnt, "eager run 2")
    torch.cuda.current_stream(dev).wait_stream(s)
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph, stream=s):
        pipe.step(frames)
    for _ in range(3):
        pipe.out.fill_(float("nan"))
        pipe.host.fill_(-1.0)
        graph.replay()
        torch.cuda.synchronize()
        assert torch.equal(pipe.out, heads), "replayed heads differ from the eager step"
        _same(pipe.host, pipe.host_counts, rec, cnt, "replay")
    assert int(cnt.sum()) > 0
