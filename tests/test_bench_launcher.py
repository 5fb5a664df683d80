"""bench.py's multi-rank launch, on CPU: `--gpus N` outside torch.distributed.run starts N
ranks (one torch.distributed.run child), each rank all-gathers its frames' packed records
through RecordGather over gloo, and rank 0's line reports the ranks the collective saw and
the gathered frame count; a --gpus / WORLD_SIZE mismatch is refused."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def run_bench(*argv, env=None):
    e = dict(os.environ)
    e.pop("WORLD_SIZE", None)
    if env:
        e.update(env)
    r = subprocess.run([sys.executable, BENCH, *argv], capture_output=True, text=True, timeout=240, env=e,
                       cwd="/tmp")
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    return r, (json.loads(lines[-1]) if lines else None)


@pytest.mark.parametrize("gpus,batch", [(2, 4), (3, 3)])
def test_launcher_spawns_ranks_and_gathers(gpus, batch):
    r, line = run_bench("--gpus", str(gpus), "--cpu-dryrun", "--batch", str(batch), "--steps", "2")
    assert r.returncode == 0, r.stderr[-2000:]
    assert line["ranks"] == gpus and line["n_gpus"] == gpus and line["backend"] == "gloo"
    assert line["gathered_frames"] == gpus * batch
    assert line["gather_ok"], "gathered records differ from the single-process records of the same frames"


def test_single_process_dryrun_matches():
    r, line = run_bench("--cpu-dryrun", "--batch", "8", "--steps", "1")
    assert r.returncode == 0, r.stderr[-2000:]
    assert line["ranks"] == 1 and line["gathered_frames"] == 8 and line["gather_ok"]


def test_world_size_mismatch_refused():
    r, line = run_bench("--gpus", "1", "--cpu-dryrun", env={"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode != 0 and line is None
    assert "WORLD_SIZE" in r.stderr
