"""The driver's bench contract, rehearsed on CPU/gloo: ``bench.py`` under
``torch.distributed.run`` (one rank per device) prints ONE JSON line on rank 0
with the whole-job aggregate."""
import json
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _bench(world, extra, tmp_path, launcher=True):
    args = ["--gpus", str(world), "--steps", "2", "--warmup", "1", "--cpu", "--model", "tiny",
            "--prompts-per-gpu", "3", "--prefix-len", "24", "--suffix-len", "4"] + extra
    if world > 1 and launcher:
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
               "--master-addr", "127.0.0.1", "--master-port", str(_port()), os.path.join(ROOT, "bench.py")] + args
    else:
        cmd = [sys.executable, os.path.join(ROOT, "bench.py")] + args
    env = dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="1")
    r = subprocess.run(cmd, cwd=str(tmp_path), env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    return json.loads(lines[0])


@pytest.mark.parametrize("world,mode,stages", [(1, "auto", "round_robin"), (2, "auto", "round_robin"),
                                               (2, "mp", "round_robin"), (3, "auto", "round_robin"),
                                               (6, "mp", "round_robin"), (3, "mp", "contiguous"),
                                               (8, "auto", "round_robin")])
def test_bench_contract(tmp_path, world, mode, stages):
    # world 6 on the 5-layer tiny model: the MP shard padding leaves rank 5 with no layers;
    # world 8 DP = the driver's 8-GPU scaling point (every layer scatter-loaded 1/8 per rank + all-gather)
    out = _bench(world, ["--mode", mode, "--stages", stages], tmp_path)
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
              "scaling", "vs_baseline", "dtype", "data", "config"):
        assert k in out
    assert out["n_gpus"] == world and out["steps"] == 2 and out["warmup"] == 1
    assert out["scores_finite"] is True and out["value"] > 0
    tok = out["config"]["tokens_per_step"]
    # value is the whole-job aggregate: tokens per step (summed over ranks) / seconds per step
    assert abs(out["value"] - tok / (out["ms_per_step"] / 1e3)) / out["value"] < 0.02
    if world > 1:
        want = "pp" if mode == "mp" else "dp"
        assert out["config"]["parallelism"].startswith(want)
    # weak scaling: per-rank work fixed, global batch grows with the rank count
    assert out["config"]["global_batch"] == 3 * world


def test_bench_spawns_its_own_ranks(tmp_path):
    """`bench.py --gpus 3` with no torchrun environment starts the 3 rank processes itself
    and rank 0 prints one JSON line for the whole job; the JSON names the process group size."""
    out = _bench(3, [], tmp_path, launcher=False)
    assert out["n_gpus"] == 3 and out["world"] == 3 and out["process_group_ranks"] == 3
    assert len(out["rank_devices"]) == 3 and out["backend"] == "gloo"
    assert out["config"]["parallelism"].startswith("dp3") and out["scores_finite"] is True


@pytest.mark.parametrize("world", [1, 2])
def test_bench_stream_weights(tmp_path, world):
    """--weights stream: per-layer files written once, re-read every pass (DP: each rank its 1/G
    slice + all-gather); the JSON reports the host pinned / RSS footprint."""
    out = _bench(world, ["--weights", "stream", "--unique-layers", "1", "--ckpt-dir", str(tmp_path / "ck")],
                 tmp_path, launcher=False)
    assert out["config"]["weights"] == "stream" and out["scores_finite"] is True
    assert "host_pinned_gb" in out and "host_peak_rss_gb" in out
    assert os.path.exists(tmp_path / "ck" / "model.layers.1.safetensors")
