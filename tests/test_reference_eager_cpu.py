"""The reference-algorithm eager baseline script (scripts/reference_eager_bench.py) runs and scores."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_reference_eager_baseline_tiny_cpu():
    cmd = [sys.executable, os.path.join(ROOT, "scripts", "reference_eager_bench.py"), "--device", "cpu",
           "--layers", "2", "--hidden", "128", "--inter", "256", "--heads", "4", "--kv-heads", "2",
           "--vocab", "500", "--prompts", "2", "--prefix-len", "16", "--n-suffix", "3", "--suffix-len", "4"]
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=300, check=True).stdout
    rec = json.loads(out.strip().splitlines()[-1])
    assert rec["tokens_per_step"] == 2 * (16 + 3 * 4)
    assert rec["scores_finite"] and rec["value"] > 0
