import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs under gpurun)")
    config.addinivalue_line("markers", "slow: long-running test")


def gpu_available() -> bool:
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


@pytest.fixture(scope="session")
def tiny_model(tmp_path_factory):
    """A tiny random-init per-layer checkpoint directory (config + tokenizer + layer files)."""
    from flexible_llm_sharding_amd.config import preset
    from flexible_llm_sharding_amd.utils.synthetic import write_synthetic_checkpoint
    d = tmp_path_factory.mktemp("tiny_model")
    cfg = preset("tiny")
    write_synthetic_checkpoint(cfg, str(d), seed=1, std=0.05)
    return str(d), cfg
