"""Non-finite scores from the engine path on random-init presets (debug aid)."""
import argparse
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from flexible_llm_sharding_amd.config import preset  # noqa: E402
from flexible_llm_sharding_amd.engine import ShardedRunner  # noqa: E402
from flexible_llm_sharding_amd.runtime.weights import HostStore  # noqa: E402
from flexible_llm_sharding_amd.utils.synthetic import synthetic_prompts  # noqa: E402
from flexible_llm_sharding_amd.utils.tokenizer import load_tokenizer, write_synthetic_tokenizer  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--model", default="llama2-70b")
ap.add_argument("--layers", type=int, default=8)
ap.add_argument("--prompts", type=int, default=2)
ap.add_argument("--budget", type=int, default=16384)
ap.add_argument("--storage", default="cpu")
a = ap.parse_args()
dev = torch.device("cuda", 0)
cfg = preset(a.model, num_hidden_layers=a.layers)
store = HostStore.synthetic(cfg, dev, seed=0)
td = f"/tmp/tok_{os.getpid()}"
write_synthetic_tokenizer(td, cfg.vocab_size)
tok = load_tokenizer(td)
prompts = synthetic_prompts(a.prompts, 1024, 5, 64, cfg.vocab_size, seed=0)
r = ShardedRunner(cfg, store, dev, tok, layer_num_per_shard=1, storage_location=a.storage, token_budget=a.budget)
out = r(prompts)
bad = [int((~np.isfinite(o.astype(np.float32))).sum()) for o in out]
print(f"layers={a.layers} prompts={a.prompts} budget={a.budget} storage={a.storage} mb={r.stats['micro_batches']}"
      f" non-finite per prompt: {bad[:8]} total {sum(bad)}", flush=True)
