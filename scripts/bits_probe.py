"""Which plan knob changes the scores' bits?  Llama-2-7B geometry (4 layers), 12 prompts of
1,024 + 5 x 64 tokens, one uncapped runner; the same call with the attention phase in
prompt-aligned row groups, with MLP row chunks, and with each v11 selection mode, against the
default whole-micro-batch run: bitwise equal or the max |difference|.

    python scripts/bits_probe.py
"""
import os
import sys
import tempfile

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from flexible_llm_sharding_amd.config import preset  # noqa: E402
from flexible_llm_sharding_amd.engine import ShardedRunner  # noqa: E402
from flexible_llm_sharding_amd.runtime.weights import HostStore  # noqa: E402
from flexible_llm_sharding_amd.utils.synthetic import synthetic_prompts  # noqa: E402
from flexible_llm_sharding_amd.utils.tokenizer import load_tokenizer, write_synthetic_tokenizer  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    cfg = preset("llama2-7b", num_hidden_layers=4)
    store = HostStore.synthetic(cfg, dev, seed=11)
    d = tempfile.mkdtemp()
    write_synthetic_tokenizer(os.path.join(d, "tok"), cfg.vocab_size)
    tok = load_tokenizer(os.path.join(d, "tok"))
    prompts = synthetic_prompts(12, 1024, 5, 64, cfg.vocab_size, seed=12)
    r = ShardedRunner(cfg, store, dev, tok, layer_num_per_shard=1, storage_location="cpu")
    k = r.ops.k

    def run():
        outs = r(prompts)
        torch.cuda.synchronize()
        return np.concatenate([o.reshape(-1) for o in outs]).astype(np.float32)

    base = run()
    cases = [("repeat", {}, None), ("attn_rows 12288", {"attn_rows": 12288}, None),
             ("mlp_chunk 9216", {"mlp_chunk": 9216}, None),
             ("attn_rows 12288 + mlp_chunk 9216", {"attn_rows": 12288, "mlp_chunk": 9216}, None),
             ("v11 mode 0 (v10)", {}, 0), ("v11 mode 2", {}, 2)]
    for name, ctx_kw, v11 in cases:
        saved = {a: getattr(r.ctx, a) for a in ctx_kw}
        for a, v in ctx_kw.items():
            setattr(r.ctx, a, v)
        old = k.fls_gemm_set_v11(v11) if v11 is not None else None
        got = run()
        if old is not None:
            k.fls_gemm_set_v11(old)
        for a, v in saved.items():
            setattr(r.ctx, a, v)
        eq = np.array_equal(got, base)
        print(f"{name:36s} bitwise {eq}  max |diff| {np.abs(got - base).max():.3e}", flush=True)
    # without the pruned last layer (every layer's attention phase in groups)
    r.ctx.prune_last = False
    base = run()
    r.ctx.attn_rows = 4096
    got = run()
    r.ctx.attn_rows = 0
    print(f"{'no pruning: attn_rows 4096':36s} bitwise {np.array_equal(got, base)}  "
          f"max |diff| {np.abs(got - base).max():.3e}", flush=True)


if __name__ == "__main__":
    main()
