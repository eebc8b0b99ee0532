"""Where do non-finite values first appear in a random-init model's forward?

Runs embed + decoder layers one at a time on one packed micro-batch of the
bench's prompt shape and prints, per layer, max |x| of the residual stream and
the number of non-finite entries.

    python scripts/nan_probe.py [--model llama2-70b] [--layers 80] [--prompts 2]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from flexible_llm_sharding_amd.config import preset  # noqa: E402
from flexible_llm_sharding_amd.models.layout import layer_layout  # noqa: E402
from flexible_llm_sharding_amd.models.llama import (ExecContext, rope_tables, run_decoder, run_embed,  # noqa: E402
                                                     run_head, run_norm)
from flexible_llm_sharding_amd.ops import get_ops  # noqa: E402
from flexible_llm_sharding_amd.runtime.batch import pack_prompts  # noqa: E402
from flexible_llm_sharding_amd.utils.tokenizer import TokenizedPrompt  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama2-70b")
    ap.add_argument("--layers", type=int, default=80)
    ap.add_argument("--prompts", type=int, default=2)
    ap.add_argument("--std", type=float, default=0.02)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    cfg = preset(a.model)
    ops = get_ops(dev)
    names = cfg.layer_names()
    g = torch.Generator().manual_seed(0)
    tps = [TokenizedPrompt(torch.randint(3, cfg.vocab_size, (1024,), generator=g).tolist(),
                           [torch.randint(3, cfg.vocab_size, (64,), generator=g).tolist() for _ in range(5)],
                           64, [63] * 5) for _ in range(a.prompts)]
    b = pack_prompts(tps, list(range(a.prompts)))
    meta = b.device_tensors(dev)
    cos, sin = rope_tables(cfg, 4096, torch.float16, dev)
    ctx = ExecContext(cfg, ops, dev, torch.float16, cos, sin)

    def layer(name):
        lay = layer_layout(cfg, "decoder" if ".layers." in name else
                           ("embed" if "embed" in name else ("norm" if name == "model.norm" else "head")))
        buf = torch.empty(lay.nbytes, dtype=torch.uint8, device=dev)
        ops.fill_layer_random(buf, lay, seed=names.index(name), std=a.std)
        return lay.views(buf, torch.float16)

    x = run_embed(ctx, layer(names[0]), meta)
    for i in range(a.layers):
        x = run_decoder(ctx, layer(names[1 + i]), x, b, meta, names[1 + i])
        bad = (~torch.isfinite(x)).sum().item()
        print(f"layer {i:3d}: max|x| {x.float().abs().max().item():10.2f}  rms {x.float().pow(2).mean().sqrt().item():8.3f}"
              f"  non-finite {bad}", flush=True)
        if bad:
            break
    h = run_norm(ctx, layer("model.norm"), x, meta)
    p = run_head(ctx, layer("lm_head"), h)
    print("probs non-finite:", (~torch.isfinite(p)).sum().item(), "of", p.numel())


if __name__ == "__main__":
    main()
