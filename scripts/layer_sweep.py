"""Per-token cost of one Llama-2-70B decoder layer vs micro-batch size / MLP chunk.

Times ``run_decoder`` (rmsnorm, QKV+RoPE GEMM, shared-prefix attention, O+residual,
rmsnorm, gate/up+SwiGLU, down+residual) on packed batches of the bench's prompt
shape (1024-token prefix + 5 x 64-token suffixes), interleaving the variants over
several rounds in one process (guide §5.4 rule 24).

    python scripts/layer_sweep.py [--prompts 12,18,24,32] [--chunks 16384,24576,65536] [--rounds 3]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from flexible_llm_sharding_amd.config import preset  # noqa: E402
from flexible_llm_sharding_amd.models.layout import layer_layout  # noqa: E402
from flexible_llm_sharding_amd.models.llama import ExecContext, layer_flops, rope_tables, run_decoder  # noqa: E402
from flexible_llm_sharding_amd.ops import get_ops  # noqa: E402
from flexible_llm_sharding_amd.runtime.batch import pack_prompts  # noqa: E402
from flexible_llm_sharding_amd.utils.tokenizer import TokenizedPrompt  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--prompts", default="12,16,18,24,32")
    ap.add_argument("--chunks", default="16384,24576,65536")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--iters", type=int, default=3)
    ap.add_argument("--prefix-len", type=int, default=1024)
    ap.add_argument("--suffix-len", type=int, default=64)
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    cfg = preset("llama2-70b")
    ops = get_ops(dev)
    lay = layer_layout(cfg, "decoder")
    buf = torch.empty(lay.nbytes, dtype=torch.uint8, device=dev)
    ops.fill_layer_random(buf, lay, seed=1)
    W = lay.views(buf, torch.float16)
    cos, sin = rope_tables(cfg, 4096, torch.float16, dev)
    g = torch.Generator().manual_seed(0)

    def prompt():
        pre = torch.randint(3, cfg.vocab_size, (a.prefix_len,), generator=g).tolist()
        sufs = [torch.randint(3, cfg.vocab_size, (a.suffix_len,), generator=g).tolist() for _ in range(5)]
        return TokenizedPrompt(pre, sufs, a.suffix_len, [a.suffix_len - 1] * 5)

    variants = []
    for npr in [int(x) for x in a.prompts.split(",")]:
        tps = [prompt() for _ in range(npr)]
        b = pack_prompts(tps, list(range(npr)))
        meta = b.device_tensors(dev)
        x0 = (torch.randn(b.num_tokens, cfg.hidden_size, device=dev) * 0.5).half()
        for ch in [int(x) for x in a.chunks.split(",")]:
            if ch > b.num_tokens and ch != max(int(x) for x in a.chunks.split(",")):
                continue
            variants.append({"prompts": npr, "tokens": b.num_tokens, "mlp_chunk": ch, "batch": b,
                             "meta": meta, "x0": x0, "ms": []})
    for r in range(a.rounds):
        for v in variants:
            ctx = ExecContext(cfg, ops, dev, torch.float16, cos, sin, v["mlp_chunk"])
            x = v["x0"].clone()
            run_decoder(ctx, W, x, v["batch"], v["meta"])       # warm
            torch.cuda.synchronize()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(a.iters):
                x = run_decoder(ctx, W, x, v["batch"], v["meta"])
            e.record()
            torch.cuda.synchronize()
            v["ms"].append(s.elapsed_time(e) / a.iters)
    out = []
    for v in variants:
        ms = sorted(v["ms"])[len(v["ms"]) // 2]
        fl = layer_flops(cfg, v["batch"])
        row = {"prompts": v["prompts"], "tokens": v["tokens"], "mlp_chunk": v["mlp_chunk"],
               "ms_median": round(ms, 3), "ms_all": [round(t, 3) for t in v["ms"]],
               "us_per_token": round(ms * 1e3 / v["tokens"], 4), "tflops": round(fl / ms / 1e9, 1)}
        out.append(row)
        print(json.dumps(row), flush=True)
    if a.json:
        with open(a.json, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
