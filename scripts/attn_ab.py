"""A/B of attention kernel launch variants on the 70B bench batch (interleaved rounds, one
process): heads per block (``fls_attention_set_hpb``).  Prints TFLOP/s per variant and checks the
outputs are bitwise equal.

    python scripts/attn_ab.py [--variants 4,8] [--rounds 5]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from flexible_llm_sharding_amd.config import preset  # noqa: E402
from flexible_llm_sharding_amd.models.llama import layer_flops  # noqa: E402
from flexible_llm_sharding_amd.ops.hip_backend import HipOps  # noqa: E402
from flexible_llm_sharding_amd.runtime.batch import pack_prompts  # noqa: E402
from flexible_llm_sharding_amd.utils.tokenizer import TokenizedPrompt  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variants", default="4,8")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--prefix", type=int, default=1024)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    ops = HipOps()
    cfg = preset("llama2-70b")
    nh, nkv, hd = cfg.num_attention_heads, cfg.num_key_value_heads, cfg.head_dim
    n = 32 if a.prefix == 1024 else max(1, 32 * 1024 // a.prefix)
    tps = [TokenizedPrompt(list(range(a.prefix)), [list(range(64))] * 5, 64, [63] * 5) for _ in range(n)]
    b = pack_prompts(tps, list(range(n)), "bidirectional")
    meta = b.device_tensors(dev)
    g = torch.Generator(device=dev).manual_seed(0)
    qkv = torch.randn(b.num_tokens, cfg.qkv_size, device=dev, generator=g).half()
    fl = layer_flops(cfg, b) - 2.0 * b.num_tokens * cfg.decoder_layer_params()
    variants = [int(v) for v in a.variants.split(",")]
    outs, times = {}, {v: [] for v in variants}

    def run(v):
        ops.k.fls_attention_set_hpb(v)
        return ops.attention(qkv, meta["work"], nh, nkv, hd, seg_lo=meta["seg_lo"])

    for v in variants:
        outs[v] = run(v).clone()
    for _ in range(a.rounds):
        for v in variants:
            for _ in range(3):
                run(v)
            torch.cuda.synchronize()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(a.iters):
                run(v)
            e.record()
            torch.cuda.synchronize()
            times[v].append(s.elapsed_time(e) / a.iters / 1e3)
    ops.k.fls_attention_set_hpb(0)
    base = variants[0]
    for v in variants:
        ts = sorted(times[v])
        print(json.dumps({"hpb": v, "median_ms": ts[len(ts) // 2] * 1e3, "min_ms": ts[0] * 1e3,
                          "tflops_median": fl / ts[len(ts) // 2] / 1e12,
                          "bitwise_equal_to_first": bool(torch.equal(outs[v], outs[base]))}), flush=True)


if __name__ == "__main__":
    main()
