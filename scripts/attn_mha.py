"""Attention for MHA (Llama-2-7B heads: 32 q / 32 kv, hd 128): v1 (16 rows/wave) vs the v2 / v3 kernel with
one head per block.  12 prompts x (1024 prefix + 5 x 64 suffixes); interleaved rounds, median."""
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from flexible_llm_sharding_amd.config import preset  # noqa: E402
from flexible_llm_sharding_amd.models.llama import layer_flops  # noqa: E402
from flexible_llm_sharding_amd.ops.hip_backend import HipOps  # noqa: E402
from flexible_llm_sharding_amd.runtime.batch import pack_prompts  # noqa: E402
from flexible_llm_sharding_amd.utils.tokenizer import TokenizedPrompt  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    ops = HipOps()
    cfg = preset("llama2-7b")
    nh, nkv, hd = cfg.num_attention_heads, cfg.num_key_value_heads, cfg.head_dim
    out = {}
    for plen, n in ((1024, 12), (4096, 3)):
        tps = [TokenizedPrompt(list(range(plen)), [list(range(64))] * 5, 64, [63] * 5) for _ in range(n)]
        b = pack_prompts(tps, list(range(n)), "bidirectional")
        meta = b.device_tensors(dev)
        b128 = pack_prompts(tps, list(range(n)), "bidirectional", q_block=128)
        meta128 = b128.device_tensors(dev)
        qkv = torch.randn(b.num_tokens, (nh + 2 * nkv) * hd, device=dev).half()
        fl = layer_flops(cfg, b) - 2.0 * b.num_tokens * cfg.decoder_layer_params()
        arms = {"v1": (1, 0), "v2_hpb1": (2, 1), "v3_hpb1_db": (3, 1), "q128_4waves": (3, 0)}
        ts = {k: [] for k in arms}
        ref = None
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        for rnd in range(7):
            for k, (var, mha) in arms.items():
                ops.k.fls_attn_set_variant(var)
                ops.k.fls_attn_set_mha_v2(mha)
                qb = 128 if k == "q128_4waves" else 64
                wk = meta128["work"] if qb == 128 else meta["work"]
                o = ops.attention(qkv, wk, nh, nkv, hd, q_block=qb)
                if rnd == 0:
                    if ref is None:
                        ref = o.float()
                    err = (o.float() - ref).abs().max().item()
                    assert err < 2e-2, (k, err)
                ev[0].record()
                for _ in range(5):
                    ops.attention(qkv, wk, nh, nkv, hd, q_block=qb)
                ev[1].record()
                torch.cuda.synchronize()
                ts[k].append(ev[0].elapsed_time(ev[1]) / 5)
        ops.k.fls_attn_set_variant(3)
        ops.k.fls_attn_set_mha_v2(0)
        row = {k: {"ms": round(statistics.median(v[1:]), 4), "tflops": round(fl / statistics.median(v[1:]) / 1e9, 1)}
               for k, v in ts.items()}
        out[f"p{plen}"] = row
        print(json.dumps({f"p{plen}": row}), flush=True)


if __name__ == "__main__":
    main()
