"""Which op breaks bitwise row-exactness at 70B geometry (debug): the row-exact GEMMs on a subset of
rows vs the same rows inside a big launch (v10 vs v11), and the reused-step attention (range 0 + range
2 over 64-aligned cache regions, decode kernel) vs the full step's attention (range 0 + range 1,
single-suffix items) for the same query rows.

    python scripts/exact_reuse_probe.py
"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from flexible_llm_sharding_amd.config import ModelConfig  # noqa: E402
from flexible_llm_sharding_amd.models.llama import rope_tables  # noqa: E402
from flexible_llm_sharding_amd.ops.hip_backend import HipOps  # noqa: E402
from flexible_llm_sharding_amd.runtime.batch import pack_prompts  # noqa: E402
from flexible_llm_sharding_amd.runtime.prefix_cache import PrefixEntry  # noqa: E402
from flexible_llm_sharding_amd.utils.tokenizer import TokenizedPrompt  # noqa: E402

DEV = torch.device("cuda", 0)


def rnd(*shape, scale=1.0, seed=0):
    g = torch.Generator(device="cpu").manual_seed(seed)
    return (torch.randn(*shape, generator=g) * scale).half().to(DEV)


def gemms(ops):
    M, sub = 20480, 320
    H, I, nh, nkv, hd = 8192, 28672, 64, 8, 128
    x = rnd(M, H, seed=1)
    rs = (torch.rand(M, generator=torch.Generator().manual_seed(2)) + 0.5).float().to(DEV)
    cfg = ModelConfig(hidden_size=H, num_attention_heads=nh, num_key_value_heads=nkv)
    cos, sin = [t.to(DEV) for t in rope_tables(cfg, 4096)]
    pos = torch.randint(0, 4000, (M,), dtype=torch.int32, device=DEV)
    wqkv = rnd((nh + 2 * nkv) * hd, H, scale=0.02, seed=3)
    wo = rnd(H, H, scale=0.02, seed=4)
    wgu = rnd(2 * I, H, scale=0.02, seed=5)
    r0 = rnd(M, H, seed=6)
    res = {}
    with ops.row_exact(True):
        for name, fn in (("qkv_rope", lambda a, p, s: ops.qkv_rope(a, wqkv, p, cos, sin, nh, nkv, hd, rscale=s)),
                         ("o_resid", lambda a, p, s: ops.linear_residual(a, wo, r0[:a.shape[0]].clone())),
                         ("swiglu", lambda a, p, s: ops.swiglu_up(a, wgu, rscale=s)),
                         ("head", lambda a, p, s: ops.linear(a[:, :H], wo))):
            full = fn(x, pos, rs)
            part = fn(x[:sub].contiguous(), pos[:sub].contiguous(), rs[:sub].contiguous())
            torch.cuda.synchronize()
            res[name] = bool(torch.equal(full[:sub], part))
            # the 64 x 128 mid-M kernel on the same rows (not row-exact: forced by the setters)
            with ops.row_exact(False):
                old = (ops.k.fls_gemm_set_v11(0), ops.k.fls_gemm_set_skinny(0, 0), ops.k.fls_gemm_set_splitk(0))
                try:
                    mid = fn(x[:sub].contiguous(), pos[:sub].contiguous(), rs[:sub].contiguous())
                finally:
                    ops.k.fls_gemm_set_v11(old[0])
                    ops.k.fls_gemm_set_skinny(old[1], 0)
                    ops.k.fls_gemm_set_splitk(old[2])
            torch.cuda.synchronize()
            res[name + "_mid"] = bool(torch.equal(full[:sub], mid))
    return res


def attention(ops, nh, nkv, hd, n_prompts=4, lp=300, lens=(40, 70, 64, 5, 100)):
    qs, kv = nh * hd, 2 * nkv * hd
    tps = [TokenizedPrompt(list(range(lp)), [list(range(n)) for n in lens], max(lens), [n - 1 for n in lens])
           for _ in range(n_prompts)]
    offs = [j * lp for j in range(n_prompts)]
    e = PrefixEntry("k", [lp] * n_prompts, kv, DEV, torch.float16,
                    suffix_caps=[[n + 64 for n in lens] for _ in range(n_prompts)])
    cache = e.buffer("l", create=True)
    full = pack_prompts(tps, list(range(n_prompts)), "bidirectional", prefix_offsets=offs, kv_cached=True,
                        q_block=64, suffix_rows=e.sfx_rows, single_suffix_items=True)
    T = full.num_tokens
    qkv = rnd(T, qs + kv, seed=7)
    # the prefix K/V in the cache (what step 0 stored)
    pk = rnd(n_prompts * lp, kv, seed=8)
    cache[:n_prompts * lp] = pk
    # every suffix token's K/V into its region (as the full step captures them)
    src = torch.from_numpy(full.sfx_src.astype(np.int64)).to(DEV)
    dst = torch.from_numpy(full.sfx_dst.astype(np.int64)).to(DEV)
    cache[dst] = qkv[src, qs:]
    mf = full.device_tensors(DEV)
    y_full = ops.attention(qkv.clone(), mf["work"], nh, nkv, hd, kv0=cache, q_block=64, seg_lo=mf["seg_lo"])
    # reused step: only the last token of each suffix computed; the kept ones from the regions
    keep = [[n - 1 for n in lens] for _ in range(n_prompts)]
    reuse = pack_prompts(tps, list(range(n_prompts)), "bidirectional", prefix_offsets=offs, kv_cached=True,
                         q_block=8, suffix_rows=e.sfx_rows, suffix_keep=keep)
    last = torch.from_numpy(full.last_idx.astype(np.int64)).to(DEV)
    qkv_new = qkv[last].contiguous()
    mr = reuse.device_tensors(DEV)
    with ops.row_exact(True):
        y_new = ops.attention(qkv_new.clone(), mr["work"], nh, nkv, hd, kv0=cache, q_block=8, seg_lo=mr["seg_lo"],
                              work2=mr["work2"], r2win=mr["r2win"])
    torch.cuda.synchronize()
    a, b = y_full[last][:, :qs], y_new[:, :qs]
    return {"equal": bool(torch.equal(a, b)), "max_abs": float((a.float() - b.float()).abs().max()),
            "rows_differing": int((a != b).any(-1).sum()), "rows": int(a.shape[0])}


def main():
    ops = HipOps()
    print("gemms", gemms(ops), flush=True)
    for nh, nkv, hd in ((64, 8, 128), (4, 2, 64), (8, 8, 128), (16, 2, 128)):
        print("attention", (nh, nkv, hd), attention(ops, nh, nkv, hd), flush=True)


if __name__ == "__main__" and len(sys.argv) == 1:
    main()


def engine(n_layers=2, n_prompts=8, gen=4, graphs="1", prune=True, suffix_len=64, budget=49152):
    import argparse
    from flexible_llm_sharding_amd.api import generation_loop
    from flexible_llm_sharding_amd.config import preset
    from flexible_llm_sharding_amd.engine import ShardedRunner
    from flexible_llm_sharding_amd.parallel.comm import Comm
    from flexible_llm_sharding_amd.runtime.weights import HostStore
    from flexible_llm_sharding_amd.utils.synthetic import synthetic_prompts
    from flexible_llm_sharding_amd.utils.tokenizer import load_tokenizer, write_synthetic_tokenizer
    os.environ["FLS_DECODE_GRAPHS"] = graphs
    cfg = preset("llama2-70b", num_hidden_layers=n_layers)
    store = HostStore.synthetic(cfg, DEV, seed=0, fold_norms=True)
    tok_dir = f"/tmp/fls_dbg_tok_{os.getpid()}"
    write_synthetic_tokenizer(tok_dir, cfg.vocab_size)
    tok = load_tokenizer(tok_dir)
    prompts = synthetic_prompts(n_prompts, 1024, 5, suffix_len, cfg.vocab_size, seed=0)
    args = argparse.Namespace(num_gen_token=gen, data_parallel=False, num_batch=1)
    outs = {}
    for sfx in (False, True):
        r = ShardedRunner(cfg, store, DEV, tok, layer_num_per_shard=1, prefix_kv_cache=True, suffix_kv_cache=sfx,
                          resident=True, prune_last_layer=prune, token_budget=budget)
        outs[sfx] = generation_loop(args, r, Comm(0, 1, DEV), tok, prompts)
        r.close()
    (s0, u0), (s1, u1) = outs[False], outs[True]
    per_step = [bool(all(np.array_equal(a[:, t], b[:, t]) for a, b in zip(s0, s1))) for t in range(gen)]
    diff1 = [(j, si, float(np.abs(a[si, 1].astype(np.float32) - b[si, 1].astype(np.float32)).max()))
             for j, (a, b) in enumerate(zip(s0, s1)) for si in range(a.shape[0]) if not np.array_equal(a[si, 1], b[si, 1])]
    print("step1 diffs (prompt, suffix, max abs):", diff1[:40], flush=True)
    return {"layers": n_layers, "prompts": n_prompts, "budget": budget, "graphs": graphs, "prune": prune,
            "tokens_equal": u0 == u1, "steps_bitwise": per_step}


if __name__ == "__main__" and len(sys.argv) > 1 and sys.argv[1] == "engine":
    for kw in ({"n_prompts": 24}, {"n_prompts": 40}, {"n_prompts": 48}, {"n_prompts": 64, "n_layers": 4}):
        print("engine", engine(**kw), flush=True)
