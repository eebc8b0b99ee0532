"""Whole-model numerics at the headline geometry: Llama-2-70B (random init, fp16 weights) scored by
the engine (lnps=1, storage=cpu, HIP kernels, fp16 activations) and by a layer-streamed fp32 PyTorch
oracle of the reference's forward (`models/reference.py` `_block`, HF weight names rebuilt from each
packed layer image through `models/layout.placements`) on the same prompts.

    python scripts/full70b_numerics.py [--prompts 2] [--prefix-len 1024] [--json out.json]

Reports, over every scored suffix: relative L2 error of the probability vectors, max |dp|, and
agreement of the top-1 / top-5 tokens.  Needs ~140 GB of pinned host RAM (the weights) and one GPU.
"""
import argparse
import json
import os
import sys
import tempfile
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from flexible_llm_sharding_amd.config import preset  # noqa: E402
from flexible_llm_sharding_amd.engine import ShardedRunner  # noqa: E402
from flexible_llm_sharding_amd.models.layout import placements  # noqa: E402
from flexible_llm_sharding_amd.models.llama import rope_tables  # noqa: E402
from flexible_llm_sharding_amd.models.reference import _block, _rms  # noqa: E402
from flexible_llm_sharding_amd.runtime.weights import HostStore  # noqa: E402
from flexible_llm_sharding_amd.utils.synthetic import synthetic_prompts  # noqa: E402
from flexible_llm_sharding_amd.utils.tokenizer import load_tokenizer, write_synthetic_tokenizer  # noqa: E402


def layer_state(cfg, store, name, dev, dtype=torch.float32):
    """HF-named tensors of one layer on ``dev`` from its packed pinned image."""
    buf = store.host_buffer(name).to(dev, non_blocking=True)
    sd = {}
    for pl in placements(cfg, name):
        t = buf[pl.offset:pl.offset + pl.numel * pl.elem_size].view(torch.float16).view(pl.shape)
        sd[pl.hf_name] = t.to(dtype)
    return sd


def _rms16(x, w, eps):
    """HF LlamaRMSNorm on fp16 input: statistics in fp32, cast back, then the fp16 weight."""
    xf = x.float()
    return w * (xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + eps)).to(torch.float16)


def _block16(x, sd, p, cfg, pos, cos, sin, mask, past_kv=None):
    """HF LlamaDecoderLayer (eager) in fp16, as the reference runs it (utils.py:272-279): fp16
    matmuls (fp32 accumulate), RMSNorm statistics and softmax in fp32, fp16 residual stream."""
    from flexible_llm_sharding_amd.models.reference import _rope
    B, T, H = x.shape
    nh, nkv, hd = cfg.num_attention_heads, cfg.num_key_value_heads, cfg.head_dim
    g = lambda n: sd[f"{p}.{n}"]
    h = _rms16(x, g("input_layernorm.weight"), cfg.rms_norm_eps)
    q = (h @ g("self_attn.q_proj.weight").t()).view(B, T, nh, hd).transpose(1, 2)
    k = (h @ g("self_attn.k_proj.weight").t()).view(B, T, nkv, hd).transpose(1, 2)
    v = (h @ g("self_attn.v_proj.weight").t()).view(B, T, nkv, hd).transpose(1, 2)
    q, k = _rope(q, pos, cos.half(), sin.half()), _rope(k, pos, cos.half(), sin.half())
    if past_kv is not None:
        k = torch.cat([past_kv[0], k], 2)
        v = torch.cat([past_kv[1], v], 2)
    present = (k, v)
    rep = nh // nkv
    s = q @ k.repeat_interleave(rep, 1).transpose(2, 3) / (hd ** 0.5)
    if mask is not None:
        s = s + mask.half()
    a = torch.softmax(s, -1, dtype=torch.float32).to(torch.float16) @ v.repeat_interleave(rep, 1)
    x = x + a.transpose(1, 2).reshape(B, T, nh * hd) @ g("self_attn.o_proj.weight").t()
    h = _rms16(x, g("post_attention_layernorm.weight"), cfg.rms_norm_eps)
    m = torch.nn.functional.silu(h @ g("mlp.gate_proj.weight").t()) * (h @ g("mlp.up_proj.weight").t())
    return x + m @ g("mlp.down_proj.weight").t(), present


@torch.no_grad()
def oracle(cfg, store, tok, prompts, dev, max_len=4096, fp16=False):
    """Reference forward (utils.py:246-290 semantics: bidirectional prefix, padded suffix batch
    against the expanded prefix K/V, suffix_eos gather), streamed one layer at a time: fp32
    throughout, or (``fp16``) the reference's own fp16 eager arithmetic."""
    dt = torch.float16 if fp16 else torch.float32
    blk = _block16 if fp16 else _block
    cos, sin = rope_tables(cfg, max_len)
    cos, sin = cos.to(dev), sin.to(dev)
    neg = torch.finfo(torch.float32).min
    st = []
    emb = layer_state(cfg, store, "model.embed_tokens", dev, dt)["model.embed_tokens.weight"]
    for prefix, suffixes in prompts:
        pids = torch.tensor(tok(prefix, truncation=True, max_length=max_len)["input_ids"])[None].to(dev)
        sids = torch.tensor(tok(list(suffixes), truncation=True, max_length=max_len,
                                padding=True)["input_ids"])[:, 1:].to(dev)
        eos = (sids != tok.pad_token_id).sum(1) - 1
        Lp, Ls, ns = pids.shape[1], sids.shape[1], sids.shape[0]
        full = torch.full((Lp + Ls, Lp + Ls), neg if not fp16 else -65504.0, device=dev).triu(1)
        st.append(dict(P=emb[pids], S=emb[sids], eos=eos, ns=ns,
                       ppos=torch.arange(Lp, device=dev)[None],
                       spos=torch.arange(Lp, Lp + Ls, device=dev)[None].expand(ns, -1),
                       smask=full[-Ls:, -(Lp + Ls):][None, None].expand(ns, 1, Ls, Lp + Ls)))
    del emb
    for i in range(cfg.num_hidden_layers):
        p = f"model.layers.{i}"
        sd = layer_state(cfg, store, p, dev, dt)
        for s in st:
            s["P"], (kc, vc) = blk(s["P"], sd, p, cfg, s["ppos"], cos, sin, None)
            kv = (kc.expand(s["ns"], -1, -1, -1), vc.expand(s["ns"], -1, -1, -1))
            s["S"], _ = blk(s["S"], sd, p, cfg, s["spos"], cos, sin, s["smask"], past_kv=kv)
        del sd
    norm = layer_state(cfg, store, "model.norm", dev, dt)["model.norm.weight"]
    head = layer_state(cfg, store, "lm_head", dev, dt)["lm_head.weight"]
    outs = []
    for s in st:
        last = s["S"][torch.arange(s["ns"], device=dev), s["eos"]]
        hn = _rms16(last, norm, cfg.rms_norm_eps) if fp16 else _rms(last, norm, cfg.rms_norm_eps)
        outs.append(torch.softmax((hn @ head.t()).float(), -1).to(dt).float().cpu().numpy())
    return outs


def compare(ours, ref):
    rel, mx, top1, top5, n = [], 0.0, 0, 0, 0
    for o, x in zip(ours, ref):
        o = o.reshape(o.shape[0], -1).astype(np.float64)
        x = x.reshape(x.shape[0], -1).astype(np.float64)
        for j in range(o.shape[0]):
            rel.append(float(np.linalg.norm(o[j] - x[j]) / np.linalg.norm(x[j])))
            mx = max(mx, float(np.abs(o[j] - x[j]).max()))
            top1 += int(o[j].argmax() == x[j].argmax())
            top5 += len(set(np.argsort(-o[j])[:5]) & set(np.argsort(-x[j])[:5]))
            n += 1
    return {"rel_l2_err_max": max(rel), "rel_l2_err_mean": float(np.mean(rel)), "max_abs_prob_err": mx,
            "top1_agree": top1 / n, "top5_overlap": top5 / (5 * n), "scored_suffixes": n}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--prompts", type=int, default=2)
    ap.add_argument("--prefix-len", type=int, default=1024)
    ap.add_argument("--suffix-len", type=int, default=64)
    ap.add_argument("--json", default=None)
    ap.add_argument("--model", default="llama2-70b")
    ap.add_argument("--cpu", action="store_true", help="plumbing check on the CPU backend (tiny models)")
    a = ap.parse_args()
    dev = torch.device("cpu") if a.cpu else torch.device("cuda", 0)
    cfg = preset(a.model)
    t0 = time.time()
    store = HostStore.synthetic(cfg, dev, seed=0, pinned=not a.cpu)
    print(f"weights {store.total_bytes / 1e9:.1f} GB in {time.time() - t0:.0f}s", flush=True)
    d = tempfile.mkdtemp(prefix="fls_tok_")
    write_synthetic_tokenizer(d, cfg.vocab_size)
    tok = load_tokenizer(d)
    prompts = synthetic_prompts(a.prompts, a.prefix_len, 5, a.suffix_len, cfg.vocab_size, seed=7, vary=True)
    r = ShardedRunner(cfg, store, dev, tok, layer_num_per_shard=1, storage_location="cpu")
    t0 = time.time()
    ours = r(prompts)
    if not a.cpu:
        torch.cuda.synchronize()
    print(f"engine {time.time() - t0:.1f}s", flush=True)
    r.close()
    if not a.cpu:
        torch.cuda.empty_cache()
    t0 = time.time()
    ref = oracle(cfg, store, tok, prompts, dev)
    print(f"fp32 oracle {time.time() - t0:.1f}s", flush=True)
    t0 = time.time()
    ref16 = oracle(cfg, store, tok, prompts, dev, fp16=True) if not a.cpu else ref
    print(f"fp16 eager (reference arithmetic) {time.time() - t0:.1f}s", flush=True)
    res = {"model": f"{a.model} (random init, std 0.02)", "prompts": a.prompts,
           "prefix_len_max": a.prefix_len, "suffix_len_max": a.suffix_len,
           "ref_max_prob": float(max(x.max() for x in ref)),
           "engine_vs_fp32": compare(ours, ref),
           "reference_fp16_eager_vs_fp32": compare(ref16, ref),
           "engine_vs_reference_fp16_eager": compare(ours, ref16)}
    print(json.dumps(res), flush=True)
    if a.json:
        with open(a.json, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
