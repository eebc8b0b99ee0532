"""Reference-algorithm baseline on MI355X: the reference's per-shard loop in plain PyTorch eager ops.

The reference publishes no throughput, and its pinned stack (transformers <= 4.35 eager
`LlamaDecoderLayer`) is not installed here. This script re-expresses the reference's hot path with the
same math and the same data-movement pattern, so its tokens/s on MI355X is a measured baseline for
`bench.py` on the same config (Llama-2-70B, lnps=1, storage=cpu, 32 prompts x (1024 prefix + 5 x 64)):

* per shard (= 1 layer, `utils.py:143-157`): weights H2D from pageable host tensors, one `.to()` per
  tensor, synchronous (`utils.py:121-131`; the reference additionally re-reads the file: NOT modelled,
  which favours the baseline). One random-init host layer is reused for every decoder layer (same bytes
  moved, 1.7 GB of host RAM instead of 138 GB).
* per prompt (`utils.py:223-305`): fetch activations H2D (`storage=cpu`, `utils.py:187-213`), prefix pass
  with no mask (bidirectional), suffix pass with prefix K/V expanded to n_s, concatenated
  and `repeat_kv`-materialised, additive causal mask slice from a 4096x4096 fp16 mask (`utils.py:219-221`),
  eager attention (fp32 softmax), SwiGLU MLP; activations D2H (`utils.py:159-185`).
* embed / final norm on the last real token / lm_head / fp16 softmax / D2H as `utils.py:266-291`.

Tokenisation is skipped (random ids of the tokenised shape), which also favours the baseline.
Prints one JSON line with tokens/s (same token count as bench.py: prefix + suffix tokens).
"""
import argparse
import json
import time

import torch


def rms(x, w, eps):
    v = x.float().pow(2).mean(-1, keepdim=True)
    return w * (x.float() * torch.rsqrt(v + eps)).to(x.dtype)


def rot_half(x):
    h = x.shape[-1] // 2
    return torch.cat((-x[..., h:], x[..., :h]), dim=-1)


def rope_tables(hd, n, theta, dev):
    inv = 1.0 / (theta ** (torch.arange(0, hd, 2, device=dev).float() / hd))
    f = torch.outer(torch.arange(n, device=dev).float(), inv)
    e = torch.cat((f, f), -1)
    return e.cos().half(), e.sin().half()


def decoder(x, w, pos, cos, sin, nh, nkv, hd, eps, mask=None, past=None):
    """One eager Llama decoder layer; returns (out, (k, v)) with post-RoPE k/v [B, nkv, T, hd]."""
    B, T, H = x.shape
    h = rms(x, w["in"], eps)
    q = (h @ w["q"].t()).view(B, T, nh, hd).transpose(1, 2)
    k = (h @ w["k"].t()).view(B, T, nkv, hd).transpose(1, 2)
    v = (h @ w["v"].t()).view(B, T, nkv, hd).transpose(1, 2)
    c, s = cos[pos][None, None], sin[pos][None, None]
    q = q * c + rot_half(q) * s
    k = k * c + rot_half(k) * s
    kv = (k, v)
    if past is not None:                      # suffix pass: shared prefix K/V expanded per suffix
        pk, pv = past
        k = torch.cat((pk.expand(B, -1, -1, -1), k), 2)
        v = torch.cat((pv.expand(B, -1, -1, -1), v), 2)
    rep = nh // nkv                           # repeat_kv materialises the GQA broadcast
    k = k[:, :, None].expand(B, nkv, rep, k.shape[2], hd).reshape(B, nh, k.shape[2], hd)
    v = v[:, :, None].expand(B, nkv, rep, v.shape[2], hd).reshape(B, nh, v.shape[2], hd)
    a = (q @ k.transpose(2, 3)) / hd ** 0.5
    if mask is not None:
        a = a + mask
    a = torch.softmax(a.float(), dim=-1).to(q.dtype)
    o = (a @ v).transpose(1, 2).reshape(B, T, nh * hd)
    x = x + o @ w["o"].t()
    h = rms(x, w["post"], eps)
    x = x + (torch.nn.functional.silu(h @ w["g"].t()) * (h @ w["u"].t())) @ w["d"].t()
    return x, kv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--layers", type=int, default=80)
    ap.add_argument("--hidden", type=int, default=8192)
    ap.add_argument("--inter", type=int, default=28672)
    ap.add_argument("--heads", type=int, default=64)
    ap.add_argument("--kv-heads", type=int, default=8)
    ap.add_argument("--vocab", type=int, default=32000)
    ap.add_argument("--prompts", type=int, default=32)
    ap.add_argument("--prefix-len", type=int, default=1024)
    ap.add_argument("--n-suffix", type=int, default=5)
    ap.add_argument("--suffix-len", type=int, default=64)
    ap.add_argument("--steps", type=int, default=1)
    ap.add_argument("--warmup", type=int, default=0)
    ap.add_argument("--device", default="cuda:0")
    a = ap.parse_args()
    dev = torch.device(a.device)
    H, I, nh, nkv = a.hidden, a.inter, a.heads, a.kv_heads
    hd, eps, f16 = H // nh, 1e-5, torch.float16
    g = torch.Generator().manual_seed(0)

    def rnd(*shape, std=0.02):
        return (torch.randn(*shape, generator=g) * std).to(f16)

    host_layer = {"in": torch.ones(H, dtype=f16), "post": torch.ones(H, dtype=f16),
                  "q": rnd(H, H), "k": rnd(nkv * hd, H), "v": rnd(nkv * hd, H), "o": rnd(H, H),
                  "g": rnd(I, H), "u": rnd(I, H), "d": rnd(H, I)}
    host_embed, host_head, host_norm = rnd(a.vocab, H), rnd(a.vocab, H), torch.ones(H, dtype=f16)
    Lp, ns, Ls = a.prefix_len, a.n_suffix, a.suffix_len
    ids = [(torch.randint(0, a.vocab, (1, Lp), generator=g), torch.randint(0, a.vocab, (ns, Ls), generator=g))
           for _ in range(a.prompts)]
    eos = torch.full((ns,), Ls - 1)

    def one_pass():
        maxlen = 4096
        mask = torch.full((maxlen, maxlen), torch.finfo(f16).min, device=dev, dtype=f16).triu(1)
        pos_all = torch.arange(maxlen, device=dev)
        cos, sin = rope_tables(hd, maxlen, 10000.0, dev)
        acts = [None] * a.prompts
        scores = []
        for shard in range(a.layers + 3):
            if shard == 0:
                w = host_embed.to(dev)
            elif shard <= a.layers:
                w = {k_: t.to(dev) for k_, t in host_layer.items()}
            elif shard == a.layers + 1:
                w = host_norm.to(dev)
            else:
                w = host_head.to(dev)
            for p in range(a.prompts):
                if shard == 0:
                    pre, suf = ids[p][0].to(dev), ids[p][1].to(dev)
                    xp, xs = w[pre], w[suf]
                else:
                    xp, xs = (t.to(dev) for t in acts[p])
                    if shard <= a.layers:
                        xp, kv = decoder(xp, w, pos_all[:Lp], cos, sin, nh, nkv, hd, eps)
                        xs, _ = decoder(xs, w, pos_all[Lp:Lp + Ls], cos, sin, nh, nkv, hd, eps,
                                        mask=mask[None, None, Lp:Lp + Ls, :Lp + Ls], past=kv)
                    elif shard == a.layers + 1:
                        xs = rms(xs[torch.arange(ns, device=dev), eos.to(dev)][:, None], w, eps)
                        xp = xp[:, :0]
                    else:
                        sc = torch.softmax(xs[:, 0] @ w.t(), dim=-1)
                        scores.append(sc.cpu().numpy()[:, None])
                        acts[p] = None
                        continue
                acts[p] = (xp.cpu(), xs.cpu())     # storage_location=cpu
            del w
        return scores

    for _ in range(a.warmup):
        one_pass()
    sync = (lambda: torch.cuda.synchronize(dev)) if dev.type == "cuda" else (lambda: None)
    sync()
    t0 = time.perf_counter()
    for i in range(a.steps):
        ts = time.perf_counter()
        out = one_pass()
        print(f"[ref-eager] step {i}: {time.perf_counter() - ts:.2f}s", flush=True)
    sync()
    dt = (time.perf_counter() - t0) / a.steps
    toks = a.prompts * (Lp + ns * Ls)
    finite = all(bool(abs(s).max() < float("inf")) for s in out)
    print(json.dumps({"metric": "reference-algorithm eager baseline tokens/s", "value": round(toks / dt, 2),
                      "unit": "tokens/s", "ms_per_step": round(dt * 1e3, 2), "tokens_per_step": toks,
                      "steps": a.steps, "warmup": a.warmup, "layers": a.layers, "scores_finite": finite,
                      "peak_gpu_mem_gb": round(torch.cuda.max_memory_allocated(dev) / 1e9, 3) if dev.type == "cuda" else None}))


if __name__ == "__main__":
    main()
