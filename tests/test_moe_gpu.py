"""Mixture-of-experts kernels (csrc/kernels/moe.hip) vs plain PyTorch fp32, and MoE models through
the engine vs the fp32 oracle, on an MI355X."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():
    pytest.skip("no GPU", allow_module_level=True)

from flexible_llm_sharding_amd import _native  # noqa: E402
from flexible_llm_sharding_amd.ops.hip_backend import HipOps  # noqa: E402

DEV = torch.device("cuda", 0)


@pytest.fixture(scope="module")
def ops():
    o = HipOps()
    assert _native.loaded_libraries().get("k"), "libfls_kernels.so not loaded"
    return o


def rnd(*shape, scale=1.0, seed=0):
    g = torch.Generator(device="cpu").manual_seed(seed)
    return (torch.randn(*shape, generator=g) * scale).to(torch.float16).to(DEV)


@pytest.mark.parametrize("T,E,k,norm,r16", [(1, 4, 2, True, False), (333, 8, 2, True, False),
                                            (1000, 128, 8, False, True), (257, 256, 8, True, False),
                                            (64, 3, 3, True, False), (3000, 8, 2, True, False),
                                            (5000, 64, 8, True, False)])   # last two: multi-block sort
def test_moe_route_and_plan(ops, T, E, k, norm, r16):
    """Top-k of the fp32 softmax (any tie order), renormalised / fp16-rounded weights, and the
    plan = a stable sort of the (token, slot) entries by expert."""
    logits = rnd(T, E, seed=T + E)
    r = ops.moe_route_logits(logits, k, norm, r16)
    torch.cuda.synchronize()
    p = torch.softmax(logits.float().cpu(), -1)
    top, _ = torch.topk(p, k, -1)
    ids = r.ids.cpu().long().view(T, k)
    got_p = torch.gather(p, 1, ids)
    assert torch.allclose(got_p, top, rtol=1e-6, atol=0)                 # the k largest, best first
    assert all(len(set(row.tolist())) == k for row in ids)               # distinct experts
    want_w = top / top.sum(-1, keepdim=True) if norm else top
    if r16:
        want_w = want_w.half().float()
    # fast exp on the device: fp16-rounded weights may land one fp16 step away (2^-11 relative)
    assert torch.allclose(r.w.cpu().view(T, k), want_w, rtol=1e-3 if r16 else 1e-5, atol=1e-7)
    # plan
    flat = ids.reshape(-1)
    counts = torch.bincount(flat, minlength=E)
    offs = torch.cat([torch.zeros(1, dtype=torch.long), counts.cumsum(0)])
    assert torch.equal(r.offs.cpu().long(), offs)
    tiles = torch.cat([torch.zeros(1, dtype=torch.long), ((counts + 255) // 256).cumsum(0)])
    assert torch.equal(r.tiles.cpu().long(), tiles)
    order = torch.sort(flat, stable=True).indices                        # entries grouped by expert
    assert torch.equal(r.rows.cpu().long(), order // k)
    dest = torch.empty_like(order)
    dest[order] = torch.arange(order.numel())
    assert torch.equal(r.dest.cpu().long(), dest)


@pytest.mark.parametrize("T,H,E,k", [(1, 256, 4, 2), (777, 4096, 8, 2), (130, 2048, 64, 8), (64, 256, 16, 3)])
def test_fused_router_route(ops, T, H, E, k):
    """E <= 64: router logits computed inside the routing kernel (fp32 sums, fp16-rounded logits) ==
    torch's fp16 Linear + softmax + top-k, up to near-ties flipped by the summation order."""
    h = rnd(T, H, seed=7)
    wr = rnd(E, H, scale=H ** -0.5, seed=8)
    r = ops.moe_route(h, wr, k, True)
    torch.cuda.synchronize()
    logits = (h.float() @ wr.float().t()).half().float().cpu()
    p = torch.softmax(logits, -1)
    top, _ = torch.topk(p, k, -1)
    got = torch.gather(p, 1, r.ids.cpu().long().view(T, k))
    assert torch.allclose(got, top, rtol=2e-2, atol=1e-4)
    assert torch.allclose(r.w.cpu().view(T, k), top / top.sum(-1, keepdim=True), rtol=2e-2, atol=1e-4)
    assert int(r.offs[-1].item()) == T * k


def _torch_experts(h, x, wgu, wdown, ids, w, k):
    """HF's expert loop in fp32 math with its fp16 roundings (per-expert GEMM outputs, weighted
    contribution, fp16 accumulation in expert order, residual add)."""
    T, H = h.shape
    E, I2, _ = wgu.shape
    I = I2 // 2
    idx, ww = ids.long().view(T, k), w.view(T, k)
    acc = torch.zeros(T, H, dtype=torch.float16, device=h.device)
    for e in range(E):
        tok, slot = torch.where(idx == e)
        if tok.numel() == 0:
            continue
        gu = (h[tok].float() @ wgu[e].float().t())
        m = (torch.nn.functional.silu(gu[:, :I]) * gu[:, I:]).half()
        y = (m.float() @ wdown[e].float().t()).half()
        acc.index_add_(0, tok, (y.float() * ww[tok, slot, None]).half())
    return (x.float() + acc.float()).half()


@pytest.mark.parametrize("T,H,I,E,k", [(200, 256, 256, 4, 2),          # tiny-Mixtral geometry
                                       (1500, 512, 512, 8, 2),         # several 256-row tiles per expert
                                       (300, 256, 128, 128, 8),        # Qwen3-MoE-like: many empty experts
                                       (2, 256, 256, 8, 2),            # fewer tokens than experts
                                       (100, 256, 96, 4, 2)])          # N = 192: per-expert fallback
def test_moe_experts_match_torch(ops, T, H, I, E, k):
    h = rnd(T, H, seed=1)
    x = rnd(T, H, seed=2)
    wr = rnd(E, H, scale=H ** -0.5, seed=3)
    wgu = rnd(E, 2 * I, H, scale=0.05, seed=4)
    wdown = rnd(E, H, I, scale=0.05, seed=5)
    route = ops.moe_route(h, wr, k, True)
    out = ops.moe_experts(h, x.clone(), wgu, wdown, route)
    again = ops.moe_experts(h, x.clone(), wgu, wdown, route)
    torch.cuda.synchronize()
    assert torch.equal(out, again)                                       # deterministic
    want = _torch_experts(h, x, wgu, wdown, route.ids, route.w, k)
    d_got, d_want = (out.float() - x.float()), (want.float() - x.float())
    assert ((d_got - d_want).norm() / d_want.norm()).item() < 5e-3
    # whole op (router GEMM + routing + experts) == route + experts
    full = ops.moe_ffn(h, x.clone(), wr, wgu, wdown, k, True)
    torch.cuda.synchronize()
    assert torch.equal(full, out)
    # Qwen2-MoE: the gated shared-expert output joins the experts' fp16 sum before the residual
    sh = rnd(T, H, seed=6)
    with_sh = ops.moe_experts(h, x.clone(), wgu, wdown, route, shared=sh)
    torch.cuda.synchronize()
    acc = (out.float() - x.float())               # the experts' sum as the combine rounded it
    ref_sh = (x.float() + (acc + sh.float()).half().float()).half()
    assert ((with_sh.float() - ref_sh.float()).norm() / (ref_sh.float() - x.float()).norm()).item() < 2e-3


@pytest.mark.parametrize("lnps", [1, 3])
@pytest.mark.parametrize("family", ["tiny-mixtral", "tiny-qwen3-moe", "tiny-qwen2-moe"])
def test_moe_families_on_gpu(tmp_path, family, lnps):
    """Mixtral (8 experts -> tiny 4, top-2, renormalised), Qwen3-MoE (q/k norm, top-3 of 8,
    fp16 routing weights, no renormalisation) and Qwen2-MoE (q/k/v biases, a sigmoid-gated shared
    expert) end to end through the HIP engine vs the fp32 oracle, incl. the pruned last layer;
    storage cpu so activations cross PCIe between shards."""
    from flexible_llm_sharding_amd.config import preset
    from flexible_llm_sharding_amd.engine import ShardedRunner
    from flexible_llm_sharding_amd.models.reference import reference_scores
    from flexible_llm_sharding_amd.runtime.weights import HostStore
    from flexible_llm_sharding_amd.utils.synthetic import (load_full_state_dict, synthetic_prompts,
                                                           write_synthetic_checkpoint)
    from flexible_llm_sharding_amd.utils.tokenizer import load_tokenizer
    cfg = preset(family)
    path = str(tmp_path / family)
    write_synthetic_checkpoint(cfg, path, seed=21, std=0.05)
    tok = load_tokenizer(path)
    prompts = synthetic_prompts(5, 90, 3, 12, cfg.vocab_size, seed=22, vary=True)
    ref = reference_scores(cfg, load_full_state_dict(cfg, path), tok, prompts)
    r = ShardedRunner(cfg, HostStore.from_model_path(cfg, path), "cuda:0", tok, layer_num_per_shard=lnps,
                      storage_location="cpu")
    for o, rf in zip(r(prompts), ref):
        assert np.abs(o.astype(np.float32) - rf).max() < 3e-3
    r.close()
