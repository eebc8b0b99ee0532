"""HIP kernel numerics vs plain-PyTorch fp32 references (run on an MI355X)."""
import math

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():
    pytest.skip("no GPU", allow_module_level=True)

from flexible_llm_sharding_amd.ops.hip_backend import HipOps, EPI_NONE, EPI_RESID, EPI_SWIGLU, EPI_ROPE  # noqa: E402
from flexible_llm_sharding_amd.ops.torch_backend import TorchOps  # noqa: E402
from flexible_llm_sharding_amd import _native  # noqa: E402

DEV = torch.device("cuda", 0)


@pytest.fixture(scope="module")
def ops():
    o = HipOps()
    assert _native.loaded_libraries().get("k"), "libfls_kernels.so not loaded"
    return o


@pytest.fixture(scope="module")
def ref():
    return TorchOps(torch.float32)


def rnd(*shape, scale=1.0, seed=0):
    g = torch.Generator(device="cpu").manual_seed(seed)
    return (torch.randn(*shape, generator=g) * scale).to(torch.float16).to(DEV)


def rel_err(a, b):
    a, b = a.float(), b.float()
    return ((a - b).norm() / (b.norm() + 1e-12)).item()


@pytest.mark.parametrize("M,N,K", [(256, 256, 64), (300, 512, 256), (1, 256, 128), (517, 768, 192),
                                   (64, 96, 40), (33, 48, 100), (1024, 1024, 1024)])
def test_gemm_plain(ops, M, N, K):
    x = rnd(M, K, seed=1)
    w = rnd(N, K, scale=0.05, seed=2)
    y = ops.gemm(x, w)
    torch.cuda.synchronize()
    r = x.float() @ w.float().t()
    assert rel_err(y, r) < 2e-3


def test_gemm_asymmetric_exact(ops):
    # A = identity-like, asymmetric B: catches transposed C writes (guide §3 check)
    M = N = K = 256
    x = torch.eye(M, K, dtype=torch.float16, device=DEV)
    w = (torch.arange(N * K, device=DEV).reshape(N, K) % 17).to(torch.float16)
    y = ops.gemm(x, w)
    torch.cuda.synchronize()
    assert torch.equal(y, w.t().contiguous())


@pytest.mark.parametrize("M,N,K", [(300, 512, 256), (40, 96, 64)])
def test_gemm_resid_inplace(ops, M, N, K):
    x = rnd(M, K, seed=3)
    w = rnd(N, K, scale=0.05, seed=4)
    r0 = rnd(M, N, seed=5)
    ref_out = r0.float() + x.float() @ w.float().t()
    r = r0.clone()
    out = ops.linear_residual(x, w, r)
    torch.cuda.synchronize()
    assert out.data_ptr() == r.data_ptr()
    assert rel_err(out, ref_out) < 2e-3


@pytest.mark.parametrize("M,I,K", [(300, 256, 256), (70, 48, 64)])
def test_gemm_swiglu(ops, ref, M, I, K):
    x = rnd(M, K, seed=6)
    wgu = rnd(2 * I, K, scale=0.05, seed=7)
    y = ops.swiglu_up(x, wgu)
    r = ref.swiglu_up(x.float().cpu(), wgu.float().cpu())
    torch.cuda.synchronize()
    assert rel_err(y.cpu(), r) < 3e-3


@pytest.mark.parametrize("nh,nkv,hd,M", [(4, 2, 64, 300), (2, 1, 128, 257), (8, 8, 128, 64), (4, 4, 96, 300)])
def test_gemm_rope(ops, ref, nh, nkv, hd, M):
    from flexible_llm_sharding_amd.config import ModelConfig
    from flexible_llm_sharding_amd.models.llama import rope_tables
    H = 256
    cfg = ModelConfig(hidden_size=nh * hd, num_attention_heads=nh, num_key_value_heads=nkv)
    N = (nh + 2 * nkv) * hd
    x = rnd(M, H, seed=8)
    w = rnd(N, H, scale=0.05, seed=9)
    pos = torch.randint(0, 4000, (M,), dtype=torch.int32, device=DEV)
    cos, sin = rope_tables(cfg, 4096)
    y = ops.qkv_rope(x, w, pos, cos.to(DEV), sin.to(DEV), nh, nkv, hd)
    r = ref.qkv_rope(x.float().cpu(), w.float().cpu(), pos.cpu(), cos, sin, nh, nkv, hd)
    torch.cuda.synchronize()
    assert rel_err(y.cpu(), r) < 3e-3


def _attn_case(nh, nkv, hd, prompts, prefix_attention, seed=0, q_block=64):
    from flexible_llm_sharding_amd.runtime.batch import pack_prompts
    from flexible_llm_sharding_amd.utils.tokenizer import TokenizedPrompt
    g = torch.Generator().manual_seed(seed)
    tps = []
    for lp, lens in prompts:
        tps.append(TokenizedPrompt(list(range(lp)), [list(range(l)) for l in lens], max(lens), [l - 1 for l in lens]))
    b = pack_prompts(tps, list(range(len(tps))), prefix_attention, q_block=q_block)
    T = b.num_tokens
    qkv = (torch.randn(T, (nh + 2 * nkv) * hd, generator=g)).to(torch.float16)
    return b, qkv


@pytest.mark.parametrize("nh,nkv,hd", [(4, 4, 128), (6, 2, 64), (4, 2, 128), (3, 3, 64), (4, 4, 96)])
@pytest.mark.parametrize("mode", ["bidirectional", "causal"])
def test_attention_128_row_items(ops, ref, nh, nkv, hd, mode):
    """128-row work items (multi-head models): 4 waves per query head share each K/V tile;
    ragged segments (1..200 rows) cross the 128-row boundary."""
    prompts = [(70, [5, 64, 1]), (1, [3]), (130, [65, 17, 129]), (200, [33, 64])]
    b, qkv = _attn_case(nh, nkv, hd, prompts, mode, q_block=128)
    assert int(b.work[:, 1].max()) == 128
    meta = b.device_tensors(DEV)
    y = ops.attention(qkv.to(DEV), meta["work"], nh, nkv, hd, q_block=128, seg_lo=meta["seg_lo"])
    r = ref.attention(qkv.float(), b.segments, nh, nkv, hd)
    torch.cuda.synchronize()
    assert rel_err(y.cpu(), r) < 5e-3


@pytest.mark.parametrize("nh,nkv,hd", [(4, 2, 64), (8, 1, 128), (2, 2, 128), (16, 2, 128), (12, 2, 64),
                                        (4, 4, 96), (4, 2, 96)])
@pytest.mark.parametrize("mode", ["bidirectional", "causal"])
def test_attention_shared_prefix(ops, ref, nh, nkv, hd, mode):
    prompts = [(70, [5, 64, 1]), (1, [3]), (130, [65, 17, 129]), (200, [33, 64])]
    b, qkv = _attn_case(nh, nkv, hd, prompts, mode)
    meta = b.device_tensors(DEV)
    y = ops.attention(qkv.to(DEV), meta["work"], nh, nkv, hd, seg_lo=meta["seg_lo"])
    r = ref.attention(qkv.float(), b.segments, nh, nkv, hd)
    torch.cuda.synchronize()
    assert rel_err(y.cpu(), r) < 5e-3


@pytest.mark.parametrize("nh,nkv,hd", [(8, 1, 128), (2, 2, 128), (4, 2, 64), (4, 4, 96)])
def test_attention_prefix_from_cache(ops, ref, nh, nkv, hd):
    """Range 0 read from a separate prefix K/V tensor (prefix cache) == the full packed pass."""
    from flexible_llm_sharding_amd.runtime.batch import pack_prompts
    from flexible_llm_sharding_amd.utils.tokenizer import TokenizedPrompt
    prompts = [(70, [5, 64, 1]), (130, [65, 17]), (9, [3, 40])]
    tps = [TokenizedPrompt(list(range(lp)), [list(range(l)) for l in ls], max(ls), [l - 1 for l in ls])
           for lp, ls in prompts]
    offs, t = [], 0
    for lp, _ in prompts:
        offs.append(t)
        t += lp
    full = pack_prompts(tps, [0, 1, 2], "bidirectional", prefix_offsets=offs)
    g = torch.Generator().manual_seed(5)
    qkv = torch.randn(full.num_tokens, (nh + 2 * nkv) * hd, generator=g).half()
    qs, kv = nh * hd, 2 * nkv * hd
    cache = torch.zeros(t, kv, dtype=torch.float16)
    cache[torch.from_numpy(full.pfx_dst)] = qkv[torch.from_numpy(full.pfx_src), qs:qs + kv]
    cached = pack_prompts(tps, [0, 1, 2], "bidirectional", prefix_offsets=offs, kv_cached=True)
    keep = np.setdiff1d(np.arange(full.num_tokens), full.pfx_src)       # suffix rows, in packed order
    qkv_s = qkv[torch.from_numpy(keep)].contiguous()
    cm = cached.device_tensors(DEV)
    y = ops.attention(qkv_s.to(DEV), cm["work"], nh, nkv, hd, kv0=cache.to(DEV), seg_lo=cm["seg_lo"])
    r = ref.attention(qkv.float(), full.segments, nh, nkv, hd)[torch.from_numpy(keep)]
    torch.cuda.synchronize()
    assert rel_err(y.cpu(), r) < 5e-3


@pytest.mark.parametrize("nh,nkv,hd,q_block", [(64, 8, 128, 64), (8, 2, 128, 64), (4, 4, 128, 128), (8, 1, 128, 64),
                                              (8, 2, 64, 64), (4, 4, 64, 128), (12, 2, 64, 64)])
@pytest.mark.parametrize("mode", ["bidirectional", "causal"])
@pytest.mark.parametrize("cached", [False, True])
def test_attention_persistent_bitwise(ops, ref, nh, nkv, hd, q_block, mode, cached):
    """The persistent full-pass kernel (a grid of about one block per CU walking (work item, head
    group) units, the K/V tile pipeline and the next unit's Q load running across unit boundaries)
    == one block per unit, bitwise, on ragged prompts, multi-suffix items, padding items (q_len 0)
    and range 0 from a prefix K/V cache; and == the fp32 oracle."""
    from flexible_llm_sharding_amd.runtime.batch import pack_prompts
    from flexible_llm_sharding_amd.utils.tokenizer import TokenizedPrompt
    prompts = [(70, [5, 64, 1]), (1, [3]), (130, [65, 17, 129]), (200, [33, 64]), (1024, [64] * 5), (40, [30] * 5)]
    tps = [TokenizedPrompt(list(range(lp)), [list(range(l)) for l in ls], max(ls), [l - 1 for l in ls])
           for lp, ls in prompts]
    offs, t = [], 0
    for lp, _ in prompts:
        offs.append(t)
        t += lp
    full = pack_prompts(tps, list(range(len(tps))), mode, prefix_offsets=offs, q_block=q_block)
    g = torch.Generator().manual_seed(17)
    qkv = torch.randn(full.num_tokens, (nh + 2 * nkv) * hd, generator=g).half()
    r = ref.attention(qkv.float(), full.segments, nh, nkv, hd)
    kw = {}
    if cached and mode == "bidirectional":
        qs, kv = nh * hd, 2 * nkv * hd
        cache = torch.zeros(t, kv, dtype=torch.float16)
        cache[torch.from_numpy(full.pfx_dst)] = qkv[torch.from_numpy(full.pfx_src), qs:qs + kv]
        b = pack_prompts(tps, list(range(len(tps))), mode, prefix_offsets=offs, kv_cached=True, q_block=q_block)
        keep = torch.from_numpy(np.setdiff1d(np.arange(full.num_tokens), full.pfx_src))
        q, r = qkv[keep].contiguous(), r[keep]
        kw["kv0"] = cache.to(DEV)
    else:
        b, q = full, qkv
    meta = b.device_tensors(DEV)
    work = torch.cat([meta["work"], torch.zeros(3, 8, dtype=torch.int32, device=DEV)])   # padding items
    q = q.to(DEV)
    old = ops.k.fls_attention_set_persistent(1)
    try:
        y = ops.attention(q, work, nh, nkv, hd, q_block=q_block, seg_lo=meta["seg_lo"], **kw)
        ops.k.fls_attention_set_persistent(0)
        y0 = ops.attention(q, work, nh, nkv, hd, q_block=q_block, seg_lo=meta["seg_lo"], **kw)
    finally:
        ops.k.fls_attention_set_persistent(old)
    torch.cuda.synchronize()
    assert torch.equal(y, y0)
    assert rel_err(y.cpu(), r) < 5e-3


def test_attention_softmax_spike(ops, ref):
    # force the online-softmax rescale path: one huge key late in the sequence
    nh, nkv, hd = 2, 1, 128
    b, qkv = _attn_case(nh, nkv, hd, [(200, [40])], "bidirectional", seed=3)
    qs = nh * hd
    qkv[150, qs:qs + hd] = 8.0          # key 150 of the prefix
    qkv[:, :qs] = qkv[:, :qs].clamp(-1, 1) + 0.5
    meta = b.device_tensors(DEV)
    y = ops.attention(qkv.to(DEV), meta["work"], nh, nkv, hd, seg_lo=meta["seg_lo"])
    r = ref.attention(qkv.float(), b.segments, nh, nkv, hd)
    torch.cuda.synchronize()
    assert torch.isfinite(y).all()
    assert rel_err(y.cpu(), r) < 5e-3


@pytest.mark.parametrize("q_block", [64, 128])
@pytest.mark.parametrize("nh,nkv,hd", [(8, 2, 128), (4, 4, 128), (4, 2, 64), (4, 4, 96)])
def test_attention_multi_suffix_items(ops, ref, q_block, nh, nkv, hd):
    """Work items holding several suffixes of one prompt (short suffixes, one crossing an item
    boundary): block-diagonal range 1 via seg_lo; the same rows computed with one suffix per item
    (runtime.batch._work_items) give the same result."""
    from flexible_llm_sharding_amd.runtime.batch import _work_items
    prompts = [(100, [3, 5, 1, 10, 7, 2, 60, 9]), (40, [30, 30, 30, 30, 30]), (1, [1, 2])]
    b, qkv = _attn_case(nh, nkv, hd, prompts, "bidirectional", seed=21, q_block=q_block)
    assert (b.work[:, 7] > b.work[:, 1]).any() or (b.work[:, 2] > 0).any()    # items span suffixes
    meta = b.device_tensors(DEV)
    q = qkv.to(DEV)
    y = ops.attention(q, meta["work"], nh, nkv, hd, q_block=q_block, seg_lo=meta["seg_lo"])
    single = torch.from_numpy(_work_items(b.segments, q_block)).to(DEV)
    y1 = ops.attention(q, single, nh, nkv, hd, q_block=q_block, seg_lo=meta["seg_lo"])
    r = ref.attention(qkv.float(), b.segments, nh, nkv, hd)
    torch.cuda.synchronize()
    assert rel_err(y.cpu(), r) < 5e-3
    assert rel_err(y1.cpu(), r) < 5e-3


@pytest.mark.parametrize("q_block", [64, 128])
def test_attention_softmax_ramp(ops, ref, q_block):
    """Scores that grow along the keys, tile after tile, by a little more or a little less than the
    deferred-rescale threshold (2^8): v4 alternates between keeping the old running max (P up to
    256) and rescaling O and l; both paths must agree with the fp32 reference."""
    nh, nkv, hd = 4, 2 if q_block == 64 else 4, 128
    b, qkv = _attn_case(nh, nkv, hd, [(600, [64, 40]), (300, [130])], "bidirectional", seed=9, q_block=q_block)
    qs = nh * hd
    T = qkv.shape[0]
    ramp = torch.linspace(0.0, 6.0, T).unsqueeze(1)
    qkv[:, :qs] = 0.25
    qkv[:, qs:qs + nkv * hd] = ramp + 0.05 * qkv[:, qs:qs + nkv * hd]
    meta = b.device_tensors(DEV)
    y = ops.attention(qkv.to(DEV), meta["work"], nh, nkv, hd, q_block=q_block, seg_lo=meta["seg_lo"])
    r = ref.attention(qkv.float(), b.segments, nh, nkv, hd)
    torch.cuda.synchronize()
    assert torch.isfinite(y).all()
    assert rel_err(y.cpu(), r) < 5e-3


@pytest.mark.parametrize("H", [256, 4096, 8192, 5120])
def test_rmsnorm(ops, ref, H):
    x = rnd(37, H, scale=3.0, seed=11)
    w = rnd(H, scale=0.5, seed=12)
    y = ops.rmsnorm(x, w, 1e-5)
    r = ref.rmsnorm(x.cpu(), w.cpu(), 1e-5)
    torch.cuda.synchronize()
    assert (y.cpu().float() - r.float()).abs().max().item() < 2e-2


def test_gather_rmsnorm(ops, ref):
    x = rnd(50, 1024, seed=13)
    w = rnd(1024, seed=14)
    idx = torch.tensor([3, 49, 0, 7], dtype=torch.int32)
    y = ops.gather_rmsnorm(x, idx.to(DEV), w, 1e-6)
    r = ref.gather_rmsnorm(x.cpu(), idx, w.cpu(), 1e-6)
    torch.cuda.synchronize()
    assert (y.cpu().float() - r.float()).abs().max().item() < 2e-2


def test_embed(ops):
    table = rnd(1000, 512, seed=15)
    ids = torch.randint(0, 1000, (77,), dtype=torch.int32, device=DEV)
    y = ops.embed(ids, table, torch.float16)
    torch.cuda.synchronize()
    assert torch.equal(y, table[ids.long()])


@pytest.mark.parametrize("V", [32000, 1000, 37])
def test_softmax(ops, V):
    x = rnd(9, V, scale=4.0, seed=16)
    y = ops.softmax(x)
    r = torch.softmax(x.float(), -1)
    torch.cuda.synchronize()
    assert (y.float() - r).abs().max().item() < 1e-3
    assert abs(y.float().sum(-1) - 1).max().item() < 1e-2


def test_fill_random(ops):
    buf = torch.empty(1 << 20, dtype=torch.float16, device=DEV)
    _native.kernels().fls_fill_random(buf.data_ptr(), buf.numel(), 7, 0.0, 1.0,
                                      torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    f = buf.float()
    assert abs(f.mean().item()) < 0.01 and abs(f.std().item() - 1) < 0.01


@pytest.mark.parametrize("M", [17, 100, 517])
def test_gemm_mid_rope64(ops, ref, M):
    """mid-M kernel, RoPE epilogue with head_dim 64 (partner column 2 subtiles away) vs fp32."""
    from flexible_llm_sharding_amd.config import ModelConfig
    from flexible_llm_sharding_amd.models.llama import rope_tables
    H, nh, nkv, hd = 512, 8, 2, 64
    x = rnd(M, H, seed=51)
    wqkv = rnd((nh + 2 * nkv) * hd, H, scale=0.05, seed=52)
    pos = torch.randint(0, 4000, (M,), dtype=torch.int32, device=DEV)
    cfg = ModelConfig(hidden_size=nh * hd, num_attention_heads=nh, num_key_value_heads=nkv)
    cos, sin = rope_tables(cfg, 4096)
    y = ops.gemm(x, wqkv, EPI_ROPE, positions=pos, cos=cos.to(DEV), sin=sin.to(DEV),
                 rope_cols=(nh + nkv) * hd, head_dim=hd)
    r = ref.qkv_rope(x.float().cpu(), wqkv.float().cpu(), pos.cpu(), cos, sin, nh, nkv, hd)
    assert rel_err(y.cpu(), r) < 3e-3


@pytest.mark.parametrize("M", [1, 17, 64, 100, 416, 517, 1000])
def test_gemm_mid_all_epilogues(ops, ref, M):
    """64x128-tile mid-M kernel (chosen when 256x256 tiles cannot fill the chip) vs fp32 references."""
    from flexible_llm_sharding_amd.config import ModelConfig
    from flexible_llm_sharding_amd.models.llama import rope_tables
    H, I, nh, nkv, hd = 512, 768, 4, 2, 128
    x = rnd(M, H, seed=41)
    w = rnd(H, H, scale=0.05, seed=42)
    assert rel_err(ops.gemm(x, w), x.float() @ w.float().t()) < 2e-3
    r0 = rnd(M, H, seed=43)
    out = ops.gemm(x, w, EPI_RESID, out=r0.clone(), resid=r0.clone())
    assert rel_err(out, r0.float() + x.float() @ w.float().t()) < 2e-3
    wgu = rnd(2 * I, H, scale=0.05, seed=44)
    assert rel_err(ops.gemm(x, wgu, EPI_SWIGLU).cpu(), ref.swiglu_up(x.float().cpu(), wgu.float().cpu())) < 3e-3
    wqkv = rnd((nh + 2 * nkv) * hd, H, scale=0.05, seed=45)
    pos = torch.randint(0, 4000, (M,), dtype=torch.int32, device=DEV)
    cfg = ModelConfig(hidden_size=nh * hd, num_attention_heads=nh, num_key_value_heads=nkv)
    cos, sin = rope_tables(cfg, 4096)
    y = ops.gemm(x, wqkv, EPI_ROPE, positions=pos, cos=cos.to(DEV), sin=sin.to(DEV),
                 rope_cols=(nh + nkv) * hd, head_dim=hd)
    r = ref.qkv_rope(x.float().cpu(), wqkv.float().cpu(), pos.cpu(), cos, sin, nh, nkv, hd)
    assert rel_err(y.cpu(), r) < 3e-3
    # bias epilogue (Qwen2) and exactness of the fragment orientation
    b = rnd(H, scale=0.5, seed=46)
    yb = ops.gemm(x, w, bias=b)
    assert rel_err(yb, x.float() @ w.float().t() + b.float()) < 2e-3
    torch.cuda.synchronize()


def test_gemm_mid_asymmetric_exact(ops):
    M, N, K = 100, 256, 128
    x = torch.eye(M, K, dtype=torch.float16, device=DEV)
    w = (torch.arange(N * K, device=DEV).reshape(N, K) % 17).to(torch.float16)
    y = ops.gemm(x, w)
    torch.cuda.synchronize()
    assert torch.equal(y, w.t().contiguous()[:M])


def test_gemm_main_all_epilogues(ops, ref):
    """The main kernel (v10) against fp32 references, with all four epilogues and a ragged M."""
    from flexible_llm_sharding_amd.config import ModelConfig
    from flexible_llm_sharding_amd.models.llama import rope_tables
    M, H, I, nh, nkv, hd = 517, 512, 768, 4, 2, 128
    ops.k.fls_gemm_set_mid(0)           # these shapes would otherwise take the 64x128 mid-M kernel
    try:
        x = rnd(M, H, seed=31)
        w = rnd(H, H, scale=0.05, seed=32)
        assert rel_err(ops.gemm(x, w), x.float() @ w.float().t()) < 2e-3
        r0 = rnd(M, H, seed=33)
        out = ops.gemm(x, w, EPI_RESID, out=r0.clone(), resid=r0.clone())
        assert rel_err(out, r0.float() + x.float() @ w.float().t()) < 2e-3
        wgu = rnd(2 * I, H, scale=0.05, seed=34)
        assert rel_err(ops.gemm(x, wgu, EPI_SWIGLU).cpu(), ref.swiglu_up(x.float().cpu(), wgu.float().cpu())) < 3e-3
        wqkv = rnd((nh + 2 * nkv) * hd, H, scale=0.05, seed=35)
        pos = torch.randint(0, 4000, (M,), dtype=torch.int32, device=DEV)
        cfg = ModelConfig(hidden_size=nh * hd, num_attention_heads=nh, num_key_value_heads=nkv)
        cos, sin = rope_tables(cfg, 4096)
        y = ops.gemm(x, wqkv, EPI_ROPE, positions=pos, cos=cos.to(DEV), sin=sin.to(DEV),
                     rope_cols=(nh + nkv) * hd, head_dim=hd)
        r = ref.qkv_rope(x.float().cpu(), wqkv.float().cpu(), pos.cpu(), cos, sin, nh, nkv, hd)
        assert rel_err(y.cpu(), r) < 3e-3
        torch.cuda.synchronize()
    finally:
        ops.k.fls_gemm_set_mid(1)


@pytest.mark.parametrize("hd", [128, 64])
def test_gemm_row_exact_small_m_bitwise(ops, ref, hd):
    """Row-exact small-M GEMMs (generation steps): every row of M = 1 / 17 / 64 / 160 / 320 equals,
    bit for bit, the same row of a 1,000-row row-exact GEMM, with the mid-M kernel's 64-column
    blocks and its 128-column blocks of 4 and 8 waves, 64 and 128 rows (bitwise equal to each other), for all four epilogues incl. bias, per-row scale
    and RoPE (both head sizes); and the fp32 reference."""
    from flexible_llm_sharding_amd.config import ModelConfig
    from flexible_llm_sharding_amd.models.llama import rope_tables
    Mb, H, I, nh, nkv = 1000, 1024, 1536, 8, 2
    x = rnd(Mb, H, seed=61)
    rs = (torch.rand(Mb, device=DEV) + 0.5).float()
    wo = rnd(H, H, scale=0.03, seed=62)
    r0 = rnd(Mb, H, seed=63)
    wgu = rnd(2 * I, H, scale=0.03, seed=64)
    wqkv = rnd((nh + 2 * nkv) * hd, H, scale=0.03, seed=65)
    bq = rnd((nh + 2 * nkv) * hd, scale=0.5, seed=66)
    pos = torch.randint(0, 4000, (Mb,), dtype=torch.int32, device=DEV)
    cfg = ModelConfig(hidden_size=nh * hd, num_attention_heads=nh, num_key_value_heads=nkv)
    cos, sin = rope_tables(cfg, 4096)
    cos, sin = cos.to(DEV), sin.to(DEV)

    def run(rows):
        xs, p, r = x[rows].contiguous(), pos[rows].contiguous(), rs[rows].contiguous()
        return [ops.gemm(xs, wo),
                ops.gemm(xs, wo, EPI_RESID, out=r0[rows].clone(), resid=r0[rows].clone(), rscale=r),
                ops.gemm(xs, wgu, EPI_SWIGLU, rscale=r),
                ops.gemm(xs, wqkv, EPI_ROPE, positions=p, cos=cos, sin=sin, rope_cols=(nh + nkv) * hd,
                         head_dim=hd, bias=bq, rscale=r)]

    # the mid kernel's 32-column blocks (plain / residual epilogues), 64-column blocks (4 / 8 waves), and
    # 128-column blocks of 4 and of 8 waves (64 / 128 rows)
    arms = ((128, 4, 0), (128, 8, 64), (128, 8, 128), (64, 4, 0), (64, 8, 0), (32, 8, 0))

    def forced(bn, waves, rows, fn):
        old = (ops.k.fls_gemm_set_mid_bn(bn), ops.k.fls_gemm_set_mid_waves(waves),
               ops.k.fls_gemm_set_mid_rows(rows))
        try:
            return fn()
        finally:
            ops.k.fls_gemm_set_mid_bn(old[0])
            ops.k.fls_gemm_set_mid_waves(old[1])
            ops.k.fls_gemm_set_mid_rows(old[2])

    with ops.row_exact():
        full = run(torch.arange(Mb, device=DEV))
        for arm in arms:
            for a, b in zip(forced(*arm, lambda: run(torch.arange(Mb, device=DEV))), full):
                assert torch.equal(a, b), arm
        g = torch.Generator().manual_seed(5)
        for m in (1, 17, 64, 160, 320):
            rows = torch.randperm(Mb, generator=g)[:m].to(DEV)
            for arm in arms:
                for a, b in zip(forced(*arm, lambda: run(rows)), full):
                    assert torch.equal(a, b[rows]), (m, arm)
    torch.cuda.synchronize()
    assert rel_err(full[0], x.float() @ wo.float().t()) < 2e-3
    assert rel_err(full[2].cpu(), ref.swiglu_up((x.float() * rs[:, None]).cpu(), wgu.float().cpu())) < 3e-3


def test_row_ss_matches_residual_epilogue(ops):
    """fls_row_ss on a hidden state == the partial sums of squares the residual GEMM epilogue wrote
    for the same rows (v10 / v11 tiles and the mid-M kernel + ss_partials), bit for bit, and the
    statistic from them equals the fp32 RMS to rounding: a row's norm statistic does not depend on
    whether its partials survived (pipeline hand-off, grouped attention, pruned last layer)."""
    H = 1024
    for M in (5000, 300, 7):                  # main tiles / mid-M / mid-M (few rows)
        a = rnd(M, 512, seed=71)
        w = rnd(H, 512, scale=0.05, seed=72)
        r = rnd(M, H, seed=73)
        ss = torch.zeros(M, H // 128, dtype=torch.float32, device=DEV)
        out = ops.linear_residual(a, w, r.clone(), ss=ss)
        got = ops.row_ss(out)
        torch.cuda.synchronize()
        assert torch.equal(got, ss), M
        want = (out.float() ** 2).reshape(M, H // 128, 128).sum(-1)
        assert torch.allclose(got, want, rtol=1e-4, atol=1e-3)
        # the fused statistic == partials + rstd_from_ss, bit for bit
        eps = 1e-5
        assert torch.equal(ops.row_stat(out, eps), ops.rstd_from_ss(ss, H, eps)), M
    # model widths (64 and 128 partials per row: one and two per lane), ragged row counts, and a
    # view whose rows are not 16-byte aligned (the two-launch path)
    for H2, M2 in ((8192, 37), (16384, 6), (4096, 130)):
        x = rnd(M2, H2, seed=74)
        want = ops.rstd_from_ss(ops.row_ss(x), H2, 1e-5)
        assert torch.equal(ops.row_stat(x, 1e-5), want), (H2, M2)
        xv = rnd(M2, H2 + 4, seed=74)[:, 4:]
        xv.copy_(x)
        assert torch.equal(ops.row_stat(xv, 1e-5), want), (H2, M2, "unaligned")
        assert rel_err(want, torch.rsqrt(x.float().pow(2).mean(-1) + 1e-5)) < 1e-5


@pytest.mark.parametrize("order", [8, -4, -8, 1, -1, 2, 3, -5])
def test_gemm_v10_tile_orders(ops, ref, order):
    """v10 tile orders (groups of M tiles / of N tiles, any size) only permute which block computes which tile:
    every epilogue gives the fp32 reference and the same bits as the default order."""
    M, N, K = 1100, 1536, 1024            # 5 x 6 tiles: ragged last M tile, groups split unevenly
    ops.k.fls_gemm_set_mid(0)
    try:
        x = rnd(M, K, seed=51)
        w = rnd(N, K, scale=0.05, seed=52)
        r0 = rnd(M, N, seed=53)
        base = [ops.gemm(x, w), ops.gemm(x, w, EPI_RESID, out=r0.clone(), resid=r0.clone()),
                ops.gemm(x, w, EPI_SWIGLU)]
        assert ops.k.fls_gemm_set_order(order) == 0
        got = [ops.gemm(x, w), ops.gemm(x, w, EPI_RESID, out=r0.clone(), resid=r0.clone()),
               ops.gemm(x, w, EPI_SWIGLU)]
        torch.cuda.synchronize()
        for a, b in zip(base, got):
            assert torch.equal(a, b)
        assert rel_err(got[0], x.float() @ w.float().t()) < 2e-3
        assert rel_err(got[2].cpu(), ref.swiglu_up(x.float().cpu(), w.float().cpu())) < 3e-3
    finally:
        ops.k.fls_gemm_set_order(0)
        ops.k.fls_gemm_set_mid(1)


@pytest.mark.parametrize("M,N,K", [(1, 32000, 1024), (5, 1000, 8192), (16, 33, 96), (7, 100, 160)])
def test_gemv_skinny(ops, M, N, K):
    x = rnd(M, K, seed=41)
    w = rnd(N, K, scale=0.05, seed=42)
    y = ops.gemv_skinny(x, w)
    torch.cuda.synchronize()
    assert rel_err(y, x.float() @ w.float().t()) < 2e-3
    assert ops.linear(x, w).shape == (M, N)          # linear() routes M <= 16 here


@pytest.mark.parametrize("mid", [1, 0])
def test_gemm_bias_epilogues(ops, ref, mid):
    """Per-column bias ahead of RoPE (Qwen2 q/k/v) and ahead of the residual add (o_proj), on the
    mid-M kernel (this M's default) and on v10."""
    from flexible_llm_sharding_amd.config import ModelConfig
    from flexible_llm_sharding_amd.models.llama import rope_tables
    M, H, nh, nkv, hd = 300, 512, 4, 2, 128
    ops.k.fls_gemm_set_mid(mid)
    try:
        x = rnd(M, H, seed=51)
        wqkv = rnd((nh + 2 * nkv) * hd, H, scale=0.05, seed=52)
        b = rnd((nh + 2 * nkv) * hd, scale=0.5, seed=53)
        pos = torch.randint(0, 4000, (M,), dtype=torch.int32, device=DEV)
        cfg = ModelConfig(hidden_size=nh * hd, num_attention_heads=nh, num_key_value_heads=nkv)
        cos, sin = rope_tables(cfg, 4096)
        y = ops.qkv_rope(x, wqkv, pos, cos.to(DEV), sin.to(DEV), nh, nkv, hd, bias=b)
        r = ref.qkv_rope(x.float().cpu(), wqkv.float().cpu(), pos.cpu(), cos, sin, nh, nkv, hd, bias=b.float().cpu())
        assert rel_err(y.cpu(), r) < 3e-3
        wo = rnd(H, H, scale=0.05, seed=54)
        bo = rnd(H, scale=0.5, seed=55)
        r0 = rnd(M, H, seed=56)
        out = ops.linear_residual(x, wo, r0.clone(), bias=bo)
        assert rel_err(out, r0.float() + x.float() @ wo.float().t() + bo.float()) < 2e-3
        torch.cuda.synchronize()
    finally:
        ops.k.fls_gemm_set_mid(1)


@pytest.mark.parametrize("nq,nk,hd", [(8, 2, 128), (4, 4, 64), (0, 2, 128), (6, 0, 128), (4, 4, 96)])
def test_qkv_norm_rope(ops, ref, nq, nk, hd):
    """Qwen3 projection: GEMM + per-head q/k RMSNorm + RoPE (headnorm_rope_kernel) vs the fp32
    torch backend; V columns untouched; q-only and k/v-only forms (the pruned last layer)."""
    from flexible_llm_sharding_amd.config import preset
    from flexible_llm_sharding_amd.models.llama import rope_tables
    K, M = 512, 70
    nv = nk
    N = (nq + nk + nv) * hd
    x = rnd(M, K, seed=31)
    w = rnd(N, K, scale=0.05, seed=32)
    qn = (1 + 0.1 * torch.randn(hd)).half().to(DEV)
    kn = (1 + 0.1 * torch.randn(hd)).half().to(DEV)
    pos = torch.randint(0, 4000, (M,), dtype=torch.int32)
    cfg = preset("tiny-qwen3", explicit_head_dim=hd)
    cos, sin = rope_tables(cfg, 4096, torch.float16)
    y = ops.qkv_norm_rope(x, w, pos.to(DEV), cos.to(DEV), sin.to(DEV), nq, nk, hd, qn, kn, 1e-6)
    r = ref.qkv_norm_rope(x.cpu(), w.cpu(), pos, cos, sin, nq, nk, hd, qn.cpu(), kn.cpu(), 1e-6)
    torch.cuda.synchronize()
    assert y.shape == r.shape
    assert (y.cpu().float() - r.float()).abs().max().item() < 2e-2
    if nv:
        v0 = (nq + nk) * hd
        assert rel_err(y[:, v0:], (x.float() @ w.float().t())[:, v0:]) < 2e-3


@pytest.mark.parametrize("q_block", [64, 32, 8])
@pytest.mark.parametrize("split", [0, 1, 3, 8])
@pytest.mark.parametrize("nh,nkv,hd", [(8, 1, 128), (16, 2, 128), (8, 2, 64), (4, 4, 64), (4, 4, 96)])
def test_attention_suffix_rows_from_cache(ops, ref, nh, nkv, hd, split, q_block):
    """Suffix K/V reuse: the kept rows of each suffix read from the cache as range 2 (with the
    prefix as range 0) and only the new rows computed == the full packed pass on those rows.
    split: key-tile slices of the split-KV kernel (0 = by grid size, which splits this small grid;
    1 = one block per item and head; hd 96 never splits).  q_block 32: one wave per head, 4 or 8
    heads of a KV group per block (groups of < 4 heads fall back to the 2-wave kernel).  q_block 8:
    the packed-GQA decode kernel (a KV group's heads x rows in 64-row passes: these items hold up
    to 13 new rows, so the 8-head groups take two passes; hd 96 falls back)."""
    old = ops.k.fls_attention_set_split(split)
    try:
        _suffix_rows_from_cache(ops, ref, nh, nkv, hd, q_block=q_block)
    finally:
        ops.k.fls_attention_set_split(old)


def test_attention_decode_split_matches_unsplit(ops, ref):
    """Decode-like step at 70B heads (12 prompts x 5 suffixes, one new row each after 40 kept rows,
    600-row prefixes): the split-KV kernel (by grid size) == one block per item to fp32-partials
    rounding, and both == the fp32 oracle."""
    prompts = [(600, [41] * 5)] * 12
    keep = [[40] * 5] * 12
    ys = []
    for split, qb in ((1, 64), (0, 64), (1, 32), (0, 32), (1, 8), (0, 8)):
        old = ops.k.fls_attention_set_split(split)
        try:
            ys.append(_suffix_rows_from_cache(ops, ref, 64, 8, 128, prompts, keep, q_block=qb))
        finally:
            ops.k.fls_attention_set_split(old)
    assert rel_err(ys[1], ys[0]) < 2e-3
    # one wave per head, 8 heads per block: the same per-row math as the 2-wave kernel, unsplit
    assert torch.equal(ys[2], ys[0])
    assert rel_err(ys[3], ys[0]) < 2e-3
    # packed-GQA decode kernel (8 heads x 5 rows in one 64-row pass), unsplit and split
    assert rel_err(ys[4], ys[0]) < 2e-3
    assert rel_err(ys[5], ys[0]) < 2e-3


def _suffix_rows_from_cache(ops, ref, nh, nkv, hd, prompts=None, keep=None, q_block=64):
    from flexible_llm_sharding_amd.runtime.batch import pack_prompts
    from flexible_llm_sharding_amd.utils.tokenizer import TokenizedPrompt
    prompts = prompts or [(70, [5, 80, 1]), (130, [65, 17]), (9, [3, 140])]
    keep = keep or [[3, 70, 0], [64, 5], [0, 139]]
    tps = [TokenizedPrompt(list(range(lp)), [list(range(l)) for l in ls], max(ls), [l - 1 for l in ls])
           for lp, ls in prompts]
    offs, t = [], 0
    for lp, _ in prompts:
        offs.append(t)
        t += lp
    rows = []
    for lp, ls in prompts:
        rows.append([])
        for l in ls:
            rows[-1].append(t)
            t += l
    full = pack_prompts(tps, [0, 1, 2], "bidirectional", prefix_offsets=offs, suffix_rows=rows)
    g = torch.Generator().manual_seed(6)
    qkv = torch.randn(full.num_tokens, (nh + 2 * nkv) * hd, generator=g).half()
    qs, kv = nh * hd, 2 * nkv * hd
    cache = torch.zeros(t, kv, dtype=torch.float16)
    cache[torch.from_numpy(full.pfx_dst)] = qkv[torch.from_numpy(full.pfx_src), qs:qs + kv]
    cache[torch.from_numpy(full.sfx_dst)] = qkv[torch.from_numpy(full.sfx_src), qs:qs + kv]
    reuse = pack_prompts(tps, [0, 1, 2], "bidirectional", prefix_offsets=offs, kv_cached=True, suffix_rows=rows,
                         suffix_keep=keep)
    # packed rows of the full pass that the reuse pass computes: each suffix's rows after its kept ones
    sel = []
    si = 0
    for j, (lp, ls) in enumerate(prompts):
        for s, l in enumerate(ls):
            sg = [x for x in full.segments if x.r1_len][si]
            sel.extend(range(sg.q_start + keep[j][s], sg.q_start + l))
            si += 1
    sel = torch.tensor(sel)
    qkv_new = qkv[sel].contiguous()
    m = reuse.device_tensors(DEV)
    if q_block == 32:                                     # one wave per head: items of <= 32 rows
        q_block = 32 if int(reuse.work[:, 1].max()) <= 32 else 64
    y = ops.attention(qkv_new.to(DEV), m["work"], nh, nkv, hd, kv0=cache.to(DEV), seg_lo=m["seg_lo"],
                      work2=m["work2"], r2win=m["r2win"], q_block=q_block)
    want = ref.attention(qkv.float(), full.segments, nh, nkv, hd)[sel]
    got_ref = ref.attention(qkv_new.float(), reuse.segments, nh, nkv, hd, kv0=cache.float())
    torch.cuda.synchronize()
    assert rel_err(got_ref, want) < 1e-5                 # the oracle agrees with itself across layouts
    assert rel_err(y.cpu(), want) < 5e-3
    return y.cpu()


@pytest.mark.parametrize("M", [1, 7, 64, 160, 300, 512])
@pytest.mark.parametrize("epi", ["none_bias", "resid", "swiglu", "rope128", "rope64"])
def test_gemm_small_m_splitk(ops, ref, M, epi):
    """Small-M split-K path (fp32 partial slabs + reduce with the epilogue) == the fp32 reference,
    == the non-split kernels to rounding, and bitwise reproducible."""
    from flexible_llm_sharding_amd.config import ModelConfig
    from flexible_llm_sharding_amd.models.llama import rope_tables
    K, N = 2048, 1024
    x = rnd(M, K, seed=11)
    if epi == "swiglu":
        w = rnd(2 * N, K, scale=0.05, seed=12)
        run = lambda: ops.swiglu_up(x, w)                                         # noqa: E731
        want = ref.swiglu_up(x.float().cpu(), w.float().cpu())
    elif epi.startswith("rope"):
        hd = int(epi[4:])
        nh, nkv = N // hd // 2, N // hd // 4
        n = (nh + 2 * nkv) * hd
        w = rnd(n, K, scale=0.05, seed=13)
        b = rnd(n, scale=0.5, seed=14)
        cfg = ModelConfig(hidden_size=nh * hd, num_attention_heads=nh, num_key_value_heads=nkv)
        cos, sin = rope_tables(cfg, 4096)
        pos = torch.randint(0, 4000, (M,), dtype=torch.int32, device=DEV)
        run = lambda: ops.qkv_rope(x, w, pos, cos.to(DEV), sin.to(DEV), nh, nkv, hd, bias=b)   # noqa: E731
        want = ref.qkv_rope(x.float().cpu(), w.float().cpu(), pos.cpu(), cos, sin, nh, nkv, hd, bias=b.float().cpu())
    else:
        w = rnd(N, K, scale=0.05, seed=15)
        r0 = rnd(M, N, seed=16)
        b = rnd(N, scale=0.5, seed=17)
        if epi == "resid":
            run = lambda: ops.linear_residual(x, w, r0.clone(), bias=b)           # noqa: E731
            want = r0.float().cpu() + x.float().cpu() @ w.float().cpu().t() + b.float().cpu()
        else:
            run = lambda: ops.gemm(x, w, EPI_NONE, bias=b)                         # noqa: E731
            want = x.float().cpu() @ w.float().cpu().t() + b.float().cpu()
    got, again = run(), run()
    old = ops.k.fls_gemm_set_splitk(0)
    try:
        plain = run()
    finally:
        ops.k.fls_gemm_set_splitk(old)
    torch.cuda.synchronize()
    assert torch.equal(got, again)
    assert rel_err(got.cpu(), want) < 3e-3
    assert rel_err(got.cpu(), plain.cpu()) < 2e-3


@pytest.mark.parametrize("bn", [128, 256])
@pytest.mark.parametrize("blocks", [0, 1])
@pytest.mark.parametrize("M", [1, 7, 17, 33, 100, 160, 256])
@pytest.mark.parametrize("epi", ["none_bias", "resid", "swiglu", "rope128", "rope64"])
def test_gemm_skinny_m(ops, ref, M, epi, blocks, bn):
    """Skinny-M kernel (gemm_skinny.h: every row of M in one block, weights and activations by
    LDS-DMA) == the fp32 reference and == the other small-M paths to rounding, bitwise
    reproducible.  blocks 0: the default K split (fp32 partials + reduce); blocks 1: no split, the
    NONE / RESID / SWIGLU epilogues applied in the kernel.  bn: weight rows per block (256: four
    subtiles per wave, refill after the barrier; M > 160 falls back to 128).  M < 17 only runs
    here with the path forced (mode 2)."""
    from flexible_llm_sharding_amd.config import ModelConfig
    from flexible_llm_sharding_amd.models.llama import rope_tables
    K, N = 2048, 1024
    x = rnd(M, K, seed=61)
    if epi == "swiglu":
        w = rnd(2 * N, K, scale=0.05, seed=62)
        run = lambda: ops.swiglu_up(x, w)                                         # noqa: E731
        want = ref.swiglu_up(x.float().cpu(), w.float().cpu())
    elif epi.startswith("rope"):
        hd = int(epi[4:])
        nh, nkv = N // hd // 2, N // hd // 4
        n = (nh + 2 * nkv) * hd
        w = rnd(n, K, scale=0.05, seed=63)
        b = rnd(n, scale=0.5, seed=64)
        cfg = ModelConfig(hidden_size=nh * hd, num_attention_heads=nh, num_key_value_heads=nkv)
        cos, sin = rope_tables(cfg, 4096)
        pos = torch.randint(0, 4000, (M,), dtype=torch.int32, device=DEV)
        run = lambda: ops.qkv_rope(x, w, pos, cos.to(DEV), sin.to(DEV), nh, nkv, hd, bias=b)   # noqa: E731
        want = ref.qkv_rope(x.float().cpu(), w.float().cpu(), pos.cpu(), cos, sin, nh, nkv, hd, bias=b.float().cpu())
    else:
        w = rnd(N, K, scale=0.05, seed=65)
        r0 = rnd(M, N, seed=66)
        b = rnd(N, scale=0.5, seed=67)
        if epi == "resid":
            run = lambda: ops.linear_residual(x, w, r0.clone(), bias=b)           # noqa: E731
            want = r0.float().cpu() + x.float().cpu() @ w.float().cpu().t() + b.float().cpu()
        else:
            run = lambda: ops.gemm(x, w, EPI_NONE, bias=b)                         # noqa: E731
            want = x.float().cpu() @ w.float().cpu().t() + b.float().cpu()
    old = ops.k.fls_gemm_set_skinny(0, 0)
    old_bn = ops.k.fls_gemm_set_skinny_bn(bn)
    try:
        plain = run()                                   # the mid / split-K / generic paths
        ops.k.fls_gemm_set_skinny(2, blocks)
        got, again = run(), run()
    finally:
        ops.k.fls_gemm_set_skinny(old, 0)
        ops.k.fls_gemm_set_skinny_bn(old_bn)
    torch.cuda.synchronize()
    assert torch.equal(got, again)
    assert rel_err(got.cpu(), want) < 3e-3
    assert rel_err(got.cpu(), plain.cpu()) < 2e-3


@pytest.mark.parametrize("bn", [0, 256])
def test_gemm_skinny_70b_generation_shapes(ops, bn):
    """The 70B projections at a generation step's 160 rows (QKV + RoPE, O + residual, gate/up +
    SwiGLU, down + residual) on the skinny kernel (mode 2: every projection, bn 0 = the default
    block) == the same GEMMs with it off, to rounding."""
    from flexible_llm_sharding_amd.config import preset
    from flexible_llm_sharding_amd.models.llama import rope_tables
    cfg = preset("llama2-70b")
    M, H, I = 160, cfg.hidden_size, cfg.intermediate_size
    nh, nkv, hd = cfg.num_attention_heads, cfg.num_key_value_heads, cfg.head_dim
    cos, sin = rope_tables(cfg, 4096)
    cos, sin = cos.to(DEV), sin.to(DEV)
    pos = torch.randint(0, 4000, (M,), dtype=torch.int32, device=DEV)
    x = rnd(M, H, seed=71)
    xi = rnd(M, I, seed=72)
    wqkv = rnd((nh + 2 * nkv) * hd, H, scale=0.02, seed=73)
    wo = rnd(H, H, scale=0.02, seed=74)
    wgu = rnd(2 * I, H, scale=0.02, seed=75)
    wd = rnd(H, I, scale=0.02, seed=76)
    r0 = rnd(M, H, seed=77)
    runs = [lambda: ops.qkv_rope(x, wqkv, pos, cos, sin, nh, nkv, hd),
            lambda: ops.linear_residual(x, wo, r0.clone()),
            lambda: ops.swiglu_up(x, wgu),
            lambda: ops.linear_residual(xi, wd, r0.clone())]
    for run in runs:
        old = ops.k.fls_gemm_set_skinny(2, 0)
        old_bn = ops.k.fls_gemm_set_skinny_bn(bn)
        try:
            got = run()
            ops.k.fls_gemm_set_skinny(0, 0)
            plain = run()
        finally:
            ops.k.fls_gemm_set_skinny(old, 0)
            ops.k.fls_gemm_set_skinny_bn(old_bn)
        torch.cuda.synchronize()
        assert rel_err(got, plain) < 2e-3


@pytest.mark.parametrize("epi", ["resid", "rope", "swiglu"])
def test_gemm_row_chunks_bitwise(ops, epi):
    """Main-path GEMMs over more than 16,384 rows run as row-chunk launches (the activation panel
    then fits the Infinity Cache): bitwise equal to one launch over all rows."""
    from flexible_llm_sharding_amd.config import ModelConfig
    from flexible_llm_sharding_amd.models.llama import rope_tables
    M, K = 17000, 256
    x = rnd(M, K, seed=21)
    pos = torch.randint(0, 4000, (M,), dtype=torch.int32, device=DEV)
    cfg = ModelConfig(hidden_size=1024, num_attention_heads=8, num_key_value_heads=4)
    cos, sin = rope_tables(cfg, 4096)
    cos, sin = cos.to(DEV), sin.to(DEV)
    # N = 2048: each 8,704-row chunk is 272 tiles of 256 x 256 (the chunks stay on the main path)
    w = rnd(2048, K, scale=0.05, seed=22)
    r0 = rnd(M, 2048, seed=23)

    def run():
        if epi == "resid":
            return ops.linear_residual(x, w, r0.clone())
        if epi == "rope":
            return ops.qkv_rope(x, w, pos, cos, sin, 8, 4, 128)
        return ops.swiglu_up(x, w)
    a = run()
    old = ops.k.fls_gemm_set_row_chunk(0)
    try:
        b = run()
    finally:
        ops.k.fls_gemm_set_row_chunk(old)
    torch.cuda.synchronize()
    assert torch.equal(a, b)


@pytest.mark.parametrize("M", [384, 768, 1000, 1537])
@pytest.mark.parametrize("epi", ["none", "resid", "rope", "rope64", "swiglu", "bias"])
def test_gemm_v11_bitwise_vs_v10(ops, ref, M, epi):
    """gemm_nt_v11 (384 x 256 tile, gemm_v11.hip) accumulates every output in the same k order as
    v10, so every epilogue but RoPE (FMA contraction, <= 1 ulp) is bitwise equal to v10 -- including ragged M, where v11's last tile is
    shifted back and must not store its neighbour's rows twice (in-place residual)."""
    from flexible_llm_sharding_amd.config import ModelConfig
    from flexible_llm_sharding_amd.models.llama import rope_tables
    K = 384                                            # 6 K-tiles (v11 needs an even count)
    x = rnd(M, K, seed=31)
    pos = torch.randint(0, 4000, (M,), dtype=torch.int32, device=DEV)
    hd = 64 if epi == "rope64" else 128
    cfg = ModelConfig(hidden_size=1024, num_attention_heads=1024 // hd, num_key_value_heads=2)
    cos, sin = rope_tables(cfg, 4096)
    cos, sin = cos.to(DEV), sin.to(DEV)
    w = rnd(1024, K, scale=0.05, seed=32)
    b = rnd(1024, scale=0.1, seed=33)
    r0 = rnd(M, 1024, seed=34)

    def run():
        if epi == "resid":
            return ops.linear_residual(x, w, r0.clone())
        if epi.startswith("rope"):
            nh = 1024 // hd
            return ops.qkv_rope(x, w, pos, cos, sin, nh - 4, 2, hd)
        if epi == "swiglu":
            return ops.swiglu_up(x, w)
        if epi == "bias":
            return ops.linear_residual(x, w, r0.clone(), bias=b)
        return ops.linear(x, w)
    old = ops.k.fls_gemm_set_v11(2)
    old_mid = ops.k.fls_gemm_set_mid(0)      # the v10 arm runs v10, not the 64 x 128 mid-M kernel
    try:
        a = run()
        ops.k.fls_gemm_set_v11(0)
        v10 = run()
    finally:
        ops.k.fls_gemm_set_v11(old)
        ops.k.fls_gemm_set_mid(old_mid)
    torch.cuda.synchronize()
    if epi.startswith("rope"):
        nh = 1024 // hd
        r = ref.qkv_rope(x.float().cpu(), w.float().cpu(), pos.cpu(), cos.cpu(), sin.cpu(), nh - 4, 2, hd)
        assert rel_err(a.cpu(), r) < 3e-3
        # the rotation's FMA contraction may differ between the two kernels' epilogues: <= 1 ulp
        af, bf = a.float(), v10.float()
        assert bool(((af - bf).abs() <= torch.maximum(af.abs(), bf.abs()) * 2.0 ** -10 + 1e-7).all())
    else:
        assert torch.equal(a, v10)
    if epi == "none":
        assert rel_err(a, x.float() @ w.float().t()) < 2e-3


def test_gemm_v11_production_shape_bitwise(ops):
    """A 70B O-projection-sized launch (43,008 x 8,192 x 8,192 would take 2 GB; 4,608 rows keep the
    full N / K): v11 in auto mode vs v10, bitwise, and vs fp32 on a row sample."""
    M, N, K = 4608, 8192, 8192
    x = rnd(M, K, seed=41)
    w = rnd(N, K, scale=0.02, seed=42)
    r0 = rnd(M, N, seed=43)
    old = ops.k.fls_gemm_set_v11(1)
    try:
        a = ops.linear_residual(x, w, r0.clone())
        ops.k.fls_gemm_set_v11(0)
        b = ops.linear_residual(x, w, r0.clone())
    finally:
        ops.k.fls_gemm_set_v11(old)
    torch.cuda.synchronize()
    assert torch.equal(a, b)
    rows = torch.arange(0, M, 97, device=DEV)
    want = x[rows].float() @ w.float().t() + r0[rows].float()
    assert rel_err(a[rows], want) < 2e-3


# ------------------------------------------------------------------ fused RMSNorm (round 5)
@pytest.mark.parametrize("H", [256, 1000 // 8 * 8, 4096, 8192, 5120])
@pytest.mark.parametrize("gather", [False, True])
def test_row_rstd(ops, H, gather):
    """Row statistics of the fused RMSNorm: rsqrt(mean(x^2) + eps) in fp32 per row (or per
    gathered row) == the fp32 reference."""
    x = rnd(61, H, scale=3.0, seed=101)
    idx = torch.tensor([3, 60, 0, 7, 7], dtype=torch.int32, device=DEV) if gather else None
    r = ops.row_rstd(x, 1e-5, row_idx=idx)
    xs = x.float()[idx.long()] if gather else x.float()
    want = torch.rsqrt(xs.pow(2).mean(-1) + 1e-5)
    torch.cuda.synchronize()
    assert r.dtype == torch.float32 and r.shape == want.shape
    assert ((r - want).abs() / want).max().item() < 1e-5


def test_fold_norm_bitwise(ops):
    """W[n, k] *= gamma[k] in place == torch's fp16(fp32 product), bitwise (a strided W view too)."""
    w = rnd(300, 1024, scale=0.05, seed=102)
    g = rnd(1024, scale=0.7, seed=103) + 1.0
    want = (w.float() * g.float()).half()
    ops.fold_norm(w, g)
    big = rnd(64, 2048, scale=0.05, seed=104)
    view = big[:, 1024:]                                   # row stride 2048
    want_v = (view.float() * g.float()).half()
    ops.fold_norm(view, g)
    torch.cuda.synchronize()
    assert torch.equal(w, want)
    assert torch.equal(big[:, 1024:], want_v)


def test_copy_rows(ops):
    """Row gather / scatter / both (the pruned layer's rows, the prefix K/V capture) == torch."""
    x = rnd(50, 2048, seed=105)
    src = torch.tensor([4, 49, 0, 17], dtype=torch.int32, device=DEV)
    dst = torch.tensor([9, 1, 30, 2], dtype=torch.int32, device=DEV)
    g = ops.gather_rows(x, src)
    y = torch.zeros(40, 2048, dtype=torch.float16, device=DEV)
    ops.scatter_rows(g, dst, y)
    z = torch.zeros(40, 512, dtype=torch.float16, device=DEV)
    ops.copy_rows(x[:, 1024:1536], src, z, dst)            # strided source columns
    torch.cuda.synchronize()
    assert torch.equal(g, x[src.long()])
    want = torch.zeros_like(y)
    want[dst.long()] = x[src.long()]
    assert torch.equal(y, want)
    assert torch.equal(z, want[:, 1024:1536])


@pytest.mark.parametrize("M,path", [(1, "auto"), (7, "auto"), (100, "auto"), (160, "auto"), (300, "auto"),
                                    (517, "auto"), (1000, "v11"), (1000, "v10"), (1000, "mid"), (33, "generic")])
@pytest.mark.parametrize("epi", ["none_bias", "resid_alpha", "swiglu", "rope128", "rope64"])
def test_gemm_row_scale_every_path(ops, ref, M, path, epi):
    """Per-row scale of the raw product (the fused RMSNorm statistic) and the residual alpha
    (Granite) on every GEMM path: auto (skinny / split-K / mid by M), and v11, v10 main, mid-M and
    the generic kernel forced: == the fp32 reference of the row-scaled product, and a unit scale /
    alpha == no scale, bitwise."""
    from flexible_llm_sharding_amd.config import ModelConfig
    from flexible_llm_sharding_amd.models.llama import rope_tables
    K, N = 2048, 1024
    x = rnd(M, K, seed=111)
    rs = (torch.rand(M, generator=torch.Generator().manual_seed(112)) * 2 + 0.1).to(DEV)
    ones = torch.ones(M, dtype=torch.float32, device=DEV)
    xs = x.float().cpu() * rs.cpu()[:, None]
    if epi == "swiglu":
        w = rnd(2 * N, K, scale=0.05, seed=113)
        run = lambda s: ops.swiglu_up(x, w, rscale=s)                                          # noqa: E731
        want = ref.swiglu_up(xs, w.float().cpu())
    elif epi.startswith("rope"):
        hd = int(epi[4:])
        nh, nkv = N // hd // 2, N // hd // 4
        n = (nh + 2 * nkv) * hd
        w = rnd(n, K, scale=0.05, seed=114)
        b = rnd(n, scale=0.5, seed=115)
        cfg = ModelConfig(hidden_size=nh * hd, num_attention_heads=nh, num_key_value_heads=nkv)
        cos, sin = rope_tables(cfg, 4096)
        pos = torch.randint(0, 4000, (M,), dtype=torch.int32, device=DEV)
        run = lambda s: ops.qkv_rope(x, w, pos, cos.to(DEV), sin.to(DEV), nh, nkv, hd, bias=b, rscale=s)  # noqa: E731
        want = ref.qkv_rope(xs, w.float().cpu(), pos.cpu(), cos, sin, nh, nkv, hd, bias=b.float().cpu())
    else:
        w = rnd(N, K, scale=0.05, seed=116)
        r0 = rnd(M, N, seed=117)
        b = rnd(N, scale=0.5, seed=118)
        if epi == "resid_alpha":
            run = lambda s: ops.gemm(x, w, EPI_RESID, out=r0.clone(), resid=r0, bias=b, rscale=s,      # noqa: E731
                                     alpha=0.7 if s is not None else 1.0)
            want = r0.float().cpu() + 0.7 * (xs @ w.float().cpu().t() + b.float().cpu())
        else:
            run = lambda s: ops.gemm(x, w, EPI_NONE, bias=b, rscale=s)                         # noqa: E731
            want = xs @ w.float().cpu().t() + b.float().cpu()
    modes = {"auto": (1, 1, 1), "v11": (2, 1, 1), "v10": (0, 0, 1), "mid": (0, 2, 1), "generic": (0, 0, 0)}[path]
    k = ops.k
    old = (k.fls_gemm_set_v11(modes[0]), k.fls_gemm_set_mid(modes[1]), k.fls_gemm_set_skinny(modes[2], 0),
           k.fls_gemm_set_splitk(modes[2]))
    try:
        if path == "generic":
            x = x[:, :K - 8]                               # an odd K keeps every tiled kernel out
            xs = xs[:, :K - 8]
            w = w[:, :K - 8]
            want = {"none_bias": lambda: xs @ w.float().cpu().t() + b.float().cpu(),
                    "resid_alpha": lambda: r0.float().cpu() + 0.7 * (xs @ w.float().cpu().t() + b.float().cpu()),
                    "swiglu": lambda: ref.swiglu_up(xs, w.float().cpu()),
                    "rope128": lambda: ref.qkv_rope(xs, w.float().cpu(), pos.cpu(), cos, sin, nh, nkv, hd,
                                                    bias=b.float().cpu()),
                    "rope64": lambda: ref.qkv_rope(xs, w.float().cpu(), pos.cpu(), cos, sin, nh, nkv, hd,
                                                   bias=b.float().cpu())}[epi]()
        got = run(rs)
        unscaled, unit = run(None), (ops.gemm(x, w, EPI_RESID, out=r0.clone(), resid=r0, bias=b, rscale=ones)
                                     if epi == "resid_alpha" else run(ones))
    finally:
        k.fls_gemm_set_v11(old[0])
        k.fls_gemm_set_mid(old[1])
        k.fls_gemm_set_skinny(old[2], 0)
        k.fls_gemm_set_splitk(old[3])
    torch.cuda.synchronize()
    assert rel_err(got.cpu(), want) < 3e-3
    assert torch.equal(unit, unscaled)


@pytest.mark.parametrize("path,M", [("v11", 3072), ("v10", 1024), ("mid", 300), ("skinny", 160), ("splitk", 40),
                                    ("generic", 300)])
def test_resid_gemm_row_sum_squares(ops, path, M):
    """RESID GEMMs with ``ss`` also write each output row's partial sums of squares per 128 columns
    (the v10 / v11 epilogue, or the fallback kernel after the small-M paths): equal to the sums
    over the fp16 output, the output itself bitwise unchanged; the statistic from them matches
    row_rstd of the output."""
    N, K = 2048, 1024
    x = rnd(M, K, seed=131)
    w = rnd(N, K, scale=0.05, seed=132)
    r0 = rnd(M, N, seed=133)
    modes = {"v11": (2, 1, 1, 1), "v10": (0, 0, 0, 1), "mid": (0, 1, 0, 0), "skinny": (0, 1, 2, 0),
             "splitk": (0, 0, 0, 1), "generic": (0, 0, 0, 0)}[path]
    k = ops.k
    old = (k.fls_gemm_set_v11(modes[0]), k.fls_gemm_set_mid(modes[1]), k.fls_gemm_set_skinny(modes[2], 0),
           k.fls_gemm_set_splitk(modes[3]))
    try:
        if path == "generic":
            x, w = x[:, :K - 8], w[:, :K - 8]
        ss = torch.full((M + 3, N // 128 + 2), -1.0, dtype=torch.float32, device=DEV)
        plain = ops.linear_residual(x, w, r0.clone())
        got = ops.linear_residual(x, w, r0.clone(), ss=ss)
        rs = ops.rstd_from_ss(ss[:M], N, 1e-5)
    finally:
        k.fls_gemm_set_v11(old[0])
        k.fls_gemm_set_mid(old[1])
        k.fls_gemm_set_skinny(old[2], 0)
        k.fls_gemm_set_splitk(old[3])
    torch.cuda.synchronize()
    assert torch.equal(got, plain)
    want = (got.float() ** 2).view(M, N // 128, 128).sum(-1)
    assert torch.allclose(ss[:M, :N // 128], want, rtol=1e-5, atol=1e-5)
    assert (ss[M:] == -1).all() and (ss[:, N // 128:] == -1).all()       # nothing outside [M, N/128]
    rr = ops.row_rstd(got, 1e-5)
    assert torch.allclose(rs, rr, rtol=2e-6, atol=0)


@pytest.mark.parametrize("v11", [0, 2])
def test_row_scale_past_row_chunk(ops, v11):
    """The fused norm's per-row scale on a launch cut into row chunks (v10: <= 16,384 rows a launch):
    every chunk reads its own rows' statistic (a second chunk once read the first chunk's)."""
    M, N, K = 16384 + 700, 256, 128
    x = rnd(M, K, seed=141)
    w = rnd(N, K, scale=0.05, seed=142)
    rs = (torch.rand(M, generator=torch.Generator().manual_seed(143)) + 0.5).float().to(DEV)
    old = ops.k.fls_gemm_set_v11(v11)
    try:
        y = ops.gemm(x, w, rscale=rs)
    finally:
        ops.k.fls_gemm_set_v11(old)
    torch.cuda.synchronize()
    want = (x.float() @ w.float().t()) * rs[:, None]
    assert rel_err(y, want) < 3e-3
    assert rel_err(y[16384:], want[16384:]) < 3e-3


def test_embed_scaled(ops, ref):
    """Granite's embedding_multiplier inside the gather: fp16(e * m) == torch, bitwise."""
    table = rnd(1000, 512, seed=121)
    ids = torch.randint(0, 1000, (77,), dtype=torch.int32, device=DEV)
    y = ops.embed(ids, table, torch.float16, scale=12.0)
    out = torch.empty(77, 512, dtype=torch.float16, device=DEV)
    y2 = ops.embed(ids, table, torch.float16, out=out)
    torch.cuda.synchronize()
    assert torch.equal(y, (table[ids.long()].float() * 12.0).half())
    assert y2.data_ptr() == out.data_ptr() and torch.equal(out, table[ids.long()])


@pytest.mark.parametrize("V", [32000, 37])
def test_softmax_scaled(ops, V):
    """Granite's logits_scaling inside the softmax: softmax(fp16(l / s)) == torch."""
    x = rnd(9, V, scale=8.0, seed=122)
    y = ops.softmax(x, logits_scaling=8.0)
    r = torch.softmax((x / 8.0).float(), -1)
    torch.cuda.synchronize()
    assert (y.float() - r).abs().max().item() < 1e-3


def test_argmax_rows_first_index(ops):
    """Greedy tokens on the device == numpy's argmax of the fp16 probabilities (first index on
    ties, the reference's np.argmax, main.py:85-88)."""
    x = torch.softmax(rnd(37, 32000, scale=3.0, seed=131).float(), -1).half()
    x[3, 100] = x[3, 2000] = 0.5                          # a tie: the first index wins
    x[5] = 0                                              # all equal
    got = ops.argmax_rows(x)
    torch.cuda.synchronize()
    assert np.array_equal(got.cpu().numpy(), np.argmax(x.cpu().numpy(), axis=-1))
    assert got[3].item() == 100 and got[5].item() == 0
