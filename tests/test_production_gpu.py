"""Numerics at production geometry: one Llama-2-70B-shaped decoder layer (H 8192, 64 / 8 heads,
I 28672) on 8,064 packed tokens (6 prompts x (1024 prefix + 5 x 64 suffixes)) through the HIP
kernels, against the same layer computed in fp32 PyTorch from the same packed fp16 weights; then
the LM head + vocab softmax at V = 32000 on the scored rows.  Reference: the per-layer dispatch
of ``/root/reference/utils.py:269-290``."""
import pytest
import torch

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():
    pytest.skip("no GPU", allow_module_level=True)

from flexible_llm_sharding_amd import _native  # noqa: E402
from flexible_llm_sharding_amd.config import preset  # noqa: E402
from flexible_llm_sharding_amd.models.layout import layer_layout  # noqa: E402
from flexible_llm_sharding_amd.models.llama import ExecContext, Workspace, rope_tables, run_decoder  # noqa: E402
from flexible_llm_sharding_amd.ops.hip_backend import HipOps  # noqa: E402
from flexible_llm_sharding_amd.ops.torch_backend import TorchOps  # noqa: E402
from flexible_llm_sharding_amd.runtime.batch import pack_prompts  # noqa: E402
from flexible_llm_sharding_amd.utils.tokenizer import TokenizedPrompt  # noqa: E402

DEV = torch.device("cuda", 0)


@pytest.fixture(scope="module")
def layer70b():
    cfg = preset("llama2-70b", num_hidden_layers=1)
    ops = HipOps()
    lay = layer_layout(cfg, "decoder")
    buf = torch.empty(lay.nbytes, dtype=torch.uint8, device=DEV)
    ops.fill_layer_random(buf, lay, seed=11, std=0.02)
    W16 = lay.views(buf, torch.float16)
    head = torch.empty(cfg.vocab_size, cfg.hidden_size, dtype=torch.float16, device=DEV)
    _native.kernels().fls_fill_random(head.data_ptr(), head.numel(), 77, 0.0, 0.02,
                                      torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    return cfg, ops, W16, head


def _rel(a, b):
    a, b = a.float(), b.float()
    return ((a - b).norm() / b.norm()).item()


@pytest.mark.parametrize("mode", ["bidirectional", "causal"])
def test_70b_layer_and_head_vs_fp32(layer70b, mode):
    cfg, ops, W16, head = layer70b
    assert _native.loaded_libraries().get("k")
    tps = [TokenizedPrompt(list(range(1024)), [list(range(64))] * 5, 64, [63] * 5) for _ in range(6)]
    b = pack_prompts(tps, list(range(6)), mode)
    assert b.num_tokens == 6 * (1024 + 5 * 64)
    meta = b.device_tensors(DEV)
    g = torch.Generator(device=DEV).manual_seed(3)
    x16 = torch.randn(b.num_tokens, cfg.hidden_size, generator=g, device=DEV).half()
    cos, sin = rope_tables(cfg, 4096, torch.float16, DEV)

    # HIP path: the engine's decoder block (workspace arena, fused epilogues, shared-prefix attention)
    ctx = ExecContext(cfg, ops, DEV, torch.float16, cos, sin, mlp_chunk=16384)
    ctx.ws = Workspace(DEV, torch.float16)
    ctx.prune_last = False
    y16 = run_decoder(ctx, W16, x16.clone(), b, meta, "model.layers.0")

    # fp32 PyTorch reference of the same block from the same fp16 weights
    ref = TorchOps(torch.float32)
    W32 = {k: v.float() for k, v in W16.items()}
    rctx = ExecContext(cfg, ref, DEV, torch.float32, cos, sin, mlp_chunk=1 << 30)
    rctx.prune_last = False
    y32 = run_decoder(rctx, W32, x16.float(), b, meta, "model.layers.0")
    torch.cuda.synchronize()
    assert torch.isfinite(y16).all()
    err = _rel(y16, y32)
    assert err < 5e-3, err
    # the layer's update (y - x) is what the fp16 path has to get right, not the residual stream
    err_d = _rel(y16.float() - x16.float(), y32 - x16.float())
    assert err_d < 2e-2, err_d

    # LM head + softmax at V = 32000 on the 30 scored rows (rmsnorm of the gathered rows first)
    idx = meta["last_idx"]
    norm_w = W16["ln1"]
    h16 = ops.gather_rmsnorm(y16, idx, norm_w, cfg.rms_norm_eps)
    p16 = ops.lm_head_softmax(h16, head)
    h32 = ref.gather_rmsnorm(y32, idx, norm_w.float(), cfg.rms_norm_eps)
    p32 = torch.softmax(h32 @ head.float().t(), dim=-1)
    torch.cuda.synchronize()
    assert p16.shape == (30, cfg.vocab_size)
    assert (p16.float() - p32).abs().max().item() < 2e-3
    assert (p16.float().argmax(-1) == p32.argmax(-1)).float().mean().item() >= 0.9
    assert abs(p16.float().sum(-1) - 1).max().item() < 1e-2
