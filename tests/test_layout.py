"""Packed HBM layout: pack/unpack round trip, RoPE pair permutation, gate/up interleave."""
import torch

from flexible_llm_sharding_amd.config import preset
from flexible_llm_sharding_amd.models.layout import (deinterleave_gate_up, interleave_gate_up, layer_layout,
                                                     pack_layer, permute_head_cols, rope_row_perm,
                                                     unpack_layer, unpermute_head_cols)
from flexible_llm_sharding_amd.models.llama import rope_tables
from flexible_llm_sharding_amd.models.reference import _rope
from flexible_llm_sharding_amd.ops.torch_backend import TorchOps
from flexible_llm_sharding_amd.utils.synthetic import synthetic_layer_state_dict


def test_rope_perm_is_permutation():
    for hd in (64, 128):
        p = rope_row_perm(hd)
        assert sorted(p) == list(range(hd))
        # blocks of 16 alternate first half / second half
        assert p[:16] == list(range(16)) and p[16:32] == list(range(hd // 2, hd // 2 + 16))


def test_pack_roundtrip():
    cfg = preset("tiny")
    for name in cfg.layer_names():
        sd = synthetic_layer_state_dict(cfg, name, seed=3)
        buf = pack_layer(cfg, name, sd)
        assert buf.numel() == layer_layout(cfg, {"model.embed_tokens": "embed", "model.norm": "norm",
                                                 "lm_head": "head"}.get(name, "decoder")).nbytes
        back = unpack_layer(cfg, name, buf)
        assert set(back) == set(sd)
        for k in sd:
            assert torch.equal(back[k], sd[k]), k


def test_layout_alignment():
    cfg = preset("llama2-70b")
    lay = layer_layout(cfg, "decoder")
    assert all(s.offset % 256 == 0 for s in lay.slots)
    assert abs(lay.nbytes - 1.711e9) / 1.711e9 < 0.01


def test_interleave_roundtrip():
    g, u = torch.randn(64, 8), torch.randn(64, 8)
    w = interleave_gate_up(g, u)
    assert torch.equal(w[16:32], u[:16])
    g2, u2 = deinterleave_gate_up(w)
    assert torch.equal(g, g2) and torch.equal(u, u2)


def test_rope_on_permuted_layout_equals_hf_rope():
    """qkv_rope on packed (permuted) weights == HF rotate-half RoPE on HF-layout q/k, permuted."""
    cfg = preset("tiny")
    nh, nkv, hd = cfg.num_attention_heads, cfg.num_key_value_heads, cfg.head_dim
    name = "model.layers.0"
    sd = synthetic_layer_state_dict(cfg, name, seed=5, dtype=torch.float32)
    buf = pack_layer(cfg, name, sd, dtype=torch.float32)
    W = layer_layout(cfg, "decoder", 4).views(buf, torch.float32)
    T = 9
    x = torch.randn(T, cfg.hidden_size)
    pos = torch.tensor([0, 1, 2, 5, 77, 1000, 3, 4095, 12], dtype=torch.int32)
    cos, sin = rope_tables(cfg, 4096, table_dtype=torch.float32)
    y = TorchOps().qkv_rope(x, W["wqkv"], pos, cos, sin, nh, nkv, hd)
    q = x @ sd[f"{name}.self_attn.q_proj.weight"].t()
    k = x @ sd[f"{name}.self_attn.k_proj.weight"].t()
    qh = _rope(q.view(1, T, nh, hd).transpose(1, 2), pos.long()[None], cos, sin).transpose(1, 2).reshape(T, -1)
    kh = _rope(k.view(1, T, nkv, hd).transpose(1, 2), pos.long()[None], cos, sin).transpose(1, 2).reshape(T, -1)
    qs, ks = nh * hd, nkv * hd
    assert torch.allclose(unpermute_head_cols(y[:, :qs], nh, hd), qh, atol=1e-4)
    assert torch.allclose(unpermute_head_cols(y[:, qs:qs + ks], nkv, hd), kh, atol=1e-4)
    assert torch.allclose(permute_head_cols(qh, nh, hd), y[:, :qs], atol=1e-4)
    v = x @ sd[f"{name}.self_attn.v_proj.weight"].t()
    assert torch.allclose(y[:, qs + ks:], v, atol=1e-4)


def test_int8_rejected():
    cfg = preset("tiny")
    sd = {"model.norm.weight": torch.ones(cfg.hidden_size, dtype=torch.int8)}
    try:
        pack_layer(cfg, "model.norm", sd)
    except AssertionError as e:
        assert "int8" in str(e)
    else:
        raise AssertionError("int8 accepted")
