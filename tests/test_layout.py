"""Packed HBM layout: placements, pack/unpack round trip, natural-order RoPE / SwiGLU oracle."""
import pytest
import torch
import torch.nn.functional as F

from flexible_llm_sharding_amd.config import preset
from flexible_llm_sharding_amd.models.layout import layer_layout, pack_layer, placements, unpack_layer
from flexible_llm_sharding_amd.models.llama import rope_tables
from flexible_llm_sharding_amd.models.reference import _rope
from flexible_llm_sharding_amd.ops.torch_backend import TorchOps
from flexible_llm_sharding_amd.utils.synthetic import synthetic_layer_state_dict


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


@pytest.mark.parametrize("model", ["tiny", "tiny-qwen2", "llama2-70b"])
def test_placements_tile_the_slots(model):
    """Every checkpoint tensor lands inside its slot, tensors never overlap, and the stacked
    slots (wqkv = q|k|v, wgu = gate|up) are exactly filled — no permutation, no gaps."""
    cfg = preset(model)
    name = "model.layers.0"
    lay = layer_layout(cfg, "decoder")
    pls = sorted(placements(cfg, name), key=lambda p: p.offset)
    for a, b in zip(pls, pls[1:]):
        assert a.offset + a.nbytes <= b.offset
    for slot, parts in (("wqkv", ("q_proj.weight", "k_proj.weight", "v_proj.weight")),
                        ("wgu", ("gate_proj.weight", "up_proj.weight"))):
        s = lay.slot(slot)
        ps = [p for p in pls if any(p.hf_name.endswith(x) for x in parts)]
        assert ps[0].offset == s.offset
        assert sum(p.nbytes for p in ps) == 2 * s.numel
    assert all(s.offset % 256 == 0 for s in lay.slots)


def test_layout_alignment():
    cfg = preset("llama2-70b")
    lay = layer_layout(cfg, "decoder")
    assert all(s.offset % 256 == 0 for s in lay.slots)
    assert abs(lay.nbytes - 1.711e9) / 1.711e9 < 0.01


def test_qkv_rope_oracle_equals_hf_rope():
    """qkv_rope on the packed [q; k; v] weight == HF rotate-half RoPE on HF q/k, v untouched."""
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
    assert torch.allclose(y[:, :qs], qh, atol=1e-4)
    assert torch.allclose(y[:, qs:qs + ks], kh, atol=1e-4)
    v = x @ sd[f"{name}.self_attn.v_proj.weight"].t()
    assert torch.allclose(y[:, qs + ks:], v, atol=1e-4)


def test_swiglu_oracle_on_stacked_gate_up():
    cfg = preset("tiny")
    name = "model.layers.1"
    sd = synthetic_layer_state_dict(cfg, name, seed=6, dtype=torch.float32)
    W = layer_layout(cfg, "decoder", 4).views(pack_layer(cfg, name, sd, dtype=torch.float32), torch.float32)
    x = torch.randn(7, cfg.hidden_size)
    y = TorchOps().swiglu_up(x, W["wgu"])
    ref = F.silu(x @ sd[f"{name}.mlp.gate_proj.weight"].t()) * (x @ sd[f"{name}.mlp.up_proj.weight"].t())
    assert torch.allclose(y, ref, atol=1e-5)


def test_int8_rejected():
    cfg = preset("tiny")
    sd = {"model.norm.weight": torch.ones(cfg.hidden_size, dtype=torch.int8)}
    with pytest.raises(AssertionError, match="int8"):
        pack_layer(cfg, "model.norm", sd)


def test_decoder_image_splits_into_attention_and_mlp_pieces():
    """Sub-layer streaming (PiecePoolPrefetcher) frees the attention piece before the MLP phase:
    every tensor the MLP phase reads (ln2, gate/up, down) must sit at or after mlp_offset, every
    attention tensor before it."""
    from flexible_llm_sharding_amd.config import preset
    from flexible_llm_sharding_amd.models.layout import layer_layout, mlp_offset
    for name in ("tiny", "tiny-qwen2", "llama2-70b"):
        lay = layer_layout(preset(name), "decoder")
        split = mlp_offset(lay)
        for ts in lay.slots:
            assert (ts.offset >= split) == (ts.name in ("ln2", "wgu", "wdown")), (name, ts.name)
