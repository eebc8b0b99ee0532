"""Safetensors reader/writer (python + native), layer conversion (prepare_weights)."""
import json
import os

import pytest
import torch

from flexible_llm_sharding_amd import _native
from flexible_llm_sharding_amd.config import preset
from flexible_llm_sharding_amd.runtime import hostmem
from flexible_llm_sharding_amd.utils.layer_format import layer_of_param, split_into_layers
from flexible_llm_sharding_amd.utils.safetensors_io import load_file, read_header, save_file


@pytest.fixture(scope="module", autouse=True)
def _build_runtime():
    from flexible_llm_sharding_amd._native import build
    build.build_runtime()


def sample_tensors():
    g = torch.Generator().manual_seed(0)
    return {"a.weight": torch.randn(5, 7, generator=g).half(),
            "b": torch.randn(3, generator=g),
            "c.bf": torch.randn(2, 2, generator=g).bfloat16(),
            "d.i": torch.arange(6, dtype=torch.int64).view(2, 3),
            "e.empty": torch.empty(0, 4)}


def test_roundtrip_with_reference_library(tmp_path):
    safetensors = pytest.importorskip("safetensors.torch")
    t = sample_tensors()
    p1 = str(tmp_path / "ours.safetensors")
    save_file(t, p1, metadata={"format": "pt"})
    theirs = safetensors.load_file(p1)
    for k in t:
        assert torch.equal(theirs[k], t[k])
    p2 = str(tmp_path / "theirs.safetensors")
    safetensors.save_file(t, p2)
    ours = load_file(p2)
    for k in t:
        assert torch.equal(ours[k], t[k])


def test_native_header_and_pread(tmp_path):
    assert _native.runtime_or_none() is not None
    t = sample_tensors()
    p = str(tmp_path / "x.safetensors")
    save_file(t, p)
    py, _ = read_header(p)
    nat = hostmem.read_header_native(p)
    assert py == nat
    got = hostmem.read_safetensors(p)
    for k in t:
        assert torch.equal(got[k], t[k])


def test_native_header_rejects_garbage(tmp_path):
    p = tmp_path / "bad.safetensors"
    p.write_bytes(b"\x05\x00\x00\x00\x00\x00\x00\x00{bad}")
    with pytest.raises(ValueError):
        hostmem.read_header_native(str(p))


def test_pwrite_pread_roundtrip(tmp_path):
    x = torch.randint(0, 255, (40 << 20,), dtype=torch.uint8)   # > one 16 MiB chunk
    p = str(tmp_path / "blob")
    hostmem.pwrite_from(p, x)
    y = torch.empty_like(x)
    hostmem.pread_into(p, 0, x.numel(), y)
    assert torch.equal(x, y)
    z = torch.empty(100, dtype=torch.uint8)
    hostmem.pread_into(p, 12345, 100, z)
    assert torch.equal(z, x[12345:12445])


def test_gather_blocks():
    rt = _native.runtime()
    src = torch.arange(64, dtype=torch.int32)
    perm = torch.tensor([3, 0, 2, 1, 7, 6, 5, 4], dtype=torch.int64)
    dst = torch.empty_like(src)
    rt.fls_gather_blocks(dst.data_ptr(), src.data_ptr(), 32, perm.data_ptr(), 8, 4)
    assert torch.equal(dst.view(8, 8), src.view(8, 8)[perm])


def test_layer_of_param():
    assert layer_of_param("model.layers.3.self_attn.q_proj.weight") == "model.layers.3"
    assert layer_of_param("model.embed_tokens.weight") == "model.embed_tokens"
    assert layer_of_param("model.norm.weight") == "model.norm"
    assert layer_of_param("lm_head.weight") == "lm_head"


def _hf_checkpoint(tmp_path, fmt, name="tiny", tied=False):
    from flexible_llm_sharding_amd.utils.synthetic import synthetic_layer_state_dict
    from flexible_llm_sharding_amd.utils.tokenizer import write_synthetic_tokenizer
    cfg = preset(name, tie_word_embeddings=tied)
    d = tmp_path / f"hf_{fmt}"
    d.mkdir()
    cfg.save(str(d))
    write_synthetic_tokenizer(str(d), cfg.vocab_size)
    sd = {}
    for n in cfg.layer_names():
        sd.update(synthetic_layer_state_dict(cfg, n, seed=2))
    if tied:
        del sd["lm_head.weight"]             # HF tied checkpoints store no lm_head
    names = sorted(sd)
    halves = [names[: len(names) // 2], names[len(names) // 2:]]
    wmap = {}
    for i, part in enumerate(halves):
        fn = f"model-{i:05d}.{'bin' if fmt == 'bin' else 'safetensors'}"
        chunk = {k: sd[k] for k in part}
        if fmt == "bin":
            torch.save(chunk, str(d / fn))
        else:
            save_file(chunk, str(d / fn))
        wmap.update({k: fn for k in part})
    idx = "pytorch_model.bin.index.json" if fmt == "bin" else "model.safetensors.index.json"
    (d / idx).write_text(json.dumps({"metadata": {}, "weight_map": wmap}))
    return cfg, d, sd


@pytest.mark.parametrize("fmt", ["bin", "safetensors"])
def test_split_into_layers(tmp_path, fmt):
    cfg, src, sd = _hf_checkpoint(tmp_path, fmt)
    out = tmp_path / f"layers_{fmt}"
    written = split_into_layers(str(src), str(out), verbose=False)
    assert sorted(written) == sorted(cfg.layer_names())
    assert (out / "config.json").exists() and (out / "tokenizer.json").exists()
    assert not any(f.endswith(".bin") for f in os.listdir(out))
    for n in cfg.layer_names():
        got = load_file(str(out / f"{n}.safetensors"))
        for k, v in got.items():
            assert layer_of_param(k) == n
            assert torch.equal(v, sd[k])


def test_split_tied_qwen2_checkpoint(tmp_path):
    """Qwen2 (q/k/v biases) with tie_word_embeddings: the converter materialises lm_head,
    and the packed layer round-trips biases through the RoPE row permutation."""
    from flexible_llm_sharding_amd.models.layout import pack_layer, unpack_layer
    cfg, src, sd = _hf_checkpoint(tmp_path, "safetensors", name="tiny-qwen2", tied=True)
    out = tmp_path / "layers_tied"
    written = split_into_layers(str(src), str(out), verbose=False)
    assert sorted(written) == sorted(cfg.layer_names())
    head = load_file(str(out / "lm_head.safetensors"))["lm_head.weight"]
    assert torch.equal(head, sd["model.embed_tokens.weight"])
    layer = load_file(str(out / "model.layers.1.safetensors"))
    assert "model.layers.1.self_attn.q_proj.bias" in layer
    back = unpack_layer(cfg, "model.layers.1", pack_layer(cfg, "model.layers.1", layer))
    for k, v in layer.items():
        assert torch.equal(back[k], v), k


@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16, torch.float32])
def test_file_source_reads_checkpoint_bytes(tmp_path, dtype):
    """The streaming source builds each packed image from file byte ranges only: equal to
    pack_layer of the loaded state dict for fp16 / bf16 / fp32 checkpoints, and any byte range
    [lo, hi) (a data-parallel rank's slice) reads only the file bytes it covers."""
    from flexible_llm_sharding_amd.runtime.stream import FileLayerSource
    from flexible_llm_sharding_amd.utils.synthetic import load_full_state_dict, write_synthetic_checkpoint
    from flexible_llm_sharding_amd.models.layout import pack_layer
    cfg = preset("tiny-qwen2")
    d = str(tmp_path / "ck")
    write_synthetic_checkpoint(cfg, d, seed=4, dtype=dtype)
    sd = load_full_state_dict(cfg, d)
    src = FileLayerSource(cfg, d)
    for n in cfg.layer_names():
        nb = src.nbytes(n)
        full = torch.zeros(nb, dtype=torch.uint8)
        src.read_into(n, full)
        assert torch.equal(full, pack_layer(cfg, n, sd)), n
        for G in (2, 3):
            c = (nb + G - 1) // G // 2 * 2 + 2
            for r in range(G):
                lo, hi = min(nb, r * c), min(nb, (r + 1) * c)
                part = torch.zeros(max(1, hi - lo), dtype=torch.uint8)
                before = src.read_bytes
                src.read_range_into(n, part, lo, hi)
                assert torch.equal(part[:hi - lo], full[lo:hi]), (n, G, r)
                # file bytes read == the tensor bytes this range covers (x 2 for fp32), not the file
                want = sum(max(0, min(hi, r.img_off + 2 * r.numel) - max(lo, r.img_off)) * r.src_es // 2
                           for r in src.plan(n).runs)
                assert src.read_bytes - before == want


def test_f32_to_f16_rounding_matches_torch():
    """The streamer's host fp32 -> fp16 conversion == torch .to(float16) (RNE, subnormals, inf, nan)."""
    import ctypes
    import numpy as np
    from flexible_llm_sharding_amd import _native
    rt = _native.runtime_or_none()
    if rt is None:
        pytest.skip("native runtime not built")
    vals = torch.cat([torch.randn(10000) * 3, torch.randn(1000) * 1e-5, torch.randn(1000) * 1e-8,
                      torch.tensor([65504., 65519.9, 65520., 1e6, -1e6, 0., -0., 2 ** -24, 2 ** -25, 3 * 2 ** -26,
                                    float("inf"), float("-inf"), 5.960464477539063e-08, 6.103515625e-05,
                                    6.097555160522461e-05, 1.0009765625, 1.00048828125, 1.00146484375])])
    src = vals.float().contiguous()
    out = torch.empty(src.numel(), dtype=torch.int16)
    rt.fls_f32_to_f16(src.data_ptr(), out.data_ptr(), src.numel())
    assert torch.equal(out.view(torch.float16), src.to(torch.float16))
    nan = torch.tensor([float("nan")])
    rt.fls_f32_to_f16(nan.data_ptr(), out.data_ptr(), 1)
    assert torch.isnan(out[:1].view(torch.float16)).all()


def test_dp_slices_read_only_their_range(tiny_model):
    """SlicedHostStore.from_source: rank r's slice of every layer piece (attention / MLP piece of a
    decoder, the whole image otherwise) == bytes [lo + r*c, lo + (r+1)*c) of the full image, and
    the G ranks together read each layer file's tensor bytes exactly once."""
    from flexible_llm_sharding_amd.parallel.data_parallel import SlicedHostStore
    from flexible_llm_sharding_amd.runtime.stream import FileLayerSource
    path, cfg = tiny_model
    full_src = FileLayerSource(cfg, path)
    G = 3
    total = 0
    for rank in range(G):
        src = FileLayerSource(cfg, path)
        st = SlicedHostStore.from_source(src, rank, G, pinned=False)
        total += src.read_bytes
        for n in cfg.layer_names():
            nb = st.nbytes(n)
            full = torch.zeros(nb, dtype=torch.uint8)
            full_src.read_into(n, full)
            sl = st.slices(n)
            assert len(sl) == (2 if n.startswith("model.layers.") else 1)
            assert sl[0].lo == 0 and sl[-1].hi == nb and st.buffers[n].numel() == st.chunk_bytes(n)
            for p in sl:
                a, b = p.rank_range(rank)
                assert torch.equal(st.buffers[n][p.buf_off:p.buf_off + b - a], full[a:b]), (rank, n)
    assert total == sum(full_src.plan(n).file_bytes for n in cfg.layer_names())


@pytest.mark.parametrize("family", ["mixtral", "qwen3_moe"])
def test_hf_moe_checkpoint_converts_and_matches(tmp_path, family):
    """An HF MoE checkpoint (transformers save_pretrained: Mixtral's per-expert w1/w2/w3, Qwen3-MoE's
    per-expert gate/up/down_proj) -> prepare_weights' per-layer files -> the engine == HF logits;
    the v5 stacked in-memory form (mlp.experts.gate_up_proj) converts to the same files."""
    transformers = pytest.importorskip("transformers")
    import numpy as np
    import torch
    from flexible_llm_sharding_amd.config import ModelConfig
    from flexible_llm_sharding_amd.engine import ShardedRunner
    from flexible_llm_sharding_amd.utils.tokenizer import tokenize_prompt
    from flexible_llm_sharding_amd.runtime.stream import FileLayerSource
    from flexible_llm_sharding_amd.utils.layer_format import layer_file, normalize_expert_names
    from flexible_llm_sharding_amd.utils.safetensors_io import load_file
    from flexible_llm_sharding_amd.utils.synthetic import synthetic_prompts
    from flexible_llm_sharding_amd.utils.tokenizer import load_tokenizer, write_synthetic_tokenizer
    common = dict(hidden_size=128, intermediate_size=256, num_attention_heads=4, num_key_value_heads=2,
                  num_hidden_layers=2, vocab_size=300, tie_word_embeddings=False, max_position_embeddings=4096)
    torch.manual_seed(0)
    if family == "mixtral":
        hf = transformers.MixtralForCausalLM(transformers.MixtralConfig(num_local_experts=4, **common))
    else:
        hf = transformers.Qwen3MoeForCausalLM(transformers.Qwen3MoeConfig(
            num_experts=6, num_experts_per_tok=3, moe_intermediate_size=64, norm_topk_prob=True, head_dim=32,
            **common))
    hf = hf.float().eval()
    with torch.no_grad():                       # make routing non-trivial (HF inits the router to zeros)
        for n, p in hf.named_parameters():
            if n.endswith("mlp.gate.weight"):
                p.normal_(0, 0.3)
    src, out = tmp_path / "hf", tmp_path / "layers"
    hf.save_pretrained(str(src), safe_serialization=True)
    write_synthetic_tokenizer(str(src), common["vocab_size"])
    split_into_layers(str(src), str(out), verbose=False)
    cfg = ModelConfig.from_pretrained(str(out))
    assert cfg.is_moe and cfg.model_type == family
    # the stacked v5 state dict of layer 0 normalises to exactly the file's tensors
    v5 = {k: v for k, v in hf.state_dict().items() if k.startswith("model.layers.0.")}
    disk = load_file(layer_file(str(out), "model.layers.0"))
    norm = normalize_expert_names(family, v5)
    assert sorted(norm) == sorted(disk) and all(torch.equal(norm[k], disk[k]) for k in disk)
    tok = load_tokenizer(str(out))
    prompts = synthetic_prompts(2, 16, 2, 4, common["vocab_size"], seed=3, vary=True)
    got = ShardedRunner(cfg, FileLayerSource(cfg, str(out)), "cpu", tok, prefix_attention="causal")(prompts)
    for (prefix, sufs), o in zip(prompts, got):
        tp = tokenize_prompt(tok, prefix, sufs)
        for j, s in enumerate(tp.suffixes):
            with torch.no_grad():
                logits = hf(torch.tensor([tp.prefix + s])).logits[0, -1].float()
            assert np.abs(o[j, 0].astype(np.float32) - torch.softmax(logits, -1).numpy()).max() < 2e-3
