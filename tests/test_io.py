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


def test_packed_cache_source(tiny_model, tmp_path):
    """--weight_cache packed: images equal the in-RAM packing, stale caches are rebuilt,
    and a rank's byte slice can be read on its own."""
    from flexible_llm_sharding_amd.runtime.packed import PackedFileSource, build_packed_cache, packed_path
    from flexible_llm_sharding_amd.runtime.weights import FileLayerSource
    path, cfg = tiny_model
    src = FileLayerSource(cfg, path)
    cache = str(tmp_path / "pk")
    assert build_packed_cache(src, cache) == len(cfg.layer_names())
    assert build_packed_cache(src, cache) == 0                      # up to date
    pk = PackedFileSource(cfg, cache)
    for n in cfg.layer_names():
        a = torch.zeros(src.nbytes(n), dtype=torch.uint8)
        b = torch.zeros(src.nbytes(n), dtype=torch.uint8)
        src.read_into(n, a)
        pk.read_into(n, b)
        assert torch.equal(a, b), n
        part = torch.zeros(100, dtype=torch.uint8)
        pk.read_range_into(n, part, 300, 400)
        assert torch.equal(part, a[300:400])
    # a cache written for another config is stale -> refused, then rebuilt
    other = preset("tiny", rms_norm_eps=1e-6)
    with pytest.raises(FileNotFoundError):
        PackedFileSource(other, cache)
    with open(packed_path(cache, "lm_head"), "r+b") as f:
        f.write(b"garbage!")
    assert build_packed_cache(src, cache) == 1


def test_dp_slices_from_packed_cache(tiny_model, tmp_path):
    from flexible_llm_sharding_amd.parallel.data_parallel import SlicedHostStore
    from flexible_llm_sharding_amd.runtime.packed import PackedFileSource, build_packed_cache
    from flexible_llm_sharding_amd.runtime.weights import FileLayerSource
    path, cfg = tiny_model
    src = FileLayerSource(cfg, path)
    build_packed_cache(src, str(tmp_path / "pk"))
    for rank in range(3):
        a = SlicedHostStore.from_source(src, rank, 3, pinned=False)
        b = SlicedHostStore.from_source(PackedFileSource(cfg, str(tmp_path / "pk")), rank, 3, pinned=False)
        for n in cfg.layer_names():
            nb, c = a.nbytes(n), a.chunk_bytes(n)
            valid = max(0, min(nb, (rank + 1) * c) - rank * c)
            assert torch.equal(a.buffers[n][:valid], b.buffers[n][:valid]), (rank, n)
