"""main.py / prepare_weights.py CLI parity (reference main.py:30-98, prepare_weights.py:56-62)."""
import os
import pickle
import subprocess
import sys

import numpy as np
import pytest

from flexible_llm_sharding_amd.api import batch_ranges
from flexible_llm_sharding_amd.utils.cli import parse_args

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_reference_flags_and_defaults():
    a = parse_args(["--prompt_pickle", "p.pkl", "--output_file", "o.pkl"])
    assert a.model_path == "./" and a.num_batch == 1 and a.layer_num_per_shard == 1
    assert a.storage_location == "cpu" and a.max_activation_in_cpu == 100
    assert a.data_parallel is False and a.disk_folder == "./temp" and a.num_gen_token == 1
    with pytest.raises(SystemExit):
        parse_args(["--output_file", "o.pkl"])          # prompt_pickle required


@pytest.mark.parametrize("val,exp", [("True", True), ("False", False), ("1", True), ("0", False)])
def test_data_parallel_bool(val, exp):
    # reference type=bool turned "False" into True; we parse it as a boolean
    a = parse_args(["--prompt_pickle", "p", "--output_file", "o", "--data_parallel", val])
    assert a.data_parallel is exp
    a = parse_args(["--prompt_pickle", "p", "--output_file", "o", "--data_parallel"])
    assert a.data_parallel is True


def test_batch_ranges_matches_reference():
    for n in range(0, 23):
        for nb in range(1, 6):
            ends = [n // nb * i for i in range(1, nb)] + [n]
            ref = list(zip([0] + ends[:-1], ends))
            assert batch_ranges(n, nb) == ref


def _run(args, cwd):
    env = dict(os.environ, PYTHONPATH=ROOT, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "main.py")] + args, cwd=cwd, env=env,
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    return r


@pytest.mark.parametrize("storage,lnps,nb", [("cpu", 1, 1), ("disk", 2, 2), ("gpu", 100, 3)])
def test_main_end_to_end(tiny_model, tmp_path, storage, lnps, nb):
    from flexible_llm_sharding_amd.utils.synthetic import synthetic_prompts
    path, cfg = tiny_model
    prompts = synthetic_prompts(5, 15, 3, 4, cfg.vocab_size, seed=4, vary=True)
    pp = tmp_path / "prompts.pkl"
    pickle.dump(prompts, open(pp, "wb"))
    out = tmp_path / "scores.pkl"
    _run(["--model_path", path, "--prompt_pickle", str(pp), "--output_file", str(out),
          "--num_gen_token", "3", "--layer_num_per_shard", str(lnps), "--storage_location", storage,
          "--num_batch", str(nb), "--disk_folder", str(tmp_path / "spill")], str(tmp_path))
    scores = pickle.load(open(out, "rb"))
    assert len(scores) == 5
    for (pre, sufs), s in zip(prompts, scores):
        assert s.shape == (len(sufs), 3, cfg.vocab_size) and s.dtype == np.float16
        assert np.allclose(s.astype(np.float32).sum(-1), 1.0, atol=2e-2)
    upd = pickle.load(open(tmp_path / "prompts_updated.pkl", "rb"))
    assert isinstance(upd, list) and len(upd) == 5
    for (pre, sufs), (pre2, sufs2) in zip(prompts, upd):
        assert pre2 == pre and all(b.startswith(a) and len(b) > len(a) for a, b in zip(sufs, sufs2))


def test_generation_is_greedy_rerun(tiny_model, tmp_path):
    """Step t's scores equal a fresh scoring of the prompts extended by steps < t (main.py:85-90)."""
    from flexible_llm_sharding_amd.engine import ShardedRunner
    from flexible_llm_sharding_amd.runtime.stream import FileLayerSource
    from flexible_llm_sharding_amd.utils.synthetic import synthetic_prompts
    from flexible_llm_sharding_amd.utils.tokenizer import load_tokenizer
    path, cfg = tiny_model
    prompts = synthetic_prompts(2, 12, 2, 3, cfg.vocab_size, seed=9)
    pp = tmp_path / "p.pkl"
    pickle.dump(prompts, open(pp, "wb"))
    _run(["--model_path", path, "--prompt_pickle", str(pp), "--output_file", str(tmp_path / "s.pkl"),
          "--num_gen_token", "2"], str(tmp_path))
    scores = pickle.load(open(tmp_path / "s.pkl", "rb"))
    tok = load_tokenizer(path)
    r = ShardedRunner(cfg, FileLayerSource(cfg, path), "cpu", tok)
    ext = []
    for (pre, sufs), s in zip(prompts, scores):
        t0 = np.argmax(s[:, :1], -1)
        ext.append((pre, tuple(a + tok.decode(t) for a, t in zip(sufs, t0))))
    step1 = r(ext)
    for s, o in zip(scores, step1):
        assert np.abs(s[:, 1].astype(np.float32) - o[:, 0].astype(np.float32)).max() < 1e-3


def test_prepare_weights_synthetic_cli(tmp_path):
    env = dict(os.environ, PYTHONPATH=ROOT)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "prepare_weights.py"), "tiny", str(tmp_path / "m"),
                        "--synthetic", "--num_hidden_layers", "1"], env=env, capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stderr
    files = sorted(os.listdir(tmp_path / "m"))
    assert "model.layers.0.safetensors" in files and "lm_head.safetensors" in files and "config.json" in files


def test_main_synthetic_and_max_token_len(tmp_path):
    """--synthetic PRESET (no checkpoint files) and --max_token_len truncation."""
    from flexible_llm_sharding_amd.config import preset
    from flexible_llm_sharding_amd.utils.synthetic import synthetic_prompts
    cfg = preset("tiny")
    prompts = synthetic_prompts(3, 40, 2, 6, cfg.vocab_size, seed=2)
    pp = tmp_path / "prompts.pkl"
    pickle.dump(prompts, open(pp, "wb"))
    out = tmp_path / "scores.pkl"
    mj = tmp_path / "m.json"
    _run(["--synthetic", "tiny", "--prompt_pickle", str(pp), "--output_file", str(out),
          "--max_token_len", "16", "--metrics_json", str(mj)], str(tmp_path))
    scores = pickle.load(open(out, "rb"))
    assert [s.shape for s in scores] == [(2, 1, cfg.vocab_size)] * 3
    import json
    m = json.load(open(mj))
    # prefix truncated to 16 tokens (BOS included), each suffix to 16 (after BOS drop): 3 x (16 + 2 x 6)
    assert m["stats"]["tokens"] == 3 * (16 + 2 * 6)


def test_main_weight_cache_modes_agree(tiny_model, tmp_path):
    """host / stream / disk (alias) / auto weight caches give identical scores; auto with a host
    budget below the model size streams."""
    from flexible_llm_sharding_amd.utils.synthetic import synthetic_prompts
    path, cfg = tiny_model
    pp = tmp_path / "prompts.pkl"
    pickle.dump(synthetic_prompts(3, 12, 2, 4, cfg.vocab_size, seed=3), open(pp, "wb"))
    outs = {}
    for mode, extra in (("host", []), ("stream", []), ("disk", []), ("auto", ["--host_mem_gb", "0.0001"])):
        out = tmp_path / f"s_{mode}.pkl"
        _run(["--model_path", path, "--prompt_pickle", str(pp), "--output_file", str(out),
              "--weight_cache", mode] + extra, str(tmp_path))
        outs[mode] = pickle.load(open(out, "rb"))
    for m in ("stream", "disk", "auto"):
        for a, b in zip(outs["host"], outs[m]):
            assert np.array_equal(a, b), m


def test_weight_cache_resolution(tiny_model):
    """auto -> host when the packed model fits the host budget, else stream; an explicit host that
    cannot fit is refused up front; disk is the reference-named alias of stream."""
    import types
    from flexible_llm_sharding_amd.api import resolve_weight_cache
    from flexible_llm_sharding_amd.parallel.comm import Comm
    path, cfg = tiny_model
    names = cfg.layer_names()
    comm = Comm(0, 1)

    def args(mode, gb):
        return types.SimpleNamespace(weight_cache=mode, host_mem_gb=gb, synthetic=None)
    assert resolve_weight_cache(args("auto", 100.0), cfg, comm, names, sliced=False) == "host"
    assert resolve_weight_cache(args("auto", 1e-4), cfg, comm, names, sliced=False) == "stream"
    assert resolve_weight_cache(args("disk", 100.0), cfg, comm, names, sliced=False) == "stream"
    with pytest.raises(SystemExit):
        resolve_weight_cache(args("host", 1e-4), cfg, comm, names, sliced=False)


def _torchrun(world, args, cwd):
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    env = dict(os.environ, PYTHONPATH=ROOT, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="", OMP_NUM_THREADS="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.join(ROOT, "main.py")] + args
    r = subprocess.run(cmd, cwd=cwd, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    return r


@pytest.mark.parametrize("n_prompts,num_batch,weight_cache", [(3, 2, "host"), (1, 1, "host"), (3, 2, "stream"),
                                                               (0, 1, "host")])
def test_main_data_parallel_uneven_slices(tiny_model, tmp_path, n_prompts, num_batch, weight_cache):
    """DP with scatter-loaded weights and prompt slices of different sizes (3 prompts / 2 ranks with
    2 batches: rank 1 has an empty batch; 1 prompt: rank 1 has none; 0 prompts): every rank still
    runs num_batch passes, so the weight all-gathers stay matched, and the scores equal
    a one-process run."""
    from flexible_llm_sharding_amd.utils.synthetic import synthetic_prompts
    path, cfg = tiny_model
    prompts = synthetic_prompts(n_prompts, 14, 2, 4, cfg.vocab_size, seed=8, vary=True)
    pp = tmp_path / "prompts.pkl"
    pickle.dump(prompts, open(pp, "wb"))
    common = ["--model_path", path, "--prompt_pickle", str(pp), "--num_batch", str(num_batch),
              "--weight_cache", weight_cache]
    _torchrun(2, common + ["--output_file", str(tmp_path / "dp.pkl"), "--data_parallel"], str(tmp_path))
    _run(common + ["--output_file", str(tmp_path / "one.pkl")], str(tmp_path))
    dp, one = pickle.load(open(tmp_path / "dp.pkl", "rb")), pickle.load(open(tmp_path / "one.pkl", "rb"))
    assert len(dp) == len(one) == n_prompts
    for a, b in zip(dp, one):
        assert np.abs(a.astype(np.float32) - b.astype(np.float32)).max() < 1e-5


def test_main_model_parallel_no_prompts(tiny_model, tmp_path):
    """MP with an empty prompt list returns an empty score list."""
    path, cfg = tiny_model
    pp = tmp_path / "prompts.pkl"
    pickle.dump([], open(pp, "wb"))
    _torchrun(2, ["--model_path", path, "--prompt_pickle", str(pp), "--output_file", str(tmp_path / "o.pkl")],
              str(tmp_path))
    assert pickle.load(open(tmp_path / "o.pkl", "rb")) == []


def test_repeated_pass_defaults():
    """--prefix_kv_cache / --hbm_cache_gb default to auto: on for generation / repeated passes."""
    from flexible_llm_sharding_amd.api import repeated_passes, resolve_hbm_cache_gb, resolve_prefix_kv_cache
    from flexible_llm_sharding_amd.config import preset
    import torch
    base = ["--prompt_pickle", "p.pkl", "--output_file", "o.pkl"]
    a = parse_args(base)
    assert a.prefix_kv_cache == "auto" and a.hbm_cache_gb == "auto"
    assert not repeated_passes(a) and not resolve_prefix_kv_cache(a)
    g = parse_args(base + ["--num_gen_token", "4"])
    assert repeated_passes(g) and resolve_prefix_kv_cache(g)
    assert repeated_passes(parse_args(base + ["--num_batch", "2"]))
    assert not resolve_prefix_kv_cache(parse_args(base + ["--num_gen_token", "4", "--prefix_kv_cache", "false"]))
    # a VRAM cap: the cache lives in pinned host memory (host mode), so auto stays on while the
    # host has room for it
    from flexible_llm_sharding_amd.api import host_kv_fits
    capped = parse_args(base + ["--num_gen_token", "4", "--max_vram_gb", "6"])
    assert resolve_prefix_kv_cache(capped)
    assert host_kv_fits(1 << 20) and not host_kv_fits(1 << 60)
    # suffix K/V reuse is on by default with the prefix cache on one GPU (exact: row-independent
    # kernels, engine "exact K/V reuse"); off on several ranks and without the prefix cache
    from flexible_llm_sharding_amd.api import resolve_suffix_kv_cache
    assert g.suffix_kv_cache == "auto" and resolve_suffix_kv_cache(g, 1) and not resolve_suffix_kv_cache(g, 2)
    # under a cap a step is PCIe-bound: the suffix regions cost more to stage than the suffix tokens
    # cost to recompute, so auto keeps only the prefix cache there
    assert not resolve_suffix_kv_cache(a, 1) and not resolve_suffix_kv_cache(capped, 1)
    # reuse is row-exact unless --exact_reuse false asks for the small-M kernels
    assert g.exact_reuse is True and parse_args(base + ["--exact_reuse", "false"]).exact_reuse is False
    assert not resolve_suffix_kv_cache(parse_args(base + ["--num_gen_token", "4", "--suffix_kv_cache", "false"]), 1)
    assert parse_args(base + ["--hbm_cache_gb", "12.5"]).hbm_cache_gb == 12.5
    cfg = preset("tiny")
    assert resolve_hbm_cache_gb(g, cfg, torch.device("cpu")) == 0.0       # nothing to cache on a CPU run
    assert resolve_hbm_cache_gb(parse_args(base + ["--hbm_cache_gb", "3"]), cfg, torch.device("cpu")) == 3.0


def test_greedy_tokens_equal_numpy_argmax():
    """Generation's argmax on the fp16 bit patterns == np.argmax, ties (first index) included."""
    import numpy as np
    from flexible_llm_sharding_amd.api import greedy_tokens
    rng = np.random.default_rng(0)
    a = rng.random((7, 3, 1000)).astype(np.float16)
    a[0, 0, 10] = a[0, 0, 20] = 2.0                      # tie: first index wins
    a[1, 1] = 0.0
    assert np.array_equal(greedy_tokens(a), np.argmax(a, axis=-1))
    b = a.copy()
    b[2, 2, 5] = -1.0                                     # a negative value: generic path
    assert np.array_equal(greedy_tokens(b), np.argmax(b, axis=-1))
    assert np.array_equal(greedy_tokens(a.astype(np.float32)), np.argmax(a, axis=-1))


def test_prefix_kv_bytes_counts_suffix_regions(tmp_path):
    """The --hbm_cache_gb auto reserve covers the suffix regions PrefixKVCache.begin allocates
    (len(suffix) + SUFFIX_GROWTH rows each) when suffix reuse is on."""
    from flexible_llm_sharding_amd.api import prefix_kv_bytes
    from flexible_llm_sharding_amd.config import preset
    from flexible_llm_sharding_amd.runtime.prefix_cache import PrefixKVCache
    from flexible_llm_sharding_amd.utils.tokenizer import load_tokenizer, write_synthetic_tokenizer
    cfg = preset("tiny")
    write_synthetic_tokenizer(str(tmp_path), cfg.vocab_size)
    tok = load_tokenizer(str(tmp_path))
    prompts = [("alpha beta gamma", ("x y", "z")), ("delta", ("one two three",))]
    per_row = 2 * cfg.num_key_value_heads * cfg.head_dim * 2 * 3
    pre = sum(len(tok(p[0]).input_ids) for p in prompts)
    sfx = sum(len(ids) + PrefixKVCache.SUFFIX_GROWTH for p in prompts for ids in tok(list(p[1])).input_ids)
    assert prefix_kv_bytes(cfg, tok, prompts, 3) == pre * per_row
    assert prefix_kv_bytes(cfg, tok, prompts, 3, suffix_kv_cache=True) == (pre + sfx) * per_row


def test_every_env_knob_is_registered():
    """Every FLS_* environment variable read by the package, bench.py or main.py is listed (with a
    default and a description) in knobs.py, the one documented list."""
    import pathlib
    import re

    from flexible_llm_sharding_amd import knobs
    root = pathlib.Path(__file__).resolve().parents[1]
    srcs = list((root / "flexible_llm_sharding_amd").rglob("*.py")) + [root / "bench.py", root / "main.py"]
    used = set()
    for p in srcs:
        if p.name == "knobs.py":
            continue
        used |= set(re.findall(r"\bFLS_[A-Z0-9_]+\b", p.read_text()))
    missing = sorted(used - set(knobs.KNOBS))
    assert not missing, f"unregistered FLS_* knobs: {missing}"
    for name, (default, doc) in knobs.KNOBS.items():
        assert doc.strip(), name
    # reads go through the registry: an unknown name is refused
    import pytest
    with pytest.raises(KeyError):
        knobs.get("FLS_NOT_A_KNOB")
    # the README carries the table
    readme = (root / "README.md").read_text()
    assert all(f"`{n}`" in readme for n in knobs.KNOBS), "README knob table out of date"


def test_dp_gather_comm_flag():
    """--dp_gather_comm native: the data-parallel prefetchers' gather communicator (Comm.dup) becomes
    the native RCCL one on a GPU; on the CPU (gloo tests) dup() keeps torch.distributed."""
    from flexible_llm_sharding_amd.parallel.comm import Comm
    base = ["--prompt_pickle", "p.pkl", "--output_file", "o.pkl"]
    assert parse_args(base).dp_gather_comm == "torch"
    assert parse_args(base + ["--dp_gather_comm", "native"]).dp_gather_comm == "native"
    c = Comm(0, 1, "cpu")
    c.gather_native = True
    d = c.dup()
    assert type(d) is Comm and d.world == 1
