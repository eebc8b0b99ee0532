"""CPU engine: mode equivalence, oracle parity, HF transformers parity (causal mode)."""
import os

import numpy as np
import pytest
import torch

from flexible_llm_sharding_amd.engine import ShardedRunner
from flexible_llm_sharding_amd.models.reference import reference_scores
from flexible_llm_sharding_amd.runtime.batch import pack_prompts, split_microbatches
from flexible_llm_sharding_amd.runtime.stream import FileLayerSource
from flexible_llm_sharding_amd.runtime.weights import HostStore
from flexible_llm_sharding_amd.utils.synthetic import load_full_state_dict, synthetic_prompts
from flexible_llm_sharding_amd.utils.tokenizer import load_tokenizer, tokenize_prompt


@pytest.fixture(scope="module")
def ctx(tiny_model):
    path, cfg = tiny_model
    tok = load_tokenizer(path)
    prompts = synthetic_prompts(5, 30, 3, 7, cfg.vocab_size, seed=11, vary=True)
    sd = load_full_state_dict(cfg, path)
    return path, cfg, tok, prompts, sd


def test_tokenize_contract(ctx):
    path, cfg, tok, prompts, sd = ctx
    tp = tokenize_prompt(tok, "wd we wf", ("wg wh", "wi", "wj wk wl"))
    assert tp.prefix[0] == tok.bos_token_id and len(tp.prefix) == 4
    assert tp.padded_len == 3 and tp.eos_index == [1, 0, 2]
    assert [len(s) for s in tp.suffixes] == [2, 1, 3]      # BOS dropped, padding not computed
    assert tp.padded_tokens == 4 + 3 * 3


def test_batched_tokenize_equals_per_prompt(ctx):
    """tokenize_prompts (two batched tokenizer calls) == tokenize_prompt per prompt, incl. truncation,
    suffixes of different lengths and empty suffix strings."""
    from flexible_llm_sharding_amd.utils.tokenizer import tokenize_prompts
    path, cfg, tok, prompts, sd = ctx
    extra = [("wd we wf", ("wg wh", "", "wj wk wl wm")), ("wa " * 50, ("wb",))]
    for max_len in (4096, 16):
        got = tokenize_prompts(tok, list(prompts) + extra, max_len)
        want = [tokenize_prompt(tok, p, s, max_len) for p, s in list(prompts) + extra]
        assert [vars(g) for g in got] == [vars(w) for w in want]


def test_microbatch_split():
    from flexible_llm_sharding_amd.utils.tokenizer import TokenizedPrompt
    tps = [TokenizedPrompt([1] * 10, [[1] * 5], 5, [4]) for _ in range(7)]   # 15 tokens each
    g = split_microbatches(tps, 40)
    assert g == [[0, 1], [2, 3], [4, 5], [6]]
    assert split_microbatches(tps, 5) == [[i] for i in range(7)]
    # as many micro-batches as greedy filling needs, evened out (bench --prompts-per-gpu 128 under
    # its 24,576-token plan: 8 x 16 prompts, not 7 x 18 + 2)
    big = [TokenizedPrompt([1] * 1024, [[1] * 64] * 5, 64, [63] * 5) for _ in range(128)]
    assert [len(x) for x in split_microbatches(big, 24576)] == [16] * 8
    assert [len(x) for x in split_microbatches(big[:32], 16384)] == [11, 11, 10]
    # a prompt larger than the budget never raises the packing limit above it (the capped plan
    # sizes the arena for token_budget rows): [1000, 30000, 20000, 5000] under 24,576
    odd = [TokenizedPrompt([1] * (n - 1), [[1]], 1, [0]) for n in (1000, 30000, 20000, 5000)]
    g = split_microbatches(odd, 24576)
    assert sorted(i for x in g for i in x) == [0, 1, 2, 3]
    for x in g:
        assert len(x) == 1 or sum(odd[i].num_tokens for i in x) <= 24576


def test_pack_segments():
    from flexible_llm_sharding_amd.utils.tokenizer import TokenizedPrompt
    tp = TokenizedPrompt([1, 5, 6], [[7, 8], [9]], 2, [1, 0])
    b = pack_prompts([tp, tp], [0, 1], "bidirectional")
    assert b.num_tokens == 12
    assert b.positions.tolist() == [0, 1, 2, 3, 4, 3] * 2
    assert b.last_idx.tolist() == [4, 5, 10, 11]
    # per prompt: one prefix item + one item over both suffixes (block-diagonal range 1)
    assert b.work.shape == (4, 8)
    assert b.work[1].tolist() == [3, 3, 0, 0, 3, 0, 3, 3]
    assert b.seg_lo.tolist() == [0, 0, 0, 3, 3, 5, 6, 6, 6, 9, 9, 11]


@pytest.mark.parametrize("q_block", [64, 128])
@pytest.mark.parametrize("prefix_attention", ["bidirectional", "causal"])
def test_work_items_cover_segments(q_block, prefix_attention):
    """Every packed query row sees, through the work items + seg_lo (the attention kernel's
    semantics), exactly the keys its segment defines: the whole prefix (or its causal part) and
    its own suffix up to itself — with suffixes of many lengths sharing items."""
    from flexible_llm_sharding_amd.runtime.batch import visible_keys
    from flexible_llm_sharding_amd.utils.tokenizer import TokenizedPrompt
    rng = np.random.default_rng(3)
    tps = []
    for lp, lens in [(70, [5, 64, 1, 3, 100]), (1, [3]), (130, [65, 17, 129, 2]), (200, [33, 64] * 4)]:
        tps.append(TokenizedPrompt(list(range(lp)), [list(rng.integers(0, 9, l)) for l in lens], max(lens),
                                   [l - 1 for l in lens]))
    b = pack_prompts(tps, list(range(len(tps))), prefix_attention, q_block=q_block)
    assert int(b.work[:, 1].max()) <= q_block
    covered = np.zeros(b.num_tokens, np.int32)
    for q_start, q_len, *_ in b.work.tolist():
        covered[q_start:q_start + q_len] += 1
    assert (covered == 1).all()                        # every row in exactly one item
    for sg in b.segments:
        for i in range(sg.q_len):
            row = sg.q_start + i
            want = []
            if sg.r0_len:
                qi = sg.q_off + i
                want.append((0, sg.r0_start, sg.r0_start + (min(sg.r0_len - 1, qi) if sg.r0_causal else sg.r0_len - 1)))
            if sg.r1_len:
                want.append((1, sg.r1_start, sg.r1_start + i))
            assert visible_keys(b.work, b.seg_lo, row) == want, (row, sg)
    n_sfx_items = int((b.work[:, 7] > 0).sum())
    assert n_sfx_items == sum(-(-sum(len(s) for s in tp.suffixes) // q_block) for tp in tps)


@pytest.mark.parametrize("storage", ["gpu", "cpu", "disk"])
@pytest.mark.parametrize("lnps", [1, 2, 7])
@pytest.mark.parametrize("budget", [25, 100000])
def test_engine_matches_oracle(ctx, tmp_path, storage, lnps, budget):
    path, cfg, tok, prompts, sd = ctx
    r = ShardedRunner(cfg, FileLayerSource(cfg, path), "cpu", tok, layer_num_per_shard=lnps,
                      storage_location=storage, disk_folder=str(tmp_path), token_budget=budget)
    out = r(prompts)
    ref = reference_scores(cfg, sd, tok, prompts)
    for o, rf in zip(out, ref):
        assert o.shape == rf.shape and o.dtype == np.float16
        assert np.abs(o.astype(np.float32) - rf).max() < 1e-4
    # probabilities are not degenerate
    assert max(float(o.max()) for o in out) > 3.0 / cfg.vocab_size


def test_host_store_equals_file_source(ctx):
    path, cfg, tok, prompts, sd = ctx
    a = ShardedRunner(cfg, FileLayerSource(cfg, path), "cpu", tok)(prompts)
    b = ShardedRunner(cfg, HostStore.from_model_path(cfg, path, pinned=False), "cpu", tok,
                      layer_num_per_shard=3)(prompts)
    for x, y in zip(a, b):
        assert np.array_equal(x, y)


def test_causal_prefix_matches_hf_transformers(ctx):
    """--prefix_attention causal == HF LlamaForCausalLM on prefix+suffix (parity anchor)."""
    transformers = pytest.importorskip("transformers")
    path, cfg, tok, prompts, sd = ctx
    hf_cfg = transformers.LlamaConfig(
        hidden_size=cfg.hidden_size, intermediate_size=cfg.intermediate_size,
        num_attention_heads=cfg.num_attention_heads, num_key_value_heads=cfg.num_key_value_heads,
        num_hidden_layers=cfg.num_hidden_layers, vocab_size=cfg.vocab_size, rms_norm_eps=cfg.rms_norm_eps,
        rope_theta=cfg.rope_theta, max_position_embeddings=cfg.max_position_embeddings,
        tie_word_embeddings=False)
    model = transformers.LlamaForCausalLM(hf_cfg).float().eval()
    model.load_state_dict({k: v.float() for k, v in sd.items()}, strict=False)
    r = ShardedRunner(cfg, FileLayerSource(cfg, path), "cpu", tok, prefix_attention="causal")
    out = r(prompts)
    for (prefix, sufs), o in zip(prompts, out):
        tp = tokenize_prompt(tok, prefix, sufs)
        for j, s in enumerate(tp.suffixes):
            ids = torch.tensor([tp.prefix + s])
            with torch.no_grad():
                logits = model(ids).logits[0, -1].float()
            p = torch.softmax(logits, -1).numpy()
            # our fp32 path uses fp16-rounded cos/sin tables like the reference; HF uses fp32
            assert np.abs(o[j, 0].astype(np.float32) - p).max() < 2e-3


def test_bidirectional_differs_from_causal(ctx):
    path, cfg, tok, prompts, sd = ctx
    a = ShardedRunner(cfg, FileLayerSource(cfg, path), "cpu", tok, prefix_attention="causal")(prompts)
    b = ShardedRunner(cfg, FileLayerSource(cfg, path), "cpu", tok)(prompts)
    assert any(np.abs(x.astype(np.float32) - y.astype(np.float32)).max() > 1e-4 for x, y in zip(a, b))
    ref = reference_scores(cfg, sd, tok, prompts, prefix_attention="causal")
    for x, rf in zip(a, ref):
        assert np.abs(x.astype(np.float32) - rf).max() < 1e-4


def test_checkpoint_resume_after_fault(ctx, tmp_path, monkeypatch):
    """--resume_dir: a run that dies at shard 3 restarts from the step-2 checkpoint and matches a clean run."""
    path, cfg, tok, prompts, sd = ctx
    src = FileLayerSource(cfg, path)

    def runner():
        return ShardedRunner(cfg, src, "cpu", tok, layer_num_per_shard=1, storage_location="cpu",
                             token_budget=40, resume_dir=str(tmp_path / "ck"), checkpoint_every=2)

    clean = ShardedRunner(cfg, src, "cpu", tok, layer_num_per_shard=1, token_budget=40)(prompts)
    monkeypatch.setenv("FLS_FAULT", "0:3")          # tiny: 5 layers = 5 shards, checkpoint after shards 1, 3
    with pytest.raises(RuntimeError, match="FLS_FAULT"):
        runner()(prompts)
    assert sorted(os.listdir(tmp_path / "ck" / "rank0")) == ["step2"]
    monkeypatch.delenv("FLS_FAULT")
    r = runner()
    out = r(prompts)
    assert r.stats["resumed_from_shard"] == 2
    assert not (tmp_path / "ck").exists()             # cleared on completion
    for a, b in zip(out, clean):
        np.testing.assert_array_equal(a, b)
    # different prompts -> fingerprint mismatch -> no resume
    monkeypatch.setenv("FLS_FAULT", "0:4")
    with pytest.raises(RuntimeError):
        runner()(prompts)
    monkeypatch.delenv("FLS_FAULT")
    r = runner()
    r(prompts[:3])
    assert r.stats["resumed_from_shard"] == 0
    # keep-last-two pruning
    from flexible_llm_sharding_amd.runtime.checkpoint import RunCheckpoint
    ck = RunCheckpoint(str(tmp_path / "k2"), "fp")
    for k in (1, 2, 3):
        ck.save_state(k, 0, torch.ones(2, 3))
        ck.commit(k, [0], torch.float32)
    assert ck.available() == [2, 3]
    assert torch.equal(ck.load(3)[0], torch.ones(2, 3))


# Llama checkpoints whose RoPE tables or head geometry differ from Llama-2 (Llama-3.1's llama3
# scaling, linear and YaRN scaling, an explicit head_dim with nh*hd != hidden as in Mistral-Nemo)
LLAMA_VARIANTS = {
    "llama3_rope": dict(rope_theta=500000.0, rope_scaling={
        "rope_type": "llama3", "factor": 8.0, "low_freq_factor": 1.0, "high_freq_factor": 4.0,
        "original_max_position_embeddings": 64}),
    "linear_rope": dict(rope_scaling={"rope_type": "linear", "factor": 4.0}),
    "yarn_rope": dict(rope_theta=1e6, rope_scaling={"rope_type": "yarn", "factor": 4.0,
                                                    "original_max_position_embeddings": 1024}),
    "head_dim_32": dict(explicit_head_dim=32),
}


def _hf_family_case(tmp_path, family):
    """tiny random checkpoint of another Llama-structured family + its HF model."""
    transformers = pytest.importorskip("transformers")
    from flexible_llm_sharding_amd.config import preset
    from flexible_llm_sharding_amd.utils.synthetic import write_synthetic_checkpoint
    from flexible_llm_sharding_amd.utils.tokenizer import write_synthetic_tokenizer
    if family == "qwen2":
        cfg = preset("tiny-qwen2")
        hf_cfg = transformers.Qwen2Config(
            hidden_size=cfg.hidden_size, intermediate_size=cfg.intermediate_size,
            num_attention_heads=cfg.num_attention_heads, num_key_value_heads=cfg.num_key_value_heads,
            num_hidden_layers=cfg.num_hidden_layers, vocab_size=cfg.vocab_size, rms_norm_eps=cfg.rms_norm_eps,
            rope_theta=cfg.rope_theta, max_position_embeddings=cfg.max_position_embeddings,
            tie_word_embeddings=False, use_sliding_window=False)
        model = transformers.Qwen2ForCausalLM(hf_cfg)
    elif family == "qwen3":
        cfg = preset("tiny-qwen3")
        hf_cfg = transformers.Qwen3Config(
            hidden_size=cfg.hidden_size, intermediate_size=cfg.intermediate_size,
            num_attention_heads=cfg.num_attention_heads, num_key_value_heads=cfg.num_key_value_heads,
            num_hidden_layers=cfg.num_hidden_layers, vocab_size=cfg.vocab_size, rms_norm_eps=cfg.rms_norm_eps,
            rope_theta=cfg.rope_theta, max_position_embeddings=cfg.max_position_embeddings,
            head_dim=cfg.head_dim, tie_word_embeddings=False, use_sliding_window=False, attention_bias=False)
        model = transformers.Qwen3ForCausalLM(hf_cfg)
    elif family in ("phi3", "phi3_mini"):
        cfg = (preset("tiny-phi3", sliding_window=64) if family == "phi3"
               else preset("tiny-phi3-mini", rope_theta=10000.0))
        rs = dict(cfg.rope_scaling or {"rope_type": "default"}, rope_theta=cfg.rope_theta)
        hf_cfg = transformers.Phi3Config(
            hidden_size=cfg.hidden_size, intermediate_size=cfg.intermediate_size,
            num_attention_heads=cfg.num_attention_heads, num_key_value_heads=cfg.num_key_value_heads,
            num_hidden_layers=cfg.num_hidden_layers, vocab_size=cfg.vocab_size, rms_norm_eps=cfg.rms_norm_eps,
            max_position_embeddings=cfg.max_position_embeddings, original_max_position_embeddings=4096,
            rope_parameters=rs, sliding_window=cfg.sliding_window, tie_word_embeddings=False, pad_token_id=0)
        model = transformers.Phi3ForCausalLM(hf_cfg)
    elif family == "mixtral":
        cfg = preset("tiny-mixtral")
        hf_cfg = transformers.MixtralConfig(
            hidden_size=cfg.hidden_size, intermediate_size=cfg.intermediate_size,
            num_attention_heads=cfg.num_attention_heads, num_key_value_heads=cfg.num_key_value_heads,
            num_hidden_layers=cfg.num_hidden_layers, vocab_size=cfg.vocab_size, rms_norm_eps=cfg.rms_norm_eps,
            rope_theta=cfg.rope_theta, max_position_embeddings=cfg.max_position_embeddings,
            num_local_experts=cfg.num_local_experts, num_experts_per_tok=cfg.num_experts_per_tok,
            tie_word_embeddings=False, sliding_window=None)
        model = transformers.MixtralForCausalLM(hf_cfg)
    elif family == "qwen3_moe":
        cfg = preset("tiny-qwen3-moe")
        hf_cfg = transformers.Qwen3MoeConfig(
            hidden_size=cfg.hidden_size, intermediate_size=cfg.intermediate_size,
            moe_intermediate_size=cfg.moe_intermediate_size, num_experts=cfg.num_local_experts,
            num_experts_per_tok=cfg.num_experts_per_tok, norm_topk_prob=cfg.norm_topk_prob,
            num_attention_heads=cfg.num_attention_heads, num_key_value_heads=cfg.num_key_value_heads,
            num_hidden_layers=cfg.num_hidden_layers, vocab_size=cfg.vocab_size, rms_norm_eps=cfg.rms_norm_eps,
            rope_theta=cfg.rope_theta, max_position_embeddings=cfg.max_position_embeddings,
            head_dim=cfg.head_dim, tie_word_embeddings=False, use_sliding_window=False, attention_bias=False)
        model = transformers.Qwen3MoeForCausalLM(hf_cfg)
    elif family == "qwen2_moe":
        cfg = preset("tiny-qwen2-moe")
        hf_cfg = transformers.Qwen2MoeConfig(
            hidden_size=cfg.hidden_size, intermediate_size=cfg.intermediate_size,
            moe_intermediate_size=cfg.moe_intermediate_size, num_experts=cfg.num_local_experts,
            num_experts_per_tok=cfg.num_experts_per_tok, norm_topk_prob=cfg.norm_topk_prob,
            shared_expert_intermediate_size=cfg.shared_expert_intermediate_size,
            num_attention_heads=cfg.num_attention_heads, num_key_value_heads=cfg.num_key_value_heads,
            num_hidden_layers=cfg.num_hidden_layers, vocab_size=cfg.vocab_size, rms_norm_eps=cfg.rms_norm_eps,
            rope_theta=cfg.rope_theta, max_position_embeddings=cfg.max_position_embeddings,
            tie_word_embeddings=False, use_sliding_window=False, qkv_bias=True)
        model = transformers.Qwen2MoeForCausalLM(hf_cfg)
    elif family == "granite":
        cfg = preset("tiny-granite")
        hf_cfg = transformers.GraniteConfig(
            hidden_size=cfg.hidden_size, intermediate_size=cfg.intermediate_size,
            num_attention_heads=cfg.num_attention_heads, num_key_value_heads=cfg.num_key_value_heads,
            num_hidden_layers=cfg.num_hidden_layers, vocab_size=cfg.vocab_size, rms_norm_eps=cfg.rms_norm_eps,
            rope_theta=cfg.rope_theta, max_position_embeddings=cfg.max_position_embeddings,
            embedding_multiplier=cfg.embedding_multiplier, residual_multiplier=cfg.residual_multiplier,
            attention_multiplier=cfg.attention_multiplier, logits_scaling=cfg.logits_scaling,
            tie_word_embeddings=False)
        model = transformers.GraniteForCausalLM(hf_cfg)
    elif family in LLAMA_VARIANTS:
        over = dict(LLAMA_VARIANTS[family])
        cfg = preset("tiny", **over)
        hf_cfg = transformers.LlamaConfig(
            hidden_size=cfg.hidden_size, intermediate_size=cfg.intermediate_size,
            num_attention_heads=cfg.num_attention_heads, num_key_value_heads=cfg.num_key_value_heads,
            num_hidden_layers=cfg.num_hidden_layers, vocab_size=cfg.vocab_size, rms_norm_eps=cfg.rms_norm_eps,
            rope_theta=cfg.rope_theta, max_position_embeddings=cfg.max_position_embeddings,
            tie_word_embeddings=False, rope_scaling=cfg.rope_scaling, head_dim=cfg.head_dim)
        model = transformers.LlamaForCausalLM(hf_cfg)
    else:
        cfg = preset("tiny", model_type="mistral", architectures=["MistralForCausalLM"], rope_theta=1e6,
                     sliding_window=4096)
        hf_cfg = transformers.MistralConfig(
            hidden_size=cfg.hidden_size, intermediate_size=cfg.intermediate_size,
            num_attention_heads=cfg.num_attention_heads, num_key_value_heads=cfg.num_key_value_heads,
            num_hidden_layers=cfg.num_hidden_layers, vocab_size=cfg.vocab_size, rms_norm_eps=cfg.rms_norm_eps,
            rope_theta=cfg.rope_theta, max_position_embeddings=cfg.max_position_embeddings,
            tie_word_embeddings=False, sliding_window=4096)
        model = transformers.MistralForCausalLM(hf_cfg)
    path = str(tmp_path / family)
    write_synthetic_checkpoint(cfg, path, seed=5, std=0.05)
    write_synthetic_tokenizer(path, cfg.vocab_size)
    sd = load_full_state_dict(cfg, path)
    missing, unexpected = model.float().eval().load_state_dict(
        {k: v.float() for k, v in _hf_v5_names(cfg, sd).items()}, strict=False)
    assert not unexpected and all("rotary" in m for m in missing), (missing, unexpected)
    return path, cfg, sd, model


def _hf_v5_names(cfg, sd):
    """Per-expert checkpoint tensors (the released form our layer files keep) -> transformers v5's
    stacked expert parameters (``mlp.experts.gate_up_proj`` / ``down_proj``, router ``mlp.gate``)."""
    if not cfg.is_moe:
        return sd
    from flexible_llm_sharding_amd.models.layout import expert_names, router_name
    out = dict(sd)
    for i in range(cfg.num_hidden_layers):
        p = f"model.layers.{i}"
        names = [expert_names(cfg, p, e) for e in range(cfg.num_local_experts)]
        out[f"{p}.mlp.experts.gate_up_proj"] = torch.stack([torch.cat([out.pop(g), out.pop(u)]) for g, u, _ in names])
        out[f"{p}.mlp.experts.down_proj"] = torch.stack([out.pop(d) for _, _, d in names])
        out[f"{p}.mlp.gate.weight"] = out.pop(router_name(cfg, p))
    return out


@pytest.mark.parametrize("family", ["qwen2", "qwen3", "phi3", "phi3_mini", "mistral", "mixtral", "qwen3_moe",
                                    "qwen2_moe", "granite"] + sorted(LLAMA_VARIANTS))
def test_other_llama_families_match_hf(tmp_path, family):
    """Qwen2 (q/k/v biases, rope_theta 1e6), Qwen3 (per-head q/k RMSNorm, head_dim 128 on a
    256-wide residual), Phi-3 (fused qkv_proj / gate_up_proj, LongRoPE with its attention factor,
    sliding window covering the prompts), Mistral, the MoE families (Mixtral, Qwen3-MoE, Qwen2-MoE
    with its sigmoid-gated shared expert), Granite (embedding / residual / attention multipliers,
    logits scaling) == HF transformers in causal mode, and == the fp32 oracle in the reference's
    bidirectional-prefix mode."""
    from flexible_llm_sharding_amd.config import ModelConfig
    path, cfg, sd, model = _hf_family_case(tmp_path, family)
    assert ModelConfig.from_pretrained(path).attention_bias == (family in ("qwen2", "qwen2_moe"))
    assert ModelConfig.from_pretrained(path).qk_norm == (family in ("qwen3", "qwen3_moe"))
    assert ModelConfig.from_pretrained(path).num_local_experts == cfg.num_local_experts
    tok = load_tokenizer(path)
    prompts = synthetic_prompts(3, 20, 2, 5, cfg.vocab_size, seed=9, vary=True)
    out = ShardedRunner(cfg, FileLayerSource(cfg, path), "cpu", tok, prefix_attention="causal")(prompts)
    for (prefix, sufs), o in zip(prompts, out):
        tp = tokenize_prompt(tok, prefix, sufs)
        for j, s in enumerate(tp.suffixes):
            with torch.no_grad():
                logits = model(torch.tensor([tp.prefix + s])).logits[0, -1].float()
            assert np.abs(o[j, 0].astype(np.float32) - torch.softmax(logits, -1).numpy()).max() < 2e-3
    bid = ShardedRunner(cfg, FileLayerSource(cfg, path), "cpu", tok, layer_num_per_shard=2)(prompts)
    for o, rf in zip(bid, reference_scores(cfg, sd, tok, prompts)):
        assert np.abs(o.astype(np.float32) - rf).max() < 1e-4


def test_unsupported_configs_rejected():
    from flexible_llm_sharding_amd.config import ModelConfig
    for bad in ({"model_type": "gemma"}, {"mlp_bias": True}, {"hidden_act": "gelu"},
                {"rope_scaling": {"rope_type": "dynamic", "factor": 2.0}},
                {"model_type": "phi3", "partial_rotary_factor": 0.75},
                {"rope_scaling": {"type": "su", "short_factor": [1.0] * 64, "long_factor": [1.0] * 64},
                 "original_max_position_embeddings": 2048}):
        with pytest.raises(NotImplementedError):
            ModelConfig.from_dict(bad)
    with pytest.raises(ValueError):           # longrope factors must cover head_dim / 2
        ModelConfig.from_dict({"rope_parameters": {"rope_type": "longrope", "rope_theta": 1e4}})


def test_llama_structured_unlisted_family(tiny_model, tmp_path):
    """An unlisted model_type whose config describes the Llama block runs as Llama (the reference's
    AutoModelForCausalLM takes any such checkpoint, utils.py:109-115): same scores as the Llama run;
    a layer file holding a tensor Llama does not read, or a config key that changes the block, is
    refused instead of run wrong."""
    import json
    import shutil
    from safetensors.torch import load_file, save_file
    from flexible_llm_sharding_amd.config import ModelConfig, llama_like_rejection
    from flexible_llm_sharding_amd.runtime.stream import FileLayerSource
    from flexible_llm_sharding_amd.utils.layer_format import layer_file
    path, cfg = tiny_model
    d = str(tmp_path / "other")
    shutil.copytree(path, d)
    with open(os.path.join(d, "config.json")) as f:
        conf = json.load(f)
    conf["model_type"], conf["architectures"] = "llama_like_family", ["LlamaLikeForCausalLM"]
    with open(os.path.join(d, "config.json"), "w") as f:
        json.dump(conf, f)
    other = ModelConfig.from_pretrained(d)
    assert other.model_type == "llama_like_family"
    tok = load_tokenizer(path)
    prompts = synthetic_prompts(3, 30, 2, 6, cfg.vocab_size, seed=4)
    want = ShardedRunner(cfg, FileLayerSource(cfg, path), "cpu", tok)(prompts)
    for src in (FileLayerSource(other, d), HostStore.from_model_path(other, d, pinned=False)):
        got = ShardedRunner(other, src, "cpu", tok)(prompts)
        for a, b in zip(got, want):
            assert np.array_equal(a, b)
    # a tensor the Llama block does not have (e.g. a q norm) -> refused at load
    lf = layer_file(d, "model.layers.0")
    sd = load_file(lf)
    sd["model.layers.0.self_attn.q_norm.weight"] = torch.ones(other.head_dim)
    save_file(sd, lf)
    with pytest.raises(NotImplementedError, match="does not have"):
        ShardedRunner(other, FileLayerSource(other, d), "cpu", tok)(prompts)
    with pytest.raises(NotImplementedError, match="does not have"):
        HostStore.from_model_path(other, d, pinned=False)
    assert "scale_emb" in llama_like_rejection(dict(conf, scale_emb=12))
    assert "hidden_act" in llama_like_rejection(dict(conf, hidden_act="gelu"))
    with pytest.raises(NotImplementedError):
        ModelConfig.from_dict(dict(conf, kv_lora_rank=512))


def test_sliding_window_must_cover_prompts(tmp_path):
    """Windowed attention is full attention while every sequence fits the window; longer prompts
    are rejected instead of silently attending past the window."""
    from flexible_llm_sharding_amd.config import preset
    cfg = preset("tiny", sliding_window=24)
    store = HostStore.synthetic(cfg, "cpu", seed=1)
    from flexible_llm_sharding_amd.utils.tokenizer import write_synthetic_tokenizer
    write_synthetic_tokenizer(str(tmp_path), cfg.vocab_size)
    r = ShardedRunner(cfg, store, "cpu", load_tokenizer(str(tmp_path)))
    ok = synthetic_prompts(2, 16, 2, 8, cfg.vocab_size, seed=2)
    assert all(np.isfinite(o).all() for o in r(ok))
    with pytest.raises(ValueError, match="sliding_window"):
        r(synthetic_prompts(2, 20, 2, 8, cfg.vocab_size, seed=2))


def test_config_rope_and_head_dim_forms(tmp_path):
    """HF v4 (rope_theta + rope_scaling) and v5 (rope_parameters) config forms; explicit head_dim
    survives save/load."""
    from flexible_llm_sharding_amd.config import ModelConfig
    v4 = ModelConfig.from_dict({"rope_theta": 5e5, "rope_scaling": {"rope_type": "llama3", "factor": 8.0}})
    v5 = ModelConfig.from_dict({"rope_parameters": {"rope_type": "llama3", "factor": 8.0, "rope_theta": 5e5}})
    assert v4.rope_theta == v5.rope_theta == 5e5 and v4.rope_scaling == v5.rope_scaling
    assert ModelConfig.from_dict({"rope_parameters": {"rope_type": "default", "rope_theta": 1e6}}).rope_scaling is None
    c = ModelConfig.from_dict({"hidden_size": 256, "num_attention_heads": 4, "num_key_value_heads": 2,
                               "head_dim": 32})
    assert c.head_dim == 32 and c.q_size == 128
    c.save(str(tmp_path))
    assert ModelConfig.from_pretrained(str(tmp_path)) == c


def test_row_exact_packing_and_regions():
    """Generation packing (engine row_exact): no work item spans two suffixes (each item's range 1
    starts at its own suffix's first token, so key tiles sit at multiples of 64 tokens from it), and
    every suffix K/V region of a cache entry starts on a 64-row tile boundary, zero-filled."""
    from flexible_llm_sharding_amd.runtime.prefix_cache import PrefixEntry
    from flexible_llm_sharding_amd.utils.tokenizer import TokenizedPrompt
    tps = [TokenizedPrompt(list(range(lp)), [list(range(n)) for n in ns], max(ns), [n - 1 for n in ns])
           for lp, ns in ((70, [5, 64, 1, 130]), (1, [3]), (9, [40, 30, 30]))]
    for kv_cached in (False, True):
        offs = [0, 70, 71]
        b = pack_prompts(tps, [0, 1, 2], "bidirectional", prefix_offsets=offs, kv_cached=kv_cached, q_block=64,
                         single_suffix_items=True)
        seen = set()
        for q_start, q_len, q_off, r0s, r0l, r0c, r1s, r1l in b.work.tolist():
            if not r1l:
                continue
            rows = range(q_start, q_start + q_len)
            assert {int(b.seg_lo[r]) for r in rows} == {r1s}                # one suffix per item
            assert q_off == q_start - r1s and r1l == q_off + q_len
            seen.update(rows)
        assert seen == {r for sg in b.segments if sg.r1_len for r in range(sg.q_start, sg.q_start + sg.q_len)}
        multi = pack_prompts(tps, [0, 1, 2], "bidirectional", prefix_offsets=offs, kv_cached=kv_cached, q_block=64)
        assert any(len({int(multi.seg_lo[r]) for r in range(w[0], w[0] + w[1])}) > 1 for w in multi.work.tolist())
    e = PrefixEntry("k", [70, 1, 9], 16, "cpu", torch.float16, suffix_caps=[[69, 128, 65, 194], [67], [104, 94, 94]])
    starts = [r for rows in e.sfx_rows for r in rows]
    assert all(r % 64 == 0 for r in starts) and starts[0] >= 80 and len(set(starts)) == len(starts)
    buf = e.buffer("model.layers.0", create=True)
    assert buf.shape[0] >= starts[-1] + 94 and not buf.any()


def _host_mode(r):
    """Swap a runner's prefix K/V cache for a host-mode one (what --max_vram_gb builds)."""
    from flexible_llm_sharding_amd.runtime.prefix_cache import PrefixKVCache
    pc = r.prefix_cache
    r.prefix_cache = PrefixKVCache(pc.kv_cols, pc.dev, pc.dtype, pc.max_entries, suffix_reuse=pc.suffix_reuse,
                                   host=True)
    r.prefix_cache.on_evict = pc.on_evict
    return r


@pytest.mark.parametrize("host", [False, True])
@pytest.mark.parametrize("num_batch_calls", [1, 2])
def test_prefix_kv_cache_generation_exact(tiny_model, num_batch_calls, host):
    """--prefix_kv_cache: later calls on the same prefixes compute only suffix tokens, same scores
    (host: the entries in host memory, staged per layer — several micro-batches per call here)."""
    from flexible_llm_sharding_amd.api import generation_loop
    from flexible_llm_sharding_amd.engine import ShardedRunner
    from flexible_llm_sharding_amd.parallel.comm import Comm
    from flexible_llm_sharding_amd.runtime.weights import HostStore
    from flexible_llm_sharding_amd.utils.synthetic import synthetic_prompts
    from flexible_llm_sharding_amd.utils.tokenizer import load_tokenizer
    import argparse
    path, cfg = tiny_model
    tok = load_tokenizer(path)
    prompts = synthetic_prompts(5, 60, 3, 6, cfg.vocab_size, seed=21, vary=True)
    src = HostStore.from_model_path(cfg, path, pinned=False)
    args = argparse.Namespace(num_gen_token=3, data_parallel=False, num_batch=num_batch_calls)
    plain = ShardedRunner(cfg, src, "cpu", tok, layer_num_per_shard=2, token_budget=150)
    s0, u0 = generation_loop(args, plain, Comm(), tok, prompts)
    from flexible_llm_sharding_amd.api import batch_ranges
    b0, b1 = batch_ranges(len(prompts), num_batch_calls)[-1]
    last = plain.tokenize(prompts[b0:b1])
    n_prefix = sum(len(tp.prefix) for tp in last)
    for sfx in (False, True):
        cached = ShardedRunner(cfg, src, "cpu", tok, layer_num_per_shard=2, token_budget=150, prefix_kv_cache=True,
                               suffix_kv_cache=sfx)
        if host:
            _host_mode(cached)
        s1, u1 = generation_loop(args, cached, Comm(), tok, prompts)
        assert u0 == u1
        for a, b in zip(s0, s1):
            assert a.shape == b.shape
            assert np.abs(a.astype(np.float32) - b.astype(np.float32)).max() < 1e-5
        pc = cached.prefix_cache
        assert pc.misses == num_batch_calls and pc.hits == 2 * num_batch_calls
        if host:
            # staged in for every reused layer call, written back after every layer call
            assert pc.stage.bytes_h2d > 0 and pc.stage.bytes_d2h > 0
            assert all(not t.is_cuda for e in pc.entries.values() for t in e.layers.values())
        assert cached.stats["prefix_cached"] == 1.0
        if not sfx:
            # the cached pass computed only the suffix tokens of the last call's prompts
            assert cached.stats["tokens"] == plain.stats["tokens"] - n_prefix
        else:
            # ... and with suffix K/V reuse only what each suffix gained since the last step (>= 1 each)
            assert sum(tp.n_suffix for tp in last) <= cached.stats["tokens"] < plain.stats["tokens"] - n_prefix
            assert cached.stats["suffix_tokens_reused"] > 0


def test_host_mode_cache_grows_and_evicts(tiny_model):
    """Host-mode prefix K/V cache (--max_vram_gb): a larger call grows the staging buffer, LRU
    eviction drops entries (and their write-back events), and every call's scores stay those of a
    runner without a cache; repeated calls hit."""
    from flexible_llm_sharding_amd.engine import ShardedRunner
    from flexible_llm_sharding_amd.runtime.weights import HostStore
    path, cfg = tiny_model
    tok = load_tokenizer(path)
    src = HostStore.from_model_path(cfg, path, pinned=False)
    r = _host_mode(ShardedRunner(cfg, src, "cpu", tok, prefix_kv_cache=True, suffix_kv_cache=True,
                                 prefix_cache_entries=2))
    ref = ShardedRunner(cfg, src, "cpu", tok)
    small = synthetic_prompts(2, 20, 2, 4, cfg.vocab_size, seed=5)
    big = synthetic_prompts(4, 60, 3, 8, cfg.vocab_size, seed=6)
    other = synthetic_prompts(3, 30, 2, 5, cfg.vocab_size, seed=7)
    sizes = []
    for ps in (small, big, small, other, big, big):
        for a, b in zip(r(ps), ref(ps)):
            assert np.abs(a.astype(np.float32) - b.astype(np.float32)).max() < 1e-5
        sizes.append(r.prefix_cache.stage.bufs[0].shape[0])
    pc = r.prefix_cache
    assert sizes[1] > sizes[0] and sizes == sorted(sizes)          # grown, never shrunk
    assert len(pc.entries) <= 2 and pc.hits >= 2
    live = {id(t) for e in pc.entries.values() for t in e.layers.values()}
    assert all(k[0] in live for k in pc.stage.layer_ev)            # no events of evicted entries


def test_prefix_cache_invalidated_by_new_prefix(tiny_model):
    from flexible_llm_sharding_amd.engine import ShardedRunner
    from flexible_llm_sharding_amd.runtime.weights import HostStore
    from flexible_llm_sharding_amd.utils.synthetic import synthetic_prompts
    from flexible_llm_sharding_amd.utils.tokenizer import load_tokenizer
    path, cfg = tiny_model
    tok = load_tokenizer(path)
    src = HostStore.from_model_path(cfg, path, pinned=False)
    r = ShardedRunner(cfg, src, "cpu", tok, prefix_kv_cache=True)
    ref = ShardedRunner(cfg, src, "cpu", tok)
    p1 = synthetic_prompts(2, 30, 2, 4, cfg.vocab_size, seed=1)
    p2 = synthetic_prompts(2, 30, 2, 4, cfg.vocab_size, seed=2)
    for ps in (p1, p2, p1):
        out = r(ps)
        for a, b in zip(out, ref(ps)):
            assert np.abs(a.astype(np.float32) - b.astype(np.float32)).max() < 1e-5
    assert r.prefix_cache.hits == 1 and r.prefix_cache.misses == 2


@pytest.mark.parametrize("prefix_attention", ["bidirectional", "causal"])
def test_last_layer_pruning_is_exact(ctx, prefix_attention):
    """The last decoder layer computing only the scored rows (K/V for every token) gives the
    full computation's scores and fewer FLOPs; the final norm then skips its gather."""
    path, cfg, tok, prompts, sd = ctx
    src = FileLayerSource(cfg, path)
    full = ShardedRunner(cfg, src, "cpu", tok, prefix_attention=prefix_attention, token_budget=60,
                         prune_last_layer=False)
    pr = ShardedRunner(cfg, src, "cpu", tok, prefix_attention=prefix_attention, token_budget=60)
    a, b = full(prompts), pr(prompts)
    for x, y in zip(a, b):
        assert np.abs(x.astype(np.float32) - y.astype(np.float32)).max() < 1e-5
    assert pr.stats["decoder_flops"] < full.stats["decoder_flops"]


def test_prefetcher_slot_map_tiny_shards():
    """lnps=1 on a Llama-2-70B-shaped plan: the final RMSNorm (16 KB) owns a small buffer, the
    full-size shards alternate between the two slots in their own order, so the LM head's slot is
    not the last decoder layer's (it loads while that layer computes)."""
    from flexible_llm_sharding_amd.config import preset
    from flexible_llm_sharding_amd.parallel.planner import make_plan
    from flexible_llm_sharding_amd.runtime.prefetch import ShardPrefetcher
    from flexible_llm_sharding_amd.runtime.weights import HostStore
    cfg = preset("llama2-70b")
    names = cfg.layer_names()
    plan = make_plan(len(names), 1, 1, 0, False)
    shards = [s for s in plan.my_shards if len(s)]
    pf = ShardPrefetcher(HostStore(cfg, names=[]), names, shards, "cpu", n_slots=2)
    k_norm, k_head, k_last = len(shards) - 2, len(shards) - 1, len(shards) - 3
    assert pf.slot_of(k_norm) >= 2 and pf._slot_sizes[pf.slot_of(k_norm)] == pf.shard_bytes(k_norm)
    assert {pf.slot_of(k) for k in range(len(shards)) if k != k_norm} == {0, 1}
    assert pf.slot_of(k_head) != pf.slot_of(k_last)
    assert pf.slot_of(0) != pf.slot_of(1)
    assert pf.planned_hbm_bytes() == 2 * pf.slot_bytes + pf.shard_bytes(k_norm)
    # lnps = 8: no tiny shard, plain alternation
    plan8 = make_plan(len(names), 8, 1, 0, False)
    sh8 = [s for s in plan8.my_shards if len(s)]
    pf8 = ShardPrefetcher(HostStore(cfg, names=[]), names, sh8, "cpu", n_slots=2)
    assert [pf8.slot_of(k) for k in range(len(sh8))] == [k % 2 for k in range(len(sh8))]


@pytest.mark.parametrize("lnps,n_slots", [(1, 3), (1, 2), (8, 3), (3, 4)])
def test_prefetcher_slots_rotate_across_calls(lnps, n_slots):
    """The engine prefetches n_slots - 1 shards ahead and, past the last shard, the next call's first
    shards (epoch + 1).  Replaying that order over several calls: every load lands in a slot whose
    previous occupant was already released, and two shards live at the same time never share one."""
    from flexible_llm_sharding_amd.config import preset
    from flexible_llm_sharding_amd.parallel.planner import make_plan
    from flexible_llm_sharding_amd.runtime.prefetch import ShardPrefetcher
    from flexible_llm_sharding_amd.runtime.weights import HostStore
    cfg = preset("llama2-70b")
    names = cfg.layer_names()
    shards = [s for s in make_plan(len(names), lnps, 1, 0, False).my_shards if len(s)]
    pf = ShardPrefetcher(HostStore(cfg, names=[]), names, shards, "cpu", n_slots=n_slots)
    n, depth = len(shards), n_slots - 1
    occupant = {}                 # slot -> (epoch, shard) loaded last
    released, loaded = set(), set()

    def load(e, k):
        if (e, k) in loaded:
            return
        s = pf.slot_of(k, e)
        prev = occupant.get(s)
        assert prev is None or prev in released, (e, k, s, prev)
        occupant[s] = (e, k)
        loaded.add((e, k))

    for e in range(4):
        pf.epoch = e
        for k in range(min(n_slots, n)):        # __call__: the first shards (no-op if already loaded)
            load(e, k)
        for k in range(n):
            if k:
                released.add((e, k - 1))
            load(e, k)                          # acquire
            issued, j = 0, k + 1                # ShardedRunner._prefetch_ahead
            while issued < depth and j < k + 1 + n:
                ee, kk = (e, j) if j < n else (e + 1, j - n)   # past the end: the next call's shards
                load(ee, kk)
                issued += n_slots < 3 or pf.in_rotation(kk)   # own buffers: free lookahead (3+ slots)
                j += 1
        released.add((e, n - 1))
    if n_slots >= 3 and lnps == 1:              # embedding and LM head own buffers: rotation = decoders
        assert not pf.in_rotation(0) and not pf.in_rotation(n - 1) and pf.in_rotation(1)


def test_choose_kept_shards_spread_and_budget():
    from flexible_llm_sharding_amd.runtime.prefetch import choose_kept_shards
    sizes = [5] + [17] * 80 + [1, 5]                    # embed, 80 layers, norm, head (GB-ish units)
    for budget in (0, 17, 100, 17 * 40, 1000, sum(sizes)):
        keep = choose_kept_shards(sizes, budget)
        assert sum(sizes[k] for k in keep) <= budget
        assert keep == sorted(set(keep))
    assert choose_kept_shards(sizes, sum(sizes)) == list(range(len(sizes)))
    half = choose_kept_shards(sizes, sum(sizes) // 2)
    gaps = np.diff(half)
    assert len(half) >= 35 and gaps.max() <= 3         # kept shards interleave with streamed ones


@pytest.mark.parametrize("frac", [0.5, 1.0])
def test_hbm_cache_keeps_shards_and_matches(ctx, frac):
    """--hbm_cache_gb: some (or all) shards stay loaded across calls, the rest stream; scores equal
    the plain streaming run on every call, kept shards are never re-read."""
    path, cfg, tok, prompts, sd = ctx
    src = FileLayerSource(cfg, path)
    gb = frac * sum(src.nbytes(n) for n in cfg.layer_names()) / 1e9
    base = ShardedRunner(cfg, FileLayerSource(cfg, path), "cpu", tok, layer_num_per_shard=1, token_budget=60)
    r = ShardedRunner(cfg, src, "cpu", tok, layer_num_per_shard=1, token_budget=60, hbm_cache_gb=gb)
    pf = r.prefetcher
    kept = sorted(pf._sticky)
    assert kept and (frac < 1.0) == (len(kept) < len(r.my_shards))
    want = base(prompts)
    for _ in range(2):
        got = r(prompts)
        for a, b in zip(got, want):
            assert np.array_equal(a, b)
    assert all(pf.is_kept_loaded(k) for k in kept)
    assert not any(pf.is_kept_loaded(k) for k in range(len(r.my_shards)) if k not in kept)


def test_mp_micro_budget_fills_pipeline():
    """Model parallel: the per-call micro-batch budget shrinks so each of G stages sees >= 2
    micro-batches (not below 8k tokens); single / data parallel keep --token_budget."""
    from types import SimpleNamespace
    from flexible_llm_sharding_amd.utils.tokenizer import TokenizedPrompt
    tps = [TokenizedPrompt([1] * 1024, [[1] * 64] * 5, 64, [63] * 5) for _ in range(256)]   # 344k tokens
    total = sum(tp.num_tokens for tp in tps)
    for mode, world, want in (("mp", 8, -(-total // 16)), ("mp", 2, 49152), ("single", 1, 49152),
                              ("dp", 8, 49152)):
        r = SimpleNamespace(token_budget=49152, plan=SimpleNamespace(mode=mode), comm=SimpleNamespace(world=world),
                            MP_MICRO_PER_STAGE=2, MP_MIN_BUDGET=8192)
        b = ShardedRunner.micro_budget(r, tps)
        assert b == want, (mode, world, b)
        if mode == "mp":
            assert len(split_microbatches(tps, b)) >= 2 * world
    small = tps[:8]                                  # 10.8k tokens: the 8k floor wins
    r = SimpleNamespace(token_budget=49152, plan=SimpleNamespace(mode="mp"), comm=SimpleNamespace(world=8),
                        MP_MICRO_PER_STAGE=2, MP_MIN_BUDGET=8192)
    assert ShardedRunner.micro_budget(r, small) == 8192


def test_chunked_qkv_and_mlp_rows_match(tiny_model):
    """Row-chunked RMSNorm + QKV (the --max_vram_gb layout) and small MLP chunks give the same
    scores as whole-micro-batch projections."""
    from flexible_llm_sharding_amd.engine import ShardedRunner
    from flexible_llm_sharding_amd.models.llama import balanced_step
    from flexible_llm_sharding_amd.runtime.stream import FileLayerSource
    from flexible_llm_sharding_amd.utils.synthetic import synthetic_prompts
    from flexible_llm_sharding_amd.utils.tokenizer import load_tokenizer
    path, cfg = tiny_model
    tok = load_tokenizer(path)
    prompts = synthetic_prompts(5, 30, 3, 6, cfg.vocab_size, seed=4, vary=True)
    want = ShardedRunner(cfg, FileLayerSource(cfg, path), "cpu", tok)(prompts)
    r = ShardedRunner(cfg, FileLayerSource(cfg, path), "cpu", tok, mlp_chunk=24)
    r.ctx.qkv_chunk = 17
    got = r(prompts)
    for a, b in zip(want, got):
        assert np.abs(a.astype(np.float32) - b.astype(np.float32)).max() < 1e-5
    assert balanced_step(43008, 16384) == 15360 and balanced_step(100, 0) == 100
    assert balanced_step(43008, 8192) == 7680 and balanced_step(500, 1000) == 500
    assert balanced_step(43008, 16384, align=256) == 14336 and balanced_step(1000, 800) == 768


@pytest.mark.parametrize("prune", [True, False])
def test_grouped_attention_phase_matches(tiny_model, prune):
    """--max_vram_gb's attention phase in prompt-aligned row groups (group-relative work items)
    gives the whole-micro-batch scores, with and without the pruned last layer."""
    from flexible_llm_sharding_amd.engine import ShardedRunner
    from flexible_llm_sharding_amd.runtime.batch import pack_prompts
    from flexible_llm_sharding_amd.runtime.stream import FileLayerSource
    from flexible_llm_sharding_amd.utils.synthetic import synthetic_prompts
    from flexible_llm_sharding_amd.utils.tokenizer import load_tokenizer, tokenize_prompts
    path, cfg = tiny_model
    tok = load_tokenizer(path)
    prompts = synthetic_prompts(6, 30, 3, 6, cfg.vocab_size, seed=5, vary=True)
    want = ShardedRunner(cfg, FileLayerSource(cfg, path), "cpu", tok, prune_last_layer=prune)(prompts)
    r = ShardedRunner(cfg, FileLayerSource(cfg, path), "cpu", tok, prune_last_layer=prune)
    r.ctx.attn_rows = 70
    got = r(prompts)
    for a, b in zip(want, got):
        assert np.abs(a.astype(np.float32) - b.astype(np.float32)).max() < 1e-5
    # the groups cover every row / work item / scored row once, prompt-aligned
    tps = tokenize_prompts(tok, prompts, 4096)
    pb = pack_prompts(tps, list(range(len(tps))))
    gs = pb.attn_groups(70)
    assert gs[0]["r0"] == 0 and gs[-1]["r1"] == pb.num_tokens and len(gs) > 1
    assert sum(len(g["work"]) for g in gs) == len(pb.work)
    assert sum(len(g["last_local"]) for g in gs) == pb.n_scored
    for g in gs:
        assert (g["work"][:, 0] >= 0).all() and (g["work"][:, 0] + g["work"][:, 1] <= g["r1"] - g["r0"]).all()


@pytest.mark.parametrize("family", ["tiny-mixtral", "tiny-qwen3-moe"])
def test_moe_chunks_shards_storage_match_oracle(tmp_path, family):
    """MoE decoder layers through every engine path that reshapes the MLP phase: token chunks of
    the expert FFN (routing per chunk), multi-layer shards, activations spilled to disk — all equal
    the fp32 oracle of HF's MoE block."""
    from flexible_llm_sharding_amd.config import preset
    from flexible_llm_sharding_amd.engine import ShardedRunner
    from flexible_llm_sharding_amd.runtime.stream import FileLayerSource
    from flexible_llm_sharding_amd.utils.synthetic import synthetic_prompts, write_synthetic_checkpoint
    cfg = preset(family)
    path = str(tmp_path / family)
    write_synthetic_checkpoint(cfg, path, seed=3, std=0.05)
    tok = load_tokenizer(path)
    prompts = synthetic_prompts(4, 30, 3, 6, cfg.vocab_size, seed=5, vary=True)
    ref = reference_scores(cfg, load_full_state_dict(cfg, path), tok, prompts)
    for kw in ({}, {"mlp_chunk": 24}, {"layer_num_per_shard": 2, "storage_location": "disk",
                                       "disk_folder": str(tmp_path / "spill"), "token_budget": 64}):
        out = ShardedRunner(cfg, FileLayerSource(cfg, path), "cpu", tok, **kw)(prompts)
        for o, rf in zip(out, ref):
            assert np.abs(o.astype(np.float32) - rf).max() < 1e-4, kw


@pytest.mark.parametrize("host", [False, True])
def test_suffix_kv_reuse_partial_and_overflow(tiny_model, host):
    """Suffix K/V reuse keeps only the common token prefix with the last call: suffixes edited in
    the middle, grown past their cache region (reuse off for that call), shortened, or dropped —
    every call's scores equal a runner without any cache."""
    from flexible_llm_sharding_amd.engine import ShardedRunner
    from flexible_llm_sharding_amd.runtime.prefix_cache import PrefixKVCache
    from flexible_llm_sharding_amd.runtime.stream import FileLayerSource
    from flexible_llm_sharding_amd.utils.synthetic import synthetic_prompts
    from flexible_llm_sharding_amd.utils.tokenizer import load_tokenizer
    path, cfg = tiny_model
    tok = load_tokenizer(path)
    base = synthetic_prompts(3, 40, 3, 8, cfg.vocab_size, seed=31, vary=True)
    words = [p[0].split()[:30] for p in base]
    step2 = [(pre, (sufs[0] + " " + " ".join(words[i][:2]),                     # grew by 2 words
                    " ".join(words[i][3:6]) + sufs[1][len(sufs[1]) // 2:],      # edited in the middle
                    sufs[2]))
             for i, (pre, sufs) in enumerate(base)]
    step3 = [(pre, (sufs[0], sufs[1], sufs[2] + " " + " ".join(words[i][:28])))      # one outgrows its region
             for i, (pre, sufs) in enumerate(step2)]
    step4 = [(pre, (sufs[0][:max(1, len(sufs[0]) // 2)],)) for pre, sufs in step3]   # shorter, fewer
    plain = ShardedRunner(cfg, FileLayerSource(cfg, path), "cpu", tok)
    old = PrefixKVCache.SUFFIX_GROWTH
    PrefixKVCache.SUFFIX_GROWTH = 8
    try:
        r = ShardedRunner(cfg, FileLayerSource(cfg, path), "cpu", tok, prefix_kv_cache=True, suffix_kv_cache=True)
        if host:
            _host_mode(r)
        reused = []
        for prompts in (base, step2, step3, step4):
            got, want = r(prompts), plain(prompts)
            for a, b in zip(got, want):
                assert np.abs(a.astype(np.float32) - b.astype(np.float32)).max() < 1e-5
            reused.append(r.stats["suffix_tokens_reused"])
        # a suffix without a region (grown past it) turns reuse off for that call
        assert reused[0] == 0 and reused[1] > 0 and reused[2] == 0
    finally:
        PrefixKVCache.SUFFIX_GROWTH = old


def test_pack_suffix_reuse_work_items():
    """Packing with kept suffix rows: only the new tokens, at their true positions; each suffix's
    items see the prefix (range 0), its kept rows (range 2) and its new rows causally (range 1)."""
    from flexible_llm_sharding_amd.runtime.batch import pack_prompts, visible_keys
    from flexible_llm_sharding_amd.utils.tokenizer import TokenizedPrompt
    tp = TokenizedPrompt(prefix=list(range(10)), suffixes=[[1, 2, 3, 4], [5, 6, 7]], padded_len=4,
                         eos_index=[3, 2])
    b = pack_prompts([tp], [0], prefix_offsets=[0], kv_cached=True, suffix_rows=[[20, 40]],
                     suffix_keep=[[2, 0]])
    assert b.ids.tolist() == [3, 4, 5, 6, 7] and b.positions.tolist() == [12, 13, 10, 11, 12]
    assert b.sfx_src.tolist() == [0, 1, 2, 3, 4] and b.sfx_dst.tolist() == [22, 23, 40, 41, 42]
    assert b.last_idx.tolist() == [1, 4]
    # the new rows' K/V are read back from the cache (captured before the attention runs): each row
    # sees its suffix's region up to and including itself, so the items need no range 1
    assert b.r2win.tolist() == [[20, 23], [20, 24], [40, 41], [40, 42], [40, 43]]
    assert b.work.tolist() == [[0, 5, 0, 0, 10, 0, 0, 0]] and b.work2.tolist() == [[20, 23]]
    assert visible_keys(b.work, b.seg_lo, 1, b.work2, b.r2win) == [(0, 0, 9), (2, 20, 23)]
    assert visible_keys(b.work, b.seg_lo, 3, b.work2, b.r2win) == [(0, 0, 9), (2, 40, 41)]
    assert b.work_last[:, :2].tolist() == [[1, 1], [4, 1]] and b.work2_last.tolist() == [[20, 4], [40, 3]]
    # at most 8 rows per item: the packed-GQA decode kernel (q_block 8)
    assert b.r2_q_block == 8
    mid = TokenizedPrompt(prefix=list(range(10)), suffixes=[list(range(20))], padded_len=20, eos_index=[19])
    b1 = pack_prompts([mid], [0], prefix_offsets=[0], kv_cached=True, suffix_rows=[[20]], suffix_keep=[[2]])
    assert int(b1.work[:, 1].max()) == 18 and b1.r2_q_block == 32      # one wave per head
    long = TokenizedPrompt(prefix=list(range(10)), suffixes=[list(range(40))], padded_len=40, eos_index=[39])
    b2 = pack_prompts([long], [0], prefix_offsets=[0], kv_cached=True, suffix_rows=[[20]], suffix_keep=[[2]])
    assert int(b2.work[:, 1].max()) == 38 and b2.r2_q_block == b2.q_block
    full = pack_prompts([tp], [0], prefix_offsets=[0], suffix_rows=[[20, 40]])
    assert full.r2_q_block == full.q_block               # no range 2: the batch's own q_block


def test_qwen2_moe_config_forms():
    """A released Qwen1.5-MoE config.json maps to q/k/v biases (no o_proj bias), 60 routed
    experts (top 4, not renormalised) and the shared expert; dense layers between MoE layers and
    a shared expert in a Qwen3-MoE config are rejected."""
    from flexible_llm_sharding_amd.config import ModelConfig, preset
    d = {"model_type": "qwen2_moe", "architectures": ["Qwen2MoeForCausalLM"], "hidden_size": 2048,
         "intermediate_size": 5632, "moe_intermediate_size": 1408, "shared_expert_intermediate_size": 5632,
         "num_experts": 60, "num_experts_per_tok": 4, "norm_topk_prob": False, "num_attention_heads": 16,
         "num_key_value_heads": 16, "num_hidden_layers": 24, "vocab_size": 151936, "rope_theta": 1000000.0,
         "rms_norm_eps": 1e-06, "decoder_sparse_step": 1, "mlp_only_layers": [], "use_sliding_window": False,
         "sliding_window": 32768, "hidden_act": "silu"}
    cfg = ModelConfig.from_dict(d)
    assert cfg.attention_bias and not cfg.o_proj_bias
    assert (cfg.num_local_experts, cfg.num_experts_per_tok, cfg.expert_intermediate) == (60, 4, 1408)
    assert cfg.shared_expert_intermediate_size == 5632 and not cfg.norm_topk_prob and cfg.sliding_window is None
    ref = preset("qwen1.5-moe-a2.7b")
    assert cfg.decoder_layer_params() == ref.decoder_layer_params()
    # 14.3B parameters in all (the released model card's count)
    assert abs(cfg.total_params() / 1e9 - 14.32) < 0.05
    assert not ModelConfig.from_dict(dict(d, qkv_bias=False)).attention_bias
    for bad in (dict(d, mlp_only_layers=[3]), dict(d, decoder_sparse_step=2),
                dict(d, model_type="qwen3_moe")):
        with pytest.raises(NotImplementedError):
            ModelConfig.from_dict(bad)


def test_vram_plan_resident_states():
    """plan_for_vram (Llama-2-70B, 6 GB, the piece pool's 3.12 GB of weight buffers): a 43k-token
    call is one micro-batch; under a 16k token budget its three micro-batches' states together fit,
    so every state keeps a ring slot (resident: nothing parked in host memory); 128 prompts'
    172k tokens do not fit and go through the two-slot ring."""
    from flexible_llm_sharding_amd.config import preset
    from flexible_llm_sharding_amd.runtime.memplan import STATES, activation_bytes, plan_for_vram
    cfg = preset("llama2-70b")
    kw = dict(max_prompt_rows=1344, overhead=int(0.9e9), weight_bytes=int(3.12e9), fused_norm=True)
    tb, mc, ar, qc, est, res = plan_for_vram(cfg, int(6e9), 1, 2, 49152, 16384, total_tokens=43008, **kw)
    assert tb >= 43008 and res and est <= 6e9
    tb, mc, ar, qc, est, res = plan_for_vram(cfg, int(6e9), 1, 2, 16384, 16384, total_tokens=43008, **kw)
    assert tb == 16384 and res and est <= 6e9
    # the estimate charges one state per micro-batch
    assert est == int(3.12e9) + int(0.9e9) + activation_bytes(cfg, 16384, mc, states=3, fused_norm=True)
    tb, mc, ar, qc, est, res = plan_for_vram(cfg, int(6e9), 1, 2, 49152, 16384, total_tokens=172032, **kw)
    assert not res and est <= 6e9
    assert est == int(3.12e9) + int(0.9e9) + activation_bytes(cfg, tb, mc, states=STATES, fused_norm=True)


def test_activation_store_buffer_bound():
    """ActivationStore.max_buffers: past the bound a new pinned buffer of a size is not allocated;
    the oldest pending reload of that size is waited for and its buffer reused (a reload whose
    copy already completed goes back to the pool first).  No bound: the pool grows."""
    from flexible_llm_sharding_amd.runtime.activations import ActivationStore

    class Ev:
        def __init__(self, done):
            self.done, self.waited = done, False

        def query(self):
            return self.done

        def synchronize(self):
            self.waited = True
            self.done = True

    st = ActivationStore("cpu", "cpu")
    st.max_buffers = 2
    n = 3 << 20
    a, b = st._get_host(n), st._get_host(n)
    ea, eb = Ev(False), Ev(False)
    st._recycle += [(a, ea), (b, eb)]          # both still being read by their reloads
    c = st._get_host(n)                        # bound reached: waits for the oldest, reuses it
    assert c is a and ea.waited and not eb.waited and st.buffer_waits == 1
    eb.done = True
    assert st._get_host(n) is b                # a completed reload's buffer comes from the pool
    st._recycle.append((c, Ev(False)))
    other = st._get_host(5 << 20)              # another size has its own count
    assert other.numel() == 5 << 20 and st.buffer_waits == 1
    st.max_buffers = None
    assert st._get_host(n) is not c            # unbounded: a new buffer
    st.trim()


def test_gemm_v11_round_rule():
    """The GEMM launcher's v10 / v11 choice (csrc/kernels/gemm_v11.hip v11_pays, a host-side rule):
    whole 256-CU tile rounds of each kernel, a 384 x 256 tile priced at 1.45 256 x 256 tiles
    (profiles/r5_resident/gemm_m.log).  Needs the built kernel library (host code only)."""
    from flexible_llm_sharding_amd import _native
    try:
        k = _native.kernels()
    except Exception as e:  # noqa: BLE001 (library not built in this checkout)
        pytest.skip(f"kernel library unavailable: {e}")
    pays = k.fls_gemm_v11_pays
    H, I2, Q = 8192, 2 * 28672, 10240
    # the headline's whole-round shapes keep v11
    for M, N in ((43008, Q), (43008, H), (15360, I2), (12288, I2), (15360, H), (12288, H)):
        assert pays(M, N) == 1, (M, N)
    # a 16k-budget micro-batch of 11 prompts: v11 5 rounds vs v10 8 (O / down)
    assert pays(14784, H) == 1
    # 16,128 rows: v11 needs 6 rounds, v10 8: 6 x 1.45 > 8
    assert pays(16128, H) == 0
