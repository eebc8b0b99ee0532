"""Model configuration (Llama family) read from an HF ``config.json``.

The reference builds the model shell from ``AutoConfig.from_pretrained``
(``/root/reference/utils.py:101``) and instantiates HF ``LlamaForCausalLM`` on
the meta device (``utils.py:111-113``).  We only need the architecture
numbers: the model itself is our own packed-weight implementation.
"""
from __future__ import annotations

import json
import os
from dataclasses import asdict, dataclass, field
from typing import Optional

# Reference hard-codes the maximum sequence length (utils.py:14).
MAX_TOKEN_LEN = 4096


@dataclass
class ModelConfig:
    hidden_size: int = 4096
    intermediate_size: int = 11008
    num_attention_heads: int = 32
    num_key_value_heads: int = 32
    num_hidden_layers: int = 32
    vocab_size: int = 32000
    rms_norm_eps: float = 1e-5
    rope_theta: float = 10000.0
    max_position_embeddings: int = 4096
    tie_word_embeddings: bool = False
    attention_bias: bool = False        # q/k/v projection biases (Qwen2; Llama attention_bias)
    o_proj_bias: bool = False           # o_proj bias (Llama attention_bias=True)
    qk_norm: bool = False               # Qwen3: RMSNorm over head_dim on every q / k head, before RoPE
    # Mistral / Phi-3: every call's sequences must fit the window (checked per call by the runner)
    sliding_window: Optional[int] = None
    # RoPE frequency scaling (HF ``rope_scaling`` / v5 ``rope_parameters``): linear, llama3, yarn,
    # longrope (Phi-3)
    rope_scaling: Optional[dict] = None
    explicit_head_dim: Optional[int] = None   # HF ``head_dim`` when != hidden / heads (Mistral-Nemo)
    # sparse mixture-of-experts FFN (Mixtral, Qwen3-MoE): 0 = dense SwiGLU MLP.  Each token's
    # post-attention RMSNorm output goes to its top-k experts (router softmax in fp32, top-k,
    # renormalised when norm_topk_prob), each a SwiGLU MLP of moe_intermediate_size (Mixtral:
    # intermediate_size), and the weighted expert outputs are summed into the residual
    num_local_experts: int = 0
    num_experts_per_tok: int = 2
    moe_intermediate_size: Optional[int] = None
    norm_topk_prob: bool = True
    # Qwen2-MoE: a dense SwiGLU "shared expert" of this width on every token, scaled by
    # sigmoid(h . shared_expert_gate) and added to the routed experts' sum (0: none)
    shared_expert_intermediate_size: int = 0
    # Granite (HF GraniteModel / GraniteDecoderLayer / GraniteForCausalLM): token embeddings x
    # embedding_multiplier; each sub-layer output x residual_multiplier before the residual add;
    # attention scores x attention_multiplier (instead of head_dim^-1/2); logits / logits_scaling
    embedding_multiplier: float = 1.0
    residual_multiplier: float = 1.0
    attention_multiplier: Optional[float] = None
    logits_scaling: float = 1.0
    bos_token_id: int = 1
    eos_token_id: int = 2
    torch_dtype: str = "float16"
    model_type: str = "llama"
    architectures: list = field(default_factory=lambda: ["LlamaForCausalLM"])

    # ------------------------------------------------------------------ derived
    @property
    def head_dim(self) -> int:
        return self.explicit_head_dim or self.hidden_size // self.num_attention_heads

    @property
    def attn_scale(self) -> float:
        """Softmax scale of the attention scores (Granite: attention_multiplier)."""
        return self.attention_multiplier if self.attention_multiplier is not None else self.head_dim ** -0.5

    @property
    def is_moe(self) -> bool:
        return self.num_local_experts > 0

    @property
    def expert_intermediate(self) -> int:
        """Rows of one expert's gate (= up) projection (the dense MLP's for non-MoE models)."""
        return self.moe_intermediate_size or self.intermediate_size

    @property
    def fused_projections(self) -> bool:
        """Phi-3 checkpoints store ``qkv_proj`` ([q; k; v] rows) and ``gate_up_proj`` ([gate; up]
        rows) as single tensors: the same row order as the packed ``wqkv`` / ``wgu`` slots."""
        return self.model_type == "phi3"

    @property
    def q_size(self) -> int:
        return self.num_attention_heads * self.head_dim

    @property
    def kv_size(self) -> int:
        return self.num_key_value_heads * self.head_dim

    @property
    def qkv_size(self) -> int:
        return self.q_size + 2 * self.kv_size

    @property
    def num_layers_total(self) -> int:
        """embed + decoder layers + final norm + lm_head (reference utils.py:106-107)."""
        return self.num_hidden_layers + 3

    def layer_names(self) -> list:
        """Ordered layer list, identical to ``ShardedLlama.layer_names`` (utils.py:106-107)."""
        return (["model.embed_tokens"]
                + [f"model.layers.{i}" for i in range(self.num_hidden_layers)]
                + ["model.norm", "lm_head"])

    def decoder_layer_params(self) -> int:
        """Parameters stored per decoder layer (every expert of an MoE layer)."""
        return self._decoder_params(self.num_local_experts)

    def decoder_active_params(self) -> int:
        """Parameters one token multiplies per decoder layer (MoE: router + its top-k experts)."""
        return self._decoder_params(self.num_experts_per_tok) if self.is_moe else self.decoder_layer_params()

    def _decoder_params(self, experts: int) -> int:
        h = self.hidden_size
        n = h * self.qkv_size + self.q_size * h + 2 * h
        if self.is_moe:
            n += self.num_local_experts * h + experts * 3 * h * self.expert_intermediate
            n += 3 * h * self.shared_expert_intermediate_size + (h if self.shared_expert_intermediate_size else 0)
        else:
            n += 3 * h * self.intermediate_size
        return (n + (self.qkv_size if self.attention_bias else 0) + (h if self.o_proj_bias else 0)
                + (2 * self.head_dim if self.qk_norm else 0))

    def total_params(self) -> int:
        emb = self.vocab_size * self.hidden_size
        head = 0 if self.tie_word_embeddings else emb
        return emb + head + self.hidden_size + self.num_hidden_layers * self.decoder_layer_params()

    def validate(self) -> None:
        if self.explicit_head_dim is None and self.hidden_size % self.num_attention_heads:
            raise ValueError("hidden_size must be divisible by num_attention_heads")
        if self.num_attention_heads % self.num_key_value_heads:
            raise ValueError("num_attention_heads must be a multiple of num_key_value_heads")
        if self.head_dim % 32:
            raise ValueError("head_dim must be a multiple of 32 (RoPE pair blocks of 16)")
        if self.is_moe and not 1 <= self.num_experts_per_tok <= min(self.num_local_experts, MAX_TOP_K):
            raise ValueError(f"num_experts_per_tok must be in 1..min(num_local_experts, {MAX_TOP_K})")
        if self.is_moe and self.residual_multiplier != 1.0:
            # the MoE combine kernel adds the experts' sum to the residual unscaled
            raise NotImplementedError("residual_multiplier with a mixture-of-experts MLP")
        if self.num_local_experts > MAX_EXPERTS:
            raise NotImplementedError(f"num_local_experts={self.num_local_experts} > {MAX_EXPERTS}")
        rs = self.rope_scaling
        if rs:
            kind = rs.get("rope_type", rs.get("type"))
            if kind not in ROPE_SCALING_TYPES:
                raise NotImplementedError(f"rope_scaling type {kind!r}: supported are {sorted(ROPE_SCALING_TYPES)}"
                                          " (dynamic NTK depends on each call's length: not supported)")
            if float(rs.get("factor") or 1.0) <= 0:
                raise ValueError(f"rope_scaling factor must be > 0: {rs}")
            if kind == "longrope":
                for key in ("short_factor", "long_factor"):
                    if len(rs.get(key) or ()) != self.head_dim // 2:
                        raise ValueError(f"longrope {key} must hold head_dim/2 = {self.head_dim // 2} values")
                orig = int(rs.get("original_max_position_embeddings") or self.max_position_embeddings)
                if orig < MAX_TOKEN_LEN:
                    # HF switches to long_factor once a sequence exceeds the original context;
                    # static tables are exact only while no sequence can
                    raise NotImplementedError(f"longrope with original_max_position_embeddings={orig} < the "
                                              f"{MAX_TOKEN_LEN}-token cap (length-dependent tables)")

    # ---------------------------------------------------------------------- io
    @classmethod
    def from_dict(cls, d: dict) -> "ModelConfig":
        kw = {}
        for f in cls.__dataclass_fields__:
            if f in d and d[f] is not None:
                kw[f] = d[f]
        if "num_key_value_heads" not in d or d.get("num_key_value_heads") is None:
            kw["num_key_value_heads"] = d.get("num_attention_heads", cls.num_attention_heads)
        rp = d.get("rope_parameters")          # transformers v5 form: {"rope_type", "rope_theta", ...}
        if isinstance(rp, dict):
            if "rope_theta" in rp:
                kw["rope_theta"] = rp["rope_theta"]
            if rp.get("rope_type", "default") != "default":
                kw["rope_scaling"] = {k: v for k, v in rp.items() if k != "rope_theta"}
        rs = kw.get("rope_scaling")
        if rs and rs.get("rope_type", rs.get("type")) == "default":
            kw.pop("rope_scaling")
        rs = kw.get("rope_scaling")
        if rs and rs.get("rope_type", rs.get("type")) in ("su", "longrope"):
            # Phi-3: "su" is the old name; the pretraining context sits at the config's top level
            rs = dict(rs, rope_type="longrope")
            rs.pop("type", None)
            if "original_max_position_embeddings" not in rs and d.get("original_max_position_embeddings"):
                rs["original_max_position_embeddings"] = d["original_max_position_embeddings"]
            kw["rope_scaling"] = rs
        for src in (d, rp if isinstance(rp, dict) else {}, rs or {}):
            if float(src.get("partial_rotary_factor", 1.0) or 1.0) != 1.0:
                raise NotImplementedError("partial_rotary_factor < 1 (RoPE on part of each head) is not supported")
        mt = d.get("model_type", "llama")
        if mt not in SUPPORTED_MODEL_TYPES:
            why = llama_like_rejection(d)
            if why:
                raise NotImplementedError(f"model_type={mt!r}: supported are {sorted(SUPPORTED_MODEL_TYPES)}, or a "
                                          f"Llama-structured config ({why})")
            # an unlisted family with the Llama block: run as Llama; every layer file must then hold
            # exactly the Llama tensors (models/layout.py check_layer_tensors), so a different block
            # structure fails at load instead of running wrong
            kw["model_type"] = mt
        if mt in ("qwen3_moe", "qwen2_moe"):
            kw["num_local_experts"] = int(d.get("num_experts") or d.get("num_local_experts") or 0)
            if mt == "qwen3_moe" and d.get("shared_expert_intermediate_size"):
                raise NotImplementedError("shared experts in a Qwen3-MoE config")
            if d.get("mlp_only_layers") or int(d.get("decoder_sparse_step", 1) or 1) != 1:
                raise NotImplementedError("dense layers between the MoE layers (mlp_only_layers / "
                                          "decoder_sparse_step) are not supported")
        if mt == "mixtral":
            kw["norm_topk_prob"] = True           # HF MixtralTopKRouter always renormalises
        elif mt in ("qwen3_moe", "qwen2_moe"):
            kw["norm_topk_prob"] = bool(d.get("norm_topk_prob", False))     # HF Qwen3MoeConfig default
        if d.get("mlp_bias"):
            raise NotImplementedError("mlp_bias=True is not supported")
        hdim = d.get("head_dim")
        if hdim is not None and hdim * d.get("num_attention_heads", cls.num_attention_heads) != d.get(
                "hidden_size", cls.hidden_size):
            kw["explicit_head_dim"] = int(hdim)
        if d.get("hidden_act", "silu") != "silu":
            raise NotImplementedError(f"hidden_act={d.get('hidden_act')!r} (SwiGLU/silu only)")
        if mt == "qwen2" or (mt == "qwen2_moe" and d.get("qkv_bias", d.get("attention_bias", True))):
            # HF Qwen2Attention / Qwen2MoeAttention (qkv_bias, default True): q/k/v Linear with
            # bias, o_proj without
            kw["attention_bias"], kw["o_proj_bias"] = True, False
        elif d.get("attention_bias"):
            kw["attention_bias"], kw["o_proj_bias"] = True, True
        if mt in ("qwen3", "qwen3_moe"):
            # HF Qwen3Attention: q_norm / k_norm (RMSNorm over head_dim) on every head before RoPE;
            # q/k/v/o biases only with attention_bias (off in every released Qwen3 config)
            kw["qk_norm"] = True
        # HF Phi3Model / Mixtral apply their sliding_window whenever it is set; Qwen2/3 only with
        # use_sliding_window
        if not d.get("use_sliding_window", mt in ("mistral", "phi3", "mixtral")):
            kw.pop("sliding_window", None)
        if isinstance(kw.get("eos_token_id"), list):
            kw["eos_token_id"] = kw["eos_token_id"][0]
        cfg = cls(**kw)
        cfg.validate()
        return cfg

    @classmethod
    def from_pretrained(cls, model_path: str) -> "ModelConfig":
        with open(os.path.join(model_path, "config.json")) as f:
            return cls.from_dict(json.load(f))

    def to_dict(self) -> dict:
        d = asdict(self)
        d["head_dim"] = self.head_dim
        return d

    def save(self, model_path: str) -> None:
        os.makedirs(model_path, exist_ok=True)
        d = asdict(self)
        d["head_dim"] = self.head_dim           # HF key (also read back by from_dict)
        if self.model_type in ("qwen3_moe", "qwen2_moe"):
            d["num_experts"] = self.num_local_experts          # the HF key of these families
        with open(os.path.join(model_path, "config.json"), "w") as f:
            json.dump(d, f, indent=2)


# Llama-structured causal LMs (model.embed_tokens / model.layers.N / model.norm / lm_head with
# q/k/v/o + gate/up/down + two RMSNorms per layer) -- what the reference's AutoModelForCausalLM
# path (utils.py:101-115) runs in practice.
SUPPORTED_MODEL_TYPES = {"llama", "mistral", "qwen2", "qwen3", "phi3", "mixtral", "qwen3_moe", "qwen2_moe",
                         "granite"}

# config keys of other families whose block differs from Llama's while its tensors may look the same
# (MiniCPM's embedding / depth scales, Gemma-2's soft-capping, DeepSeek's latent attention, Cohere's
# logit scale, parallel attention + MLP blocks, experts under other names)
_NON_LLAMA_KEYS = ("scale_emb", "scale_depth", "dim_model_base", "attn_logit_softcapping",
                   "final_logit_softcapping", "query_pre_attn_scalar", "kv_lora_rank", "q_lora_rank",
                   "logit_scale", "use_parallel_residual", "parallel_attn", "parallel_block", "n_routed_experts",
                   "num_experts", "num_local_experts", "moe_intermediate_size", "use_qk_norm", "qk_layernorm",
                   "layer_norm_eps", "norm_epsilon", "embedding_multiplier", "residual_multiplier")


def llama_like_rejection(d: dict) -> str:
    """'' when an unlisted model_type's config.json describes the Llama block (the fields Llama reads,
    SwiGLU, RMSNorm, full RoPE, none of the keys that change the block), else the reason not."""
    need = ("hidden_size", "intermediate_size", "num_attention_heads", "num_hidden_layers", "vocab_size",
            "rms_norm_eps")
    missing = [k for k in need if k not in d]
    if missing:
        return f"missing {', '.join(missing)}"
    # (1 / 0 / false are the neutral values: this framework's own config.json lists every field)
    extra = [k for k in _NON_LLAMA_KEYS if d.get(k) not in (None, False, 0, 1)]
    if extra:
        return f"{', '.join(extra)} change the block"
    if d.get("hidden_act", "silu") != "silu":
        return f"hidden_act={d.get('hidden_act')!r}"
    return ""
# MoE limits of the routing kernels (csrc/kernels/moe.hip): experts per layer, experts per token
MAX_EXPERTS = 256
MAX_TOP_K = 8
# static RoPE scalings: they only change the cos/sin tables (models/llama.py rope_inv_freq)
ROPE_SCALING_TYPES = {"linear", "llama3", "yarn", "longrope"}

# Standard HF configs (computed sizes in SURVEY.md §2.3).
PRESETS = {
    "llama2-7b": dict(hidden_size=4096, intermediate_size=11008, num_attention_heads=32,
                      num_key_value_heads=32, num_hidden_layers=32),
    "llama2-13b": dict(hidden_size=5120, intermediate_size=13824, num_attention_heads=40,
                       num_key_value_heads=40, num_hidden_layers=40),
    "llama2-70b": dict(hidden_size=8192, intermediate_size=28672, num_attention_heads=64,
                       num_key_value_heads=8, num_hidden_layers=80),
    "mistral-7b": dict(hidden_size=4096, intermediate_size=14336, num_attention_heads=32,
                       num_key_value_heads=8, num_hidden_layers=32, rope_theta=1e6,
                       model_type="mistral", architectures=["MistralForCausalLM"]),
    "qwen2-7b": dict(hidden_size=3584, intermediate_size=18944, num_attention_heads=28,
                     num_key_value_heads=4, num_hidden_layers=28, vocab_size=152064, rope_theta=1e6,
                     rms_norm_eps=1e-6, attention_bias=True, model_type="qwen2",
                     architectures=["Qwen2ForCausalLM"]),
    # tiny configs for tests (GQA 2:1, head_dim 64)
    "tiny": dict(hidden_size=256, intermediate_size=512, num_attention_heads=4,
                 num_key_value_heads=2, num_hidden_layers=2, vocab_size=512,
                 max_position_embeddings=4096),
    "tiny-qwen2": dict(hidden_size=256, intermediate_size=512, num_attention_heads=4,
                       num_key_value_heads=2, num_hidden_layers=2, vocab_size=512, rope_theta=1e6,
                       rms_norm_eps=1e-6, attention_bias=True, model_type="qwen2",
                       architectures=["Qwen2ForCausalLM"]),
    # Qwen3 dense: per-head q/k RMSNorm, explicit head_dim 128 (hidden 4096 = 32 x 128 here)
    "qwen3-8b": dict(hidden_size=4096, intermediate_size=12288, num_attention_heads=32,
                     num_key_value_heads=8, num_hidden_layers=36, vocab_size=151936, rope_theta=1e6,
                     rms_norm_eps=1e-6, qk_norm=True, explicit_head_dim=128, max_position_embeddings=40960,
                     model_type="qwen3", architectures=["Qwen3ForCausalLM"]),
    "tiny-qwen3": dict(hidden_size=256, intermediate_size=512, num_attention_heads=4,
                       num_key_value_heads=2, num_hidden_layers=2, vocab_size=512, rope_theta=1e6,
                       rms_norm_eps=1e-6, qk_norm=True, explicit_head_dim=128, model_type="qwen3",
                       architectures=["Qwen3ForCausalLM"]),
    # Phi-3 family: fused qkv_proj / gate_up_proj tensors; Phi-3-medium-4k (sliding window 2047)
    # and Phi-4 (14B, 100k vocab) have head_dim 128
    "phi3-medium": dict(hidden_size=5120, intermediate_size=17920, num_attention_heads=40,
                        num_key_value_heads=10, num_hidden_layers=40, vocab_size=32064, sliding_window=2047,
                        eos_token_id=32000, model_type="phi3", architectures=["Phi3ForCausalLM"]),
    "phi4": dict(hidden_size=5120, intermediate_size=17920, num_attention_heads=40, num_key_value_heads=10,
                 num_hidden_layers=40, vocab_size=100352, rope_theta=250000.0, max_position_embeddings=16384,
                 bos_token_id=100257, eos_token_id=100265, model_type="phi3", architectures=["Phi3ForCausalLM"]),
    # Phi-3-mini-4k: multi-head attention with head_dim 96 (unfused RoPE pass, 12-chunk LDS rows)
    "phi3-mini": dict(hidden_size=3072, intermediate_size=8192, num_attention_heads=32, num_key_value_heads=32,
                      num_hidden_layers=32, vocab_size=32064, sliding_window=2047, eos_token_id=32000,
                      model_type="phi3", architectures=["Phi3ForCausalLM"]),
    "tiny-phi3-mini": dict(hidden_size=384, intermediate_size=768, num_attention_heads=4, num_key_value_heads=4,
                           num_hidden_layers=2, vocab_size=512, model_type="phi3",
                           architectures=["Phi3ForCausalLM"]),
    # tiny Phi-3-128k-style config: longrope short/long factors, attention factor from 131072 / 4096
    "tiny-phi3": dict(hidden_size=256, intermediate_size=512, num_attention_heads=4, num_key_value_heads=2,
                      num_hidden_layers=2, vocab_size=512, max_position_embeddings=131072,
                      rope_scaling={"rope_type": "longrope", "original_max_position_embeddings": 4096,
                                    "short_factor": [1.0 + 0.05 * i for i in range(32)],
                                    "long_factor": [2.0 + 0.5 * i for i in range(32)]},
                      model_type="phi3", architectures=["Phi3ForCausalLM"]),
    # Llama-3.1 geometry (GQA 8:1, 128k vocab, llama3 RoPE scaling)
    "llama3.1-8b": dict(hidden_size=4096, intermediate_size=14336, num_attention_heads=32,
                        num_key_value_heads=8, num_hidden_layers=32, vocab_size=128256, rope_theta=500000.0,
                        max_position_embeddings=131072, bos_token_id=128000, eos_token_id=128001,
                        rope_scaling={"rope_type": "llama3", "factor": 8.0, "low_freq_factor": 1.0,
                                      "high_freq_factor": 4.0, "original_max_position_embeddings": 8192}),
    # sparse MoE: Mixtral-8x7B (8 experts, top-2, 32k vocab) and Qwen3-30B-A3B (128 experts of
    # 768 rows, top-8, q/k norm); tiny variants keep every GEMM on the grouped MFMA path
    "mixtral-8x7b": dict(hidden_size=4096, intermediate_size=14336, num_attention_heads=32, num_key_value_heads=8,
                         num_hidden_layers=32, vocab_size=32000, rope_theta=1e6, max_position_embeddings=32768,
                         num_local_experts=8, num_experts_per_tok=2, model_type="mixtral",
                         architectures=["MixtralForCausalLM"]),
    "qwen3-30b-a3b": dict(hidden_size=2048, intermediate_size=6144, num_attention_heads=32, num_key_value_heads=4,
                          num_hidden_layers=48, vocab_size=151936, rope_theta=1e6, rms_norm_eps=1e-6, qk_norm=True,
                          explicit_head_dim=128, max_position_embeddings=40960, num_local_experts=128,
                          num_experts_per_tok=8, moe_intermediate_size=768, norm_topk_prob=True,
                          model_type="qwen3_moe", architectures=["Qwen3MoeForCausalLM"]),
    "tiny-mixtral": dict(hidden_size=256, intermediate_size=256, num_attention_heads=4, num_key_value_heads=2,
                         num_hidden_layers=2, vocab_size=512, rope_theta=1e6, num_local_experts=4,
                         num_experts_per_tok=2, model_type="mixtral", architectures=["MixtralForCausalLM"]),
    "tiny-qwen3-moe": dict(hidden_size=256, intermediate_size=512, num_attention_heads=4, num_key_value_heads=2,
                           num_hidden_layers=2, vocab_size=512, rope_theta=1e6, rms_norm_eps=1e-6, qk_norm=True,
                           explicit_head_dim=128, num_local_experts=8, num_experts_per_tok=3,
                           moe_intermediate_size=128, norm_topk_prob=False, model_type="qwen3_moe",
                           architectures=["Qwen3MoeForCausalLM"]),
    # Qwen1.5-MoE-A2.7B: 60 routed experts (top 4, not renormalised) + a gated shared expert
    "qwen1.5-moe-a2.7b": dict(hidden_size=2048, intermediate_size=5632, num_attention_heads=16,
                              num_key_value_heads=16, num_hidden_layers=24, vocab_size=151936, rope_theta=1e6,
                              rms_norm_eps=1e-6, attention_bias=True, num_local_experts=60, num_experts_per_tok=4,
                              moe_intermediate_size=1408, shared_expert_intermediate_size=5632,
                              norm_topk_prob=False, bos_token_id=151643, eos_token_id=151643,
                              model_type="qwen2_moe", architectures=["Qwen2MoeForCausalLM"]),
    "tiny-qwen2-moe": dict(hidden_size=256, intermediate_size=512, num_attention_heads=4, num_key_value_heads=2,
                           num_hidden_layers=2, vocab_size=512, rope_theta=1e6, rms_norm_eps=1e-6,
                           attention_bias=True, num_local_experts=8, num_experts_per_tok=3,
                           moe_intermediate_size=128, shared_expert_intermediate_size=256, norm_topk_prob=False,
                           model_type="qwen2_moe", architectures=["Qwen2MoeForCausalLM"]),
    # Granite-3.0-8B: Llama geometry with the four Granite scalars and a tied 49k head
    "granite-3-8b": dict(hidden_size=4096, intermediate_size=12800, num_attention_heads=32, num_key_value_heads=8,
                         num_hidden_layers=40, vocab_size=49155, rope_theta=10000.0, tie_word_embeddings=True,
                         embedding_multiplier=12.0, residual_multiplier=0.22, attention_multiplier=0.0078125,
                         logits_scaling=16.0, bos_token_id=0, eos_token_id=0, model_type="granite",
                         architectures=["GraniteForCausalLM"]),
    "tiny-granite": dict(hidden_size=256, intermediate_size=512, num_attention_heads=4, num_key_value_heads=2,
                         num_hidden_layers=2, vocab_size=512, embedding_multiplier=6.0, residual_multiplier=0.4,
                         attention_multiplier=0.09, logits_scaling=3.0, model_type="granite",
                         architectures=["GraniteForCausalLM"]),
    "small": dict(hidden_size=1024, intermediate_size=2816, num_attention_heads=8,
                  num_key_value_heads=2, num_hidden_layers=4, vocab_size=32000),
}


def preset(name: str, **overrides) -> ModelConfig:
    if name not in PRESETS:
        raise KeyError(f"unknown preset {name!r}; choose from {sorted(PRESETS)}")
    d = dict(PRESETS[name])
    d.update(overrides)
    cfg = ModelConfig(**d)
    cfg.validate()
    return cfg


def resolve_dtype(name: Optional[str]):
    import torch
    table = {"float16": torch.float16, "fp16": torch.float16, "half": torch.float16,
             "bfloat16": torch.bfloat16, "bf16": torch.bfloat16,
             "float32": torch.float32, "fp32": torch.float32}
    if name is None:
        return torch.float16
    if name not in table:
        raise ValueError(f"unsupported dtype {name}")
    return table[name]
