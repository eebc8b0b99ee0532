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
        h, i = self.hidden_size, self.intermediate_size
        n = h * self.qkv_size + self.q_size * h + 3 * h * i + 2 * h
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
            raise NotImplementedError(f"model_type={mt!r}: supported are {sorted(SUPPORTED_MODEL_TYPES)}")
        if d.get("mlp_bias"):
            raise NotImplementedError("mlp_bias=True is not supported")
        hdim = d.get("head_dim")
        if hdim is not None and hdim * d.get("num_attention_heads", cls.num_attention_heads) != d.get(
                "hidden_size", cls.hidden_size):
            kw["explicit_head_dim"] = int(hdim)
        if d.get("hidden_act", "silu") != "silu":
            raise NotImplementedError(f"hidden_act={d.get('hidden_act')!r} (SwiGLU/silu only)")
        if mt == "qwen2":
            # HF Qwen2Attention: q/k/v Linear with bias, o_proj without
            kw["attention_bias"], kw["o_proj_bias"] = True, False
        elif d.get("attention_bias"):
            kw["attention_bias"], kw["o_proj_bias"] = True, True
        if mt == "qwen3":
            # HF Qwen3Attention: q_norm / k_norm (RMSNorm over head_dim) on every head before RoPE;
            # q/k/v/o biases only with attention_bias (off in every released Qwen3 config)
            kw["qk_norm"] = True
        # HF Phi3Model applies its sliding_window whenever it is set; Qwen2/3 only with use_sliding_window
        if not d.get("use_sliding_window", mt in ("mistral", "phi3")):
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
        with open(os.path.join(model_path, "config.json"), "w") as f:
            json.dump(d, f, indent=2)


# Llama-structured causal LMs (model.embed_tokens / model.layers.N / model.norm / lm_head with
# q/k/v/o + gate/up/down + two RMSNorms per layer) -- what the reference's AutoModelForCausalLM
# path (utils.py:101-115) runs in practice.
SUPPORTED_MODEL_TYPES = {"llama", "mistral", "qwen2", "qwen3", "phi3"}
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
