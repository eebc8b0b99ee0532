"""flexible_llm_sharding_amd — MI355X-native layer-sharded LLM inference.

A from-scratch rebuild of the capabilities of eyedealism/flexible-LLM-sharding
(reference: ``main.py``, ``utils.py``, ``prepare_weights.py``) designed for
AMD Instinct MI355X (gfx950 / CDNA4):

* per-layer safetensors checkpoints streamed shard-by-shard into HBM through a
  pinned-memory, double-buffered copy engine on dedicated HIP streams;
* every transformer-block op is a hand-written HIP kernel (MFMA GEMMs with
  fused RoPE / SwiGLU / residual epilogues, GQA-native shared-prefix flash
  attention, RMSNorm, embedding gather, vocab softmax) — see ``csrc/kernels``;
* multi-GPU as one process per GPU over ``torch.distributed`` (RCCL on ROCm):
  a round-robin layer pipeline (reference default "model parallel") and a
  data-parallel mode whose per-layer weights are scatter-loaded over each
  GPU's own PCIe link and all-gathered over xGMI;
* a torch-CPU backend for plumbing runs and as the numerics oracle.

The importable package name uses underscores; ``flexible-llm-sharding_amd`` is
a symlink kept for discoverability.
"""

__version__ = "0.1.0"

from .config import ModelConfig  # noqa: F401
