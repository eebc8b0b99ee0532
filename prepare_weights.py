"""Split an HF checkpoint into per-layer safetensors files (reference
``prepare_weights.py``), or write a synthetic random-init model directory.

    python prepare_weights.py <hf_dir> <new_file_dir>
    python prepare_weights.py --synthetic llama2-7b <new_file_dir> [--seed 0] [--dtype bfloat16]
                              [--unique_layers K]   (decoder layers >= K hard-link to layer i % K)
"""
import argparse
import sys

from flexible_llm_sharding_amd.utils.layer_format import split_into_layers


def main(argv=None):
    ap = argparse.ArgumentParser(description="Split model weights into layers.")
    ap.add_argument("bin_dir", type=str, help="Path to the HF weights directory (or preset name with --synthetic)")
    ap.add_argument("new_file_dir", type=str, help="Path to the new layer-wise file directory")
    ap.add_argument("--synthetic", action="store_true",
                    help="treat bin_dir as a preset name (tiny, small, llama2-7b, llama2-13b, llama2-70b) "
                         "and write random-init weights")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--std", type=float, default=0.02)
    ap.add_argument("--num_hidden_layers", type=int, default=None)
    ap.add_argument("--dtype", choices=["float16", "bfloat16", "float32"], default="float16",
                    help="--synthetic: checkpoint dtype")
    ap.add_argument("--unique_layers", type=int, default=0,
                    help="--synthetic: write K distinct decoder layers, hard-link the rest (disk-limited boxes)")
    a = ap.parse_args(argv)
    if a.synthetic:
        import torch
        from flexible_llm_sharding_amd.config import preset
        from flexible_llm_sharding_amd.utils.synthetic import write_synthetic_checkpoint
        kw = {} if a.num_hidden_layers is None else {"num_hidden_layers": a.num_hidden_layers}
        write_synthetic_checkpoint(preset(a.bin_dir, **kw), a.new_file_dir, seed=a.seed, std=a.std,
                                   dtype=getattr(torch, a.dtype), unique_layers=a.unique_layers)
    else:
        split_into_layers(a.bin_dir, a.new_file_dir)
    return 0


if __name__ == "__main__":
    sys.exit(main())
