"""CLI entry point — same flags, pickles and output semantics as the reference
``main.py`` (see ``flexible_llm_sharding_amd/utils/cli.py`` and ``api.py``).

    python main.py --model_path <layer dir> --prompt_pickle prompts.pkl \
        --output_file scores.pkl [--layer_num_per_shard 1] [--storage_location cpu] ...
"""
import sys

from flexible_llm_sharding_amd.api import main

if __name__ == "__main__":
    sys.exit(main())
