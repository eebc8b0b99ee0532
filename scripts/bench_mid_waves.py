"""bench.py with the mid-M kernel's 128-column blocks forced to 4 or 8 waves (0: the default
dispatch), for same-box A/B runs:  python scripts/bench_mid_waves.py WAVES [bench.py args]"""
import os
import runpy
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402,F401  (first: the kernel library binds to torch's HIP runtime, as in bench.py)
from flexible_llm_sharding_amd import _native  # noqa: E402

_native.kernels().fls_gemm_set_mid_waves(int(sys.argv[1]))
sys.argv = ["bench.py"] + sys.argv[2:]
runpy.run_path(os.path.join(ROOT, "bench.py"), run_name="__main__")
