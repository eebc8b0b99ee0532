import json, os, sys
import torch
sys.path.insert(0, os.environ["GRAFT_REPO_ROOT"]); sys.path.insert(0, os.environ["GRAFT_REPO_ROOT"] + "/scripts")
from flexible_llm_sharding_amd.ops.hip_backend import HipOps, EPI_SWIGLU, EPI_NONE
from kernel_bench import timeit
dev = torch.device("cuda", 0); ops = HipOps(); M = 14336
orders = [int(v) for v in sys.argv[1].split(",")]
for epi in (EPI_SWIGLU, EPI_NONE):
    x = (torch.rand(M, 8192, device=dev) * 2 - 1).half(); w = ((torch.rand(57344, 8192, device=dev) * 2 - 1) * 0.02).half()
    fl = 2.0 * M * 57344 * 8192; ts = {o: [] for o in orders}
    for _ in range(3):
        for o in orders:
            ops.k.fls_gemm_set_order(o); ts[o].append(timeit(lambda: ops.gemm(x, w, epi), 20))
    print(json.dumps({"epi": epi, **{str(o): round(fl / sorted(v)[1] / 1e12, 1) for o, v in ts.items()}}), flush=True)
