import sys, torch
sys.path.insert(0, '/root/repo')
from flexible_llm_sharding_amd.ops.hip_backend import HipOps, EPI_ROPE
from flexible_llm_sharding_amd.config import ModelConfig
from flexible_llm_sharding_amd.models.llama import rope_tables
ops = HipOps(); DEV = torch.device('cuda', 0)
M, K, hd = 384, 384, 64
g = torch.Generator().manual_seed(0)
x = torch.randn(M, K, generator=g).half().to(DEV); w = (torch.randn(1024, K, generator=g) * 0.05).half().to(DEV)
pos = torch.randint(0, 4000, (M,), dtype=torch.int32, device=DEV)
cfg = ModelConfig(hidden_size=1024, num_attention_heads=16, num_key_value_heads=2)
cos, sin = rope_tables(cfg, 4096); cos, sin = cos.to(DEV), sin.to(DEV)
ops.k.fls_gemm_set_mid(0)
def run(mode, p):
    ops.k.fls_gemm_set_v11(mode)
    return ops.gemm(x, w, EPI_ROPE, positions=p, cos=cos, sin=sin, rope_cols=14 * 64, head_dim=64)
for pname, p in [("pos", pos), ("pos0", torch.zeros_like(pos))]:
    a = run(2, p).float(); b = run(0, p).float(); torch.cuda.synchronize()
    d = (a - b).abs() > 1e-2
    print(pname, "bad", int(d.sum()), "rows", d.any(1).nonzero().flatten()[:20].tolist(), "cols", d.any(0).nonzero().flatten()[:64].tolist())
