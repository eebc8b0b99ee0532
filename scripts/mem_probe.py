"""Where does device memory outside the caching allocator come from during a capped 70B pass?
Prints hipMemGetInfo used - allocator reserved - raw weight slots at checkpoints, and the peak of
that quantity during a pass (sampler thread), plus the first launch of each kernel family in
isolation.   python scripts/mem_probe.py"""
import os
import sys
import threading
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("PYTORCH_HIP_ALLOC_CONF", "expandable_segments:True")

from flexible_llm_sharding_amd.config import preset  # noqa: E402
from flexible_llm_sharding_amd.engine import ShardedRunner  # noqa: E402
from flexible_llm_sharding_amd.runtime.weights import HostStore  # noqa: E402
from flexible_llm_sharding_amd.utils.synthetic import synthetic_prompts  # noqa: E402
from flexible_llm_sharding_amd.utils.tokenizer import load_tokenizer, write_synthetic_tokenizer  # noqa: E402

dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)


def outside(slots=0):
    free, total = torch.cuda.mem_get_info(dev)
    return (total - free - torch.cuda.memory_reserved(dev) - slots) / 1e6


print(f"[probe] start: outside {outside():.0f} MB", flush=True)
cfg = preset("llama2-70b")
store = HostStore.synthetic(cfg, dev, seed=0)
torch.cuda.synchronize()
torch.cuda.empty_cache()
print(f"[probe] after weight generation: outside {outside():.0f} MB, reserved "
      f"{torch.cuda.memory_reserved(dev) / 1e6:.0f} MB", flush=True)
d = "/tmp/fls_probe_tok"
write_synthetic_tokenizer(d, cfg.vocab_size)
tok = load_tokenizer(d)
prompts = synthetic_prompts(32, 1024, 5, 64, cfg.vocab_size, seed=0)
r = ShardedRunner(cfg, store, dev, tok, layer_num_per_shard=1, storage_location="cpu", max_vram_gb=6.0)
slots = lambda: r.prefetcher.hbm_bytes()  # noqa: E731
print(f"[probe] runner init: outside {outside(slots()):.0f} MB (slots {slots() / 1e6:.0f} MB, planned "
      f"{r.prefetcher.planned_hbm_bytes() / 1e6:.0f}), plan outside {r._outside / 1e6:.0f} MB", flush=True)
peak = {"v": 0.0, "used": 0.0}
stop = threading.Event()


def sample():
    torch.cuda.set_device(dev)
    while not stop.is_set():
        free, total = torch.cuda.mem_get_info(dev)
        used = total - free
        peak["used"] = max(peak["used"], used / 1e9)
        peak["v"] = max(peak["v"], (used - torch.cuda.memory_reserved(dev) - slots()) / 1e6)
        stop.wait(0.005)


t = threading.Thread(target=sample, daemon=True)
t.start()
def stats():
    st = torch.cuda.memory_stats(dev)
    return {k: st.get(k, 0) for k in ("num_alloc_retries", "num_device_alloc", "num_device_free", "num_ooms")}


for i in range(3):
    t0 = time.perf_counter()
    s0 = stats()
    r(prompts)
    torch.cuda.synchronize()
    s1 = stats()
    print(f"[probe] allocator during call {i}: " + ", ".join(f"{k} +{s1[k] - s0[k]}" for k in s0), flush=True)
    print(f"[probe] call {i}: {time.perf_counter() - t0:.2f}s outside-now {outside(slots()):.0f} MB, peak outside "
          f"{peak['v']:.0f} MB, peak used {peak['used']:.3f} GB, reserved peak "
          f"{torch.cuda.max_memory_reserved(dev) / 1e9:.3f} GB", flush=True)
stop.set()
t.join()
