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


timeline = []          # (time, outside MB) for the last call
events = []            # (time, host call name, '>' enter / '<' exit) for the last call


def _wrap(obj, name):
    f = getattr(obj, name, None)
    if f is None or not callable(f):
        return
    tag = f"{type(obj).__name__}.{name}"

    def w(*a, **k):
        events.append((time.perf_counter(), tag, ">"))
        try:
            return f(*a, **k)
        finally:
            events.append((time.perf_counter(), tag, "<"))
    setattr(obj, name, w)


for _n in dir(r.ops):
    if not _n.startswith("_") or _n in ("_splitk_ws",):
        _wrap(r.ops, _n)
for _n in ("_copy_piece", "_try_issue", "_wait", "acquire", "release", "_release_gid", "discard_loaded"):
    _wrap(r.prefetcher, _n)
for _n in [n for n in dir(r) if n.startswith("_") and not n.startswith("__")]:
    if callable(getattr(r, _n, None)) and _n not in ("_workspace",):
        try:
            _wrap(r, _n)
        except (AttributeError, TypeError):
            pass


def sample():
    torch.cuda.set_device(dev)
    while not stop.is_set():
        free, total = torch.cuda.mem_get_info(dev)
        used = total - free
        peak["used"] = max(peak["used"], used / 1e9)
        o = (used - torch.cuda.memory_reserved(dev) - slots()) / 1e6
        peak["v"] = max(peak["v"], o)
        timeline.append((time.perf_counter(), o))
        stop.wait(0.002)


t = threading.Thread(target=sample, daemon=True)
t.start()
def excursions(t0, label):
    """Intervals of the call where the outside-allocator memory rose > 50 MB above its median,
    with the host calls made around each."""
    steady = sorted(o for _, o in timeline)[len(timeline) // 2]
    segs, cur = [], None
    for t, o in timeline:
        if o > steady + 50:
            cur = [t, t, o] if cur is None else [cur[0], t, max(cur[2], o)]
        elif cur is not None:
            segs.append(cur)
            cur = None
    if cur is not None:
        segs.append(cur)
    print(f"[probe] {label}: {len(timeline)} samples, steady outside {steady:.0f} MB, "
          f"{len(segs)} excursions > +50 MB", flush=True)
    for a_, b_, m_ in segs[:8]:
        print(f"[probe]   {a_ - t0:7.3f}-{b_ - t0:7.3f} s  max {m_:.0f} MB; host calls around it:", flush=True)
        for t, n, d in [(t - t0, n, d) for t, n, d in events if a_ - 0.006 <= t <= b_ + 0.003][-60:]:
            print(f"[probe]     {t:8.4f} {d} {n}", flush=True)


def stats():
    st = torch.cuda.memory_stats(dev)
    return {k: st.get(k, 0) for k in ("num_alloc_retries", "num_device_alloc", "num_device_free", "num_ooms")}


for i in range(int(os.environ.get("PROBE_CALLS", "3"))):
    t0 = time.perf_counter()
    timeline.clear()
    events.clear()
    s0 = stats()
    r(prompts)
    torch.cuda.synchronize()
    s1 = stats()
    print(f"[probe] allocator during call {i}: " + ", ".join(f"{k} +{s1[k] - s0[k]}" for k in s0), flush=True)
    print(f"[probe] call {i}: {time.perf_counter() - t0:.2f}s outside-now {outside(slots()):.0f} MB, peak outside "
          f"{peak['v']:.0f} MB, peak used {peak['used']:.3f} GB, reserved peak "
          f"{torch.cuda.max_memory_reserved(dev) / 1e9:.3f} GB", flush=True)
    excursions(t0, f"call {i}")
stop.set()
t.join()
