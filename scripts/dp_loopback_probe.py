"""Probe of the data-parallel prefetcher over loopback thread ranks on one GPU: after every
acquire, synchronise and compare the slot's gathered layer bytes with the full model's
(diagnostic for tests/test_multigpu_gpu.py::test_data_parallel_loopback_7b)."""
import os
import sys
import threading

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from flexible_llm_sharding_amd.config import preset  # noqa: E402
from flexible_llm_sharding_amd.engine import ShardedRunner  # noqa: E402
from flexible_llm_sharding_amd.parallel.comm import LoopbackComm, LoopbackHub  # noqa: E402
from flexible_llm_sharding_amd.parallel.data_parallel import AllGatherPrefetcher, SlicedHostStore  # noqa: E402
from flexible_llm_sharding_amd.parallel.planner import make_plan  # noqa: E402
from flexible_llm_sharding_amd.runtime.weights import HostStore  # noqa: E402
from flexible_llm_sharding_amd.utils.synthetic import synthetic_prompts  # noqa: E402
from flexible_llm_sharding_amd.utils.tokenizer import load_tokenizer, write_synthetic_tokenizer  # noqa: E402

G = int(sys.argv[1]) if len(sys.argv) > 1 else 2
SYNC = os.environ.get("PROBE_SYNC", "0") == "1"
cfg = preset("llama2-7b", num_hidden_layers=4)
dev = torch.device("cuda", 0)
full = HostStore.synthetic(cfg, dev, seed=5)
write_synthetic_tokenizer("/tmp/probe_tok", cfg.vocab_size)
tok = load_tokenizer("/tmp/probe_tok")
names = cfg.layer_names()
bad = []
orig_acquire = AllGatherPrefetcher.acquire


def acquire(self, k):
    views = orig_acquire(self, k)
    torch.cuda.current_stream(self.dev).synchronize()
    for i in self.shards[k]:
        n = self.names[i]
        nb = self.store.nbytes(n)
        ev, v, s = self._ready[k]
        slot = self._slot(s)
        # the views sit at the start of the region of this layer in the slot
        first = next(iter(v[n].values()))
        off = first.data_ptr() - slot.data_ptr()
        got = slot[off:off + nb].cpu()
        want = full.buffers[n][:nb]
        if not torch.equal(got, want):
            diff = (got != want).nonzero()
            bad.append((self.comm.rank, self.epoch, k, n, s, int(diff.numel()), int(diff[0]), nb))
    return views


AllGatherPrefetcher.acquire = acquire
if SYNC:
    orig_load = AllGatherPrefetcher._load

    def _load(self, k, epoch=None):
        r = orig_load(self, k, epoch)
        torch.cuda.synchronize()
        return r
    AllGatherPrefetcher._load = _load

stores = [SlicedHostStore.synthetic(cfg, dev, r, G, seed=5) for r in range(G)]
prompts = synthetic_prompts(4 * G, 1024, 5, 64, cfg.vocab_size, seed=G)
idx = np.array_split(np.arange(len(prompts)), G)
hub = LoopbackHub(G, timeout_s=120)
res = {}


def run(r):
    try:
        torch.cuda.set_device(0)
        comm = LoopbackComm(hub, r, "cuda:0")
        plan = make_plan(len(names), 1, G, r, True)
        pf = AllGatherPrefetcher(stores[r], names, [s for s in plan.my_shards if len(s)], dev, comm)
        rr = ShardedRunner(cfg, stores[r], "cuda:0", tok, layer_num_per_shard=1, storage_location="gpu",
                           comm=comm, data_parallel=True, prefetcher=pf, token_budget=4096)
        res[r] = [rr(prompts_r) for prompts_r in [[prompts[i] for i in idx[r]]] * 2]
    except BaseException as e:  # noqa: BLE001
        import traceback
        traceback.print_exc()
        res[r] = e


ts = [threading.Thread(target=run, args=(r,)) for r in range(G)]
for t in ts:
    t.start()
for t in ts:
    t.join()
print("mismatched layer loads (rank, epoch, shard, layer, slot, n_bytes_bad, first_bad, nbytes):")
for b in bad:
    print("  ", b)
one = ShardedRunner(cfg, full, "cuda:0", tok, layer_num_per_shard=1, storage_location="gpu", token_budget=4096)
for r in range(G):
    want = one([prompts[i] for i in idx[r]])
    for c, call in enumerate(res[r]):
        d = max(float(np.abs(a.astype(np.float32) - b.astype(np.float32)).max()) for a, b in zip(want, call))
        print(f"rank {r} call {c}: max |score diff| vs 1 GPU {d:.3e}")
