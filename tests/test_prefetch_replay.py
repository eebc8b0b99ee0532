"""Weight-slot rotation across calls: a normal call, then an empty call or a call
that faults mid-pass, then normal calls.  Replays every load / release of the prefetcher and
asserts that no load lands in a slot whose current shard has not been released (or dropped
unused) — on CPU the slot arithmetic is the same as on the GPU, only no bytes move."""
import numpy as np
import pytest

from flexible_llm_sharding_amd.engine import ShardedRunner
from flexible_llm_sharding_amd.runtime.prefetch import ShardPrefetcher
from flexible_llm_sharding_amd.runtime.stream import FileLayerSource
from flexible_llm_sharding_amd.utils.synthetic import synthetic_prompts
from flexible_llm_sharding_amd.utils.tokenizer import load_tokenizer


class _Tracker:
    def __init__(self, pf: ShardPrefetcher):
        self.pf = pf
        self.owner = {}            # slot -> shard loaded there and not yet released / dropped
        self.violations = []
        load, release, discard = pf._load, pf.release, pf.discard_loaded

        def _load(k, epoch=None):
            r = load(k, epoch)
            s = r[2]
            if pf.in_rotation(k):
                if s in self.owner and self.owner[s] != k:
                    self.violations.append((k, s, self.owner[s]))
                self.owner[s] = k
            return r

        def _release(k):
            ent = pf._ready.get(k)
            release(k)
            if ent is not None and pf.in_rotation(k) and self.owner.get(ent[2]) == k:
                del self.owner[ent[2]]

        def _discard():
            kept = {k: e[2] for k, e in pf._ready.items()}
            discard()
            for k, s in kept.items():
                if k not in pf._ready and self.owner.get(s) == k:
                    del self.owner[s]

        pf._load, pf.release, pf.discard_loaded = _load, _release, _discard


@pytest.mark.parametrize("slots", [2, 3])
@pytest.mark.parametrize("middle", ["empty", "fault"])
def test_no_load_overwrites_an_unreleased_slot(tiny_model, monkeypatch, slots, middle):
    path, cfg = tiny_model
    tok = load_tokenizer(path)
    prompts = synthetic_prompts(5, 20, 2, 5, cfg.vocab_size, seed=3, vary=True)
    r = ShardedRunner(cfg, FileLayerSource(cfg, path), "cpu", tok, layer_num_per_shard=1, token_budget=40,
                      n_slots=slots)
    tr = _Tracker(r.prefetcher)
    want = r(prompts)
    if middle == "empty":
        assert r([]) == []
    else:
        r._fault = 2                               # FLS_FAULT: raise entering local shard 2
        with pytest.raises(RuntimeError, match="FLS_FAULT"):
            r(prompts)
        r._fault = None
    for _ in range(3):
        got = r(prompts)
        for a, b in zip(want, got):
            assert np.array_equal(a, b)
    assert not tr.violations, tr.violations
