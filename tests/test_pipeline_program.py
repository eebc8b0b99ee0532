"""Model-parallel hand-off program: deadlock freedom on the worst-case queue model, the
"receive (j+1, b) only after send (j, b)" rule, and the bounded inbox — on CPU.

The engine's real runs use RCCL, whose ``wait()`` does not block the host; these tests check
the submission ORDER instead: every rank's recorded sends / receives are replayed on a model
where each rank owns ONE in-order queue (every stream sharing one hardware queue) and sends /
receives rendezvous.  A program that completes there cannot deadlock on any stream -> queue
mapping (``parallel/pipeline.py``)."""
import threading

import numpy as np
import pytest
import torch

from flexible_llm_sharding_amd.parallel.pipeline import (build_programs, program_ops, rank_items,
                                                         simulate_single_queue)
from flexible_llm_sharding_amd.parallel.planner import make_plan


def _programs(L, lnps, G, B, stages="round_robin", mb_major=False, start=0):
    plans = {r: make_plan(L, lnps, G, r, False, stages) for r in range(G)}
    return plans, build_programs(plans, B, mb_major, start)


CASES = [(L, lnps, G, B, st)
         for L in (5, 9, 83)
         for lnps in (1, 2, 3)
         for G in (2, 3, 4, 5, 8)
         for B in (1, 2, 3, 7, 17)
         for st in ("round_robin", "contiguous")
         if not (L == 83 and B == 17 and G < 4)]


@pytest.mark.parametrize("L,lnps,G,B,stages", CASES)
def test_programs_complete_on_single_queue(L, lnps, G, B, stages):
    plans, progs = _programs(L, lnps, G, B, stages)
    ok, left = simulate_single_queue({r: program_ops(p) for r, p in progs.items()})
    assert ok, left
    for r, p in progs.items():
        assert p.items == rank_items([s for s in plans[r].my_shards if s], B)
        idx = {it: i for i, it in enumerate(p.items)}
        for i, (k, b) in enumerate(p.items):
            if p.src[i] is None:
                continue
            post = p.post_index(i)
            assert post <= i
            # never ahead of this rank's own work on the same micro-batch at an earlier shard
            if k > 0 and (k - 1, b) in idx:
                assert post > idx[(k - 1, b)]
            if stages == "contiguous" or r != 0:
                assert i not in p.parked           # only the wrap-around edge (-> rank 0) parks
        # the receive order on every edge is the send order of the producer
        for src in set(s for s in p.src if s is not None):
            mine = [i for lst in p.posts for i in lst if p.src[i] == src]
            prod = progs[src]
            sent = [it for j, it in enumerate(prod.items) if prod.dst[j] == r]
            assert [p.items[i][1] for i in mine] == [b for _, b in sent]


@pytest.mark.parametrize("G,B", [(2, 4), (4, 8), (8, 16)])
def test_round_robin_wrap_edge_parks_backlog(G, B):
    """70B lnps=1 over G GPUs: rank 0 parks one round of wrap-around inputs (posted right after
    its own send of the same micro-batch), every other rank receives at the point of use."""
    _, progs = _programs(83, 1, G, B)
    p0 = progs[0]
    rx0 = [i for i, s in enumerate(p0.src) if s is not None]
    assert rx0 and set(rx0) == set(p0.parked)
    for i in rx0:
        k, b = p0.items[i]
        assert p0.post_index(i) == p0.items.index((k - 1, b)) + 1
    for r in range(1, G):
        assert not progs[r].parked


def _naive_ops(prog, posts_at):
    """The round-2 receiver: all of a shard's receives posted at ``posts_at`` items ahead."""
    ops, seq = [], {}
    pending = [i for i, s in enumerate(prog.src) if s is not None]
    r = prog.rank
    for p in range(len(prog.items)):
        while pending and pending[0] <= p + posts_at:
            c = pending.pop(0)
            e = (prog.src[c], r)
            ops.append(("recv", e[0], e[1], seq.get(("r",) + e, 0)))
            seq[("r",) + e] = seq.get(("r",) + e, 0) + 1
        ops.append(("compute", p))
        if prog.dst[p] is not None:
            e = (r, prog.dst[p])
            ops.append(("send", e[0], e[1], seq.get(("s",) + e, 0)))
            seq[("s",) + e] = seq.get(("s",) + e, 0) + 1
    return ops


def test_simulator_catches_receives_posted_ahead():
    """Posting receives far ahead (the round-2 StageReceiver posted a whole pass at once) can
    deadlock once streams share a queue: the model must report it."""
    _, progs = _programs(9, 1, 2, 4)
    ok, _ = simulate_single_queue({r: _naive_ops(p, 10 ** 6) for r, p in progs.items()})
    assert not ok
    ok, _ = simulate_single_queue({r: program_ops(p) for r, p in progs.items()})
    assert ok


@pytest.mark.parametrize("G", [2, 3, 4])
def test_micro_batch_major_contiguous_and_resume(G):
    _, progs = _programs(20, 1, G, 6, "contiguous", mb_major=True)
    assert simulate_single_queue({r: program_ops(p) for r, p in progs.items()})[0]
    for p in progs.values():
        assert not p.parked
    # resume at a stage boundary (round robin, layer 7): nothing before it, no receive into it
    plans, progs = _programs(20, 1, G, 5, start=7)
    assert simulate_single_queue({r: program_ops(p) for r, p in progs.items()})[0]
    for r, p in progs.items():
        for i, (k, b) in enumerate(p.items):
            sh = [s for s in plans[r].my_shards if s][k]
            assert sh[0] >= 7
            if sh[0] == 7:
                assert p.src[i] is None


# --------------------------------------------------------------------------- engine runs


@pytest.fixture(scope="module")
def deep6(tmp_path_factory):
    from flexible_llm_sharding_amd.config import preset
    from flexible_llm_sharding_amd.engine import ShardedRunner
    from flexible_llm_sharding_amd.runtime.stream import FileLayerSource
    from flexible_llm_sharding_amd.utils.synthetic import synthetic_prompts, write_synthetic_checkpoint
    from flexible_llm_sharding_amd.utils.tokenizer import load_tokenizer
    cfg = preset("tiny", num_hidden_layers=6)
    path = str(tmp_path_factory.mktemp("pp6"))
    write_synthetic_checkpoint(cfg, path, seed=2, std=0.05)
    tok = load_tokenizer(path)
    prompts = synthetic_prompts(7, 25, 3, 6, cfg.vocab_size, seed=22, vary=True)
    out = ShardedRunner(cfg, FileLayerSource(cfg, path), "cpu", tok)(prompts)
    return cfg, path, tok, prompts, out


def _run_loopback(deep6, tmp_path, G, storage, stages, max_act, window=2, calls=2, resident=False):
    from flexible_llm_sharding_amd.engine import ShardedRunner
    from flexible_llm_sharding_amd.parallel.comm import LoopbackComm, LoopbackHub
    from flexible_llm_sharding_amd.runtime.stream import FileLayerSource
    cfg, path, tok, prompts, ref = deep6
    hub = LoopbackHub(G, timeout_s=60)
    res, runners = {}, {}

    def run(r):
        try:
            rr = ShardedRunner(cfg, FileLayerSource(cfg, path), "cpu", tok, layer_num_per_shard=1,
                               storage_location=storage, disk_folder=str(tmp_path / f"spill{r}"),
                               comm=LoopbackComm(hub, r, "cpu"), token_budget=40, pipeline_stages=stages,
                               max_activation_in_cpu=max_act, rx_window=window, resident=resident)
            runners[r] = rr
            res[r] = [rr(prompts) for _ in range(calls)]
        except BaseException as e:  # noqa: BLE001
            res[r] = e

    torch.set_num_threads(1)
    ts = [threading.Thread(target=run, args=(r,)) for r in range(G)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    for r in range(G):
        if isinstance(res[r], BaseException):
            raise res[r]
    return hub, res, runners, ref


@pytest.mark.parametrize("G,storage,stages,max_act", [
    (2, "cpu", "round_robin", 1), (3, "gpu", "round_robin", 100), (4, "disk", "round_robin", 100),
    (5, "cpu", "round_robin", 2), (2, "gpu", "contiguous", 100), (3, "cpu", "contiguous", 1),
    (8, "gpu", "round_robin", 1)])
def test_engine_follows_program_over_recording_comm(deep6, tmp_path, G, storage, stages, max_act):
    """G runners as threads over a recording loopback comm: scores equal the one-process run,
    every rank's recorded send/receive order equals its program and replays deadlock-free on the
    one-queue model, at most ``rx_window`` ring receives are in flight and parked activations
    never pass ``--max_activation_in_cpu`` per tier."""
    hub, res, runners, ref = _run_loopback(deep6, tmp_path, G, storage, stages, max_act)
    owner = [res[r] for r in range(G) if res[r][0] and res[r][0][0] is not None]
    assert len(owner) == 1
    for outs in owner[0]:
        for a, b in zip(outs, ref):
            assert np.abs(a.astype(np.float32) - b.astype(np.float32)).max() < 1e-5
    ok, left = simulate_single_queue({r: hub.log[r] for r in range(G)})
    assert ok, left
    nb = int(runners[0].stats["micro_batches"])
    for r in range(G):
        prog = runners[r]._mp_program(nb)
        want = [op for op in program_ops(prog) if op[0] != "compute"]
        # two calls, same program (edge sequence numbers run on across calls)
        assert [op[:3] for op in hub.log[r]] == [op[:3] for op in want] * 2
        st = runners[r].stats
        assert st.get("rx_max_ring_in_use", 0) <= runners[r].rx_window
        for tier in ("gpu", "cpu"):
            assert st.get(f"rx_max_parked_{tier}", 0) <= max_act
        if r == 0 and stages == "round_robin" and storage != "disk":
            assert st["rx_parked"] > 0


def test_engine_contiguous_resident_micro_batch_major(deep6, tmp_path):
    hub, res, runners, ref = _run_loopback(deep6, tmp_path, 3, "gpu", "contiguous", 100, resident=True)
    assert runners[0].schedule(3)[:2] == [(0, 0), (1, 0)]
    owner = [res[r] for r in range(3) if res[r][0] and res[r][0][0] is not None][0]
    for a, b in zip(owner[0], ref):
        assert np.abs(a.astype(np.float32) - b.astype(np.float32)).max() < 1e-5
    assert simulate_single_queue({r: hub.log[r] for r in range(3)})[0]


def test_loopback_all_gather_in_place_and_dup():
    """LoopbackComm.all_gather_into (the data-parallel weight gather over thread ranks): every
    rank's slice lands in every rank's buffer, in place, across repeated rounds on a dup()'ed
    communicator."""
    from flexible_llm_sharding_amd.parallel.comm import LoopbackComm, LoopbackHub
    hub = LoopbackHub(3, timeout_s=30)
    res = {}

    def run(r):
        c = LoopbackComm(hub, r, "cpu").dup()
        for it in range(3):
            out = torch.zeros(12, dtype=torch.uint8)
            mine = out[r * 4:(r + 1) * 4]
            mine.fill_(10 * it + r + 1)
            assert c.all_gather_into(out, mine).wait()
            res[(r, it)] = out.tolist()

    ts = [threading.Thread(target=run, args=(r,)) for r in range(3)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    for r in range(3):
        for it in range(3):
            assert res[(r, it)] == sum([[10 * it + q + 1] * 4 for q in range(3)], [])


@pytest.mark.parametrize("G,n", [(2, 7), (3, 7), (9, 7)])
def test_data_parallel_over_loopback_threads(deep6, G, n):
    """Data parallel with G ranks as threads (AllGatherPrefetcher: 1/G slices + loopback
    all-gather into the weight slot): each rank's scores == a one-process run on its prompts,
    over two calls (slot rotation across calls); G > prompts: ranks with no prompts join every
    gather of both calls."""
    import numpy as np
    from flexible_llm_sharding_amd.engine import ShardedRunner
    from flexible_llm_sharding_amd.parallel.comm import LoopbackComm, LoopbackHub
    from flexible_llm_sharding_amd.parallel.data_parallel import AllGatherPrefetcher, SlicedHostStore
    from flexible_llm_sharding_amd.parallel.planner import make_plan
    from flexible_llm_sharding_amd.runtime.stream import FileLayerSource
    cfg, path, tok, prompts, _ = deep6
    prompts = prompts[:n]
    torch.set_num_threads(1)
    idx = np.array_split(np.arange(len(prompts)), G)
    hub = LoopbackHub(G, timeout_s=60)
    names = cfg.layer_names()
    res = {}

    def run(r):
        try:
            comm = LoopbackComm(hub, r, "cpu")
            store = SlicedHostStore.from_source(FileLayerSource(cfg, path), r, G, pinned=False)
            plan = make_plan(len(names), 1, G, r, True)
            pf = AllGatherPrefetcher(store, names, [s for s in plan.my_shards if len(s)], torch.device("cpu"), comm)
            rr = ShardedRunner(cfg, store, "cpu", tok, layer_num_per_shard=1, storage_location="gpu", comm=comm,
                               data_parallel=True, prefetcher=pf, token_budget=40)
            mine = [prompts[i] for i in idx[r]]
            res[r] = [rr(mine) for _ in range(2)]
        except BaseException as e:  # noqa: BLE001
            res[r] = e

    ts = [threading.Thread(target=run, args=(r,)) for r in range(G)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    for r in range(G):
        if isinstance(res[r], BaseException):
            raise res[r]
        if not len(idx[r]):
            assert all(call == [] for call in res[r])
            continue
        want = ShardedRunner(cfg, FileLayerSource(cfg, path), "cpu", tok, token_budget=40)([prompts[i] for i in idx[r]])
        for call in res[r]:
            assert len(call) == len(want)
            for a, b in zip(call, want):
                assert np.abs(a.astype(np.float32) - b.astype(np.float32)).max() < 1e-5


def test_runner_warms_every_communicator_at_construction(deep6, tmp_path):
    """No VRAM cap: a model-parallel runner still warms the default group and every directed
    hand-off edge in its constructor (VERDICT r3 #2b), so no communicator is created lazily
    inside the first pass."""
    from flexible_llm_sharding_amd.engine import ShardedRunner
    from flexible_llm_sharding_amd.parallel.comm import LoopbackComm, LoopbackHub
    from flexible_llm_sharding_amd.runtime.stream import FileLayerSource
    cfg, path, tok, prompts, ref = deep6
    calls = []

    class Recording(LoopbackComm):
        def warmup(self):
            calls.append((self.rank, "warmup"))

        def warmup_p2p(self):
            calls.append((self.rank, "warmup_p2p"))

    hub = LoopbackHub(2, timeout_s=60)
    for r in range(2):
        ShardedRunner(cfg, FileLayerSource(cfg, path), "cpu", tok, comm=Recording(hub, r, "cpu")).close()
    assert sorted(calls) == [(0, "warmup"), (0, "warmup_p2p"), (1, "warmup"), (1, "warmup_p2p")]
