"""Model-parallel hand-off and multi-rank paths on MI355X.

* One GPU: two pipeline ranks as threads over :class:`LoopbackComm` (device copies ordered
  by events, no RCCL) at Llama-2-7B geometry drive the real :class:`StageInbox` — fixed HBM
  receive ring, wrap-around parking in HBM / pinned RAM / disk — and must reproduce the 1-GPU
  scores bitwise with memory high-water marks that do not grow with the micro-batch count;
  2 / 4 data-parallel ranks as threads drive the real :class:`AllGatherPrefetcher` (1/G slices
  H2D'd into their places in the HBM slot, loopback all-gather) to the same bitwise standard.
* Two or more GPUs (skipped below that): model-parallel (round-robin and contiguous stages,
  storage gpu / cpu / disk) and data-parallel (pinned slices and streamed files) over RCCL
  against the 1-GPU run, and ``bench.py --gpus 2`` on a real 2-rank ``nccl`` group.
"""
import json
import os
import pickle
import socket
import subprocess
import sys
import threading

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():
    pytest.skip("no GPU", allow_module_level=True)

from flexible_llm_sharding_amd.engine import ShardedRunner  # noqa: E402
from flexible_llm_sharding_amd.parallel.comm import LoopbackComm, LoopbackHub  # noqa: E402
from flexible_llm_sharding_amd.parallel.pipeline import simulate_single_queue  # noqa: E402
from flexible_llm_sharding_amd.runtime.weights import HostStore  # noqa: E402
from flexible_llm_sharding_amd.utils.synthetic import synthetic_prompts  # noqa: E402
from flexible_llm_sharding_amd.utils.tokenizer import load_tokenizer, write_synthetic_tokenizer  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
multi = pytest.mark.skipif(torch.cuda.device_count() < 2, reason="needs >= 2 GPUs")


@pytest.fixture(scope="module")
def seven_b(tmp_path_factory):
    """Llama-2-7B shapes, 4 decoder layers, random-init in pinned host RAM."""
    from flexible_llm_sharding_amd.config import preset
    cfg = preset("llama2-7b", num_hidden_layers=4)
    store = HostStore.synthetic(cfg, torch.device("cuda", 0), seed=5)
    d = str(tmp_path_factory.mktemp("tok"))
    write_synthetic_tokenizer(d, cfg.vocab_size)
    return cfg, store, load_tokenizer(d)


def _loopback_pass(cfg, store, tok, prompts, storage, tmp, max_act=1, window=2, stages="round_robin"):
    hub = LoopbackHub(2, timeout_s=120)
    res, runners = {}, {}

    def run(r):
        try:
            torch.cuda.set_device(0)
            rr = ShardedRunner(cfg, store, "cuda:0", tok, layer_num_per_shard=1, storage_location=storage,
                               disk_folder=os.path.join(tmp, f"spill{r}"), comm=LoopbackComm(hub, r, "cuda:0"),
                               token_budget=4096, max_activation_in_cpu=max_act, rx_window=window,
                               pipeline_stages=stages)
            runners[r] = rr
            res[r] = rr(prompts)
        except BaseException as e:  # noqa: BLE001
            res[r] = e

    ts = [threading.Thread(target=run, args=(r,)) for r in range(2)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=300)
    for r in range(2):
        assert not isinstance(res.get(r), BaseException), res.get(r)
    assert simulate_single_queue({r: hub.log[r] for r in range(2)})[0]
    owner = [res[r] for r in range(2) if res[r] and res[r][0] is not None]
    assert len(owner) == 1
    stats = {r: dict(runners[r].stats) for r in range(2)}
    ring = {r: runners[r]._inbox.ring_bytes() if runners[r]._inbox is not None else 0 for r in range(2)}
    for rr in runners.values():
        rr.close()
    return owner[0], stats, ring


@pytest.mark.parametrize("storage", ["gpu", "cpu", "disk"])
def test_stage_inbox_loopback_7b_bounded(seven_b, tmp_path, storage):
    """Two pipeline ranks on one GPU, 4 vs 8 micro-batches per pass, --max_activation_in_cpu 1:
    scores bitwise equal to the 1-GPU run; the receive ring and the parked bytes per tier stay
    the same when the micro-batch count doubles (the wrap-around backlog spills to the next
    tier instead of growing)."""
    cfg, store, tok = seven_b
    seen = {}
    for n_prompts in (12, 24):
        prompts = synthetic_prompts(n_prompts, 1024, 5, 64, cfg.vocab_size, seed=n_prompts)
        one = ShardedRunner(cfg, store, "cuda:0", tok, layer_num_per_shard=1, storage_location="gpu",
                            token_budget=4096)
        want = one(prompts)
        one.close()
        got, stats, ring = _loopback_pass(cfg, store, tok, prompts, storage, str(tmp_path))
        for a, b in zip(want, got):
            assert np.isfinite(a.astype(np.float32)).all()
            assert np.array_equal(a, b)
        nb = stats[0]["micro_batches"]
        assert nb >= (4 if n_prompts == 12 else 8)
        s0 = stats[0]
        assert s0["rx_parked"] > 0                      # rank 0 parks the wrap-around inputs
        assert s0["rx_max_parked_gpu"] <= 1 and s0["rx_max_parked_cpu"] <= 1
        assert stats[1]["rx_max_ring_in_use"] <= 2
        seen[n_prompts] = (ring, s0["rx_max_parked_bytes_gpu"], s0["rx_max_parked_bytes_cpu"])
    (ra, ga, ca), (rb, gb, cb) = seen[12], seen[24]
    assert ra == rb and ga == gb and ca == cb


@pytest.mark.parametrize("storage", ["gpu", "cpu"])
def test_contiguous_stages_loopback_7b(seven_b, tmp_path, storage):
    """Contiguous stages (rank r owns one block of layers): rank 1's first shard computes on a
    received state IN its receive-ring slot (the residual GEMMs are in place) and keeps the result
    on the rank for its next shard, while later receives reuse the ring (window 2, >= 3
    micro-batches).  The state must leave the slot before release: scores bitwise
    equal to the 1-GPU run."""
    cfg, store, tok = seven_b
    prompts = synthetic_prompts(12, 1024, 5, 64, cfg.vocab_size, seed=77)
    one = ShardedRunner(cfg, store, "cuda:0", tok, layer_num_per_shard=1, storage_location="gpu",
                        token_budget=4096)
    want = one(prompts)
    one.close()
    got, stats, _ = _loopback_pass(cfg, store, tok, prompts, storage, str(tmp_path), stages="contiguous")
    assert stats[1]["micro_batches"] >= 3
    for a, b in zip(want, got):
        assert np.isfinite(a.astype(np.float32)).all()
        assert np.array_equal(a, b)


@pytest.mark.parametrize("G,pool,n_prompts", [(2, "layer", 8), (4, "layer", 16), (2, "pieces", 8),
                                               (4, "pieces", 3)])
def test_data_parallel_loopback_7b(seven_b, G, pool, n_prompts):
    """Data parallel with G ranks as threads on ONE GPU: each rank holds 1/G of every layer in
    pinned RAM, H2Ds only its slice into its place in the HBM slot on the prefetcher's copy stream,
    and the loopback all-gather (device copies ordered by events, parallel/comm.py) completes the
    layer before compute; two calls (slot rotation across calls).  Each rank's scores must equal
    the 1-GPU run on its prompts bitwise: the weights are assembled exactly.  ``pieces``: the
    sub-layer piece pool of the --max_vram_gb mode (AllGatherPiecePool: one attention + two MLP
    slots, each piece all-gathered on its own), with 3 prompts on 4 ranks (an empty rank acquires
    and releases every layer, its pieces still gathered in pass order)."""
    cfg, full, tok = seven_b
    prompts = synthetic_prompts(n_prompts, 1024, 5, 64, cfg.vocab_size, seed=G)
    _dp_loopback_check(cfg, full, tok, G, pool, prompts, seed=5)             # seven_b's seed


def test_data_parallel_loopback_70b_eight_ranks(tmp_path):
    """The scaling run's default path (bench.py --gpus 8: data parallel, sub-layer pieces all-gathered
    under the 6 GB plan, AllGatherPiecePool) with 8 ranks as threads on one MI355X at Llama-2-70B
    layer geometry (2 decoder layers: 70B-sized attention / MLP pieces, 8-way slices of them),
    12 prompts over 8 ranks (uneven slices), two calls each: every rank's scores equal the 1-GPU run
    on its prompts bitwise."""
    from flexible_llm_sharding_amd.config import preset
    cfg = preset("llama2-70b", num_hidden_layers=2)
    full = HostStore.synthetic(cfg, torch.device("cuda", 0), seed=7)
    d = str(tmp_path / "tok")
    write_synthetic_tokenizer(d, cfg.vocab_size)
    tok = load_tokenizer(d)
    prompts = synthetic_prompts(12, 1024, 5, 64, cfg.vocab_size, seed=8)
    _dp_loopback_check(cfg, full, tok, 8, "pieces", prompts, seed=7)


def _dp_loopback_check(cfg, full, tok, G, pool, prompts, seed):
    from flexible_llm_sharding_amd.parallel.data_parallel import (AllGatherPiecePool, AllGatherPrefetcher,
                                                                  SlicedHostStore)
    from flexible_llm_sharding_amd.parallel.planner import make_plan
    dev = torch.device("cuda", 0)
    idx = np.array_split(np.arange(len(prompts)), G)
    names = cfg.layer_names()
    stores = [SlicedHostStore.synthetic(cfg, dev, r, G, seed=seed) for r in range(G)]
    hub = LoopbackHub(G, timeout_s=300)
    res, runners = {}, {}

    def run(r):
        try:
            torch.cuda.set_device(0)
            comm = LoopbackComm(hub, r, "cuda:0")
            plan = make_plan(len(names), 1, G, r, True)
            shards = [s for s in plan.my_shards if len(s)]
            pf = (AllGatherPiecePool(stores[r], names, shards, dev, comm) if pool == "pieces"
                  else AllGatherPrefetcher(stores[r], names, shards, dev, comm))
            rr = ShardedRunner(cfg, stores[r], "cuda:0", tok, layer_num_per_shard=1, storage_location="gpu",
                               comm=comm, data_parallel=True, prefetcher=pf, token_budget=4096)
            if pool == "pieces":
                # one attention + two MLP piece slots (+ small own buffers) < the double buffer
                dec = next(n for n in names if n.startswith("model.layers."))
                assert pf.planned_hbm_bytes() < 2 * full.nbytes(dec)
            runners[r] = rr
            mine = [prompts[i] for i in idx[r]]
            res[r] = [rr(mine) for _ in range(2)]
        except BaseException as e:  # noqa: BLE001
            res[r] = e

    ts = [threading.Thread(target=run, args=(r,)) for r in range(G)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=600)
    for r in range(G):
        assert not isinstance(res.get(r), BaseException), res.get(r)
    torch.cuda.synchronize()
    for rr in runners.values():
        rr.close()
    del stores
    one = ShardedRunner(cfg, full, "cuda:0", tok, layer_num_per_shard=1, storage_location="gpu", token_budget=4096)
    for r in range(G):
        if not len(idx[r]):
            assert all(call == [] for call in res[r])
            continue
        want = one([prompts[i] for i in idx[r]])
        for call in res[r]:
            for a, b in zip(want, call):
                assert np.isfinite(a.astype(np.float32)).all()
                assert np.array_equal(a, b)
    one.close()


# --------------------------------------------------------------------------- >= 2 GPUs


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _mp_worker(rank, world, port, out_dir, storage, stages, dp, weights, cap=None, n_prompts=16):
    os.environ.update({"RANK": str(rank), "WORLD_SIZE": str(world), "LOCAL_RANK": str(rank),
                       "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port)})
    from flexible_llm_sharding_amd.config import preset
    from flexible_llm_sharding_amd.parallel.comm import Comm
    from flexible_llm_sharding_amd.parallel.data_parallel import build_dp_sharded_runner
    from flexible_llm_sharding_amd.utils.synthetic import write_synthetic_checkpoint
    from types import SimpleNamespace
    comm = Comm.from_env("cuda", timeout_s=300)
    cfg = preset("llama2-7b", num_hidden_layers=4)
    ck = os.path.join(out_dir, "ckpt")
    if rank == 0 and not os.path.exists(os.path.join(ck, "config.json")):
        write_synthetic_checkpoint(cfg, ck, seed=5, device=comm.device, unique_layers=2)
    comm.barrier()
    tok = load_tokenizer(ck)
    prompts = synthetic_prompts(16, 1024, 5, 64, cfg.vocab_size, seed=3)[:n_prompts]
    if dp:
        args = SimpleNamespace(model_path=ck, layer_num_per_shard=1, storage_location=storage,
                               disk_folder=os.path.join(out_dir, f"spill{rank}"), max_activation_in_cpu=100,
                               prefix_attention="bidirectional", token_budget=4096, resident=False, dtype=None,
                               verbose=False, max_vram_gb=cap)
        r = build_dp_sharded_runner(args, cfg, comm.device, comm, tok, weight_cache=weights)
        if cap:
            # the capped data-parallel default: sub-layer pieces all-gathered per piece
            assert type(r.prefetcher).__name__ == "AllGatherPiecePool"
        idx = np.array_split(np.arange(len(prompts)), world)[rank]
        outs = r([prompts[i] for i in idx])
        outs = r([prompts[i] for i in idx])           # second call: the piece / slot rotation
    else:
        from flexible_llm_sharding_amd.runtime.stream import FileLayerSource
        r = ShardedRunner(cfg, FileLayerSource(cfg, ck), comm.device, tok, layer_num_per_shard=1,
                          storage_location=storage, disk_folder=os.path.join(out_dir, f"spill{rank}"),
                          comm=comm, token_budget=4096, pipeline_stages=stages, max_activation_in_cpu=2)
        outs = r(prompts)
        outs = r(prompts)                             # the runner-lifetime inbox, second call
    allv = comm.gather_scores(outs, dst=0)           # the production score path (api.run_all)
    if rank == 0:
        with open(os.path.join(out_dir, "out.pkl"), "wb") as f:
            pickle.dump(allv, f)
    r.close()
    comm.destroy()


@pytest.fixture(scope="module")
def one_gpu_ref(tmp_path_factory):
    from flexible_llm_sharding_amd.config import preset
    from flexible_llm_sharding_amd.runtime.stream import FileLayerSource
    from flexible_llm_sharding_amd.utils.synthetic import write_synthetic_checkpoint
    d = str(tmp_path_factory.mktemp("mgpu"))
    cfg = preset("llama2-7b", num_hidden_layers=4)
    ck = os.path.join(d, "ckpt")
    write_synthetic_checkpoint(cfg, ck, seed=5, device=torch.device("cuda", 0), unique_layers=2)
    prompts = synthetic_prompts(16, 1024, 5, 64, cfg.vocab_size, seed=3)
    r = ShardedRunner(cfg, FileLayerSource(cfg, ck), "cuda:0", load_tokenizer(ck), layer_num_per_shard=1,
                      storage_location="gpu", token_budget=4096)
    out = r(prompts)
    r.close()
    return d, out


def _spawn(d, world, *args):
    import torch.multiprocessing as mp
    world = min(world, torch.cuda.device_count())
    mp.start_processes(_mp_worker, args=(world, _port(), d) + args, nprocs=world, start_method="spawn", join=True)
    return pickle.load(open(os.path.join(d, "out.pkl"), "rb"))


@multi
@pytest.mark.parametrize("stages,storage", [("round_robin", "gpu"), ("round_robin", "cpu"),
                                            ("round_robin", "disk"), ("contiguous", "cpu")])
def test_model_parallel_rccl_matches_one_gpu(one_gpu_ref, stages, storage):
    d, want = one_gpu_ref
    allv = _spawn(d, 2, storage, stages, False, "host")
    owner = [v for v in allv if v and v[0] is not None]
    assert len(owner) == 1
    for a, b in zip(owner[0], want):
        assert np.array_equal(a, b)


@multi
@pytest.mark.parametrize("weights", ["host", "stream"])
def test_data_parallel_rccl_matches_one_gpu(one_gpu_ref, weights):
    d, want = one_gpu_ref
    got = sum(_spawn(d, 2, "cpu", "round_robin", True, weights), [])
    assert len(got) == len(want)
    for a, b in zip(got, want):
        assert np.abs(a.astype(np.float32) - b.astype(np.float32)).max() < 2e-3


@multi
@pytest.mark.parametrize("n_prompts", [16, 1])
def test_data_parallel_rccl_capped_piece_pool(one_gpu_ref, n_prompts):
    """The bench's data-parallel default under --max_vram_gb (AllGatherPiecePool: each rank H2Ds
    1/G of every attention / MLP piece, RCCL all-gathers complete them in pass order) over a real
    2-rank nccl group, two calls; with 1 prompt rank 1 is empty and still joins every gather."""
    d, want = one_gpu_ref
    got = sum(_spawn(d, 2, "cpu", "round_robin", True, "host", 2.4, n_prompts), [])
    assert len(got) == n_prompts
    for a, b in zip(got, want):
        assert np.abs(a.astype(np.float32) - b.astype(np.float32)).max() < 2e-3


def _main_cli(tmp, ck, n_gpus, extra):
    out = os.path.join(tmp, f"scores_{n_gpus}_{'_'.join(extra) or 'mp'}.pkl")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "main.py"), "--model_path", ck, "--prompt_pickle",
                        os.path.join(tmp, "prompts.pkl"), "--output_file", out, "--num_gpus", str(n_gpus),
                        "--storage_location", "cpu"] + extra, cwd=tmp, capture_output=True, text=True, timeout=900,
                       env=dict(os.environ, PYTHONPATH=ROOT))
    assert r.returncode == 0, r.stderr[-3000:]
    return pickle.load(open(out, "rb"))


@multi
@pytest.mark.parametrize("extra", [[], ["--data_parallel", "True"], ["--data_parallel", "True", "--max_vram_gb", "2.4"],
                                   ["--data_parallel", "True", "--dp_gather_comm", "native"]])
def test_main_cli_two_gpus_matches_one(one_gpu_ref, extra):
    """``main.py --num_gpus 2`` end to end (spawned ranks, RCCL hand-offs or all-gathers, rank-0
    score gather, output pickles): model parallel (default) and data parallel (capped too) equal
    the one-GPU CLI run; data parallel with its weight gathers on the native RCCL communicator too."""
    d, _ = one_gpu_ref
    ck = os.path.join(d, "ckpt")
    from flexible_llm_sharding_amd.config import preset
    cfg = preset("llama2-7b", num_hidden_layers=4)
    prompts = synthetic_prompts(5, 300, 4, 12, cfg.vocab_size, seed=4)
    with open(os.path.join(d, "prompts.pkl"), "wb") as f:
        pickle.dump(prompts, f)
    one = _main_cli(d, ck, 1, [x for x in extra if x not in ("True", "--data_parallel", "--dp_gather_comm", "native")])
    two = _main_cli(d, ck, 2, extra)
    assert len(one) == len(two) == len(prompts)
    for a, b in zip(one, two):
        assert a.shape == b.shape
        assert np.abs(a.astype(np.float32) - b.astype(np.float32)).max() < 2e-3


@multi
def test_bench_two_ranks_over_rccl(tmp_path):
    out = tmp_path / "b.json"
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "2",
                        "--warmup", "1", "--model", "llama2-7b", "--num-layers", "4", "--prompts-per-gpu", "4",
                        "--json-out", str(out)], cwd=ROOT, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    rec = json.load(open(out))
    assert rec["process_group_ranks"] == 2 and rec["backend"] == "nccl" and rec["n_gpus"] == 2
    assert rec["scores_finite"] and rec["value"] > 0


def test_native_rccl_communicator_one_rank():
    """The native RCCL communicator (csrc/comm/rccl_comm.cpp, --dp_gather_comm native) on one rank:
    it initialises, runs the in-place byte all-gather the weight fan-out issues on the copy stream
    (this rank's slice already in place: out unchanged), a second gather into a separate buffer, and
    tears down.  Multi-rank RCCL needs several GPUs (the driver's node)."""
    from flexible_llm_sharding_amd.parallel.comm import Comm
    from flexible_llm_sharding_amd.parallel.native_comm import NativeRcclComm
    base = Comm(0, 1, torch.device("cuda", 0))
    base.gather_native = True
    c = base.dup()
    assert isinstance(c, NativeRcclComm)
    c.warmup()
    out = torch.arange(4096, dtype=torch.int32, device="cuda:0").view(torch.uint8)
    want = out.clone()
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        c.all_gather_into(out, out[:out.numel()]).wait()
        dst = torch.zeros_like(out)
        c.all_gather_into(dst, out).wait()
    s.synchronize()
    assert torch.equal(out, want) and torch.equal(dst, want)
    c.destroy()
