"""Shard planner parity with the reference formulas (utils.py:143-157)."""
import math

import numpy as np
import pytest
from hypothesis import given, settings, strategies as st

from flexible_llm_sharding_amd.parallel.planner import (make_plan, model_parallel_all_shards,
                                                        model_parallel_rank_shards, single_device_shards)


def ref_single(L, lnps):
    num_shards = np.ceil(L / lnps)
    return [tuple(int(i) for i in s) for s in np.array_split(np.arange(L), num_shards)]


def ref_mp(L, lnps, G, r):
    num_shards = np.ceil(np.ceil(L / lnps) / G) * G
    all_shards = np.array_split(np.arange(L), num_shards)
    return list(map(tuple, [tuple(int(i) for i in s) for s in all_shards[r::G]]))


@settings(max_examples=200, deadline=None)
@given(L=st.integers(1, 120), lnps=st.integers(1, 40))
def test_single_matches_numpy(L, lnps):
    assert single_device_shards(L, lnps) == ref_single(L, lnps)


@settings(max_examples=200, deadline=None)
@given(L=st.integers(1, 120), lnps=st.integers(1, 40), G=st.integers(1, 8))
def test_mp_matches_numpy(L, lnps, G):
    for r in range(G):
        assert model_parallel_rank_shards(L, lnps, G, r) == ref_mp(L, lnps, G, r)
    # every layer owned exactly once
    owned = sorted(i for r in range(G) for sh in model_parallel_rank_shards(L, lnps, G, r) for i in sh)
    assert owned == list(range(L))


def test_shard_sizes_bounded():
    for L in (35, 83):
        for lnps in (1, 2, 7, 8, 100):
            assert max(len(s) for s in single_device_shards(L, lnps)) <= lnps


def test_survey_examples():
    # 7B (L=35) lnps=8 -> 5 shards of 7 layers
    sh = single_device_shards(35, 8)
    assert [len(s) for s in sh] == [7] * 5
    # 70B (L=83) lnps=8 -> 11 shards of 7-8
    sh = single_device_shards(83, 8)
    assert len(sh) == 11 and set(len(s) for s in sh) == {7, 8}
    # 70B lnps=1 G=8 -> 88 shards, 5 empty; lm_head (layer 82) on rank 2
    allsh = model_parallel_all_shards(83, 1, 8)
    assert len(allsh) == 88 and sum(1 for s in allsh if not s) == 5
    plan = make_plan(83, 1, 8, 0, False)
    assert plan.owner_of_layer(82) == 2


def test_plan_modes():
    p = make_plan(10, 3, 1, 0, False)
    assert p.mode == "single" and p.my_shards == p.all_shards
    p = make_plan(10, 3, 4, 1, True)
    assert p.mode == "dp" and len(p.my_shards) == math.ceil(10 / 3)
    p = make_plan(10, 1, 4, 1, False)
    assert p.mode == "mp" and all(p.owner_of_layer(i) == 1 for sh in p.my_shards for i in sh)


def test_invalid():
    with pytest.raises(ValueError):
        single_device_shards(10, 0)


def test_contiguous_stages():
    """--pipeline_stages contiguous: one contiguous block per rank, split into shards of <= lnps."""
    for L, lnps, G in [(83, 1, 8), (83, 3, 8), (5, 2, 3), (35, 8, 4)]:
        plans = [make_plan(L, lnps, G, r, False, "contiguous") for r in range(G)]
        assert [i for sh in plans[0].all_shards for i in sh] == list(range(L))
        for r, p in enumerate(plans):
            flat = [i for sh in p.my_shards for i in sh]
            assert flat == list(range(flat[0], flat[0] + len(flat)))
            assert all(len(sh) <= lnps for sh in p.my_shards)
            assert all(p.owner_of_layer(i) == r for i in flat)
        # hand-offs between ranks: G - 1 per pass
        owners = [plans[0].owner_of_layer(i) for i in range(L)]
        assert sum(a != b for a, b in zip(owners, owners[1:])) == G - 1
