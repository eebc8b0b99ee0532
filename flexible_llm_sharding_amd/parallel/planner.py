"""Shard planning.

Bit-compatible with the reference formulas in ``/root/reference/utils.py:143-157``:

* single GPU / data parallel: ``num_shards = ceil(L / lnps)`` and
  ``np.array_split(arange(L), num_shards)`` — balanced shards of size <= lnps;
* model parallel over G GPUs: ``num_shards = ceil(ceil(L / lnps) / G) * G``
  (padded to a multiple of G, so empty shards can appear) and rank ``r`` owns
  ``all_shards[r::G]`` (round-robin / interleaved stages).

``L`` is ``num_hidden_layers + 3`` (embed, decoders, final norm, lm_head).

Beyond the reference, ``stages="contiguous"`` gives each GPU one contiguous
slice of layers (``contiguous_stage_plan``), split into shards of <= lnps: a
micro-batch then crosses xGMI G-1 times per pass instead of at every shard
boundary (82 hand-offs for 70B lnps=1 over 8 GPUs) — the layout for resident
pipelines, where each GPU keeps its whole stage in HBM.
"""
from __future__ import annotations

import math
from dataclasses import dataclass
from typing import List, Sequence, Tuple


def _array_split(n: int, sections: int) -> List[Tuple[int, ...]]:
    """numpy.array_split(np.arange(n), sections) without numpy, as tuples."""
    if sections <= 0:
        raise ValueError("number sections must be larger than 0.")
    each, extra = divmod(n, sections)
    out, start = [], 0
    for i in range(sections):
        size = each + (1 if i < extra else 0)
        out.append(tuple(range(start, start + size)))
        start += size
    return out


def single_device_shards(num_layers: int, layer_num_per_shard: int) -> List[Tuple[int, ...]]:
    """utils.py:145-146 — used on one GPU and in data-parallel mode."""
    if layer_num_per_shard < 1:
        raise ValueError("layer_num_per_shard must be >= 1")
    num_shards = math.ceil(num_layers / layer_num_per_shard)
    return _array_split(num_layers, num_shards)


def model_parallel_all_shards(num_layers: int, layer_num_per_shard: int,
                              num_gpus: int) -> List[Tuple[int, ...]]:
    """utils.py:151-152 — the padded global shard list (may contain empty shards)."""
    if layer_num_per_shard < 1 or num_gpus < 1:
        raise ValueError("layer_num_per_shard and num_gpus must be >= 1")
    num_shards = math.ceil(math.ceil(num_layers / layer_num_per_shard) / num_gpus) * num_gpus
    return _array_split(num_layers, num_shards)


def model_parallel_rank_shards(num_layers: int, layer_num_per_shard: int, num_gpus: int,
                               rank: int) -> List[Tuple[int, ...]]:
    """utils.py:153 — shard k belongs to rank k mod G."""
    all_shards = model_parallel_all_shards(num_layers, layer_num_per_shard, num_gpus)
    return list(all_shards[rank::num_gpus])


def contiguous_stage_plan(num_layers: int, num_gpus: int) -> List[Tuple[int, ...]]:
    """One contiguous block of layers per GPU (not in the reference)."""
    return _array_split(num_layers, num_gpus)


@dataclass(frozen=True)
class ShardPlan:
    """The set of shards one rank executes, plus the global view."""
    mode: str                      # "single" | "dp" | "mp"
    rank: int
    world: int
    all_shards: Tuple[Tuple[int, ...], ...]   # global, in execution order
    my_shards: Tuple[Tuple[int, ...], ...]    # this rank, in execution order
    owners: Tuple[int, ...] = ()              # mp: rank of every global shard (default k mod G)
    stages: str = "round_robin"

    def owner_of_layer(self, layer_idx: int) -> int:
        if self.mode != "mp":
            return self.rank
        for k, sh in enumerate(self.all_shards):
            if layer_idx in sh:
                return self.owners[k] if self.owners else k % self.world
        raise KeyError(layer_idx)

    def next_nonempty_owner(self, layer_idx: int) -> int:
        """Rank that consumes the activation produced by ``layer_idx``."""
        return self.owner_of_layer(layer_idx + 1)

    def prev_owner(self, layer_idx: int) -> int:
        return self.owner_of_layer(layer_idx - 1)


PIPELINE_STAGES = ("round_robin", "contiguous")


def make_plan(num_layers: int, layer_num_per_shard: int, world: int, rank: int,
              data_parallel: bool, stages: str = "round_robin") -> ShardPlan:
    if stages not in PIPELINE_STAGES:
        raise ValueError(f"stages={stages!r}: choose from {PIPELINE_STAGES}")
    if world <= 1:
        sh = single_device_shards(num_layers, layer_num_per_shard)
        return ShardPlan("single", 0, 1, tuple(sh), tuple(sh))
    if data_parallel:
        sh = single_device_shards(num_layers, layer_num_per_shard)
        return ShardPlan("dp", rank, world, tuple(sh), tuple(sh))
    if stages == "contiguous":
        all_sh, owners = [], []
        for r, block in enumerate(contiguous_stage_plan(num_layers, world)):
            if not block:
                continue
            for sub in single_device_shards(len(block), layer_num_per_shard):
                all_sh.append(tuple(block[i] for i in sub))
                owners.append(r)
        mine = [sh for sh, o in zip(all_sh, owners) if o == rank]
        return ShardPlan("mp", rank, world, tuple(all_sh), tuple(mine), tuple(owners), stages)
    all_sh = model_parallel_all_shards(num_layers, layer_num_per_shard, world)
    mine = all_sh[rank::world]
    owners = tuple(k % world for k in range(len(all_sh)))
    return ShardPlan("mp", rank, world, tuple(all_sh), tuple(mine), owners, stages)


def shard_sizes(shards: Sequence[Sequence[int]]) -> List[int]:
    return [len(s) for s in shards]
