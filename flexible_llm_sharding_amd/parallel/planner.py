"""Shard planning.

Bit-compatible with the reference formulas in ``/root/reference/utils.py:143-157``:

* single GPU / data parallel: ``num_shards = ceil(L / lnps)`` and
  ``np.array_split(arange(L), num_shards)`` — balanced shards of size <= lnps;
* model parallel over G GPUs: ``num_shards = ceil(ceil(L / lnps) / G) * G``
  (padded to a multiple of G, so empty shards can appear) and rank ``r`` owns
  ``all_shards[r::G]`` (round-robin / interleaved stages).

``L`` is ``num_hidden_layers + 3`` (embed, decoders, final norm, lm_head).

Beyond the reference we add ``contiguous_stage_plan`` — the MI355X-friendly
alternative for resident pipelines where each GPU owns one contiguous slice.
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

    def owner_of_layer(self, layer_idx: int) -> int:
        if self.mode != "mp":
            return self.rank
        for k, sh in enumerate(self.all_shards):
            if layer_idx in sh:
                return k % self.world
        raise KeyError(layer_idx)

    def next_nonempty_owner(self, layer_idx: int) -> int:
        """Rank that consumes the activation produced by ``layer_idx``."""
        return self.owner_of_layer(layer_idx + 1)

    def prev_owner(self, layer_idx: int) -> int:
        return self.owner_of_layer(layer_idx - 1)


def make_plan(num_layers: int, layer_num_per_shard: int, world: int, rank: int,
              data_parallel: bool) -> ShardPlan:
    if world <= 1:
        sh = single_device_shards(num_layers, layer_num_per_shard)
        return ShardPlan("single", 0, 1, tuple(sh), tuple(sh))
    if data_parallel:
        sh = single_device_shards(num_layers, layer_num_per_shard)
        return ShardPlan("dp", rank, world, tuple(sh), tuple(sh))
    all_sh = model_parallel_all_shards(num_layers, layer_num_per_shard, world)
    mine = all_sh[rank::world]
    return ShardPlan("mp", rank, world, tuple(all_sh), tuple(mine))


def shard_sizes(shards: Sequence[Sequence[int]]) -> List[int]:
    return [len(s) for s in shards]
