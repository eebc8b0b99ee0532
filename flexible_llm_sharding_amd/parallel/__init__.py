"""Parallelism: shard planning, communication (RCCL / gloo), pipeline and data-parallel schedules."""
from .planner import (ShardPlan, make_plan, single_device_shards,  # noqa: F401
                      model_parallel_all_shards, model_parallel_rank_shards,
                      contiguous_stage_plan)
