# MoE throughput on one MI355X: Mixtral-8x7B / Qwen3-30B-A3B, weights streamed vs resident in HBM,
# and a kernel trace of the resident Mixtral pass (run from the repo root on the GPU box)
set -o pipefail
O=gpurun_out/r3_moe
mkdir -p $O
timeout -k 10 300 python bench.py --model mixtral-8x7b --resident --storage gpu --steps 3 --warmup 1 > $O/mixtral_resident.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --model mixtral-8x7b --prompts-per-gpu 96 --steps 3 --warmup 1 > $O/mixtral_stream_96p.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --model qwen3-30b-a3b --steps 3 --warmup 1 > $O/qwen3moe_stream.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --model qwen3-30b-a3b --resident --storage gpu --steps 3 --warmup 1 > $O/qwen3moe_resident.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/trace -o run -- python3 $GRAFT_REPO_ROOT/bench.py --model mixtral-8x7b --resident --storage gpu --steps 2 --warmup 1 > $GRAFT_REPO_ROOT/$O/trace.log 2>&1
