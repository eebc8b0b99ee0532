# after the fused router + multi-block expert sort + 64k-token MoE MLP chunks: GPU tests, Mixtral /
# Qwen3-MoE resident throughput and a kernel trace of the resident Mixtral pass
set -o pipefail
O=gpurun_out/r3_moe2
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_moe_gpu.py -x -v --timeout 120 --timeout-method thread > $O/moe_tests.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --model mixtral-8x7b --resident --storage gpu --steps 3 --warmup 1 > $O/mixtral_resident.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --model qwen3-30b-a3b --resident --storage gpu --steps 3 --warmup 1 > $O/qwen3moe_resident.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/trace -o run -- python3 $GRAFT_REPO_ROOT/bench.py --model mixtral-8x7b --resident --storage gpu --steps 2 --warmup 1 > $GRAFT_REPO_ROOT/$O/trace.log 2>&1
