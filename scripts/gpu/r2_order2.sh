# auto tile order A/B at the bench's micro-batch size, then the 1-GPU 70B bench
set -o pipefail
O=gpurun_out/r2_order2
mkdir -p $O
cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u scripts/gemm_order_ab.py --m 16128 --orders 0,-8,8,-4,7 > $O/ab16128.log 2>&1
echo "ab rc=$?"; grep -v amdgpu.ids $O/ab16128.log
timeout -k 10 700 python -u bench.py --steps 5 --warmup 2 > $O/bench.log 2>&1
echo "bench rc=$?"; grep '"metric"' $O/bench.log | cut -c1-400
