set -o pipefail
O=gpurun_out/r4_base
mkdir -p $O
timeout -k 10 300 python -u scripts/gemm_order_sweep.py --orders 0 --rounds 3 > $O/gemm.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --gpus 1 --steps 6 --warmup 2 > $O/bench.log 2>&1 || exit 1
