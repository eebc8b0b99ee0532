set -o pipefail
O=gpurun_out/r4_v11probe
mkdir -p $O
timeout -k 10 300 python -u scripts/gemm_v11_ab.py --rounds 3 --orders 0,-8 --plain > $O/ab_plain.log 2>&1 || exit 1
timeout -k 10 300 python -u scripts/gemm_v11_ab.py --rounds 3 --orders 0,-8 --only gateup_swiglu > $O/ab_gu.log 2>&1 || exit 1
