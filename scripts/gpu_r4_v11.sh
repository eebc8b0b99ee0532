set -o pipefail
O=gpurun_out/r4_v11
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -v --timeout 120 --timeout-method thread -k "v11 or gemm or rope" > $O/tests.log 2>&1 || exit 1
timeout -k 10 400 python -u scripts/gemm_v11_ab.py --rounds 3 --orders 0,-8 > $O/ab.log 2>&1 || exit 1
timeout -k 10 300 python -u scripts/gemm_v11_ab.py --rounds 3 --orders 0,-8 --plain > $O/ab_plain.log 2>&1 || exit 1
