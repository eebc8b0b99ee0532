# Skinny-M GEMM with 256 weight rows per block (gemm_skinny.h BN = 256): kernel tests, then the
# 70B small-M A/B (BN 128 / 256, K-split block targets for BN 256, hipBLASLt).
set -o pipefail
O=gpurun_out/${1:-r4_sk256}
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "skinny" --timeout 150 --timeout-method thread > $O/tests.log 2>&1 || exit 1
timeout -k 10 500 python -u scripts/gemm_skinny_ab.py --ms 64,128,160 --blocks256 256,384,512 > $O/skinny_ab.log 2>&1 || exit 1
