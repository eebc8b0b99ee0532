# packed-GQA decode attention: kernel tests first (a fault stops here), then the generation runs
# (scripts/r5/gen.sh) and the --token-budget 16384 matrix
set -o pipefail
mkdir -p gpurun_out/r5_gen
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -v --timeout 120 --timeout-method thread -k "attention" > gpurun_out/r5_gen/attn_tests.log 2>&1 || exit 1
bash scripts/r5/gen.sh r5_gen || exit 1
bash scripts/r5/tb16k_matrix.sh r5_tb16k
