# speculative generation steps: GPU tests first, then the generation runs, then the MLP-chunk probe
set -o pipefail
mkdir -p gpurun_out/r5_gen2
timeout -k 10 600 python -u -m pytest tests/test_engine_gpu.py tests/test_kernels_gpu.py -x -v --timeout 200 --timeout-method thread -k "speculative or decode_graphs or attention" > gpurun_out/r5_gen2/tests.log 2>&1 || exit 1
bash scripts/r5/gen.sh r5_gen2 || exit 1
bash scripts/r5/tb16k_chunk.sh r5_tb16k_chunk
