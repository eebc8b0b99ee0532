set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -x -q -m gpu > gpurun_out/pytest_gpu1.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -30 gpurun_out/pytest_gpu1.log
if [ $rc -le 1 ]; then
  timeout -k 10 400 python bench.py --steps 2 --warmup 1 --num-layers 8 --prompts-per-gpu 16 > gpurun_out/bench_small1.log 2>&1
  rc2=$?; echo "bench rc=$rc2"; tail -20 gpurun_out/bench_small1.log
fi
