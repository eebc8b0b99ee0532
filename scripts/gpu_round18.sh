# v9 default: full GPU tests, 70B bench (auto + hip-only), rocprof kernel breakdown (L8)
set -o pipefail
mkdir -p gpurun_out/r18
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -m pytest tests/ -x -q -m gpu > gpurun_out/r18/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r18/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --steps 3 --warmup 1 > gpurun_out/r18/bench70b_auto.log 2>&1
rc=$?; echo "bench auto rc=$rc"; grep -E "metric" gpurun_out/r18/bench70b_auto.log | cut -c1-300
[ $rc -eq 0 ] || exit $rc
FLS_GEMM_BACKEND=hip timeout -k 10 400 python bench.py --steps 3 --warmup 1 > gpurun_out/r18/bench70b_hip.log 2>&1
rc=$?; echo "bench hip rc=$rc"; grep -E "metric" gpurun_out/r18/bench70b_hip.log | cut -c1-300
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r18/prof_l8 -o run -- python bench.py --steps 2 --warmup 1 --num-layers 8 --prompts-per-gpu 16 > gpurun_out/r18/prof_l8.log 2>&1
echo "rocprof rc=$?"
