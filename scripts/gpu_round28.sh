# hand-written default: full GPU tests, 70B headline bench, 7B lnps=8 gpu-storage config, rocprof (L8)
set -o pipefail
mkdir -p gpurun_out/r28
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -m pytest tests/ -x -q -m gpu > gpurun_out/r28/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/r28/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python bench.py --steps 4 --warmup 1 > gpurun_out/r28/bench70b.log 2>&1
rc=$?; echo "bench rc=$rc"; grep -E "metric" gpurun_out/r28/bench70b.log | cut -c1-260
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --model llama2-7b --lnps 8 --storage gpu --steps 4 --warmup 1 > gpurun_out/r28/bench7b_lnps8_gpu.log 2>&1
rc=$?; echo "bench7b rc=$rc"; grep -E "metric" gpurun_out/r28/bench7b_lnps8_gpu.log | cut -c1-260
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r28/prof_l8 -o run -- python bench.py --steps 2 --warmup 1 --num-layers 8 > gpurun_out/r28/prof_l8.log 2>&1
echo "rocprof rc=$?"
