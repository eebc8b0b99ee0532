# full GPU tests + smoke + 70B headline (attention v3) + 7B lnps8 gpu + rocprof stats (8 layers)
set -o pipefail
mkdir -p gpurun_out/r38
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests/ -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/r38/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/r38/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r38/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 gpurun_out/r38/smoke.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python bench.py --steps 4 --warmup 1 > gpurun_out/r38/bench70b.log 2>&1
rc=$?; echo "bench rc=$rc"; grep -o '"value": [0-9.]*\|"peak_gpu_mem_gb": [0-9.]*' gpurun_out/r38/bench70b.log | tr '\n' ' '; echo
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --model llama2-7b --lnps 8 --storage gpu --steps 4 --warmup 1 > gpurun_out/r38/bench7b_lnps8_gpu.log 2>&1
rc=$?; echo "bench7b rc=$rc"; grep -o '"value": [0-9.]*\|"peak_gpu_mem_gb": [0-9.]*' gpurun_out/r38/bench7b_lnps8_gpu.log | tr '\n' ' '; echo
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r38/prof_l8 -o run -- python bench.py --steps 2 --warmup 1 --num-layers 8 > gpurun_out/r38/prof_l8.log 2>&1
echo "rocprof rc=$?"
