# last decoder layer on scored rows only: GPU tests + 70B / 7B benches
set -o pipefail
mkdir -p gpurun_out/r56
cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r56/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/r56/pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 4 --warmup 1 > gpurun_out/r56/bench70b.log 2>&1
rc=$?; echo "bench70b rc=$rc"; grep -o '"value": [0-9.]*\|"peak_gpu_[a-z_]*": [0-9.]*\|"scores_finite": [a-z]*' gpurun_out/r56/bench70b.log | tr '\n' ' '; grep "step 3" gpurun_out/r56/bench70b.log | cut -c1-300
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --model llama2-7b --lnps 8 --storage gpu --steps 5 --warmup 1 > gpurun_out/r56/bench7b.log 2>&1
rc=$?; echo "bench7b rc=$rc"; grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*' gpurun_out/r56/bench7b.log | tr '\n' ' '
exit $rc
