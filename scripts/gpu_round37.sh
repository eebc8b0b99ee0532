# HIP-graph replay: engine test + launch-bound 7B resident scoring with/without graphs
set -o pipefail
mkdir -p gpurun_out/r37
cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r37/pytest_engine.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r37/pytest_engine.log
[ $rc -eq 0 ] || exit $rc
for g in "" "--hip-graphs"; do
timeout -k 10 300 python bench.py --model llama2-7b --resident --storage gpu --prompts-per-gpu 4 --prefix-len 64 --suffix-len 8 --steps 10 --warmup 2 $g > gpurun_out/r37/bench7b_small$g.log 2>&1
rc=$?; echo "bench7b small $g rc=$rc"; grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*' gpurun_out/r37/bench7b_small$g.log | tr '\n' ' '; echo
[ $rc -eq 0 ] || exit $rc
done
