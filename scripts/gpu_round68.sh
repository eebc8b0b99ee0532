# v13 for RoPE GEMMs by default: full GPU suite, smoke, kernel bench, 70B/7B benches, 70B kernel stats
set -o pipefail
mkdir -p gpurun_out/r68
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r68/pytest.log 2>&1
rc=$?; echo "pytest gpu rc=$rc"; tail -2 gpurun_out/r68/pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r68/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 gpurun_out/r68/smoke.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/kernel_bench.py > gpurun_out/r68/kbench.log 2>&1
rc=$?; echo "kbench rc=$rc"; grep '"op"' gpurun_out/r68/kbench.log | head -4 | cut -c1-300
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 3 --warmup 1 > gpurun_out/r68/bench70b.log 2>&1
rc=$?; echo "bench70b rc=$rc"; grep -o '"value": [0-9.]*\|"scores_finite": [a-z]*' gpurun_out/r68/bench70b.log | tr '\n' ' '; echo
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --model llama2-7b --lnps 8 --storage gpu --steps 5 --warmup 1 > gpurun_out/r68/bench7b.log 2>&1
rc=$?; echo "bench7b rc=$rc"; grep -o '"value": [0-9.]*\|"scores_finite": [a-z]*' gpurun_out/r68/bench7b.log | tr '\n' ' '; echo
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r68/prof -o run -- python bench.py --num-layers 8 --resident --storage gpu --steps 3 --warmup 1 > gpurun_out/r68/bench_l8_prof.log 2>&1
rc=$?; echo "prof rc=$rc"
exit $rc
