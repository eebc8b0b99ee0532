# round-end rehearsal: full GPU test suite, smoke, headline bench (storage cpu with the carry window, and gpu)
set -o pipefail
mkdir -p gpurun_out/r49
cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/r49/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r49/pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r49/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; grep smoke gpurun_out/r49/smoke.log
[ $rc -eq 0 ] || exit $rc
for st in cpu gpu; do
  timeout -k 10 300 python bench.py --steps 3 --warmup 1 --storage $st > gpurun_out/r49/bench_$st.log 2>&1
  rc=$?; echo "storage=$st rc=$rc"; grep -o '"value": [0-9.]*\|"peak_gpu_[a-z_]*": [0-9.]*\|"scores_finite": [a-z]*' gpurun_out/r49/bench_$st.log | tr '\n' ' '; grep "step 2" gpurun_out/r49/bench_$st.log | cut -c1-600
  [ $rc -eq 0 ] || exit $rc
done
