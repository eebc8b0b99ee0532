# re-entry validation: full GPU tests, smoke, 70B headline bench
set -o pipefail
mkdir -p gpurun_out/r33
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests/ -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/r33/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/r33/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r33/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 gpurun_out/r33/smoke.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python bench.py --steps 3 --warmup 1 > gpurun_out/r33/bench70b.log 2>&1
rc=$?; echo "bench rc=$rc"; grep -E "metric" gpurun_out/r33/bench70b.log | cut -c1-300
exit $rc
