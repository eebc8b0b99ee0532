# after the activation-store race fix: full GPU tests, smoke, 70B headline, generation study
set -o pipefail
mkdir -p gpurun_out/r45
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests/ -x -v -m gpu --timeout 200 --timeout-method thread > gpurun_out/r45/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/r45/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r45/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 gpurun_out/r45/smoke.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python bench.py --steps 4 --warmup 1 > gpurun_out/r45/bench70b.log 2>&1
rc=$?; echo "bench rc=$rc"; grep -o '"value": [0-9.]*\|"peak_gpu_mem_gb": [0-9.]*\|"scores_finite": [a-z]*' gpurun_out/r45/bench70b.log | tr '\n' ' '; echo
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python scripts/gen_bench.py --json gpurun_out/r45/gen70b.json > gpurun_out/r45/gen70b.log 2>&1
rc=$?; echo "gen rc=$rc"; grep -v amdgpu gpurun_out/r45/gen70b.log | cut -c1-300
exit $rc
