# prefix K/V cache: kernel + engine tests, 70B generation study (rerun vs cache)
set -o pipefail
mkdir -p gpurun_out/r39
cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -x -v -k "attention or engine or prefix or graph or resident or qwen" --timeout 120 --timeout-method thread > gpurun_out/r39/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r39/pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python scripts/gen_bench.py --json gpurun_out/r39/gen70b.json > gpurun_out/r39/gen70b.log 2>&1
rc=$?; echo "gen rc=$rc"; grep -v amdgpu gpurun_out/r39/gen70b.log | cut -c1-400
exit $rc
