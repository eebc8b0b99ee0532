set -o pipefail
mkdir -p gpurun_out/r44
cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py -x -v -k "race" --timeout 200 --timeout-method thread > gpurun_out/r44/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r44/pytest.log
timeout -k 10 200 python scripts/nan_engine.py --layers 20 --prompts 32 --storage cpu 2>&1 | grep layers=
timeout -k 10 200 python scripts/nan_engine.py --layers 20 --prompts 32 --storage disk 2>&1 | grep layers=
exit $rc
