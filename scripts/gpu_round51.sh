# Llama-3.1 / YaRN RoPE tables and explicit head_dim through the HIP kernels
set -o pipefail
mkdir -p gpurun_out/r51
cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py -x -v -k "variants or qwen2" --timeout 120 --timeout-method thread > gpurun_out/r51/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -8 gpurun_out/r51/pytest.log
exit $rc
