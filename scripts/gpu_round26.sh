# K sweep: fixed per-tile cost vs per-K cost (v10 vs hipBLASLt)
set -o pipefail
mkdir -p gpurun_out/r26
cd "$GRAFT_REPO_ROOT"
FLS_GEMM_VARIANT=10 timeout -k 10 400 python scripts/k_sweep.py > gpurun_out/r26/k_sweep.log 2>&1
rc=$?; echo "rc=$rc"; grep -v amdgpu.ids gpurun_out/r26/k_sweep.log
