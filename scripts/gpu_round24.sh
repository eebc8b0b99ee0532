# row-stride padding vs LDS-DMA throughput
set -o pipefail
mkdir -p gpurun_out/r24
cd "$GRAFT_REPO_ROOT"
FLS_GEMM_VARIANT=10 timeout -k 10 500 python scripts/ld_pad.py > gpurun_out/r24/ld_pad.log 2>&1
rc=$?; echo "rc=$rc"; cat gpurun_out/r24/ld_pad.log | grep -v amdgpu.ids
