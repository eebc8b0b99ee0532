# v10 ablation: which in-loop component costs the MFMA pipe
set -o pipefail
mkdir -p gpurun_out/r23
cd "$GRAFT_REPO_ROOT"
ABL_ONLY=40 timeout -k 10 400 python scripts/gemm_ablate.py > gpurun_out/r23/ablate_v10.json 2>&1
rc=$?; echo "rc=$rc"; cat gpurun_out/r23/ablate_v10.json
