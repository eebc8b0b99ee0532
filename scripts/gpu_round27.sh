# v10 intra-phase schedule A/B (gate/up shape, interleaved rounds)
set -o pipefail
mkdir -p gpurun_out/r27
cd "$GRAFT_REPO_ROOT"
ABL_ONLY=60 timeout -k 10 400 python scripts/gemm_ablate.py > gpurun_out/r27/sched.json 2>&1
rc=$?; echo "rc=$rc"; grep -v amdgpu.ids gpurun_out/r27/sched.json | python -c "
import json,sys; d=json.load(sys.stdin); print({k:v['tflops_equiv'] for k,v in d.items()})"
