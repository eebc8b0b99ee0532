# MHA attention: v1 vs v2/v3 with one head per block (7B heads)
set -o pipefail
mkdir -p gpurun_out/r63
cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python scripts/attn_mha.py > gpurun_out/r63/attn_mha.log 2>&1
rc=$?; echo "rc=$rc"; grep "^{" gpurun_out/r63/attn_mha.log; tail -3 gpurun_out/r63/attn_mha.log
exit $rc
