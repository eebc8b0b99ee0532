# Whole-model Llama-2-70B numerics: engine (HIP, fp16) vs layer-streamed fp32 oracle (profiles/r2_numerics).
set -o pipefail
O=gpurun_out/r2_numerics
mkdir -p $O
cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u scripts/full70b_numerics.py --prompts 3 --prefix-len 1024 --suffix-len 64 --json $O/full70b.json > $O/full70b.log 2>&1
echo "rc=$?"; tail -5 $O/full70b.log
