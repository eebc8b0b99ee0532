# Round 2: full-size model families on this tree (lnps=1, storage=cpu, bench shapes), 1x MI355X.
set -o pipefail
O=gpurun_out/r2_families
mkdir -p $O
cd "$GRAFT_REPO_ROOT"
for m in llama2-7b llama2-13b mistral-7b llama3.1-8b qwen2-7b; do
  timeout -k 10 300 python -u bench.py --model $m --lnps 1 --storage cpu --steps 6 --warmup 2 > $O/$m.log 2>&1
  rc=$?; echo "$m rc=$rc $(grep -o '"value": [0-9.]*\|"peak_device_used_gb": [0-9.]*\|"scores_finite": [a-z]*' $O/$m.log | tr '\n' ' ')"
  [ $rc -eq 0 ] || exit 1
done
