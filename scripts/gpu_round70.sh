# 70B lnps=1 storage=cpu: token-budget (micro-batch size) sweep
set -o pipefail
mkdir -p gpurun_out/r70
cd "$GRAFT_REPO_ROOT"
for tb in 16384 8192 24576 45056 16384; do
  timeout -k 10 240 python bench.py --steps 3 --warmup 1 --token-budget $tb > gpurun_out/r70/bench70b_tb$tb.log 2>&1
  rc=$?; echo "tb=$tb rc=$rc $(grep -o '"value": [0-9.]*\|"peak_gpu_mem_gb": [0-9.]*\|"peak_gpu_reserved_gb": [0-9.]*\|"scores_finite": [a-z]*' gpurun_out/r70/bench70b_tb$tb.log | tr '\n' ' ')"
  [ $rc -eq 0 ] || exit $rc
done
