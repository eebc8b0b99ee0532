# A/B (stream syncs instead of a device sync): speculative next-call prefetch on/off, 7B lnps=8 storage=gpu and 70B lnps=1 (same box)
set -o pipefail
mkdir -p gpurun_out/r54
cd "$GRAFT_REPO_ROOT"
for sp in 1 0 1 0; do
  FLS_SPECULATIVE_PREFETCH=$sp timeout -k 10 300 python bench.py --model llama2-7b --lnps 8 --storage gpu --steps 5 --warmup 1 > gpurun_out/r54/bench7b_$sp.log 2>&1
  rc=$?; echo "7b spec=$sp rc=$rc"; grep -o '"value": [0-9.]*' gpurun_out/r54/bench7b_$sp.log
  [ $rc -eq 0 ] || exit $rc
done
for sp in 0 1; do
  FLS_SPECULATIVE_PREFETCH=$sp timeout -k 10 300 python bench.py --steps 3 --warmup 1 > gpurun_out/r54/bench70b_$sp.log 2>&1
  rc=$?; echo "70b spec=$sp rc=$rc"; grep -o '"value": [0-9.]*' gpurun_out/r54/bench70b_$sp.log
  [ $rc -eq 0 ] || exit $rc
done
