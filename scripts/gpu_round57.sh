# same-box A/B: last decoder layer on scored rows only (prune) vs all rows, 70B lnps=1 and 7B lnps=8
set -o pipefail
mkdir -p gpurun_out/r57
cd "$GRAFT_REPO_ROOT"
for v in prune full prune full; do
  f=""; [ $v = full ] && f="--no-prune-last"
  timeout -k 10 300 python bench.py --steps 3 --warmup 1 $f > gpurun_out/r57/bench70b_$v.log 2>&1
  rc=$?; echo "70b $v rc=$rc"; grep -o '"value": [0-9.]*' gpurun_out/r57/bench70b_$v.log
  [ $rc -eq 0 ] || exit $rc
done
for v in prune full prune full; do
  f=""; [ $v = full ] && f="--no-prune-last"
  timeout -k 10 300 python bench.py --model llama2-7b --lnps 8 --storage gpu --steps 5 --warmup 1 $f > gpurun_out/r57/bench7b_$v.log 2>&1
  rc=$?; echo "7b $v rc=$rc"; grep -o '"value": [0-9.]*' gpurun_out/r57/bench7b_$v.log
  [ $rc -eq 0 ] || exit $rc
done
