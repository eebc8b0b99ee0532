# same-box A/B of the activation-store path after the race fix: storage cpu vs gpu (70B headline bench)
set -o pipefail
mkdir -p gpurun_out/r46
cd "$GRAFT_REPO_ROOT"
for st in cpu gpu cpu; do
  timeout -k 10 300 python bench.py --steps 3 --warmup 1 --storage $st > gpurun_out/r46/bench_$st.log 2>&1
  rc=$?; echo "storage=$st rc=$rc"; grep -o '"value": [0-9.]*\|"scores_finite": [a-z]*' gpurun_out/r46/bench_$st.log | tr '\n' ' '; grep "step 2" gpurun_out/r46/bench_$st.log | cut -c1-200
  [ $rc -eq 0 ] || exit $rc
done
