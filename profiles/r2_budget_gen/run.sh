# Round 2: token-budget / MLP-chunk A/B on one box (70B lnps=1 storage=cpu), then greedy generation
# (--num_gen_token 4) with and without the prefix K/V cache, weights streamed and resident.
set -o pipefail
O=gpurun_out/r2_budget_gen
mkdir -p $O
cd "$GRAFT_REPO_ROOT"
step() {  # name, seconds, command...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.log 2>&1
  local rc=$?
  echo "$n rc=$rc $(grep -o '"value": [0-9.]*\|"peak_device_used_gb": [0-9.]*\|"speedup": [0-9.]*\|"total_s": [0-9.]*' $O/$n.log | tr '\n' ' ')"
  return $rc
}
step tb16k_a 400 python -u bench.py --steps 8 --warmup 2 || exit 1
step tb45k_mc16k 400 python -u bench.py --steps 8 --warmup 2 --token-budget 45056 || exit 1
step tb45k_mc45k 400 python -u bench.py --steps 8 --warmup 2 --token-budget 45056 --mlp-chunk 45056 || exit 1
step tb16k_b 400 python -u bench.py --steps 8 --warmup 2 || exit 1
step gen_stream 600 python -u scripts/gen_bench.py --gen 4 --json $O/gen_stream.json || exit 1
step gen_resident 600 python -u scripts/gen_bench.py --gen 4 --resident --json $O/gen_resident.json || exit 1
