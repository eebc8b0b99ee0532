# Round 2: 48k default token budget confirmed (70B default, 7B lnps=8 A/B, 6 GB cap still planned),
# then greedy generation (--num_gen_token 4) with and without the prefix K/V cache, streamed and resident.
set -o pipefail
O=gpurun_out/r2_budget_gen
mkdir -p $O
cd "$GRAFT_REPO_ROOT"
step() {  # name, seconds, command...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.log 2>&1
  local rc=$?
  echo "$n rc=$rc $(grep -o '"value": [0-9.]*\|"peak_device_used_gb": [0-9.]*\|"token_budget": [0-9]*\|"speedup": [0-9.]*\|"total_s": [0-9.]*' $O/$n.log | tr '\n' ' ')"
  return $rc
}
step default48k 400 python -u bench.py --steps 8 --warmup 2 || exit 1
step b7_tb16k 300 python -u bench.py --model llama2-7b --lnps 8 --storage gpu --steps 10 --warmup 2 --token-budget 16384 || exit 1
step b7_tb48k 300 python -u bench.py --model llama2-7b --lnps 8 --storage gpu --steps 10 --warmup 2 || exit 1
step stream_cap6 700 python -u bench.py --weights stream --ckpt-dir /tmp/ck70 --max-vram-gb 6 --steps 4 --warmup 1 || exit 1
step gen_stream 600 python -u scripts/gen_bench.py --gen 4 --json $O/gen_stream.json || exit 1
step gen_resident 600 python -u scripts/gen_bench.py --gen 4 --resident --json $O/gen_resident.json || exit 1
