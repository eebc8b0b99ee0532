# Round 2: weight slots 2 vs 3 (3: next call's first shard prefetched across the call boundary) on
# Llama-2-7B lnps=8 storage=gpu (BASELINE config 2: 5 shards of up to 8 layers, 3.2 GB each).
set -o pipefail
O=gpurun_out/r2_slots7b
mkdir -p $O
cd "$GRAFT_REPO_ROOT"
step() {  # name, seconds, command...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.log 2>&1
  local rc=$?
  echo "$n rc=$rc $(grep -o '"value": [0-9.]*\|"weight_stall_gpu_s": [0-9.]*\|"peak_device_used_gb": [0-9.]*' $O/$n.log | tail -3 | tr '\n' ' ')"
  return $rc
}
for r in 1 2; do
  step s2_$r 300 python -u bench.py --model llama2-7b --lnps 8 --storage gpu --steps 10 --warmup 2 --slots 2 || exit 1
  step s3_$r 300 python -u bench.py --model llama2-7b --lnps 8 --storage gpu --steps 10 --warmup 2 --slots 3 || exit 1
done
step l1_s2 300 python -u bench.py --model llama2-7b --lnps 1 --storage cpu --steps 10 --warmup 2 --slots 2 || exit 1
step l1_s3 300 python -u bench.py --model llama2-7b --lnps 1 --storage cpu --steps 10 --warmup 2 --slots 3 || exit 1
step l4_s2 300 python -u bench.py --lnps 4 --steps 4 --warmup 1 --slots 2 || exit 1
step l4_s3 300 python -u bench.py --lnps 4 --steps 4 --warmup 1 --slots 3 || exit 1
