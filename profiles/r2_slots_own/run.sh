# Round 2: 70B lnps=1, double buffer vs 3 decoder slots with the embedding / LM head in buffers of
# their own (lookahead reaches the next call's layer 0 during the second-to-last layer). One box.
set -o pipefail
O=gpurun_out/r2_slots_own
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
  step s2_$r 300 python -u bench.py --steps 8 --warmup 2 --slots 2 || exit 1
  step s3_$r 300 python -u bench.py --steps 8 --warmup 2 --slots 3 || exit 1
done
