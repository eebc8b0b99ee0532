# Round 2: 3 HBM weight slots + prefetch across call boundaries vs 2 slots (70B bench, one box,
# interleaved), after the GPU engine tests on this tree.
set -o pipefail
O=gpurun_out/r2_slots
mkdir -p $O
cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gputest.log 2>&1
rc=$?; echo "gputest rc=$rc $(tail -1 $O/gputest.log)"; [ $rc -eq 0 ] || exit 1
step() {  # name, seconds, command...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.log 2>&1
  local rc=$?
  echo "$n rc=$rc $(grep -o '"value": [0-9.]*\|"weight_stall_gpu_s": [0-9.]*\|"peak_device_used_gb": [0-9.]*' $O/$n.log | tail -3 | tr '\n' ' ')"
  return $rc
}
for r in 1 2; do
  step slots2_$r 300 python -u bench.py --steps 8 --warmup 2 --slots 2 || exit 1
  step slots3_$r 300 python -u bench.py --steps 8 --warmup 2 || exit 1
done
step slots3_nospec 300 env FLS_SPECULATIVE_PREFETCH=0 python -u bench.py --steps 8 --warmup 2 || exit 1
step stream3 600 python -u bench.py --weights stream --ckpt-dir /tmp/ck70 --steps 6 --warmup 2 || exit 1
