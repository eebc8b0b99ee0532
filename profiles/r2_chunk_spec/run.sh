# Round 2: MLP chunk rows (16384 default / 14336 = 3 equal chunks / 21504 = 2) and the speculative
# next-call weight prefetch (FLS_SPECULATIVE_PREFETCH), 70B bench, one box, interleaved.
set -o pipefail
O=gpurun_out/r2_chunk_spec
mkdir -p $O
cd "$GRAFT_REPO_ROOT"
step() {  # name, seconds, command...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.log 2>&1
  local rc=$?
  echo "$n rc=$rc $(grep -o '"value": [0-9.]*\|"weight_stall_gpu_s": [0-9.]*' $O/$n.log | tail -2 | tr '\n' ' ')"
  return $rc
}
for r in 1 2; do
  step mc16k_$r 300 python -u bench.py --steps 8 --warmup 2 || exit 1
  step mc14k_$r 300 python -u bench.py --steps 8 --warmup 2 --mlp-chunk 14336 || exit 1
  step mc21k_$r 300 python -u bench.py --steps 8 --warmup 2 --mlp-chunk 21504 || exit 1
  FLS_SPECULATIVE_PREFETCH=1 step spec_$r 300 python -u bench.py --steps 8 --warmup 2 || exit 1
done
