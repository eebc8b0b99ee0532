# Round 2: VRAM with fixed scratch buffers + raw weight slots (70B lnps=1 storage=cpu).
set -o pipefail
O=gpurun_out/r2_vram2
mkdir -p $O
cd "$GRAFT_REPO_ROOT"
step() {  # name, seconds, command...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.log 2>&1
  local rc=$?
  echo "$n rc=$rc $(grep -o '"value": [0-9.]*\|"peak_gpu_mem_gb": [0-9.]*\|"peak_gpu_reserved_gb": [0-9.]*\|"peak_device_used_gb": [0-9.]*\|"host_pinned_gb": [0-9.]*\|"token_budget": [0-9]*\|"mlp_chunk": [0-9]*' $O/$n.log | tr '\n' ' ') $(tail -1 $O/$n.log | cut -c1-120)"
  return $rc
}
step gputest 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread || exit 1
B="python -u bench.py --weights stream --ckpt-dir /tmp/ck70 --steps 3 --warmup 1"
step s_default 600 $B --steps 1 --warmup 0 || exit 1
step s_cap6 300 $B --max-vram-gb 6 || exit 1
step s_cap55 300 $B --max-vram-gb 5.5 || exit 1
step s_cap7 300 $B --max-vram-gb 7 || exit 1
step host_default 400 python -u bench.py --steps 5 --warmup 2 || exit 1
