# Round 2 tree: BASELINE configs on 1x MI355X + a rocprofv3 kernel breakdown (profiles/r2_configs).
set -o pipefail
O=gpurun_out/r2_configs
mkdir -p $O
cd "$GRAFT_REPO_ROOT"
step() {  # name, seconds, command...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.log 2>&1
  local rc=$?
  echo "$n rc=$rc $(grep -o '"value": [0-9.]*\|"peak_gpu_mem_gb": [0-9.]*\|"peak_device_used_gb": [0-9.]*\|"host_pinned_gb": [0-9.]*' $O/$n.log | tr '\n' ' ')"
  return $rc
}
step c3_70b_lnps1_cpu 500 python -u bench.py --steps 10 --warmup 2 || exit 1
step c2_7b_lnps8_gpu 300 python -u bench.py --model llama2-7b --lnps 8 --storage gpu --steps 10 --warmup 2 || exit 1
step c5_70b_resident 500 python -u bench.py --resident --storage gpu --steps 5 --warmup 1 || exit 1
step stream_cap6 700 python -u bench.py --weights stream --ckpt-dir /tmp/ck70 --max-vram-gb 6 --steps 4 --warmup 1 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/$O/prof" -o bench8 -- python3 "$GRAFT_REPO_ROOT/bench.py" --num-layers 8 --resident --storage gpu --steps 3 --warmup 1 > "$GRAFT_REPO_ROOT/$O/prof_bench.log" 2>&1
echo "rocprof rc=$?"
find "$GRAFT_REPO_ROOT/$O/prof" -name "*kernel_stats.csv" | head -3
