# Round 2: natural-layout GEMM epilogues + streaming weight path.
# GPU tests, then the driver bench (host weights), the stream bench (page cache, O_DIRECT) and a 6 GB VRAM cap.
set -o pipefail
O=gpurun_out/r2_stream
mkdir -p $O
cd "$GRAFT_REPO_ROOT"
step() {  # name, seconds, command...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.log 2>&1
  local rc=$?
  echo "$n rc=$rc $(grep -o '"value": [0-9.]*\|"peak_device_used_gb": [0-9.]*\|"host_pinned_gb": [0-9.]*\|"scores_finite": [a-z]*' $O/$n.log | tr '\n' ' ') $(tail -1 $O/$n.log | cut -c1-200)"
  return $rc
}
step gputest 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread || exit 1
step bench_host 400 python -u bench.py --steps 5 --warmup 2 || exit 1
step bench_stream 600 python -u bench.py --weights stream --steps 3 --warmup 1 --ckpt-dir /tmp/ck70 || exit 1
step bench_stream_direct 400 python -u bench.py --weights stream --o-direct --steps 2 --warmup 1 --ckpt-dir /tmp/ck70 || exit 1
step bench_vram6 400 python -u bench.py --steps 3 --warmup 1 --max-vram-gb 6 || exit 1
df -h /tmp > $O/df.txt
