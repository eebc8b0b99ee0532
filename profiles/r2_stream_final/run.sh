# Round 2 final tree: the reference's small-RAM mode (weights re-read from the layer files every pass),
# without a cap (three slots) and under --max-vram-gb 6 (double buffer).
set -o pipefail
O=gpurun_out/r2_stream_final
mkdir -p $O
cd "$GRAFT_REPO_ROOT"
for n in nocap cap6; do
  extra=""; [ $n = cap6 ] && extra="--max-vram-gb 6"
  timeout -k 10 700 python -u bench.py --weights stream --ckpt-dir /tmp/ck70 --steps 5 --warmup 2 $extra > $O/$n.log 2>&1
  rc=$?; echo "$n rc=$rc $(grep -o '"value": [0-9.]*\|"peak_device_used_gb": [0-9.]*\|"host_pinned_gb": [0-9.]*\|"weight_slots": [0-9]*' $O/$n.log | tr '\n' ' ')"
  [ $rc -eq 0 ] || exit 1
done
