# the streamed envelope (O_DIRECT, 6 GB cap, 128 prompts) with the pinned state buffers bounded to
# one per micro-batch + 1, against the streamer's chunk-ring depth; host RSS must stay <= 8 GB
set -o pipefail
O=gpurun_out/${1:-r5_envcap}
CK=/tmp/fls_ck70
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_engine_gpu.py -x -q --timeout 300 --timeout-method thread -k "piece_pool or stream" > $O/tests.log 2>&1 || exit 1
avail=$(df --output=avail -B1G /tmp | tail -1 | tr -d ' ')
U=$(( (avail - 10) * 100 / 175 ))
[ $U -gt 80 ] && U=80
echo "free GB $avail, distinct layers $U" > $O/disk.txt
E="python -u bench.py --weights stream --o-direct --unique-layers $U --max-vram-gb 6 --ckpt-dir $CK --warmup 1 --steps 2 --prompts-per-gpu 128"
FLS_STREAM_CHUNKS=6 timeout -k 10 900 $E > $O/ring6x64.log 2>&1 || exit 1
timeout -k 10 400 $E > $O/ring4x64.log 2>&1 || exit 1
FLS_STREAM_CHUNKS=5 timeout -k 10 400 $E > $O/ring5x64.log 2>&1 || exit 1
FLS_STREAM_CHUNKS=8 timeout -k 10 400 $E > $O/ring8x64.log 2>&1 || exit 1
