# the streamed envelope (O_DIRECT, 6 GB cap, 128 prompts) against the depth of the streamer's
# pinned chunk ring: does reading ahead of a busy piece slot close the gap to the host-RAM rate?
# (host RSS is the other limit: <= 8 GB)
set -o pipefail
O=gpurun_out/${1:-r5_envring}
CK=/tmp/fls_ck70
mkdir -p $O
avail=$(df --output=avail -B1G /tmp | tail -1 | tr -d ' ')
U=$(( (avail - 10) * 100 / 175 ))
[ $U -gt 80 ] && U=80
echo "free GB $avail, distinct layers $U" > $O/disk.txt
E="python -u bench.py --weights stream --o-direct --unique-layers $U --max-vram-gb 6 --ckpt-dir $CK --warmup 1 --steps 2 --prompts-per-gpu 128"
timeout -k 10 900 $E > $O/ring4x64.log 2>&1 || exit 1
FLS_STREAM_CHUNKS=8 timeout -k 10 400 $E > $O/ring8x64.log 2>&1 || exit 1
FLS_STREAM_CHUNKS=8 FLS_STREAM_CHUNK_MB=32 timeout -k 10 400 $E > $O/ring8x32.log 2>&1 || exit 1
FLS_STREAM_CHUNKS=6 timeout -k 10 400 $E > $O/ring6x64.log 2>&1 || exit 1
