# the reference's envelope on the final tree (defaults: 6 x 64 MB streamer ring, pinned state
# buffers bounded): O_DIRECT streamed 70B under a 6 GB cap at 64 / 96 / 128 prompts, 128 twice,
# then the host-RAM headline and 128-prompt runs on the same box
set -o pipefail
O=gpurun_out/${1:-r5_envfinal}
CK=/tmp/fls_ck70
mkdir -p $O
avail=$(df --output=avail -B1G /tmp | tail -1 | tr -d ' ')
U=$(( (avail - 10) * 100 / 175 ))
[ $U -gt 80 ] && U=80
echo "free GB $avail, distinct layers $U" > $O/disk.txt
E="python -u bench.py --weights stream --o-direct --unique-layers $U --max-vram-gb 6 --ckpt-dir $CK --warmup 1 --steps 2"
timeout -k 10 900 $E --prompts-per-gpu 128 > $O/envelope_p128.log 2>&1 || exit 1
timeout -k 10 400 $E --prompts-per-gpu 96 > $O/envelope_p96.log 2>&1 || exit 1
timeout -k 10 400 $E --prompts-per-gpu 64 > $O/envelope_p64.log 2>&1 || exit 1
timeout -k 10 400 $E --prompts-per-gpu 128 > $O/envelope_p128_2.log 2>&1 || exit 1
rm -rf $CK
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 > $O/head.log 2>&1 || exit 1
timeout -k 10 400 python -u bench.py --steps 2 --warmup 1 --prompts-per-gpu 128 > $O/p128.log 2>&1 || exit 1
