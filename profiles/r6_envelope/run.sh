# the reference's envelope on the final tree: 70B weights read from disk with O_DIRECT every pass,
# 6 GB device cap, 128 prompts, 5 timed steps (host RSS sampled through the run)
set -o pipefail
O=gpurun_out/${1:-r6_envelope}
CK=/tmp/fls_ck70
mkdir -p $O
avail=$(df --output=avail -B1G /tmp | tail -1 | tr -d ' ')
U=$(( (avail - 10) * 100 / 175 ))
[ $U -gt 80 ] && U=80
echo "free GB $avail, distinct layers $U" > $O/disk.txt
free -g >> $O/disk.txt
timeout -k 10 1000 python -u bench.py --weights stream --o-direct --unique-layers $U --max-vram-gb 6 --ckpt-dir $CK --warmup 1 --steps 5 --prompts-per-gpu 128 > $O/envelope_p128.log 2>&1 || exit 1
rm -rf $CK
