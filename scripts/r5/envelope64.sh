# the envelope at 64 prompts (86k tokens: compute ~ disk time per pass) and at 128, with the
# bench's run-time RSS sampler (host_rss_run_peak_gb); checkpoint written first, timed separately
set -o pipefail
O=gpurun_out/${1:-r5_envelope3}
CK=/tmp/fls_ck70
mkdir -p $O
avail=$(df --output=avail -B1G /tmp | tail -1 | tr -d ' ')
U=$(( (avail - 10) * 100 / 175 ))
[ $U -gt 80 ] && U=80
echo "free GB $avail, distinct layers $U" > $O/disk.txt
E="python -u bench.py --weights stream --o-direct --unique-layers $U --max-vram-gb 6 --ckpt-dir $CK --warmup 1 --steps 2"
timeout -k 10 900 $E --prompts-per-gpu 64 > $O/envelope_p64.log 2>&1 || exit 1
timeout -k 10 600 $E --prompts-per-gpu 128 > $O/envelope_p128.log 2>&1 || exit 1
