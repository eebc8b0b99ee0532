# the envelope at 96 prompts (default run-ahead and FLS_RUNAHEAD_ITEMS=6) and at 64 with the knob
set -o pipefail
O=gpurun_out/${1:-r5_envelope4}
CK=/tmp/fls_ck70
mkdir -p $O
avail=$(df --output=avail -B1G /tmp | tail -1 | tr -d ' ')
U=$(( (avail - 10) * 100 / 175 ))
[ $U -gt 80 ] && U=80
echo "free GB $avail, distinct layers $U" > $O/disk.txt
E="python -u bench.py --weights stream --o-direct --unique-layers $U --max-vram-gb 6 --ckpt-dir $CK --warmup 1 --steps 2"
timeout -k 10 900 $E --prompts-per-gpu 96 > $O/envelope_p96.log 2>&1 || exit 1
FLS_RUNAHEAD_ITEMS=6 timeout -k 10 600 $E --prompts-per-gpu 96 > $O/envelope_p96_ra6.log 2>&1 || exit 1
FLS_RUNAHEAD_ITEMS=6 timeout -k 10 600 $E --prompts-per-gpu 64 > $O/envelope_p64_ra6.log 2>&1 || exit 1
