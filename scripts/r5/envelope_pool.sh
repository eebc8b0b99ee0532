# streamed layers through the piece pool (attention / MLP pieces read from the files into their
# slots): GPU tests of the pool paths, then the envelope at 64 / 96 / 128 prompts
set -o pipefail
O=gpurun_out/${1:-r5_envelope5}
CK=/tmp/fls_ck70
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_engine_gpu.py -x -q --timeout 300 --timeout-method thread -k "piece_pool or stream" > $O/tests.log 2>&1 || exit 1
avail=$(df --output=avail -B1G /tmp | tail -1 | tr -d ' ')
U=$(( (avail - 10) * 100 / 175 ))
[ $U -gt 80 ] && U=80
echo "free GB $avail, distinct layers $U" > $O/disk.txt
E="python -u bench.py --weights stream --o-direct --unique-layers $U --max-vram-gb 6 --ckpt-dir $CK --warmup 1 --steps 2"
timeout -k 10 900 $E --prompts-per-gpu 64 > $O/envelope_p64.log 2>&1 || exit 1
timeout -k 10 600 $E --prompts-per-gpu 96 > $O/envelope_p96.log 2>&1 || exit 1
timeout -k 10 600 $E --prompts-per-gpu 128 > $O/envelope_p128.log 2>&1 || exit 1
