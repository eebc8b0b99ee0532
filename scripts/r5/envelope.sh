# The reference's whole envelope in one run: Llama-2-70B with weights read from the
# per-layer files on every pass with O_DIRECT (no page cache), device memory under the 6 GB cap,
# host RSS to be <= 8 GB; 128 prompts so the disk read hides under compute.  Then a same-box
# O_DIRECT read probe of the layer files.
# The boxes have ~79 GB of disk, not the 138 GB of 80 distinct layers: as many distinct layers as
# fit are written and the rest hard-linked to them.  With O_DIRECT that changes nothing about the
# traffic: no page cache holds a file between its reads, so every pass reads all 80 layers'
# 138 GB from the device (the streamer's counters and the read rate say so).
set -o pipefail
O=gpurun_out/${1:-r5_envelope}
CK=${CK:-/tmp/fls_ck70}
mkdir -p $O
avail=$(df --output=avail -B1G /tmp | tail -1 | tr -d ' ')
echo "free GB on /tmp: $avail" > $O/disk.txt
U=$(( (avail - 10) * 100 / 175 ))
[ $U -gt 80 ] && U=80
echo "distinct decoder layers written: $U" >> $O/disk.txt
if [ "$U" -lt 8 ]; then echo "not enough disk" >> $O/disk.txt; exit 0; fi
timeout -k 10 1000 python -u bench.py --weights stream --o-direct --unique-layers $U --max-vram-gb 6 \
  --prompts-per-gpu 128 --steps 2 --warmup 1 --ckpt-dir $CK > $O/envelope_p128.log 2>&1 || exit 1
# same-box O_DIRECT probe: 8 layer files read in parallel by dd (the streamer reads with 8 threads)
t0=$(date +%s.%N)
for f in $(ls $CK/model.layers.*.safetensors | head -8); do
  dd if=$f of=/dev/null bs=64M iflag=direct status=none &
done
wait
t1=$(date +%s.%N)
python3 -c "import sys; t=float(sys.argv[2])-float(sys.argv[1]); print(f'O_DIRECT dd x8 probe: 8 x 1.71 GB in {t:.2f} s = {8*1.711/t:.2f} GB/s')" $t0 $t1 >> $O/disk.txt
