# The reference's whole envelope in one run: Llama-2-70B with weights read from 80
# distinct per-layer files on every pass with O_DIRECT (no page cache), device memory under the
# 6 GB cap, host RSS to be <= 8 GB; 128 prompts so the disk read hides under compute.  Then a
# same-box O_DIRECT read probe of the layer files.
set -o pipefail
O=gpurun_out/${1:-r5_envelope}
CK=${CK:-/tmp/fls_ck70_u80}
mkdir -p $O
avail=$(df --output=avail -B1G /tmp | tail -1 | tr -d ' ')
echo "free GB on /tmp: $avail" > $O/disk.txt
if [ "$avail" -lt 150 ]; then echo "not enough disk for a 138 GB checkpoint" >> $O/disk.txt; exit 0; fi
timeout -k 10 1000 python -u bench.py --weights stream --o-direct --unique-layers 80 --max-vram-gb 6 \
  --prompts-per-gpu 128 --steps 2 --warmup 1 --ckpt-dir $CK > $O/envelope_p128.log 2>&1 || exit 1
# same-box O_DIRECT probe: 8 layer files read in parallel by dd (the streamer reads with 8 threads)
t0=$(date +%s.%N)
for f in $(ls $CK/model.layers.*.safetensors | head -8); do
  dd if=$f of=/dev/null bs=64M iflag=direct status=none &
done
wait
t1=$(date +%s.%N)
python3 -c "import sys; t=float(sys.argv[2])-float(sys.argv[1]); print(f'O_DIRECT dd x8 probe: 8 x 1.71 GB in {t:.2f} s = {8*1.711/t:.2f} GB/s')" $t0 $t1 >> $O/disk.txt
