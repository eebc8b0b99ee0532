# the data-parallel rank's traffic on one GPU: 1/8 of every piece over PCIe (the rank's slice) and
# 7/8 of it HBM -> HBM (the all-gather's traffic), on the CUs or on the SDMA engines
set -o pipefail
O=gpurun_out/${1:-r6_dpi_slice}
mkdir -p $O
for i in 1 2; do
  for m in none cu32 sdma blit; do
    timeout -k 10 300 python -u bench.py --steps 4 --warmup 2 --max-vram-gb 6.3 --emulate-dp-slice --emulate-dp-fanout $m > $O/bench_${m}_$i.log 2>&1 || exit 1
  done
done
