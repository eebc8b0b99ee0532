# same-box A/B of the headline bench: v11 with 768- vs 3072-row chunk alignment
set -o pipefail
O=gpurun_out/${1:-r4_bench_ab2}
mkdir -p $O
for r in 1 2; do
  FLS_CHUNK_ALIGN=768 timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 > $O/a768_$r.log 2>&1 || exit 1
  timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 > $O/a3072_$r.log 2>&1 || exit 1
done
