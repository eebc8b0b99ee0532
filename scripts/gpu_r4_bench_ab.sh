# same-box A/B of the headline bench: round-3 GEMM path (v10, 256-row chunks) vs v11 (768-row chunks)
set -o pipefail
O=gpurun_out/${1:-r4_bench_ab}
mkdir -p $O
for r in 1 2; do
  FLS_GEMM_V11=0 FLS_CHUNK_ALIGN=256 timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 > $O/v10_$r.log 2>&1 || exit 1
  timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 > $O/v11_$r.log 2>&1 || exit 1
done
