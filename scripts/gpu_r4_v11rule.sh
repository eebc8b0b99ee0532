# same-box A/B of the v11 selection rule on the capped headline (4,096-row QKV chunks)
set -o pipefail
O=gpurun_out/r4_v11rule
mkdir -p $O
for i in 1 2; do
  FLS_GEMM_V11=1 timeout -k 10 300 python -u bench.py --steps 4 --warmup 2 > $O/rule1_$i.log 2>&1 || exit 1
  FLS_GEMM_V11=3 timeout -k 10 300 python -u bench.py --steps 4 --warmup 2 > $O/rule3_$i.log 2>&1 || exit 1
done
