# MLP-phase RMSNorm overlap: bitwise tests, then same-box bench A/B (off vs on)
set -o pipefail
O=gpurun_out/r4_mlpov
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py -x -v -k "two_streams or norm_overlap or oracle" --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || exit 1
for i in 1 2; do
  FLS_MLP_NORM_OVERLAP=0 timeout -k 10 300 python -u bench.py --steps 4 --warmup 2 > $O/off_$i.log 2>&1 || exit 1
  FLS_MLP_NORM_OVERLAP=1 timeout -k 10 300 python -u bench.py --steps 4 --warmup 2 > $O/on_$i.log 2>&1 || exit 1
done
