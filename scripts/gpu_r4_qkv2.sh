# two-stream QKV chunks: bitwise test, then same-box bench A/B (1 vs 2 streams) on the capped headline
set -o pipefail
O=gpurun_out/r4_qkv2
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py -x -v -k "two_streams" --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || exit 1
for i in 1 2; do
  FLS_QKV_STREAMS=1 timeout -k 10 300 python -u bench.py --steps 4 --warmup 2 > $O/streams1_$i.log 2>&1 || exit 1
  FLS_QKV_STREAMS=2 timeout -k 10 300 python -u bench.py --steps 4 --warmup 2 > $O/streams2_$i.log 2>&1 || exit 1
done
