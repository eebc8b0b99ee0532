set -o pipefail
O=gpurun_out/${1:-r4_v2}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_vram_gpu.py tests/test_engine_gpu.py tests/test_multigpu_gpu.py -x -v --timeout 150 --timeout-method thread > $O/tests.log 2>&1 || exit 1
FLS_CHUNK_ALIGN=768 timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 > $O/bench_a768.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 > $O/bench_a3072.log 2>&1 || exit 1
timeout -k 10 400 python -u scripts/gemm_variant_ab.py --variants s2,a1,s2a1 --rounds 3 > $O/variant_ab.log 2>&1 || exit 1
