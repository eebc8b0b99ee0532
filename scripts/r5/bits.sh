# which plan knob changes the scores' bits (grouped attention, MLP chunks, v11 modes), the
# engine / multi-GPU GPU tests on the resident-state tree, then p128 (not resident) and tb16k
# with the v11 round-count rule against the padding rule, interleaved
set -o pipefail
O=gpurun_out/${1:-r5_bits}
mkdir -p $O
timeout -k 10 200 python -u scripts/bits_probe.py > $O/bits.log 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest tests/test_engine_gpu.py tests/test_multigpu_gpu.py -q --timeout 280 --timeout-method thread > $O/tests.log 2>&1
rc=$?; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 1
B="python -u bench.py --steps 3 --warmup 1"
FLS_GEMM_V11=3 timeout -k 10 300 $B --token-budget 16384 > $O/tb16k_v3.log 2>&1 || exit 1
FLS_GEMM_V11=1 timeout -k 10 300 $B --token-budget 16384 > $O/tb16k_v1.log 2>&1 || exit 1
timeout -k 10 400 $B --prompts-per-gpu 128 --steps 2 > $O/p128.log 2>&1 || exit 1
