# Resident activation states under the cap (one ring slot per micro-batch when they all fit):
# the capped-path GPU tests (run through, failures reported), then --token-budget 16384 resident
# vs parked (FLS_RESIDENT_STATES=0) and with the round-count v11 rule (FLS_GEMM_V11=3) on one
# box, the headline, then v10 vs v11 GEMM times at row counts that are not whole tile rounds
set -o pipefail
O=gpurun_out/${1:-r5_resident}
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_vram_gpu.py -q --timeout 280 --timeout-method thread > $O/tests_vram.log 2>&1
rc=$?; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 1
B="python -u bench.py --steps 3 --warmup 1"
timeout -k 10 300 $B --token-budget 16384 > $O/tb16k_res.log 2>&1 || exit 1
FLS_RESIDENT_STATES=0 timeout -k 10 300 $B --token-budget 16384 > $O/tb16k_park.log 2>&1 || exit 1
FLS_GEMM_V11=3 timeout -k 10 300 $B --token-budget 16384 > $O/tb16k_res_v3.log 2>&1 || exit 1
timeout -k 10 300 $B > $O/head.log 2>&1 || exit 1
timeout -k 10 300 python -u scripts/gemm_v10_v11_m.py > $O/gemm_m.log 2>&1 || exit 1
