set -o pipefail
O=gpurun_out/${1:-r5_vram_dbg}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_vram_gpu.py -q --timeout 280 --timeout-method thread > $O/tests.log 2>&1
FLS_RESIDENT_STATES=0 timeout -k 10 300 python -u -m pytest tests/test_vram_gpu.py -q --timeout 280 --timeout-method thread -k holds > $O/tests_park.log 2>&1
exit 0
