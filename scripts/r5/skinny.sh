# small-M projection GEMMs at generation-step row counts: automatic choice vs the skinny-M kernel
# forced with each weight-block height, and hipBLASLt
set -o pipefail
O=gpurun_out/${1:-r5_skinny}
mkdir -p $O
timeout -k 10 300 python -u scripts/skinny_bench.py --ms 96,128,160,192 > $O/skinny.log 2>&1 || exit 1
