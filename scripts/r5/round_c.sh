# decode attention ring A/B (HBM-resident caches), then piece pool vs slots under the cap
set -o pipefail
mkdir -p gpurun_out/r5_pool_ab
timeout -k 10 180 python -u scripts/attn_decode_bench.py > gpurun_out/r5_pool_ab/attn_decode_ring.log 2>&1 || exit 1
bash scripts/r5/pool_ab.sh r5_pool_ab
