# packed-GQA decode attention at the 70B generation-step shape: key tiles split over 2-4 blocks per
# (prompt, KV group) vs one block (the automatic choice at 256 blocks)
set -o pipefail
O=gpurun_out/${1:-r5_attnsplit}
mkdir -p $O
timeout -k 10 200 python -u scripts/attn_decode_bench.py > $O/attn.log 2>&1 || exit 1
