# same-box A/B of the capped headline plan with the 192 MB runtime reserve (profiles/r4_vram)
set -o pipefail
O=gpurun_out/r4_plan
mkdir -p $O
timeout -k 10 300 python -u bench.py --steps 4 --warmup 2 > $O/reserve192.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --steps 4 --warmup 2 --attn-rows 16384 > $O/reserve192_groups16k.log 2>&1 || exit 1
FLS_RUNTIME_RESERVE_MB=0 timeout -k 10 300 python -u bench.py --steps 4 --warmup 2 > $O/reserve0.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --steps 4 --warmup 2 > $O/reserve192_2.log 2>&1 || exit 1
