# same-box A/B of the headline against the round-3 tree, the model-parallel loopback rehearsal at
# 70B with 8 ranks, then the full small-RAM / small-VRAM envelope (O_DIRECT, 128 prompts)
set -o pipefail
bash scripts/r5/ab_r3.sh r5_ab_final || exit 1
mkdir -p gpurun_out/r5_loopback
timeout -k 10 400 python -u bench.py --loopback-ranks 8 --steps 2 --warmup 1 > gpurun_out/r5_loopback/lb8_70b.log 2>&1 || exit 1
bash scripts/r5/envelope.sh r5_envelope
