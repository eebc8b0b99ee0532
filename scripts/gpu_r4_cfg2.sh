set -o pipefail
O=gpurun_out/r4_cfg2
mkdir -p $O
timeout -k 10 300 python -u bench.py --model llama2-7b --lnps 8 --storage gpu --steps 6 --warmup 2 > $O/llama2_7b_lnps8_gpu.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --model llama2-7b --lnps 1 --storage cpu --steps 6 --warmup 2 > $O/llama2_7b_lnps1_cpu.log 2>&1 || exit 1
