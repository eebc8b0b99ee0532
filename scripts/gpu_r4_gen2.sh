timeout -k 10 1000 bash scripts/gpu_r4_gen.sh r4_gen2 || exit 1
