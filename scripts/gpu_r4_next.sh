# GEMM attribution (PMC) + O-projection order / row-chunk sweep + config rows + headline trace
set -o pipefail
O=gpurun_out/r4_next
mkdir -p $O
timeout -k 10 300 python -u scripts/gemm_v11_ab.py --only o_resid --orders 0,-8,4,7,14 --rows 0,21504 --rounds 3 > $O/o_sweep.log 2>&1 || exit 1
timeout -k 10 400 bash profiles/r4_pmc/run.sh > $O/pmc_run.log 2>&1 || exit 1
timeout -k 10 900 bash scripts/gpu_r4_configs.sh r4_configs > $O/configs_run.log 2>&1 || exit 1
