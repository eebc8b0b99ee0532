set -o pipefail
mkdir -p gpurun_out/r9
timeout -k 10 400 python scripts/gemm_ablate.py > gpurun_out/r9/ablate.json 2> gpurun_out/r9/ablate.err
rc=$?; echo "ablate rc=$rc"; cat gpurun_out/r9/ablate.json; tail -3 gpurun_out/r9/ablate.err
