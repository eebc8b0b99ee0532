# BASELINE config 5 per GPU: Llama-2-70B whole model resident in HBM (no weight stream), eager and HIP graphs
set -o pipefail
mkdir -p gpurun_out/r61
cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python bench.py --resident --storage gpu --steps 4 --warmup 1 > gpurun_out/r61/bench70b_resident.log 2>&1
rc=$?; echo "resident rc=$rc"; grep -o '"value": [0-9.]*\|"peak_gpu_[a-z_]*": [0-9.]*\|"scores_finite": [a-z]*' gpurun_out/r61/bench70b_resident.log | tr '\n' ' '; echo
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --resident --hip-graphs --storage gpu --steps 4 --warmup 1 > gpurun_out/r61/bench70b_resident_graphs.log 2>&1
rc=$?; echo "resident+graphs rc=$rc"; grep -o '"value": [0-9.]*\|"peak_gpu_[a-z_]*": [0-9.]*\|"scores_finite": [a-z]*' gpurun_out/r61/bench70b_resident_graphs.log | tr '\n' ' '; echo
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r61/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; grep smoke gpurun_out/r61/smoke.log
exit $rc
