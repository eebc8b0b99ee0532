# decoder-layer micro-batch / MLP-chunk sweep (70B shapes), GEMM at several M
set -o pipefail
mkdir -p gpurun_out/r35
cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python scripts/layer_sweep.py --json gpurun_out/r35/layer_sweep.json > gpurun_out/r35/layer_sweep.log 2>&1
rc=$?; echo "sweep rc=$rc"; grep prompts gpurun_out/r35/layer_sweep.log | cut -c1-200
[ $rc -eq 0 ] || exit $rc
for m in 16128 16384 24192 24576; do
timeout -k 10 200 python scripts/kernel_bench.py --m $m --json gpurun_out/r35/kb_m$m.json > gpurun_out/r35/kb_m$m.log 2>&1
rc=$?; echo "kb m=$m rc=$rc"; grep -o '"op": "[a-z_0-9]*"\|"v10_tflops": [0-9.]*' gpurun_out/r35/kb_m$m.log | tr '\n' ' '; echo
[ $rc -eq 0 ] || exit $rc
done
