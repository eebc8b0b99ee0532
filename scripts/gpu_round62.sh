# clean kernel breakdown of Llama-2-7B (MHA: 32 q / 32 kv heads), resident weights
set -o pipefail
mkdir -p gpurun_out/r62
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r62/prof -o run -- python bench.py --model llama2-7b --num-layers 8 --resident --storage gpu --steps 3 --warmup 1 > gpurun_out/r62/bench.log 2>&1
rc=$?; echo "rc=$rc"; grep '^{' gpurun_out/r62/bench.log | cut -c1-200
exit $rc
