# Model-family sweep (lnps=1, storage=cpu, bench shapes): this framework vs the reference-algorithm eager
# baseline, then rocprofv3 kernel stats of the 70B headline bench.
set -o pipefail
mkdir -p gpurun_out/r71
cd "$GRAFT_REPO_ROOT"
run() {  # name, seconds, command...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > gpurun_out/r71/$n.log 2>&1
  local rc=$?
  echo "$n rc=$rc $(grep -o '"value": [0-9.]*\|"peak_gpu_mem_gb": [0-9.]*\|"scores_finite": [a-z]*' gpurun_out/r71/$n.log | tr '\n' ' ')"
  return $rc
}
run ours_llama2-13b 300 python -u bench.py --model llama2-13b --lnps 1 --storage cpu || exit 1
run ref_llama2-13b 300 python -u scripts/reference_eager_bench.py --layers 40 --hidden 5120 --inter 13824 --heads 40 --kv-heads 40 --warmup 1 --steps 2 || exit 1
run ours_mistral-7b 300 python -u bench.py --model mistral-7b --lnps 1 --storage cpu || exit 1
run ref_mistral-7b 300 python -u scripts/reference_eager_bench.py --layers 32 --hidden 4096 --inter 14336 --heads 32 --kv-heads 8 --warmup 1 --steps 2 || exit 1
run ours_llama3.1-8b 300 python -u bench.py --model llama3.1-8b --lnps 1 --storage cpu || exit 1
run ref_llama3.1-8b 300 python -u scripts/reference_eager_bench.py --layers 32 --hidden 4096 --inter 14336 --heads 32 --kv-heads 8 --vocab 128256 --warmup 1 --steps 2 || exit 1
run ours_qwen2-7b 300 python -u bench.py --model qwen2-7b --lnps 1 --storage cpu || exit 1
run ref_qwen2-7b 300 python -u scripts/reference_eager_bench.py --layers 28 --hidden 3584 --inter 18944 --heads 28 --kv-heads 4 --vocab 152064 --warmup 1 --steps 2 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/r71/prof" -o bench70b -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 2 --warmup 1 > "$GRAFT_REPO_ROOT/gpurun_out/r71/prof70b.log" 2>&1
echo "rocprof rc=$?"
