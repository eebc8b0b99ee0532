# token-budget / storage sweep on the 70B headline bench (activation-traffic interference)
set -o pipefail
mkdir -p gpurun_out/r34
cd "$GRAFT_REPO_ROOT"
for cfg in "16384 cpu" "16384 gpu" "24576 cpu" "49152 cpu"; do
  set -- $cfg
  timeout -k 10 300 python bench.py --steps 3 --warmup 1 --token-budget $1 --storage $2 > gpurun_out/r34/bench_tb$1_$2.log 2>&1
  rc=$?; echo "tb=$1 storage=$2 rc=$rc"; grep -o '"value": [0-9.]*\|"peak_gpu_mem_gb": [0-9.]*' gpurun_out/r34/bench_tb$1_$2.log | tr '\n' ' '; echo
  [ $rc -eq 0 ] || exit $rc
done
