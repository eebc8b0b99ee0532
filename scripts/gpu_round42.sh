set -o pipefail
mkdir -p gpurun_out/r42
cd "$GRAFT_REPO_ROOT"
timeout -k 10 100 python scripts/nan_probe.py --prompts 12 --layers 4 > gpurun_out/r42/probe12.log 2>&1; tail -2 gpurun_out/r42/probe12.log
for c in "2 2 16384 cpu" "2 2 16384 gpu" "0 2 16384 cpu" "2 12 16384 cpu" "2 13 16384 cpu" "8 2 16384 cpu"; do
 set -- $c
 timeout -k 10 200 python scripts/nan_engine.py --layers $1 --prompts $2 --budget $3 --storage $4 2>&1 | grep layers=
done
