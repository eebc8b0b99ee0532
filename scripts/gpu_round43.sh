set -o pipefail
cd "$GRAFT_REPO_ROOT"
for c in "80 2 16384 cpu" "80 13 16384 cpu" "20 32 16384 cpu" "40 32 16384 gpu"; do
 set -- $c
 timeout -k 10 200 python scripts/nan_engine.py --layers $1 --prompts $2 --budget $3 --storage $4 2>&1 | grep layers=
done
