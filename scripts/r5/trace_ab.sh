set -o pipefail
bash scripts/r5/trace.sh r5_trace || exit 1
bash scripts/r5/ab_r3.sh r5_ab_r3 || exit 1
