# per-item timeline of the 128-prompt capped pass at two run-ahead bounds
set -o pipefail
O=gpurun_out/${1:-r5_probe_p128}
mkdir -p $O
for n in 0 6; do
  FLS_RUNAHEAD_ITEMS=$n timeout -k 10 400 python -u scripts/layer_timing_probe.py --prompts 128 --steps 1 > $O/ra$n.txt 2>&1 || exit 1
done
