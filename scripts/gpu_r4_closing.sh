# Closing call: validation (GPU suite, smoke, headline bench, Granite-3-8B row), then the same-box
# FLS_ATTN_DEEP traces.
set -o pipefail
bash scripts/gpu_r4_final2.sh r4_final2 || exit 1
bash scripts/gpu_r4_attndeep_trace.sh r4_attndeep_trace || exit 1
