# piece pool vs slots traces at a 16k token budget, then the eager-kernel-free traces
set -o pipefail
bash scripts/r5/trace_pool.sh r5_trace_pool || exit 1
bash scripts/r5/eager_free.sh r5_eager
