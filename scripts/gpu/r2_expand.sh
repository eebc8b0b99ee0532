# Caching-allocator configuration on the default 70B bench: device memory in use and tokens/s.
set -o pipefail
O=gpurun_out/r2_expand2
mkdir -p $O
cd "$GRAFT_REPO_ROOT"
run() {  # tag, env...
  local tag=$1; shift
  env "$@" timeout -k 10 400 python -u bench.py --steps 6 --warmup 2 > $O/$tag.log 2>&1 || return 1
  echo "$tag $(grep -o '"value": [0-9.]*\|"peak_gpu_mem_gb": [0-9.]*\|"peak_device_used_gb": [0-9.]*' $O/$tag.log | tr '\n' ' ') $(grep allocator: $O/$tag.log)"
}
run base_1 FLS_X=0 || exit 1
run exp_1 PYTORCH_CUDA_ALLOC_CONF=expandable_segments:True PYTORCH_HIP_ALLOC_CONF=expandable_segments:True || exit 1
run base_2 FLS_X=0 || exit 1
run exp_2 PYTORCH_CUDA_ALLOC_CONF=expandable_segments:True PYTORCH_HIP_ALLOC_CONF=expandable_segments:True || exit 1
