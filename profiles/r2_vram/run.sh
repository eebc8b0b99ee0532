# Round 2: device memory under a VRAM cap (70B lnps=1 storage=cpu; weights streamed from page-cache files).
set -o pipefail
O=gpurun_out/r2_vram
mkdir -p $O
cd "$GRAFT_REPO_ROOT"
step() {  # name, seconds, command...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.log 2>&1
  local rc=$?
  echo "$n rc=$rc $(grep -o '"value": [0-9.]*\|"peak_gpu_mem_gb": [0-9.]*\|"peak_gpu_reserved_gb": [0-9.]*\|"peak_device_used_gb": [0-9.]*\|"token_budget": [0-9]*\|"mlp_chunk": [0-9]*' $O/$n.log | tr '\n' ' ') $(tail -1 $O/$n.log | cut -c1-150)"
  return $rc
}
step gputest 600 python -u -m pytest tests/test_engine_gpu.py -x -q --timeout 300 --timeout-method thread || exit 1
B="python -u bench.py --weights stream --ckpt-dir /tmp/ck70 --steps 2 --warmup 1"
step s_default 600 $B || exit 1
step s_cap6 300 $B --max-vram-gb 6 || exit 1
step s_cap6_noexp 300 env PYTORCH_HIP_ALLOC_CONF=expandable_segments:False PYTORCH_CUDA_ALLOC_CONF=expandable_segments:False $B --max-vram-gb 6 || exit 1
step s_cap55 300 $B --max-vram-gb 5.5 || exit 1
step s_cap8 300 $B --max-vram-gb 8 || exit 1
python -c "
import torch; torch.cuda.init(); f,t=torch.cuda.mem_get_info(0); print('context-only device used GB', (t-f)/1e9)
import flexible_llm_sharding_amd._native as n; n.kernels(); x=torch.empty(1,device='cuda'); f,t=torch.cuda.mem_get_info(0); print('after kernels lib + 1 alloc', (t-f)/1e9)
" > $O/ctx.log 2>&1; cat $O/ctx.log
