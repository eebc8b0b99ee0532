# Generation step (verdict r3 #3): skinny-M GEMM + one-wave-per-head range-2 attention.
# Kernel tests, small-M GEMM A/B at 70B shapes, then greedy generation on Llama-2-70B with suffix
# K/V reuse (opt-in) before/after (FLS_SKINNY=0 + q_block 64 attention vs defaults), then a kernel
# trace of the after run.
set -o pipefail
O=gpurun_out/${1:-r4_gen}
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -v -k "skinny or suffix_rows or decode_split or small_m" --timeout 150 --timeout-method thread > $O/tests.log 2>&1 || exit 1
timeout -k 10 400 python -u scripts/gemm_skinny_ab.py --ms 64,160,256 > $O/skinny_ab.log 2>&1 || exit 1
python -c "import pickle,sys; sys.path.insert(0,'.'); from flexible_llm_sharding_amd.utils.synthetic import synthetic_prompts; pickle.dump(synthetic_prompts(32,1024,5,64,32000,seed=0), open('/tmp/p.pkl','wb'))" || exit 1
FLS_SKINNY=0 FLS_R2_QBLOCK=64 timeout -k 10 400 python main.py --synthetic llama2-70b --prompt_pickle /tmp/p.pkl --output_file /tmp/s_before.pkl --num_gen_token 6 --suffix_kv_cache --metrics_json $O/metrics_before.json > $O/gen_before.log 2>&1 || exit 1
timeout -k 10 400 python main.py --synthetic llama2-70b --prompt_pickle /tmp/p.pkl --output_file /tmp/s_after.pkl --num_gen_token 6 --suffix_kv_cache --metrics_json $O/metrics_after.json > $O/gen_after.log 2>&1 || exit 1
O=$O python - > $O/compare.txt 2>&1 <<'PY' || exit 1
import json, os, pickle, numpy as np
O = os.environ['O']
a = pickle.load(open('/tmp/s_before.pkl', 'rb')); b = pickle.load(open('/tmp/s_after.pkl', 'rb'))
print("step s (before):", [round(x, 4) for x in json.load(open(f'{O}/metrics_before.json'))['step_s']])
print("step s (after): ", [round(x, 4) for x in json.load(open(f'{O}/metrics_after.json'))['step_s']])
for st in range(a[0].shape[1]):
    d = max(float(np.abs(x[:, st].astype(np.float32) - y[:, st].astype(np.float32)).max()) for x, y in zip(a, b))
    same = all((x[:, st].argmax(-1) == y[:, st].argmax(-1)).all() for x, y in zip(a, b))
    print(f"  step {st}: max |score diff| {d:.3e}; same argmax tokens: {same}")
PY
R=$(pwd)
cd /tmp && export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $R/$O/trace -o run -- python3 $R/main.py --model_path $R --synthetic llama2-70b --prompt_pickle /tmp/p.pkl --output_file /tmp/s.pkl --num_gen_token 4 --suffix_kv_cache --metrics_json $R/$O/metrics_trace.json > $R/$O/trace_gen.log 2>&1 || exit 1
cd $R
db=$(ls $O/trace/*/run_results.db 2>/dev/null | head -1); [ -z "$db" ] && db=$(ls $O/trace/run_results.db | head -1)
python3 scripts/rocpd_summary.py $db --json $O/trace_passes.json > $O/trace_summary.txt 2>&1; rm -f $db; ls $O/trace/*/ 2>/dev/null | head
