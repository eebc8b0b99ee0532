# Range-2 attention with two register sets of K/V tiles (DEEP, HPB 8): attention / generation tests,
# then a kernel trace of a 70B generation run with suffix K/V reuse, and interleaved-free step times.
set -o pipefail
O=gpurun_out/${1:-r4_attndeep}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -x -q -k "attention or suffix or decode or generation or r2" --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || exit 1
python -c "import pickle,sys; sys.path.insert(0,'.'); from flexible_llm_sharding_amd.utils.synthetic import synthetic_prompts; pickle.dump(synthetic_prompts(32,1024,5,64,32000,seed=0), open('/tmp/p.pkl','wb'))" || exit 1
for r in 1 2; do
for d in 0 1; do
FLS_ATTN_DEEP=$d timeout -k 10 400 python main.py --synthetic llama2-70b --prompt_pickle /tmp/p.pkl --output_file /tmp/s_$d.pkl --num_gen_token 6 --suffix_kv_cache --metrics_json $O/metrics_d${d}_$r.json > $O/gen_d${d}_$r.log 2>&1 || exit 1
done
done
O=$O python - > $O/compare.txt 2>&1 <<'PY' || exit 1
import json, os, pickle, numpy as np
O = os.environ['O']
for d in (0, 1):
    for r in (1, 2):
        st = json.load(open(f'{O}/metrics_d{d}_{r}.json'))['step_s']
        print("deep", d, r, [round(x * 1e3, 1) for x in st], "mean later", round(sum(st[1:]) / len(st[1:]) * 1e3, 2))
a = pickle.load(open('/tmp/s_0.pkl', 'rb')); b = pickle.load(open('/tmp/s_1.pkl', 'rb'))
print("scores bitwise equal deep 0 vs 1:", all(np.array_equal(x, y) for x, y in zip(a, b)))
PY
R=$(pwd)
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/trace -o run -- python3 $R/main.py --model_path $R --synthetic llama2-70b --prompt_pickle /tmp/p.pkl --output_file /tmp/s.pkl --num_gen_token 3 --suffix_kv_cache > $R/$O/trace_gen.log 2>&1 || exit 1
cd $R
db=$(ls $O/trace/*/run_results.db 2>/dev/null | head -1); [ -z "$db" ] && db=$(ls $O/trace/run_results.db | head -1)
python3 scripts/rocpd_summary.py $db --json $O/trace_passes.json > $O/trace_summary.txt 2>&1; rm -f $db
