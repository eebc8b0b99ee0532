# greedy generation on Llama-2-70B: main.py --num_gen_token 8 --suffix_kv_cache, weights in
# the HBM cache; decode-step HIP graphs + speculative next steps (default) vs graphs without
# speculation (FLS_SPEC_DECODE=0) vs eager steps (FLS_DECODE_GRAPHS=0), same box; then a kernel
# trace of the default run
set -o pipefail
O=gpurun_out/${1:-r5_gen}
R=$(pwd)
mkdir -p $O
python -c "import pickle,sys; sys.path.insert(0,'.'); from flexible_llm_sharding_amd.utils.synthetic import synthetic_prompts; pickle.dump(synthetic_prompts(32,1024,5,64,32000,seed=0), open('/tmp/p.pkl','wb'))" || exit 1
M="python main.py --synthetic llama2-70b --prompt_pickle /tmp/p.pkl --num_gen_token 8 --suffix_kv_cache"
timeout -k 10 400 $M --output_file /tmp/s_spec.pkl --metrics_json $O/spec.json > $O/spec.log 2>&1 || exit 1
FLS_SPEC_DECODE=0 timeout -k 10 400 $M --output_file /tmp/s_graphs.pkl --metrics_json $O/graphs.json > $O/graphs.log 2>&1 || exit 1
FLS_DECODE_GRAPHS=0 timeout -k 10 400 $M --output_file /tmp/s_eager.pkl --metrics_json $O/eager.json > $O/eager.log 2>&1 || exit 1
python -c "
import json, pickle, numpy as np
for n in ('spec', 'graphs', 'eager'):
    d = json.load(open('$O/' + n + '.json'))
    print(n, [round(x, 4) for x in d['step_s']], 'speculative' if d['stats'].get('speculative') else '')
a, b, c = (pickle.load(open('/tmp/s_%s.pkl' % n, 'rb')) for n in ('spec', 'graphs', 'eager'))
print('spec == graphs bitwise:', all(np.array_equal(x, y) for x, y in zip(a, b)))
print('graphs == eager bitwise:', all(np.array_equal(x, y) for x, y in zip(b, c)))
" > $O/steps.txt 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $R/$O/trace -o run -- python3 $R/main.py --synthetic llama2-70b --prompt_pickle /tmp/p.pkl --output_file /tmp/s_t.pkl --num_gen_token 6 --suffix_kv_cache > $R/$O/trace.log 2>&1 || exit 1
cd $R
db=$(ls $O/trace/*/run_results.db 2>/dev/null | head -1); [ -z "$db" ] && db=$(ls $O/trace/run_results.db | head -1)
python3 scripts/rocpd_summary.py $db --json $O/trace_passes.json > $O/trace_summary.txt 2>&1 || exit 1
rm -f $db
