# greedy generation on Llama-2-70B: main.py --num_gen_token 8 --suffix_kv_cache, weights in
# the HBM cache; decode-step HIP graphs on (default) vs off (FLS_DECODE_GRAPHS=0), same box; then a
# kernel trace of the graphed run
set -o pipefail
O=gpurun_out/${1:-r5_gen}
R=$(pwd)
mkdir -p $O
python -c "import pickle,sys; sys.path.insert(0,'.'); from flexible_llm_sharding_amd.utils.synthetic import synthetic_prompts; pickle.dump(synthetic_prompts(32,1024,5,64,32000,seed=0), open('/tmp/p.pkl','wb'))" || exit 1
for i in 1 2; do
  timeout -k 10 400 python main.py --synthetic llama2-70b --prompt_pickle /tmp/p.pkl --output_file /tmp/s_g$i.pkl --num_gen_token 8 --suffix_kv_cache --metrics_json $O/graphs_$i.json > $O/graphs_$i.log 2>&1 || exit 1
  FLS_DECODE_GRAPHS=0 timeout -k 10 400 python main.py --synthetic llama2-70b --prompt_pickle /tmp/p.pkl --output_file /tmp/s_e$i.pkl --num_gen_token 8 --suffix_kv_cache --metrics_json $O/eager_$i.json > $O/eager_$i.log 2>&1 || exit 1
done
python -c "
import json, pickle, numpy as np
for n in ('graphs_1', 'eager_1', 'graphs_2', 'eager_2'):
    print(n, [round(x, 4) for x in json.load(open('$O/' + n + '.json'))['step_s']])
a, b = pickle.load(open('/tmp/s_g1.pkl', 'rb')), pickle.load(open('/tmp/s_e1.pkl', 'rb'))
print('graphs == eager bitwise:', all(np.array_equal(x, y) for x, y in zip(a, b)))
" > $O/steps.txt 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $R/$O/trace -o run -- python3 $R/main.py --synthetic llama2-70b --prompt_pickle /tmp/p.pkl --output_file /tmp/s_t.pkl --num_gen_token 6 --suffix_kv_cache > $R/$O/trace.log 2>&1 || exit 1
cd $R
db=$(ls $O/trace/*/run_results.db 2>/dev/null | head -1); [ -z "$db" ] && db=$(ls $O/trace/run_results.db | head -1)
python3 scripts/rocpd_summary.py $db --json $O/trace_passes.json > $O/trace_summary.txt 2>&1 || exit 1
rm -f $db
