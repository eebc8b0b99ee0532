# Range-2 attention split-KV slices on the 70B generation step (suffix K/V reuse), interleaved.
set -o pipefail
O=gpurun_out/${1:-r4_attnsplit}
mkdir -p $O
python -c "import pickle,sys; sys.path.insert(0,'.'); from flexible_llm_sharding_amd.utils.synthetic import synthetic_prompts; pickle.dump(synthetic_prompts(32,1024,5,64,32000,seed=0), open('/tmp/p.pkl','wb'))" || exit 1
for r in 1 2; do
for sp in 0 2 4; do
FLS_ATTN_SPLIT=$sp timeout -k 10 400 python main.py --synthetic llama2-70b --prompt_pickle /tmp/p.pkl --output_file /tmp/s_$sp.pkl --num_gen_token 6 --suffix_kv_cache --metrics_json $O/metrics_s${sp}_$r.json > $O/gen_s${sp}_$r.log 2>&1 || exit 1
done
done
O=$O python - > $O/compare.txt 2>&1 <<'PY' || exit 1
import json, os
O = os.environ['O']
for v in ("s0", "s2", "s4"):
    for r in (1, 2):
        st = json.load(open(f'{O}/metrics_{v}_{r}.json'))['step_s']
        print(v, r, [round(x * 1e3, 1) for x in st], "mean later", round(sum(st[1:]) / len(st[1:]) * 1e3, 2))
PY
R=$(pwd)
cd /tmp && export TMPDIR=/tmp
FLS_ATTN_SPLIT=2 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/trace -o run -- python3 $R/main.py --model_path $R --synthetic llama2-70b --prompt_pickle /tmp/p.pkl --output_file /tmp/s.pkl --num_gen_token 3 --suffix_kv_cache > $R/$O/trace_gen.log 2>&1 || exit 1
cd $R
db=$(ls $O/trace/*/run_results.db 2>/dev/null | head -1); [ -z "$db" ] && db=$(ls $O/trace/run_results.db | head -1)
python3 scripts/rocpd_summary.py $db --json $O/trace_passes.json > $O/trace_summary.txt 2>&1; rm -f $db
