# generation step before/after on the final skinny policy + trace, and the default bench
set -o pipefail
O=gpurun_out/r4_gen5
mkdir -p $O
python -c "import pickle,sys; sys.path.insert(0,'.'); from flexible_llm_sharding_amd.utils.synthetic import synthetic_prompts; pickle.dump(synthetic_prompts(32,1024,5,64,32000,seed=0), open('/tmp/p.pkl','wb'))" || exit 1
FLS_SKINNY=0 FLS_R2_QBLOCK=64 timeout -k 10 400 python main.py --synthetic llama2-70b --prompt_pickle /tmp/p.pkl --output_file /tmp/s_before.pkl --num_gen_token 6 --suffix_kv_cache --metrics_json $O/metrics_before.json > $O/gen_before.log 2>&1 || exit 1
timeout -k 10 400 python main.py --synthetic llama2-70b --prompt_pickle /tmp/p.pkl --output_file /tmp/s_after.pkl --num_gen_token 6 --suffix_kv_cache --metrics_json $O/metrics_after.json > $O/gen_after.log 2>&1 || exit 1
python -c "import json; [print(n, [round(x,4) for x in json.load(open('$O/metrics_'+n+'.json'))['step_s']]) for n in ('before','after')]" > $O/compare.txt || exit 1
R=$(pwd)
cd /tmp && export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $R/$O/trace -o run -- python3 $R/main.py --model_path $R --synthetic llama2-70b --prompt_pickle /tmp/p.pkl --output_file /tmp/s.pkl --num_gen_token 4 --suffix_kv_cache --metrics_json $R/$O/metrics_trace.json > $R/$O/trace_gen.log 2>&1 || exit 1
cd $R
db=$(ls $O/trace/*/run_results.db 2>/dev/null | head -1); [ -z "$db" ] && db=$(ls $O/trace/run_results.db | head -1)
python3 scripts/rocpd_summary.py $db --json $O/trace_passes.json > $O/trace_summary.txt 2>&1; rm -f $db
timeout -k 10 400 python -u bench.py --steps 4 --warmup 2 > $O/bench.log 2>&1 || exit 1
