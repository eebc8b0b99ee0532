# Same-box kernel traces of the 70B generation step with FLS_ATTN_DEEP=0 and 1.
set -o pipefail
O=gpurun_out/${1:-r4_attndeep_trace}
mkdir -p $O
python -c "import pickle,sys; sys.path.insert(0,'.'); from flexible_llm_sharding_amd.utils.synthetic import synthetic_prompts; pickle.dump(synthetic_prompts(32,1024,5,64,32000,seed=0), open('/tmp/p.pkl','wb'))" || exit 1
R=$(pwd)
cd /tmp && export TMPDIR=/tmp
for d in 0 1 0 1; do
FLS_ATTN_DEEP=$d timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/trace_$d -o run -- python3 $R/main.py --model_path $R --synthetic llama2-70b --prompt_pickle /tmp/p.pkl --output_file /tmp/s.pkl --num_gen_token 4 --suffix_kv_cache > $R/$O/trace_gen_$d.log 2>&1 || exit 1
db=$(ls $R/$O/trace_$d/*/run_results.db 2>/dev/null | head -1); [ -z "$db" ] && db=$(ls $R/$O/trace_$d/run_results.db | head -1)
python3 $R/scripts/rocpd_summary.py $db >> $R/$O/summary_deep$d.txt 2>&1; rm -rf $R/$O/trace_$d
done
