# kernel trace of greedy generation (Llama-2-70B, default flags, 4 tokens) on the suffix-reuse tree
set -o pipefail
O=gpurun_out/r3_sfx_trace
mkdir -p $O
python -c "import pickle,sys; sys.path.insert(0,'.'); from flexible_llm_sharding_amd.utils.synthetic import synthetic_prompts; pickle.dump(synthetic_prompts(32,1024,5,64,32000,seed=0), open('/tmp/p.pkl','wb'))"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/trace -o run -- python3 $GRAFT_REPO_ROOT/main.py --model_path $GRAFT_REPO_ROOT --synthetic llama2-70b --prompt_pickle /tmp/p.pkl --output_file /tmp/s.pkl --num_gen_token 4 --metrics_json $GRAFT_REPO_ROOT/$O/metrics.json > $GRAFT_REPO_ROOT/$O/main_gen.log 2>&1
