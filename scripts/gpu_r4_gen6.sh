set -o pipefail
O=gpurun_out/r4_gen6
mkdir -p $O
python -c "import pickle,sys; sys.path.insert(0,'.'); from flexible_llm_sharding_amd.utils.synthetic import synthetic_prompts; pickle.dump(synthetic_prompts(32,1024,5,64,32000,seed=0), open('/tmp/p.pkl','wb'))" || exit 1
timeout -k 10 400 python main.py --synthetic llama2-70b --prompt_pickle /tmp/p.pkl --output_file /tmp/s.pkl --num_gen_token 6 --suffix_kv_cache --metrics_json $O/metrics.json > $O/gen.log 2>&1 || exit 1
python -c "import json; print([round(x,4) for x in json.load(open('$O/metrics.json'))['step_s']])" > $O/steps.txt
