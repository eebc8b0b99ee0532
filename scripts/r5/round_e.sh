# host-side probe of the pool's first-micro-batch stalls; uneven skinny K slices + unpruned decode
# last layer: kernel tests, then one generation run (speculative default)
set -o pipefail
O=gpurun_out/r5_e
mkdir -p $O
timeout -k 10 300 python -u scripts/layer_timing_probe.py --token-budget 16384 --steps 1 > $O/pool_tb16k.txt 2>&1 || exit 1
FLS_PIECE_POOL=0 timeout -k 10 300 python -u scripts/layer_timing_probe.py --token-budget 16384 --steps 1 > $O/slots_tb16k.txt 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -x -q --timeout 200 --timeout-method thread -k "skinny or speculative or decode or suffix or prefix_kv or generation" > $O/tests.log 2>&1 || exit 1
python -c "import pickle,sys; sys.path.insert(0,'.'); from flexible_llm_sharding_amd.utils.synthetic import synthetic_prompts; pickle.dump(synthetic_prompts(32,1024,5,64,32000,seed=0), open('/tmp/p.pkl','wb'))" || exit 1
timeout -k 10 400 python main.py --synthetic llama2-70b --prompt_pickle /tmp/p.pkl --num_gen_token 8 --suffix_kv_cache --output_file /tmp/s.pkl --metrics_json $O/spec.json > $O/spec.log 2>&1 || exit 1
python -c "import json; d=json.load(open('$O/spec.json')); print([round(x,4) for x in d['step_s']])" > $O/steps.txt
