# full GPU suite + smoke + headline bench + 70B generation timing (argmax on fp16 bits)
set -o pipefail
O=gpurun_out/r3_check2
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit 1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --steps 5 --warmup 2 > $O/bench.log 2>&1 || exit 1
python -c "import pickle,sys; sys.path.insert(0,'.'); from flexible_llm_sharding_amd.utils.synthetic import synthetic_prompts; pickle.dump(synthetic_prompts(32,1024,5,64,32000,seed=0), open('/tmp/p.pkl','wb'))"
timeout -k 10 400 python main.py --synthetic llama2-70b --prompt_pickle /tmp/p.pkl --output_file /tmp/s.pkl --num_gen_token 6 --metrics_json $O/metrics_gen.json > $O/main_gen.log 2>&1
