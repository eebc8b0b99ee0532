# full GPU test suite on the suffix-K/V-reuse tree, then greedy generation on Llama-2-70B with the
# default flags (HBM weight cache + prefix K/V cache + suffix K/V reuse), run from the repo root
set -o pipefail
O=gpurun_out/r3_sfx
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit 1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
python -c "import pickle,sys; sys.path.insert(0,'.'); from flexible_llm_sharding_amd.utils.synthetic import synthetic_prompts; pickle.dump(synthetic_prompts(32,1024,5,64,32000,seed=0), open('/tmp/p.pkl','wb'))"
timeout -k 10 400 python main.py --synthetic llama2-70b --prompt_pickle /tmp/p.pkl --output_file /tmp/s.pkl --num_gen_token 6 --metrics_json $O/metrics.json --verbose > $O/main_gen.log 2>&1
