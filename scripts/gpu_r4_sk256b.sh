# BN = 256 skinny auto rule: kernel tests, then interleaved 70B generation runs (suffix K/V reuse)
# with BN 128 forced vs the default rule.
set -o pipefail
O=gpurun_out/${1:-r4_sk256b}
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "skinny" --timeout 150 --timeout-method thread > $O/tests.log 2>&1 || exit 1
python -c "import pickle,sys; sys.path.insert(0,'.'); from flexible_llm_sharding_amd.utils.synthetic import synthetic_prompts; pickle.dump(synthetic_prompts(32,1024,5,64,32000,seed=0), open('/tmp/p.pkl','wb'))" || exit 1
for r in 1 2; do
FLS_SKINNY_BN=128 timeout -k 10 400 python main.py --synthetic llama2-70b --prompt_pickle /tmp/p.pkl --output_file /tmp/s_128.pkl --num_gen_token 6 --suffix_kv_cache --metrics_json $O/metrics_bn128_$r.json > $O/gen_bn128_$r.log 2>&1 || exit 1
timeout -k 10 400 python main.py --synthetic llama2-70b --prompt_pickle /tmp/p.pkl --output_file /tmp/s_auto.pkl --num_gen_token 6 --suffix_kv_cache --metrics_json $O/metrics_auto_$r.json > $O/gen_auto_$r.log 2>&1 || exit 1
done
O=$O python - > $O/compare.txt 2>&1 <<'PY' || exit 1
import json, os
O = os.environ['O']
for v in ("bn128", "auto"):
    for r in (1, 2):
        print(v, r, [round(x * 1e3, 1) for x in json.load(open(f'{O}/metrics_{v}_{r}.json'))['step_s']])
PY
