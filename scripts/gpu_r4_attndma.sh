# LDS-DMA K/V ring variant of the 8-head range-2 attention: tests, micro-bench A/B, generation A/B.
set -o pipefail
O=gpurun_out/${1:-r4_attndma}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "suffix_rows or decode_split" --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || exit 1
for r in 1 2; do
for d in 0 1; do
FLS_ATTN_DMA=$d timeout -k 10 120 python -u scripts/attn_gen_one.py > $O/time_dma${d}_$r.log 2>&1 || exit 1
done
done
python -c "import pickle,sys; sys.path.insert(0,'.'); from flexible_llm_sharding_amd.utils.synthetic import synthetic_prompts; pickle.dump(synthetic_prompts(32,1024,5,64,32000,seed=0), open('/tmp/p.pkl','wb'))" || exit 1
for r in 1 2; do
for d in 0 1; do
FLS_ATTN_DMA=$d timeout -k 10 400 python main.py --synthetic llama2-70b --prompt_pickle /tmp/p.pkl --output_file /tmp/s_$d.pkl --num_gen_token 6 --suffix_kv_cache --metrics_json $O/metrics_d${d}_$r.json > $O/gen_d${d}_$r.log 2>&1 || exit 1
done
done
O=$O python - > $O/compare.txt 2>&1 <<'PY' || exit 1
import json, os, pickle, numpy as np
O = os.environ['O']
for d in (0, 1):
    for r in (1, 2):
        st = json.load(open(f'{O}/metrics_d{d}_{r}.json'))['step_s']
        print("dma", d, r, [round(x * 1e3, 1) for x in st], "mean later", round(sum(st[1:]) / len(st[1:]) * 1e3, 2))
a = pickle.load(open('/tmp/s_0.pkl', 'rb')); b = pickle.load(open('/tmp/s_1.pkl', 'rb'))
print("scores bitwise equal dma 0 vs 1:", all(np.array_equal(x, y) for x, y in zip(a, b)))
PY
