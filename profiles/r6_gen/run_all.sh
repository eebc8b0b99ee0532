# exact suffix K/V reuse: GPU kernel + engine tests, then the 70B probe + main.py comparison
set -o pipefail
O=gpurun_out/${1:-r6_gen2}
mkdir -p $O
true
O=gpurun_out/${1:-r6_gen2}; export O_NAME=${1:-r6_gen2}
timeout -k 10 900 python -u scripts/gen_exact_probe.py --prompts 64 --gen 8 --json $O/probe.json > $O/probe.log 2>&1 || exit 1
python - <<'PY' || exit 1
import pickle, sys
sys.path.insert(0, ".")
from flexible_llm_sharding_amd.utils.synthetic import synthetic_prompts
p = synthetic_prompts(64, 1024, 5, 64, 32000, seed=1)
for n in ("a", "b"):
    pickle.dump(p, open(f"/tmp/prompts_{n}.pkl", "wb"))
PY
timeout -k 10 600 python -u main.py --synthetic llama2-70b --prompt_pickle /tmp/prompts_a.pkl --output_file /tmp/out_a.pkl --num_gen_token 8 --metrics_json $O/main_default.json > $O/main_default.log 2>&1 || exit 1
timeout -k 10 600 python -u main.py --synthetic llama2-70b --prompt_pickle /tmp/prompts_b.pkl --output_file /tmp/out_b.pkl --num_gen_token 8 --suffix_kv_cache false --metrics_json $O/main_exact.json > $O/main_exact.log 2>&1 || exit 1
python - > $O/main_compare.txt <<'PY' || exit 1
import pickle, json, numpy as np
ua, ub = pickle.load(open("/tmp/prompts_a_updated.pkl", "rb")), pickle.load(open("/tmp/prompts_b_updated.pkl", "rb"))
sa, sb = pickle.load(open("/tmp/out_a.pkl", "rb")), pickle.load(open("/tmp/out_b.pkl", "rb"))
print(json.dumps({"prompts": len(ua), "updated_prompts_equal": ua == ub,
                  "greedy_tokens_equal": all(np.array_equal(np.argmax(x, -1), np.argmax(y, -1)) for x, y in zip(sa, sb)),
                  "max_abs_diff": float(max(np.abs(x.astype(np.float32) - y.astype(np.float32)).max() for x, y in zip(sa, sb)))}))
for n in ("default", "exact"):
    m = json.load(open(f"gpurun_out/{__import__('os').environ.get('O_NAME', 'r6_gen')}/main_{n}.json"))
    print(n, json.dumps({"step_s": [round(x, 4) for x in m["step_s"]], "stats": {k: m["stats"].get(k) for k in ("tokens", "suffix_tokens_reused", "speculative", "graph_replays")}}))
PY
