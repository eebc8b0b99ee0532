# decode-like attention (range-2 kernel: live-row skipping, split-KV for under-filled grids):
# kernel + engine tests, then greedy generation on Llama-2-70B with default flags (HBM weight cache,
# prefix / suffix K/V reuse), split-KV forced off (FLS_ATTN_SPLIT=1) vs the default heuristic, for
# the bench batch (32 prompts x 1k prefix x 5 suffixes) and for 2 long prompts (4k prefix), then a
# kernel trace of the bench-batch generation
set -o pipefail
O=gpurun_out/${1:-r3_splitkv}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -x -v -k "attention or suffix or generation or prefix" --timeout 150 --timeout-method thread > $O/tests.log 2>&1 || exit 1
python -c "import pickle,sys; sys.path.insert(0,'.'); from flexible_llm_sharding_amd.utils.synthetic import synthetic_prompts; pickle.dump(synthetic_prompts(32,1024,5,64,32000,seed=0), open('/tmp/p.pkl','wb')); pickle.dump(synthetic_prompts(2,4000,5,64,32000,seed=1), open('/tmp/p_long.pkl','wb'))"
for W in p p_long; do
  FLS_ATTN_SPLIT=1 timeout -k 10 400 python main.py --synthetic llama2-70b --prompt_pickle /tmp/$W.pkl --output_file /tmp/s_off_$W.pkl --num_gen_token 6 --metrics_json $O/metrics_off_$W.json > $O/main_gen_off_$W.log 2>&1 || exit 1
  timeout -k 10 400 python main.py --synthetic llama2-70b --prompt_pickle /tmp/$W.pkl --output_file /tmp/s_on_$W.pkl --num_gen_token 6 --metrics_json $O/metrics_on_$W.json > $O/main_gen_on_$W.log 2>&1 || exit 1
done
O=$O python - > $O/compare.txt 2>&1 <<'PY' || exit 1
import json, os, pickle, numpy as np
O = os.environ['O']
for w in ("p", "p_long"):
    a = pickle.load(open(f'/tmp/s_off_{w}.pkl', 'rb')); b = pickle.load(open(f'/tmp/s_on_{w}.pkl', 'rb'))
    print(w, "step s (split off):", [round(x, 4) for x in json.load(open(f'{O}/metrics_off_{w}.json'))['step_s']])
    print(w, "step s (default):  ", [round(x, 4) for x in json.load(open(f'{O}/metrics_on_{w}.json'))['step_s']])
    # scores [n_s, steps, V]: step 0 has no suffix K/V reuse; later steps may take other tokens once a
    # near-tie flips (then they diverge)
    for st in range(a[0].shape[1]):
        d = max(float(np.abs(x[:, st].astype(np.float32) - y[:, st].astype(np.float32)).max()) for x, y in zip(a, b))
        same = all((x[:, st].argmax(-1) == y[:, st].argmax(-1)).all() for x, y in zip(a, b))
        print(f"  step {st}: max |score diff| {d:.3e}; same argmax tokens: {same}")
PY
cd /tmp && export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/trace -o run -- python3 $GRAFT_REPO_ROOT/main.py --model_path $GRAFT_REPO_ROOT --synthetic llama2-70b --prompt_pickle /tmp/p.pkl --output_file /tmp/s.pkl --num_gen_token 4 --metrics_json $GRAFT_REPO_ROOT/$O/metrics_trace.json > $GRAFT_REPO_ROOT/$O/trace_gen.log 2>&1
