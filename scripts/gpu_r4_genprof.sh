set -o pipefail
O=gpurun_out/r4_genprof
mkdir -p $O
python -c "import pickle,sys; sys.path.insert(0,'.'); from flexible_llm_sharding_amd.utils.synthetic import synthetic_prompts; pickle.dump(synthetic_prompts(32,1024,5,64,32000,seed=0), open('/tmp/p.pkl','wb'))" || exit 1
FLS_PROFILE_GEN_STEPS=2,3 FLS_PROFILE_OUT=$O/prof timeout -k 10 400 python main.py --synthetic llama2-70b --prompt_pickle /tmp/p.pkl --output_file /tmp/s.pkl --num_gen_token 4 --suffix_kv_cache --metrics_json $O/metrics.json > $O/gen.log 2>&1 || exit 1
python -c "
import pstats
for st in (2, 3):
    p = pstats.Stats('$O/prof.%d' % st)
    p.sort_stats('cumulative').print_stats(45)
    p.sort_stats('tottime').print_stats(30)
" > $O/profile.txt 2>&1 || exit 1
