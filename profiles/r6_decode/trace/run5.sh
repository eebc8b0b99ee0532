# host profile (cProfile) of the 8-prompt exact generation probe: what the host does per step
set -o pipefail
O=gpurun_out/${1:-r6_decode_host}
mkdir -p $O
timeout -k 10 500 python -u -m cProfile -o $O/p8.prof scripts/gen_exact_probe.py --prompts 8 --gen 12 --only reuse > $O/p8.log 2>&1 || exit 1
python3 -c "
import pstats,sys
p=pstats.Stats(sys.argv[1]); p.sort_stats('tottime').print_stats(40)" $O/p8.prof > $O/p8_tottime.txt 2>&1 || exit 1
python3 -c "
import pstats,sys
p=pstats.Stats(sys.argv[1]); p.sort_stats('cumulative').print_stats('engine.py|graphs.py|batch.py|api.py|prefix_cache.py', 40)" $O/p8.prof > $O/p8_cum.txt 2>&1 || exit 1
