# headline bench, same box: default dispatch (8-wave mid blocks) vs 4-wave mid blocks, interleaved
set -o pipefail
O=gpurun_out/${1:-r6_mid8_head}
mkdir -p $O
for w in 0 4 0 4; do timeout -k 10 400 python -u scripts/bench_mid_waves.py $w --steps 5 --warmup 2 >> $O/bench_ab.log 2>&1 || exit 1; done
