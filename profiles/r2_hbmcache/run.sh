# Round 2: partial HBM residency (--hbm_cache_gb): GPU tests, then greedy generation on 70B with half the
# layers kept in HBM (prefix K/V cache on), and the default bench as a regression check.
set -o pipefail
O=gpurun_out/r2_hbmcache
mkdir -p $O
cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gputest.log 2>&1
rc=$?; echo "gputest rc=$rc $(tail -1 $O/gputest.log)"; [ $rc -eq 0 ] || exit 1
timeout -k 10 500 python -u scripts/gen_bench.py --gen 4 --hbm-cache-gb 70 --json $O/gen_cache70.json > $O/gen_cache70.log 2>&1
rc=$?; echo "gen70 rc=$rc"; grep '^{' $O/gen_cache70.log | cut -c1-300; [ $rc -eq 0 ] || exit 1
timeout -k 10 400 python -u bench.py --steps 6 --warmup 2 > $O/bench.log 2>&1
rc=$?; echo "bench rc=$rc $(grep -o '"value": [0-9.]*' $O/bench.log)"; [ $rc -eq 0 ] || exit 1
