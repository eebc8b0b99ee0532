# v10-only GEMM library (v13 removed): full GPU tests, smoke, bench.
set -o pipefail
O=gpurun_out/r2_v10only
mkdir -p $O
cd "$GRAFT_REPO_ROOT"
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gputest.log 2>&1
rc=$?; echo "gputest rc=$rc $(tail -1 $O/gputest.log)"; [ $rc -eq 0 ] || { tail -40 $O/gputest.log; exit 1; }
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc $(tail -1 $O/smoke.log)"; [ $rc -eq 0 ] || exit 1
timeout -k 10 500 python -u bench.py --steps 8 --warmup 2 > $O/bench.log 2>&1
echo "bench rc=$? $(grep -o '"value": [0-9.]*' $O/bench.log)"
