# Round 2 re-entry: GPU tests, smoke(), default 70B bench on the rebuilt tree.
set -o pipefail
O=gpurun_out/r2_validate
mkdir -p $O
cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gputest.log 2>&1
echo "gputest rc=$? $(tail -1 $O/gputest.log)"
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 500 python -u bench.py --steps 10 --warmup 2 > $O/bench.log 2>&1
echo "bench rc=$?"; tail -1 $O/bench.log
