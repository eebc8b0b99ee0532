# Round 2 final tree (three-slot default): GPU tests, smoke(), default 70B bench (driver command), BASELINE config 2.
set -o pipefail
O=gpurun_out/r2_final2
mkdir -p $O
cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gputest.log 2>&1
rc=$?; echo "gputest rc=$rc $(tail -1 $O/gputest.log)"; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc $(tail -1 $O/smoke.log)"; [ $rc -eq 0 ] || exit 1
timeout -k 10 500 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench70b.log 2>&1
rc=$?; echo "bench70b rc=$rc $(tail -1 $O/bench70b.log | cut -c1-400)"; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -u bench.py --model llama2-7b --lnps 8 --storage gpu --steps 10 --warmup 2 > $O/bench7b.log 2>&1
rc=$?; echo "bench7b rc=$rc $(grep -o '"value": [0-9.]*' $O/bench7b.log)"; [ $rc -eq 0 ] || exit 1
