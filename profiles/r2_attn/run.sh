# Attention (single kernel, multi-suffix items): all GPU tests, then the study (profiles/r2_attn).
set -o pipefail
O=gpurun_out/r2_attn2
mkdir -p $O
cd "$GRAFT_REPO_ROOT"
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gputest.log 2>&1
rc=$?; echo "gputest rc=$rc $(tail -1 $O/gputest.log)"; [ $rc -eq 0 ] || { tail -40 $O/gputest.log; exit 1; }
timeout -k 10 400 python -u scripts/attn_bench.py --iters 20 --json $O/attn_bench.json > $O/attn_bench.log 2>&1
echo "study rc=$?"; grep -v amdgpu.ids $O/attn_bench.log
timeout -k 10 500 python -u bench.py --steps 6 --warmup 2 > $O/bench.log 2>&1
echo "bench rc=$? $(grep -o '"value": [0-9.]*' $O/bench.log)"
