# Tiny-shard slot map (LM head loads under the last decoder layer) and speculative next-call prefetch:
# engine GPU tests, then the default 70B bench with FLS_SPECULATIVE_PREFETCH=0/1 interleaved.
set -o pipefail
O=gpurun_out/r2_spec
mkdir -p $O
cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest tests/test_engine_gpu.py -x -q --timeout 200 --timeout-method thread > $O/test.log 2>&1
rc=$?; echo "tests rc=$rc $(tail -1 $O/test.log)"; [ $rc -eq 0 ] || { tail -30 $O/test.log; exit 1; }
for i in 1 2; do
  for sp in 0 1; do
    FLS_SPECULATIVE_PREFETCH=$sp timeout -k 10 400 python -u bench.py --steps 8 --warmup 2 > $O/sp${sp}_$i.log 2>&1 || exit 1
    echo "sp=$sp run $i $(grep -o '"value": [0-9.]*' $O/sp${sp}_$i.log) $(grep -o 'weight_stall_gpu_s": [0-9.]*' $O/sp${sp}_$i.log | tail -1)"
  done
done
