# where does storage=cpu lose 5% after the race fix: GPU-side stall accounting + allocator counters
set -o pipefail
mkdir -p gpurun_out/r47
cd "$GRAFT_REPO_ROOT"
for st in cpu gpu; do
  timeout -k 10 300 python bench.py --steps 3 --warmup 1 --storage $st > gpurun_out/r47/bench_$st.log 2>&1
  rc=$?; echo "storage=$st rc=$rc"; grep -o "\"value\": [0-9.]*\|\"peak_gpu_[a-z_]*\": [0-9.]*" gpurun_out/r47/bench_$st.log | tr "\n" " "; grep "allocator\|step 2" gpurun_out/r47/bench_$st.log | cut -c1-700
  [ $rc -eq 0 ] || exit $rc
done
