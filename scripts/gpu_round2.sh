# round-1 GPU session 2: engine tests, 70B headline bench, rocprof kernel stats
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -m pytest tests/ -x -q -m gpu > gpurun_out/pytest_gpu2.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_gpu2.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 600 python bench.py --steps 2 --warmup 1 > gpurun_out/bench70b_cpu.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -6 gpurun_out/bench70b_cpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_l8 -o run -- python bench.py --steps 2 --warmup 1 --num-layers 8 --prompts-per-gpu 16 > gpurun_out/prof_l8.log 2>&1
rc=$?; echo "rocprof rc=$rc"; tail -3 gpurun_out/prof_l8.log
find gpurun_out/prof_l8 -name "*stats*" | head
