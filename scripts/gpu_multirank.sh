# multi-rank paths on one GPU: model-parallel (StageInbox) and data-parallel (AllGatherPrefetcher)
# ranks as threads over the loopback comm, against the 1-GPU run
set -o pipefail
O=gpurun_out/${1:-r3_multirank}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_multigpu_gpu.py -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1
