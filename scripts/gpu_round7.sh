# GEMM ablation + which hipBLASLt kernel runs the 70B gate/up shape
set -o pipefail
mkdir -p gpurun_out/r7
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python scripts/gemm_ablate.py > gpurun_out/r7/ablate.json 2> gpurun_out/r7/ablate.err
rc=$?; echo "ablate rc=$rc"; cat gpurun_out/r7/ablate.json
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r7/blt -o run -- python scripts/gemm_one.py -1 16128 57344 8192 3 > gpurun_out/r7/blt.log 2>&1
rc=$?; echo "blt rc=$rc"
python - <<'PY'
import csv,glob
for f in glob.glob("gpurun_out/r7/blt/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        print(r["Name"][:200], r["Calls"], r["AverageNs"])
PY
timeout -k 10 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --output-format csv -d gpurun_out/r7/bltpmc -o run -- python scripts/gemm_one.py -1 16128 57344 8192 3 > gpurun_out/r7/bltpmc.log 2>&1
echo "pmc rc=$?"
