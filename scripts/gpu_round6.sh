# PMC counters for GEMM variants (separate runs, kernel-trace only)
set -o pipefail
mkdir -p gpurun_out/pmc6
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for v in 1 3; do
  timeout -k 10 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --output-format csv -d gpurun_out/pmc6/v${v}a -o run -- python scripts/gemm_one.py $v 16128 57344 8192 5 > gpurun_out/pmc6/v${v}a.log 2>&1 || exit $?
  timeout -k 10 120 rocprofv3 --kernel-trace --pmc SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_LDS_UNALIGNED_STALL --output-format csv -d gpurun_out/pmc6/v${v}b -o run -- python scripts/gemm_one.py $v 16128 57344 8192 5 > gpurun_out/pmc6/v${v}b.log 2>&1 || exit $?
done
echo done
ls -R gpurun_out/pmc6 | head -30
