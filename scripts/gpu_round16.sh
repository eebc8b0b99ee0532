# PMC: v3 / v8 / hipBLASLt on the gate/up shape (MFMA busy, LDS, L2 hit, clock)
set -o pipefail
mkdir -p gpurun_out/r16
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for v in 3 8 -1; do
  timeout -k 10 150 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --output-format csv -d gpurun_out/r16/v${v}a -o run -- python scripts/gemm_one.py $v 16128 57344 8192 3 > gpurun_out/r16/v${v}a.log 2>&1 || exit $?
  timeout -k 10 150 rocprofv3 --kernel-trace --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_INSTS_MFMA --output-format csv -d gpurun_out/r16/v${v}b -o run -- python scripts/gemm_one.py $v 16128 57344 8192 3 > gpurun_out/r16/v${v}b.log 2>&1 || exit $?
done
ls gpurun_out/r16/*
