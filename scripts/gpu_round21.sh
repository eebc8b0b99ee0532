# PMC: v9 vs hipBLASLt on gate/up and o_proj shapes
set -o pipefail
mkdir -p gpurun_out/r21
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for v in 9 -1; do
  for shape in "16128 57344 8192" "16128 8192 8192"; do
    tag=v${v}_$(echo $shape | tr ' ' x)
    timeout -k 10 150 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --output-format csv -d gpurun_out/r21/${tag}_a -o run -- python scripts/gemm_one.py $v $shape 3 > gpurun_out/r21/${tag}_a.log 2>&1 || exit $?
    timeout -k 10 150 rocprofv3 --kernel-trace --pmc SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_INSTS_MFMA SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_VMEM TCC_HIT_sum TCC_MISS_sum --output-format csv -d gpurun_out/r21/${tag}_b -o run -- python scripts/gemm_one.py $v $shape 3 > gpurun_out/r21/${tag}_b.log 2>&1 || exit $?
  done
done
echo done
