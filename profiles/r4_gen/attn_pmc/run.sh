# The 70B generation-step attention alone (scripts/attn_gen_one.py): timing (one / two K/V register
# sets, split 2), then two PMC passes of the default kernel.
set -o pipefail
O=gpurun_out/${1:-r4_attnpmc}
mkdir -p $O
for v in "0 0" "1 0" "0 2"; do
  set -- $v
  FLS_ATTN_DEEP=$1 FLS_ATTN_SPLIT=$2 timeout -k 10 120 python -u scripts/attn_gen_one.py > $O/time_deep$1_split$2.log 2>&1 || exit 1
done
cd /tmp && export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"
A="GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"
B="FETCH_SIZE SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS"
i=0
for C in "$A" "$B"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $C -d "$R/$O/pmc$i" -o run --output-format csv -- python3 "$R/scripts/attn_gen_one.py" --iters 5 > "$R/$O/pmc$i.log" 2>&1 || exit 1
done
