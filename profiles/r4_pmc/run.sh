# PMC counters of the 70B projection GEMMs: v10 (256x256 tile) vs v11 (384x256) vs hipBLASLt (profiles/r4_pmc)
set -o pipefail
O=gpurun_out/r4_pmc
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"
C="GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE TCC_HIT_sum TCC_MISS_sum"
args=""
for shape in "15360 8192 8192 o 1" "15360 57344 8192 gateup 2" "15360 8192 28672 down 1"; do
  set -- $shape
  for which in 0 11 -1; do
    tag=$4_$([ $which -eq 0 ] && echo v10 || ([ $which -eq 11 ] && echo v11 || echo hipblaslt))
    timeout -s KILL 90 rocprofv3 --pmc $C -d "$R/$O/$tag" -o run --output-format csv -- python3 "$R/scripts/gemm_one.py" $which $1 $2 $3 5 $5 > "$R/$O/$tag.log" 2>&1
    rc=$?; echo "$tag rc=$rc"; [ $rc -eq 0 ] || exit 1
    args="$args $tag=$R/$O/$tag"
  done
done
cd "$R" && python3 scripts/pmc_summary.py $O/pmc_summary.json $args
