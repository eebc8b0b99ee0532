# every kernel of a Granite-3.0-8B pass (embedding / residual / attention / logits
# scalars) and of the 70B headline pass is a framework kernel (no torch eager kernel); rocprofv3
# kernel traces, all distinct kernel names listed and classified
set -o pipefail
O=gpurun_out/${1:-r5_eager}
R=$(pwd)
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $R/$O/granite -o run -- python3 $R/bench.py --model granite-3-8b --steps 2 --warmup 1 > $R/$O/granite.log 2>&1 || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace -d $R/$O/head -o run -- python3 $R/bench.py --steps 2 --warmup 1 > $R/$O/head.log 2>&1 || exit 1
cd $R
for n in granite head; do
  db=$(ls $O/$n/*/run_results.db 2>/dev/null | head -1); [ -z "$db" ] && db=$(ls $O/$n/run_results.db | head -1)
  python3 scripts/rocpd_summary.py $db --all-kernels > $O/${n}_kernels.txt 2>&1 || exit 1
  rm -f $db
done
