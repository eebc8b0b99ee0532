# which dispatch makes the ~185 MB device-memory excursion outside the allocator near a call's end:
# rocprofv3 scratch-memory + kernel trace (no counters) of a 2-call capped 70B probe
set -o pipefail
O=gpurun_out/r4_scratch
mkdir -p $O
R=$(pwd)
cd /tmp && export TMPDIR=/tmp
PROBE_CALLS=2 timeout -k 10 400 rocprofv3 --scratch-memory-trace --kernel-trace --output-format csv -d $R/$O/trace -o run -- python3 $R/scripts/mem_probe.py > $R/$O/probe.log 2>&1 || exit 1
cd $R
f=$(ls $O/trace/*/run_scratch_memory_trace.csv $O/trace/run_scratch_memory_trace.csv 2>/dev/null | head -1)
echo "scratch trace: $f"; wc -l $f; head -40 $f > $O/scratch_head.csv
k=$(ls $O/trace/*/run_kernel_trace.csv $O/trace/run_kernel_trace.csv 2>/dev/null | head -1)
python3 - "$f" "$k" > $O/scratch_summary.txt 2>&1 <<'PY'
import csv, sys
sf, kf = sys.argv[1], sys.argv[2]
rows = list(csv.DictReader(open(sf)))
print(len(rows), "scratch records; columns:", list(rows[0].keys()) if rows else None)
for r in rows[:60]:
    print({k: v for k, v in r.items() if v})
ks = list(csv.DictReader(open(kf)))
print(len(ks), "kernel records; columns:", list(ks[0].keys()))
scr = [r for r in ks if int(r.get("Private_Segment_Size", r.get("Scratch_Size", 0)) or 0) > 0]
names = {}
for r in scr:
    names[r["Kernel_Name"][:100]] = names.get(r["Kernel_Name"][:100], 0) + 1
print("kernels with private segment > 0:")
for n, c in sorted(names.items(), key=lambda x: -x[1]):
    print(c, n)
PY
rm -f $O/trace/*/run_kernel_trace.csv $O/trace/run_kernel_trace.csv
