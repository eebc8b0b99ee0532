# kernel + memory-copy trace of one capped 16k-budget pass with the piece pool: the slow (layer,
# micro-batch) segments next to the median one, with the copies that overlap them
set -o pipefail
O=gpurun_out/${1:-r5_seg}
R=$(pwd)
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --memory-copy-trace -d $R/$O/pool -o run -- python3 $R/scripts/layer_timing_probe.py --token-budget 16384 --steps 1 > $R/$O/pool.log 2>&1 || exit 1
cd $R
db=$(ls $O/pool/*/run_results.db 2>/dev/null | head -1); [ -z "$db" ] && db=$(ls $O/pool/run_results.db | head -1)
python3 scripts/rocpd_segments.py $db > $O/pool_segments.txt 2>&1 || exit 1
python3 -c "
import sqlite3,sys; c=sqlite3.connect(sys.argv[1])
print([r[0] for r in c.execute(\"select name from sqlite_master where type in ('table','view')\")])" $db > $O/tables.txt 2>&1
rm -f $db
