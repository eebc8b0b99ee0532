"""Per (layer, micro-batch) segments of a rocprofv3 kernel trace: a segment starts at the row
statistic / RMSNorm kernel in front of each QKV GEMM.  Prints the slowest segments next to the
median one, kernel by kernel, with the memory copies that overlap them (when the database has a
memory-copy table: --memory-copy-trace).

    python scripts/rocpd_segments.py DIR/run_results.db [--top 6]
"""
import argparse
import re
import sqlite3
import statistics


def short(name: str) -> str:
    m = re.search(r"_GLOBAL__N_1\d+(\w+?)I(Li\d+E)+", name)
    if m:
        args = re.findall(r"Li(\d+)E", name)
        return f"{m.group(1)}<{','.join(args)}>"
    m = re.search(r"_GLOBAL__N_1\d+(\w+?)E", name)
    return m.group(1) if m else name[:48]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--top", type=int, default=6)
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    ks = [(short(n), s, e) for n, s, e in c.execute("select name, start, end from kernels order by start")]
    copies = []
    for view in ("memory_copies", "memory_copy", "rocpd_memory_copy"):
        try:
            cols = [d[1] for d in c.execute(f"pragma table_info({view})")]
            if not cols:
                continue
            rows = c.execute(f"select * from {view}").fetchall()
            si, ei = cols.index("start"), cols.index("end")
            ni = next((cols.index(k) for k in ("name", "kind", "direction") if k in cols), None)
            bi = next((cols.index(k) for k in ("size", "bytes") if k in cols), None)
            copies = sorted((r[si], r[ei], r[ni] if ni is not None else "?", r[bi] if bi is not None else 0)
                            for r in rows)
            print(f"memory copies: {len(copies)} (table {view}, columns {cols})")
            break
        except sqlite3.Error:
            continue
    starts = [i for i in range(len(ks) - 1)
              if ks[i][0].startswith(("row_rstd", "rmsnorm")) and ks[i + 1][0].endswith("<3>")]
    segs = []
    for j, i0 in enumerate(starts[:-1]):
        i1 = starts[j + 1]
        t0, t1 = ks[i0][1], ks[i1][1]
        segs.append((t1 - t0, i0, i1))
    if not segs:
        print("no segments")
        return
    med = statistics.median(d for d, _, _ in segs)
    print(f"{len(segs)} segments, median {med / 1e6:.2f} ms")

    def show(tag, d, i0, i1):
        t0, t1 = ks[i0][1], ks[i1][1]
        busy = sum(e - s for _, s, e in ks[i0:i1])
        print(f"{tag}: #{i0} {d / 1e6:.2f} ms (kernel time {busy / 1e6:.2f} ms)")
        for n, s, e in ks[i0:i1]:
            if e - s > 100_000:
                print(f"    {n:36s} start +{(s - t0) / 1e6:7.2f} ms  {(e - s) / 1e6:7.2f} ms")
        for s, e, n, b in copies:
            if s < t1 and e > t0:
                print(f"    copy {n!s:24s} {b / 1e6 if b else 0:9.1f} MB  +{(s - t0) / 1e6:7.2f} .. +{(e - t0) / 1e6:7.2f} ms")

    by_d = sorted(segs, key=lambda x: x[0])
    show("median segment", *by_d[len(by_d) // 2])
    for d, i0, i1 in sorted(segs, reverse=True)[:a.top]:
        show("slow segment", d, i0, i1)


if __name__ == "__main__":
    main()
