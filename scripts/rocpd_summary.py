"""Per-pass kernel breakdown and GPU idle time from a rocprofv3 database.

    rocprofv3 --kernel-trace --stats -d DIR -o run -- python3 bench.py --steps 2 --warmup 1
    python scripts/rocpd_summary.py DIR/run_results.db [--json out.json]

Passes are delimited by the embedding kernel (one per pass).  For each pass: wall time from
its embedding to the next one (the last pass: to its last kernel), GPU busy time (union of
kernel intervals), idle = wall - busy, and per-kernel totals; the kernels before the first
pass (weight generation) are excluded.
"""
import argparse
import json
import re
import sqlite3
from collections import defaultdict


def short(name: str) -> str:
    m = re.search(r"_GLOBAL__N_1\d+(\w+?)I(Li\d+E)+", name)
    if m:
        args = re.findall(r"Li(\d+)E", name)
        return f"{m.group(1)}<{','.join(args)}>"
    m = re.search(r"_GLOBAL__N_1\d+(\w+?)E", name)
    return m.group(1) if m else name[:60]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--json", default=None)
    ap.add_argument("--embeds-per-pass", type=int, default=1,
                    help="embedding launches per pass (one per micro-batch)")
    ap.add_argument("--all-kernels", action="store_true",
                    help="list every distinct kernel of the passes, classified: framework (csrc/kernels), "
                         "HIP runtime copies, other (torch eager, libraries)")
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    rows = c.execute("select name, start, end from kernels order by start").fetchall()
    starts = [i for i, r in enumerate(rows) if "embed_kernel" in r[0]][::a.embeds_per_pass]
    passes = []
    for j, i0 in enumerate(starts):
        i1 = starts[j + 1] if j + 1 < len(starts) else len(rows)
        ks = rows[i0:i1]
        t0 = ks[0][1]
        t1 = rows[i1][1] if i1 < len(rows) else max(k[2] for k in ks)
        busy, cur_s, cur_e = 0, None, None
        per = defaultdict(float)
        for n, s, e in ks:
            per[short(n)] += (e - s) / 1e6
            if cur_e is None or s > cur_e:
                if cur_e is not None:
                    busy += cur_e - cur_s
                cur_s, cur_e = s, e
            else:
                cur_e = max(cur_e, e)
        busy += cur_e - cur_s
        passes.append({"wall_ms": (t1 - t0) / 1e6, "busy_ms": busy / 1e6, "idle_ms": (t1 - t0 - busy) / 1e6,
                       "kernels_ms": dict(sorted(per.items(), key=lambda kv: -kv[1]))})
    for i, p in enumerate(passes):
        print(f"pass {i}: wall {p['wall_ms']:.1f} ms, GPU busy {p['busy_ms']:.1f} ms, idle {p['idle_ms']:.1f} ms")
        tot = sum(p["kernels_ms"].values())
        for k, v in list(p["kernels_ms"].items())[:10]:
            print(f"    {k:40s} {v:9.1f} ms  {100 * v / tot:5.1f}%")
    if a.all_kernels and starts:
        seen = defaultdict(lambda: [0, 0.0])
        for n, s_, e in rows[starts[0]:]:
            seen[n][0] += 1
            seen[n][1] += (e - s_) / 1e6
        cls = {"framework": [], "runtime copy": [], "other": []}
        for n, (cnt, ms) in sorted(seen.items(), key=lambda kv: -kv[1][1]):
            k = ("framework" if "_GLOBAL__N_1" in n else "runtime copy" if n.startswith("__amd_rocclr") else "other")
            cls[k].append((n, cnt, ms))
        for k, lst in cls.items():
            print(f"{k} kernels: {len(lst)}")
            for n, cnt, ms in lst:
                print(f"    {short(n) if k == 'framework' else n[:100]:60s} x{cnt:<7d} {ms:9.1f} ms")
    if a.json:
        with open(a.json, "w") as f:
            json.dump(passes, f, indent=1)


if __name__ == "__main__":
    main()
