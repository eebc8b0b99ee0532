"""Where a pass idles: the GPU idle gaps of the last full pass of a rocprofv3 database, each with
the kernels before and after it (largest first), and the idle time summed by the kernel that
follows the gap.

    python scripts/rocpd_gaps.py DIR/run_results.db [--embeds-per-pass N] [--top 25]
"""
import argparse
import re
import sqlite3
from collections import defaultdict


def short(name: str) -> str:
    m = re.search(r"_GLOBAL__N_1\d+(\w+?)I", name) or re.search(r"_GLOBAL__N_1\d+(\w+?)E", name)
    return m.group(1) if m else name[:40]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--embeds-per-pass", type=int, default=3)
    ap.add_argument("--top", type=int, default=25)
    a = ap.parse_args()
    rows = sqlite3.connect(a.db).execute("select name, start, end from kernels order by start").fetchall()
    starts = [i for i, r in enumerate(rows) if "embed_kernel" in r[0]][::a.embeds_per_pass]
    if len(starts) < 2:
        print("fewer than two passes")
        return
    ks = rows[starts[-2]:starts[-1]]
    gaps, cur_e, prev = [], None, None
    for n, s, e in ks:
        if cur_e is not None and s > cur_e:
            gaps.append(((s - cur_e) / 1e3, short(prev), short(n)))
        if cur_e is None or e > cur_e:
            cur_e, prev = e, n
    by_next = defaultdict(float)
    for g, _, nxt in gaps:
        by_next[nxt] += g
    print(f"pass: {len(ks)} kernels, {len(gaps)} gaps, idle {sum(g for g, _, _ in gaps) / 1e3:.1f} ms")
    print("idle (ms) by the kernel after the gap:")
    for k, v in sorted(by_next.items(), key=lambda kv: -kv[1]):
        print(f"    {k:32s} {v / 1e3:8.2f}")
    print(f"largest {a.top} gaps (us):")
    for g, p, n in sorted(gaps, reverse=True)[:a.top]:
        print(f"    {g:9.1f}  {p} -> {n}")


if __name__ == "__main__":
    main()
