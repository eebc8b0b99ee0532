"""GPU idle time from a rocprofv3 --kernel-trace (--memory-copy-trace) CSV of bench.py: the union of
kernel intervals over the last bench steps, the gaps between them (largest first, with the kernels on
either side) and the copies in flight during each gap.

    python scripts/trace_gaps.py TRACE_DIR [--top 25]
"""
import argparse
import csv
import glob
import os


def load(d, pat):
    rows = []
    for f in glob.glob(os.path.join(d, "**", pat), recursive=True):
        with open(f) as fh:
            rows += list(csv.DictReader(fh))
    return rows


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--top", type=int, default=25)
    a = ap.parse_args()
    ks = load(a.dir, "*kernel_trace.csv")
    cs = load(a.dir, "*memory_copy_trace.csv")
    K = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:60]) for r in ks)
    C = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r.get("Direction", r.get("Kind", "?")),
                int(r.get("Bytes", r.get("Size", 0)) or 0)) for r in cs)
    # the timed region: from the first GEMM after the last fill_random (weights generated) onwards
    last_fill = max((s for s, e, n in K if "fill_random" in n), default=0)
    K = [k for k in K if k[0] > last_fill]
    t0, t1 = K[0][0], max(e for s, e, n in K)
    busy, gaps, cur_e, prev = 0, [], K[0][0], K[0]
    for s, e, n in K:
        if s > cur_e:
            gaps.append((s - cur_e, cur_e, s, prev[2], n))
        if e > cur_e:
            busy += e - max(s, cur_e)
            cur_e = e
            prev = (s, e, n)
    span = t1 - t0
    print(f"span {span / 1e6:.1f} ms (warmup + timed steps), kernels busy {busy / 1e6:.1f} ms "
          f"({100 * busy / span:.2f}%), idle {(span - busy) / 1e6:.1f} ms in {len(gaps)} gaps")
    big = sorted(gaps, reverse=True)[:a.top]
    for g, s, e, before, after in big:
        inflight = [c for c in C if c[0] < e and c[1] > s]
        cb = sum(c[3] for c in inflight)
        print(f"gap {g / 1e3:8.1f} us at +{(s - t0) / 1e6:8.1f} ms  after {before[:40]:40s} before {after[:40]:40s} "
              f"copies in flight {len(inflight)} ({cb / 1e9:.2f} GB)")
    hist = {}
    for g, *_ in gaps:
        b = "<10us" if g < 1e4 else "<100us" if g < 1e5 else "<1ms" if g < 1e6 else ">=1ms"
        hist[b] = hist.get(b, 0) + g
    print("idle by gap size:", {k: f"{v / 1e6:.1f} ms" for k, v in hist.items()})
    # the last step boundary: every kernel in a window around the last embed
    emb = [s for s, e, n in K if "embed_kernel" in n]
    if emb:
        tb = emb[-1]
        print("\nkernels around the last step start (ms relative to its embed):")
        for s, e, n in K:
            if tb - 60e6 <= s <= tb + 60e6 and ("gemm" not in n or s > tb):
                print(f"  {(s - tb) / 1e6:9.2f} .. {(e - tb) / 1e6:9.2f}  {n[:70]}")
                if s > tb and "gemm" in n:
                    break


if __name__ == "__main__":
    main()
