"""Summarise a rocprofv3 rocpd database (kernels and memory copies):
python tools/rocpd_summary.py run_results.db [--timeline N]
Prints per-kernel count / mean / total (us) and per-direction copy stats, and
optionally the first N events of the timeline (start offsets in us)."""
import sqlite3
import sys
from collections import defaultdict


def main():
    db = sqlite3.connect(sys.argv[1])
    cur = db.cursor()
    kcols = [r[1] for r in cur.execute("pragma table_info(kernels)")]
    name = "kernel_name" if "kernel_name" in kcols else "name"
    rows = cur.execute(f"select {name}, start, end, stream_id from kernels order by start").fetchall()
    mcols = [r[1] for r in cur.execute("pragma table_info(memory_copies)")]
    mrows = cur.execute("select * from memory_copies order by start").fetchall()
    agg = defaultdict(list)
    for n, s, e, _ in rows:
        agg[n].append((e - s) / 1e3)
    print(f"{'kernel':80s} {'n':>6s} {'mean_us':>10s} {'total_us':>12s}")
    for n, v in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
        print(f"{n[:80]:80s} {len(v):6d} {sum(v)/len(v):10.2f} {sum(v):12.1f}")
    if mrows:
        i_s, i_e = mcols.index("start"), mcols.index("end")
        i_sz = mcols.index("size") if "size" in mcols else None
        i_k = mcols.index("name") if "name" in mcols else None
        cagg = defaultdict(list)
        for r in mrows:
            cagg[r[i_k] if i_k is not None else "copy"].append(((r[i_e] - r[i_s]) / 1e3, r[i_sz] if i_sz is not None else 0))
        for k, v in cagg.items():
            t = sum(x for x, _ in v)
            b = sum(y for _, y in v)
            print(f"copy {k}: n={len(v)} total_us={t:.1f} bytes={b} GB/s={b / t / 1e3 if t else 0:.1f}")
    if "--timeline" in sys.argv:
        lim = int(sys.argv[sys.argv.index("--timeline") + 1])
        ev = [(s, e, n[:40], "K") for n, s, e, _ in rows]
        if mrows:
            ev += [(r[i_s], r[i_e], str(r[i_k])[:40] if i_k is not None else "copy", "C") for r in mrows]
        ev.sort()
        t0 = ev[0][0] if ev else 0
        for s, e, n, k in ev[:lim]:
            print(f"{k} {(s - t0) / 1e3:12.1f} {(e - s) / 1e3:10.1f} {n}")


if __name__ == "__main__":
    main()
