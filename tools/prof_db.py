"""Summaries of a rocprofv3 rocpd database (kernels + memory copies):
per-name count, total and average duration, plus one step's timeline.
Usage: python tools/prof_db.py <run_results.db> [--last N]"""
import sqlite3
import sys


def main(path, last=0):
    c = sqlite3.connect(path)
    kcols = [r[1] for r in c.execute("pragma table_info(kernels)")]
    name = "kernel_name" if "kernel_name" in kcols else "name"
    rows = c.execute(f"select {name}, start, end from kernels").fetchall()
    try:
        mrows = c.execute("select 'COPY ' || coalesce(name, 'memcpy') || ' ' || size, start, end "
                          "from memory_copies").fetchall()
    except sqlite3.Error:
        mrows = []
    agg = {}
    for n, s, e in rows + mrows:
        key = n.split("(")[0][:90] if not n.startswith("COPY") else " ".join(n.split()[:2])
        a = agg.setdefault(key, [0, 0.0])
        a[0] += 1
        a[1] += (e - s) / 1e6
    tot = sum(v[1] for v in agg.values())
    print(f"{'name':92s} {'calls':>6s} {'total_ms':>10s} {'avg_ms':>9s} {'pct':>6s}")
    for k, (n, t) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        print(f"{k:92s} {n:6d} {t:10.3f} {t / n:9.4f} {100 * t / tot:6.2f}")
    if last:
        ev = sorted(rows + mrows, key=lambda r: r[1])[-last:]
        t0 = ev[0][1]
        for n, s, e in ev:
            print(f"{(s - t0) / 1e3:10.1f}us {(e - s) / 1e3:9.1f}us  {n.split('(')[0][:100]}")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[3]) if len(sys.argv) > 3 and sys.argv[2] == "--last" else 0)
