"""Per-kernel duration summary from a rocprofv3 SQLite output (run_results.db):
    python tools/kstats_db.py path/to/run_results.db [--timeline N]
Prints name, calls, total / average / min / max duration (us) and share of the summed time, as
the --stats CSV would; --timeline N prints the last N dispatches (start offset, duration,
stream) to read overlap and gaps."""
import sqlite3
import sys


def main():
    db = sqlite3.connect(sys.argv[1])
    cols = [r[1] for r in db.execute("pragma table_info(kernels)")]
    name = "kernel_name" if "kernel_name" in cols else "name"
    rows = db.execute(f"select {name}, start, end, stream_id, queue_id from kernels order by start").fetchall() \
        if "stream_id" in cols else \
        [(r[0], r[1], r[2], None, None) for r in db.execute(f"select {name}, start, end from kernels order by start")]
    agg = {}
    for n, s, e, *_ in rows:
        d = (e - s) / 1e3
        a = agg.setdefault(n.split("(")[0][:60], [0, 0.0, 1e30, 0.0])
        a[0] += 1
        a[1] += d
        a[2] = min(a[2], d)
        a[3] = max(a[3], d)
    tot = sum(a[1] for a in agg.values())
    print(f"{'kernel':60s} {'calls':>6s} {'total_us':>10s} {'avg_us':>9s} {'min':>8s} {'max':>8s} {'%':>5s}")
    for n, a in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        print(f"{n:60s} {a[0]:6d} {a[1]:10.1f} {a[1] / a[0]:9.2f} {a[2]:8.2f} {a[3]:8.2f} {100 * a[1] / tot:5.1f}")
    if "--timeline" in sys.argv:
        k = int(sys.argv[sys.argv.index("--timeline") + 1])
        t0 = rows[-k][1]
        for n, s, e, st, q in rows[-k:]:
            print(f"{(s - t0) / 1e3:10.1f} {(e - s) / 1e3:8.1f} q{q} s{st} {n.split('(')[0][:50]}")


if __name__ == "__main__":
    main()
