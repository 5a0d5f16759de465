"""Per-kernel summary of a rocprofv3 --kernel-trace database (rocpd sqlite): calls,
total / average / min / max ns, share; optionally written as the CSV layout of
rocprofv3 --stats (kernel_stats.csv).  Usage: prof_db.py DB [OUT.csv] [--top N]"""
import csv
import sqlite3
import sys


def summary(db):
    con = sqlite3.connect(db)
    cols = [r[1] for r in con.execute("pragma table_info(kernels)")]
    name = "name" if "name" in cols else "kernel_name"
    rows = con.execute(f"select {name}, start, end from kernels").fetchall()
    agg = {}
    for n, s, e in rows:
        d = e - s
        a = agg.setdefault(n, [0, 0, 1 << 62, 0])
        a[0] += 1
        a[1] += d
        a[2] = min(a[2], d)
        a[3] = max(a[3], d)
    tot = sum(a[1] for a in agg.values()) or 1
    out = sorted(((n, a[0], a[1], a[1] / a[0], a[2], a[3], 100.0 * a[1] / tot) for n, a in agg.items()),
                 key=lambda r: -r[2])
    return out


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    top = int(sys.argv[sys.argv.index("--top") + 1]) if "--top" in sys.argv else 25
    rows = summary(args[0])
    if len(args) > 1 and not args[1].isdigit():
        with open(args[1], "w", newline="") as f:
            w = csv.writer(f, quoting=csv.QUOTE_NONNUMERIC)
            w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs"])
            for r in rows:
                w.writerow([r[0], r[1], r[2], round(r[3], 1), round(r[6], 3), r[4], r[5]])
    for n, c, t, avg, mn, mx, pct in rows[:top]:
        print(f"{pct:6.2f}% {c:6d} calls {avg / 1e3:10.1f} us avg  {n[:110]}")


if __name__ == "__main__":
    main()
