"""Kernel summary (calls, total / average duration in us, share) of a rocprofv3 SQLite (rocpd) trace database, and
its memory copies: `python tools/rocpd_summary.py <trace_results.db> [out.txt]`."""
import sqlite3
import sys


def main():
    db = sys.argv[1]
    out = open(sys.argv[2], "w") if len(sys.argv) > 2 else sys.stdout
    c = sqlite3.connect(db)
    print(f"{'calls':>6} {'total_ms':>12} {'avg_us':>10} {'share%':>7}  kernel   (top_kernels durations are in us)", file=out)
    for name, calls, tot, avg, pct in c.execute(
            "select name, total_calls, total_duration, average, percentage from top_kernels"):
        print(f"{calls:6d} {tot / 1e3:12.3f} {avg:10.3f} {pct:7.2f}  {name[:160]}", file=out)
    rows = c.execute("select name, count(*), sum(size), sum(duration) from memory_copies group by name").fetchall()
    for name, n, size, dur in rows:
        print(f"memory copy {name}: {n} copies, {size / 1e6:.1f} MB, {dur / 1e3:.1f} us", file=out)


if __name__ == "__main__":
    main()
