"""Timeline window of a rocprofv3 kernel trace around the n-th launch of a kernel: start / end / duration (us,
relative to that launch's start), queue, grid size and name of every kernel that starts in the window.
Usage: python tools/trace_window.py run_kernel_trace.csv KERNEL_SUBSTRING [n=20] [before_us=250] [after_us=1100]"""
import csv
import sys


def main():
    path, sub = sys.argv[1], sys.argv[2]
    n = int(sys.argv[3]) if len(sys.argv) > 3 else 20
    before = float(sys.argv[4]) if len(sys.argv) > 4 else 250.0
    after = float(sys.argv[5]) if len(sys.argv) > 5 else 1100.0
    ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0],
                 r["Queue_Id"], r["Grid_Size_X"]) for r in csv.DictReader(open(path)))
    hits = [e for e in ev if sub in e[2]]
    t0 = hits[min(n, len(hits) - 1)][0]
    for s, e, name, q, g in ev:
        if t0 - before * 1e3 < s < t0 + after * 1e3:
            print(f"{(s - t0) / 1e3:9.1f} {(e - t0) / 1e3:9.1f} {(e - s) / 1e3:8.1f}  q{q} grid {g:>7} {name[-60:]}")


if __name__ == "__main__":
    main()
