"""Per-kernel launch durations from a rocprofv3 kernel trace: count, mean, median, and the mean of the first
n launches (the bench's warmup + timed launches come first; later side legs may launch the same kernel on
smaller batches).  Usage: python tools/trace_summary.py run_kernel_trace.csv [kernel-substring] [n_first]"""
import csv
import statistics
import sys


def main():
    path = sys.argv[1]
    sub = sys.argv[2] if len(sys.argv) > 2 else ""
    nfirst = int(sys.argv[3]) if len(sys.argv) > 3 else 0
    per = {}
    for r in csv.DictReader(open(path)):
        if sub in r["Kernel_Name"]:
            per.setdefault(r["Kernel_Name"].split("(")[0], []).append(
                (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
    for name, v in sorted(per.items(), key=lambda kv: -sum(kv[1])):
        line = f"{name}: launches {len(v)} mean {statistics.mean(v):.4f} ms median {statistics.median(v):.4f} ms"
        if nfirst:
            f = v[:nfirst]
            line += f" | first {len(f)}: mean {statistics.mean(f):.4f} ms median {statistics.median(f):.4f} ms"
        print(line)


if __name__ == "__main__":
    main()
