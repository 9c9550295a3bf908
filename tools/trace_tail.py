"""Kernel timeline after the last launch of a kernel in a rocprofv3 kernel trace: start offset,
gap to the previous kernel and duration of each of the next kernels (the step tail).
    python tools/trace_tail.py TRACE.csv 'StaticLayout<8, 4, 4, 4>, false, 4, false' [--before 2] [--after 14]
"""
import argparse
import csv


def main():
    p = argparse.ArgumentParser()
    p.add_argument("trace")
    p.add_argument("kernel")
    p.add_argument("--before", type=int, default=3)
    p.add_argument("--after", type=int, default=14)
    p.add_argument("--which", type=int, default=-1, help="which launch of the kernel (default the last)")
    a = p.parse_args()
    rows = sorted(csv.DictReader(open(a.trace)), key=lambda r: int(r["Start_Timestamp"]))
    idx = [i for i, r in enumerate(rows) if a.kernel in r["Kernel_Name"]]
    i = idx[a.which]
    t0 = int(rows[i]["Start_Timestamp"])
    prev = None
    for r in rows[max(0, i - a.before): i + a.after + 1]:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        gap = (s - prev) / 1e3 if prev is not None else 0.0
        print("%9.1f us  gap %6.1f  dur %8.1f  %s" % ((s - t0) / 1e3, gap, (e - s) / 1e3,
                                                     r["Kernel_Name"].replace("(anonymous namespace)::", "")[:90]))
        prev = e


if __name__ == "__main__":
    main()
