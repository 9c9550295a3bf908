"""Average duration (us) per kernel whose name contains each given substring, from a rocprofv3
kernel trace CSV:  python tools/kavg.py TRACE.csv 'k_gbp_c<' 'k_gbp_b<' ..."""
import csv
import sys


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    out = []
    for pat in sys.argv[2:]:
        d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows if pat in r["Kernel_Name"]]
        out.append("%s n=%d avg=%.1f us" % (pat, len(d), sum(d) / len(d) if d else float("nan")))
    print(" | ".join(out))


if __name__ == "__main__":
    main()
