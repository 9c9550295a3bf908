"""Sum rocprofv3 PMC counters per kernel over one or more `-d` output directories.

    python tools/pmc_summary.py --kernel k_groupby DIR [DIR ...]
Prints {counter: value per launch} as JSON (diagnostics; not part of the product path)."""
import argparse
import csv
import glob
import json
import os
from collections import defaultdict


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--kernel", default="k_groupby")
    p.add_argument("--per-dispatch", action="store_true", help="one value per launch, in dispatch order")
    p.add_argument("dirs", nargs="+")
    a = p.parse_args()
    if a.per_dispatch:
        per = defaultdict(dict)
        for d in a.dirs:
            for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
                with open(f) as fh:
                    for row in csv.DictReader(fh):
                        if a.kernel in row["Kernel_Name"]:
                            k = int(row.get("Dispatch_Id") or row.get("Correlation_Id") or 0)
                            per[row["Counter_Name"]][k] = per[row["Counter_Name"]].get(k, 0.0) + float(row["Counter_Value"])
        print(json.dumps({c: [v[k] for k in sorted(v)] for c, v in sorted(per.items())}))
        return
    tot, launches = defaultdict(float), defaultdict(set)
    for d in a.dirs:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            with open(f) as fh:
                for row in csv.DictReader(fh):
                    if a.kernel in row["Kernel_Name"]:
                        tot[row["Counter_Name"]] += float(row["Counter_Value"])
                        launches[row["Counter_Name"]].add(row.get("Dispatch_Id", row.get("Correlation_Id", "")))
    print(json.dumps({k: v / max(1, len(launches[k])) for k, v in sorted(tot.items())}))


if __name__ == "__main__":
    main()
