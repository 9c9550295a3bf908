"""Sum rocprofv3 --pmc counters per kernel name (tools/gpu/pmc_sq.sh): one line per kernel
with the average per launch of every counter collected in the run directories under argv[1]."""
import collections
import csv
import glob
import re
import sys

acc = collections.defaultdict(lambda: collections.defaultdict(float))
launches = collections.defaultdict(set)
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = re.sub(r"\(anonymous namespace\)::", "", r["Kernel_Name"])
        k = re.sub(r"\((GbArgs|PartArgs|\(anonymous).*", "", k)[:60]
        acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
        launches[(k, r["Counter_Name"])].add(r.get("Dispatch_Id", r.get("Correlation_Id", "")))
for k, cs in sorted(acc.items(), key=lambda kv: -kv[1].get("SQ_BUSY_CYCLES", 0)):
    if not any(x in k for x in ("k_gb", "k_groupby", "k_hist", "k_compose", "k_sel", "k_np_mark", "k_andor")):
        continue
    out = []
    for c, v in sorted(cs.items()):
        n = max(1, len(launches[(k, c)]))
        out.append(f"{c}={v / n:.3g}")
    print(k, " ".join(out))
