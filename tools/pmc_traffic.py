"""Per-launch HBM traffic of one kernel from rocprofv3 PMC passes.

    python tools/pmc_traffic.py --fetch DIR_FETCH --write DIR_WRITE --kernel k_groupby \
        --config '{"events": 100000000, "keys": 1000000, "zipf": 1.1}' --out profiles/r01/traffic.json

DIR_FETCH / DIR_WRITE are the `-d` directories of two separate
`rocprofv3 --pmc FETCH_SIZE --kernel-trace ...` and `--pmc WRITE_SIZE ...` runs (one
counter per pass, MI355X_MICROARCH.md §HBM).  FETCH_SIZE and WRITE_SIZE are in KiB.
On gfx950 FETCH_SIZE counts 64 B per 128-B request of wide streaming reads, so it is
doubled (the guide's correction).  WRITE_SIZE is taken as reported.
bench.py reads the output and reports it as roofline.traffic when its config matches.
"""
import argparse
import csv
import glob
import json
import os


def _values(d, counter, kernel, exclude=()):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no counter_collection.csv under {d}")
    vals = []
    for f in files:
        with open(f) as fh:
            for row in csv.DictReader(fh):
                name = row["Kernel_Name"]
                if row["Counter_Name"] == counter and kernel in name and not any(x in name for x in exclude):
                    vals.append(float(row["Counter_Value"]))
    if not vals:
        raise SystemExit(f"no {counter} rows for kernel {kernel!r} in {d}")
    return vals


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--fetch", required=True)
    p.add_argument("--write", required=True)
    p.add_argument("--kernel", default="k_groupby")
    p.add_argument("--anchor", default=None,
                   help="a chain of kernels per update (the partitioned form): sum every --kernel match "
                        "and divide by the launches of this one")
    p.add_argument("--extra", action="append", default=[],
                   help="another kernel of the same step whose per-launch traffic is added (e.g. k_np_mark)")
    p.add_argument("--exclude", action="append", default=[],
                   help="skip kernels whose name holds this (e.g. the group-by's SAMPLE instance, ', true>')")
    p.add_argument("--config", required=True)
    p.add_argument("--out", required=True)
    a = p.parse_args()
    f = _values(a.fetch, "FETCH_SIZE", a.kernel, a.exclude)
    w = _values(a.write, "WRITE_SIZE", a.kernel, a.exclude)
    nf, nw = len(f), len(w)
    if a.anchor:
        nf = len(_values(a.fetch, "FETCH_SIZE", a.anchor))
        nw = len(_values(a.write, "WRITE_SIZE", a.anchor))
    fetch_b = 2.0 * 1024.0 * sum(f) / nf
    write_b = 1024.0 * sum(w) / nw
    for k in a.extra:
        ef, ew = _values(a.fetch, "FETCH_SIZE", k), _values(a.write, "WRITE_SIZE", k)
        fetch_b += 2.0 * 1024.0 * sum(ef) / len(ef)
        write_b += 1024.0 * sum(ew) / len(ew)
    out = {"kernel": a.kernel, "extra": a.extra, "config": json.loads(a.config),
           "fetch_bytes_per_launch": fetch_b, "write_bytes_per_launch": write_b,
           "traffic_bytes_per_launch": fetch_b + write_b, "launches": [nf, nw],
           "anchor": a.anchor, "exclude": a.exclude,
           "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes; "
                     "FETCH_SIZE x2 (gfx950 128-B requests tallied at 64 B); KiB -> bytes"}
    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    with open(a.out, "w") as fh:
        json.dump(out, fh, indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
