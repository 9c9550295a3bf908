"""Regenerate the committed golden fixtures from the reference's own test files.

Run in the build container only (the reference is not present on the GPU box):

    python tests/golden/make_golden.py /root/reference

Produces data only (inputs + expected outputs), never reference source:

* filter_table.json   -- the (filterString, expectedCount, expectError) rows of
                         pkg/columns/filter/filter_test.go:129-248 plus the five records of
                         :46-124 (values only) and the multi-filter case :287-298.
* advisor/*.input/.golden -- pkg/gadgets/advise/networkpolicy/advisor/testdata (data files
                         the reference's own golden test uses, advisor_test.go:23-51).
* ellipsis_table.json -- the (Input, MaxLength, Type, Result) rows of
                         pkg/columns/ellipsis/ellipsis_test.go:21-206.

The group_test.go and sort_test.go expectations are small enough that they are written
out by hand in tests/test_oracle_golden.py, each with its file:line.
"""
import json
import os
import re
import shutil
import sys


def main(ref):
    here = os.path.dirname(os.path.abspath(__file__))
    src = open(os.path.join(ref, "pkg/columns/filter/filter_test.go")).read()
    rows = re.findall(r'\{filterString: "((?:[^"\\]|\\.)*)", expectedCount: (\d+), '
                      r'expectError: (true|false), description: "((?:[^"\\]|\\.)*)"\}', src)
    table = [{"filter": json.loads('"' + f + '"'), "count": int(c), "error": e == "true",
              "description": d} for f, c, e, d in rows]
    records = [
        {"string": "", "v": 7}, {"string": "Demo 123", "v": 1}, {"string": "Demo 234", "v": 2},
        {"string": "Demo 234", "v": 3}, {"string": "Foobar", "v": 2}, None,
    ]
    out = {
        "source": "pkg/columns/filter/filter_test.go:23-298",
        "columns": [["int", "int"], ["int8", "int8"], ["int16", "int16"], ["int32", "int32"],
                    ["int64", "int64"], ["uint", "uint"], ["uint8", "uint8"],
                    ["uint16", "uint16"], ["uint32", "uint32"], ["uint64", "uint64"],
                    ["string", "string"], ["time", "int64"], ["float32", "float32"],
                    ["float64", "float64"], ["unsupported", "struct"]],
        "records": records,
        "rows": table,
        "multi": {"filters": ["int:1", "int8:1", "string:Demo 123"], "count": 1, "int": 1},
    }
    with open(os.path.join(here, "filter_table.json"), "w") as f:
        json.dump(out, f, indent=1)
    adv_src = os.path.join(ref, "pkg/gadgets/advise/networkpolicy/advisor/testdata")
    adv_dst = os.path.join(here, "advisor")
    os.makedirs(adv_dst, exist_ok=True)
    for fn in sorted(os.listdir(adv_src)):
        shutil.copy(os.path.join(adv_src, fn), os.path.join(adv_dst, fn))
    print(f"{len(table)} filter rows, {len(os.listdir(adv_dst))} advisor files")
    ellipsis_table(ref, here)


def ellipsis_table(ref, here):
    src = open(os.path.join(ref, "pkg/columns/ellipsis/ellipsis_test.go")).read()
    rows = re.findall(r'Input:\s+"((?:[^"\\]|\\.)*)",\s*MaxLength:\s+(\d+),\s*Type:\s+(\w+),\s*'
                      r'Result:\s+"((?:[^"\\]|\\.)*)"', src)
    out = {"source": "pkg/columns/ellipsis/ellipsis_test.go:21-206",
           "rows": [{"input": json.loads('"' + i + '"'), "max": int(m), "type": t,
                     "result": json.loads('"' + r + '"')} for i, m, t, r in rows]}
    with open(os.path.join(here, "ellipsis_table.json"), "w") as fh:
        json.dump(out, fh, indent=1, ensure_ascii=False)
    return len(rows)


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "/root/reference")
