"""Aggregate rocprofv3 counter_collection / kernel_stats CSVs into a small per-kernel JSON for profiles/.

    python tools/pmc_summary.py <out.json> <counter_collection.csv>...
"""
import collections
import csv
import json
import sys


def main() -> None:
    out, paths = sys.argv[1], sys.argv[2:]
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for p in paths:
        for r in csv.DictReader(open(p, newline="")):
            k = r["Kernel_Name"].split("(")[0]
            agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
            disp[k].add((p, r["Dispatch_Id"]))
    res = {k: {"dispatches_per_pass": len(disp[k]) // max(1, len(paths)), "totals": dict(v)}
           for k, v in sorted(agg.items(), key=lambda kv: -sum(kv[1].values()))}
    json.dump({"sources": paths, "kernels": res}, open(out, "w"), indent=1)


if __name__ == "__main__":
    main()
