"""Per-kernel totals of a rocprofv3 --pmc counter CSV (measurement aid; runs on the GPU box so that only the small
summary travels back).

    python tools/pmc_agg.py <run_counter_collection.csv> <out.json> [kernel-name-prefix ...]

out.json: {kernel: {"dispatches": n, "mean_us": ..., counter: total over the kernel's dispatches, ...}}, kernel names
with the argument list and `void ` / `uc::` stripped.  With prefixes, only kernels starting with one of them.
"""
import collections
import csv
import json
import sys


def main() -> None:
    path, out = sys.argv[1], sys.argv[2]
    want = sys.argv[3:]
    tot = collections.defaultdict(lambda: collections.defaultdict(float))
    seen = collections.defaultdict(set)
    dur = collections.defaultdict(float)
    for r in csv.DictReader(open(path, newline="")):
        k = r["Kernel_Name"].replace("void ", "").split("(")[0].replace("uc::", "")
        if want and not any(k.startswith(w) for w in want):
            continue
        tot[k][r["Counter_Name"]] += float(r["Counter_Value"])
        d = r["Dispatch_Id"]
        if d not in seen[k]:
            seen[k].add(d)
            dur[k] += float(r["End_Timestamp"]) - float(r["Start_Timestamp"])
    res = {}
    for k, v in tot.items():
        n = len(seen[k])
        res[k] = dict(dispatches=n, mean_us=dur[k] / n / 1e3 if n else None, **v)
    json.dump(res, open(out, "w"), indent=1, sort_keys=True)
    print(f"{len(res)} kernels -> {out}")


if __name__ == "__main__":
    main()
