"""Turn rocprofv3 `--pmc FETCH_SIZE` / `--pmc WRITE_SIZE` passes into measured HBM bytes per launch.

Reads the counter_collection CSV files rocprofv3 writes, averages each counter over the dispatches of
one kernel and applies the corrections of /opt/skills/guides/MI355X_MICROARCH.md (HBM section): the
counters are in KiB, and on gfx950 FETCH_SIZE reports exactly half the bytes of a wide (16 B/lane)
coalesced streaming read -- the prefilter's posting stream -- so it is doubled.

    python tools/pmc_traffic.py --fetch <csv> [--write <csv>] [--kernel k_prefilter] [--out json]
"""
import argparse
import csv
import json
import os
import sys


def per_dispatch(path: str, counter: str, kernel: str) -> list:
    vals = {}
    with open(path, newline="") as fh:
        for row in csv.DictReader(fh):
            if kernel not in row.get("Kernel_Name", "") or row.get("Counter_Name") != counter:
                continue
            key = row.get("Dispatch_Id") or row.get("Correlation_Id")
            vals[key] = vals.get(key, 0.0) + float(row["Counter_Value"])
    return list(vals.values())


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--fetch", required=True)
    ap.add_argument("--write")
    ap.add_argument("--kernel", default="k_prefilter")
    ap.add_argument("--out")
    a = ap.parse_args()
    f = per_dispatch(a.fetch, "FETCH_SIZE", a.kernel)
    if not f:
        sys.exit(f"no FETCH_SIZE rows for {a.kernel} in {a.fetch}")
    fetch = 2.0 * 1024.0 * sum(f) / len(f)  # KiB -> bytes, x2: gfx950 wide coalesced read
    write = None
    if a.write:
        w = per_dispatch(a.write, "WRITE_SIZE", a.kernel)
        write = 1024.0 * sum(w) / max(1, len(w))
    out = {"kernel": a.kernel, "dispatches": len(f), "fetch_bytes_per_launch": fetch,
           "write_bytes_per_launch": write,
           "prefilter_hbm_bytes_per_launch": fetch + (write or 0.0),
           "correction": "FETCH_SIZE KiB*1024*2 (gfx950 16 B/lane read), WRITE_SIZE KiB*1024",
           "source": [os.path.relpath(p) for p in (a.fetch, a.write) if p]}
    print(json.dumps(out))
    if a.out:
        with open(a.out, "w") as fh:
            json.dump(out, fh, indent=1)


if __name__ == "__main__":
    main()
