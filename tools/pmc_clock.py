"""Effective shader clock of one kernel during a rocprofv3 PMC run (measurement aid).

rocprofv3 --pmc GRBM_GUI_ACTIVE serialises dispatches; its counter CSV holds, per dispatch, GRBM_GUI_ACTIVE (summed over
the 8 XCDs) and the dispatch's start / end timestamps.  Clock = GRBM_GUI_ACTIVE / 8 / duration
(MI355X_MICROARCH.md "DVFS give-back": within 3 % of the in-kernel clock for dispatches of 10 ms or more, reads high
below ~0.3 ms).  Dispatches shorter than --min-us are skipped.

    python tools/pmc_clock.py <run_counter_collection.csv> <kernel name prefix> [out.json]
"""
import csv
import json
import sys


def clock(path, kernel, min_us=300.0, xcds=8):
    cyc, ns, n = 0.0, 0.0, 0
    seen = set()
    for r in csv.DictReader(open(path, newline="")):
        if r["Counter_Name"] != "GRBM_GUI_ACTIVE":
            continue
        name = r["Kernel_Name"].replace("void ", "").split("(")[0].split("::")[-1]
        if not name.startswith(kernel) or r["Dispatch_Id"] in seen:
            continue
        seen.add(r["Dispatch_Id"])
        d = float(r["End_Timestamp"]) - float(r["Start_Timestamp"])
        if d < min_us * 1e3:
            continue
        cyc += float(r["Counter_Value"]) / xcds
        ns += d
        n += 1
    return dict(kernel=kernel, dispatches=n, clock_ghz=cyc / ns if ns else None, mean_us=ns / n / 1e3 if n else None,
                source=path, note="GRBM_GUI_ACTIVE / 8 XCDs / dispatch duration, dispatches serialised by the PMC run")


if __name__ == "__main__":
    out = clock(sys.argv[1], sys.argv[2])
    print(json.dumps(out, indent=1))
    if len(sys.argv) > 3:
        json.dump(out, open(sys.argv[3], "w"), indent=1)
