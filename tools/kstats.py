"""Per-step kernel time from a rocprofv3 --stats CSV (kernel_stats): calls and ms per step by kernel family."""
import csv
import sys


def main(path, steps):
    agg = {}
    for r in csv.DictReader(open(path)):
        n = r["Name"].replace("void ", "").split("(")[0]
        if "align" in n:
            n = n.split("<")[0]
        a = agg.setdefault(n, [0, 0.0])
        a[0] += int(r["Calls"])
        a[1] += float(r["TotalDurationNs"])
    tot = sum(t for _, t in agg.values())
    for n, (c, t) in sorted(agg.items(), key=lambda x: -x[1][1]):
        print(f"{n[:44]:44s} calls/step {c / steps:8.1f}  ms/step {t / steps / 1e6:8.2f}  avg us {t / max(c, 1) / 1e3:8.1f}")
    print(f"total ms/step {tot / steps / 1e6:.2f}")


if __name__ == "__main__":
    main(sys.argv[1], float(sys.argv[2]) if len(sys.argv) > 2 else 1.0)
