"""Merge tools/bench_rows.py's JSON with the rocprofv3 kernel stats of the same run into profiles/.

    python tools/rows_summary.py <rows.json> <run_kernel_stats.csv> <out.json>
Per row: the kernels' average duration per call and the algorithmic bytes a call moves (stated below),
against the 8 TB/s HBM peak (byte work, no MFMA).
"""
import csv
import json
import sys

HBM = 8000.0


def main() -> None:
    rows_path, stats_path, out = sys.argv[1:4]
    d = json.load(open(rows_path))
    ks = {r["Name"].split("(")[0]: float(r["AverageNs"]) * 1e-9 for r in csv.DictReader(open(stats_path))}
    f1, f3, f4 = d["rows"]

    def put(row, name, t, b, note):
        row["kernel"] = dict(name=name, avg_ms=t * 1e3, algorithmic_bytes=b, achieved_gbs=b / t / 1e9, peak_gbs=HBM,
                             frac=b / t / 1e9 / HBM, note=note)
    n = f1["reads"]
    k1 = "uc::k_extract_win" if "uc::k_extract_win" in ks else "uc::k_extract"
    put(f1, k1, ks[k1], n * (73 + 68 + 2 + 24),
        "per read: its two gathered adapter windows (141 B), their lengths (2 B) and the results (24 B)")
    t3 = sum(v for k, v in ks.items() if k.startswith("uc::k_ov_"))
    put(f3, "k_ov_* (hash, insert, verify, scan, fill, pairs)", t3, f3["umis"] * (64 * 2 + 32),
        "per UMI: its 64 B read twice (hash, verify) + 4 x 8 B of hash/slot traffic; the join kernels of one call")
    kept = f4["counts"][1] - f4["counts"][2] - f4["counts"][3]
    put(f4, "k_bam_classify + k_bam_emit", ks["uc::k_bam_classify"] + ks["uc::k_bam_emit"],
        f4["records"] * (36 + 11 + 4 + 300 + 600) + kept * (1 + 10 + 10 + 600 + 1),
        "inflated record bytes read once + the FASTA bytes written for kept records")
    d["kernel_stats_source"] = stats_path
    json.dump(d, open(out, "w"), indent=1)
    for r in d["rows"]:
        print(r["row"], round(r["gpu_wall_s"] * 1e3, 2), "ms wall;", r["kernel"]["name"], round(r["kernel"]["avg_ms"], 3),
              "ms,", round(r["kernel"]["achieved_gbs"], 1), "GB/s")


if __name__ == "__main__":
    main()
