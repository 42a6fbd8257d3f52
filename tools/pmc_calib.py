"""Unit factors of the rocprofv3 SQ counters on gfx950, from the calibration kernels of tools/pmc_calib.hip
(measurement only).  Writes profiles/r03/pmc_calib.json, which bench.py's pmc_busy() reads.

    python tools/pmc_calib.py <run_counter_collection.csv> <calib stdout (JSON line)> <out.json>

* kernel cycles = GRBM_GUI_ACTIVE / 8: rocprofv3 sums that counter over the 8 XCDs (MI355X_MICROARCH.md).
* SQ_LDS_IDX_ACTIVE counts LDS-array cycles summed over the CUs: k_lds_read's conflict-free ds_read_b32 reads
  exactly 2 per wave-instruction (the guide's 2 LDS-array cycles), so the factor is 1 cycle per unit.
* SQ_ACTIVE_INST_VALU counts VALU wave-instructions; k_valu (independent v_add_u32, 8 waves per SIMD) saturates
  the VALU issue: its SIMD-cycles per instruction (CUs x 4 SIMDs x kernel cycles / instructions) is the factor
  that makes a saturated kernel read 1.0 busy.
* ds_add_u32 without conflicts (k_lds_atom<1>) issues at this many cycles per wave-instruction per CU although the
  LDS array is busy only 2 of them: the address + data transfer (MI355X_MICROARCH.md §LDS, stores).
"""
import collections
import csv
import json
import sys


def main():
    rows = list(csv.DictReader(open(sys.argv[1], newline="")))
    info = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    n = collections.defaultdict(set)
    for r in rows:
        k = r["Kernel_Name"].replace("void ", "").split("(")[0]
        per[k][r["Counter_Name"]] += float(r["Counter_Value"])
        n[k].add(r["Dispatch_Id"])
    avg = {k: {c: v / len(n[k]) for c, v in d.items()} for k, d in per.items()}
    cus, xcds = info["cus"], 8
    v, lr, la = avg["k_valu"], avg["k_lds_read"], avg["k_lds_atom<1>"]
    cyc_v = v["GRBM_GUI_ACTIVE"] / xcds
    out = dict(
        source=sys.argv[1], program="tools/pmc_calib.hip", cus=cus, xcds=xcds,
        lds_idx_active_cycles_per_unit=1.0,
        lds_idx_active_per_ds_read_b32=lr["SQ_LDS_IDX_ACTIVE"] / lr["SQ_INSTS_LDS"],
        lds_read_b32_array_busy=lr["SQ_LDS_IDX_ACTIVE"] / cus / (lr["GRBM_GUI_ACTIVE"] / xcds),
        active_inst_valu_cycles_per_unit=cus * 4 * cyc_v / v["SQ_ACTIVE_INST_VALU"],
        valu_insts_per_active_unit=v["SQ_INSTS_VALU"] / v["SQ_ACTIVE_INST_VALU"],
        ds_add_u32_cycles_per_instr_per_cu=cus * (la["GRBM_GUI_ACTIVE"] / xcds) / la["SQ_INSTS_LDS"],
        ds_add_u32_array_cycles_per_instr=la["SQ_LDS_IDX_ACTIVE"] / la["SQ_INSTS_LDS"],
        conflict32_array_cycles_per_instr=avg["k_lds_atom<32>"]["SQ_LDS_IDX_ACTIVE"] / avg["k_lds_atom<32>"]["SQ_INSTS_LDS"],
        effective_clock_ghz_k_valu=cyc_v / (info["kernels"]["k_valu"]["ms"] * 1e6),
        calib_stdout=info)
    json.dump(out, open(sys.argv[3], "w"), indent=1)
    print(json.dumps({k: v for k, v in out.items() if k != "calib_stdout"}, indent=1))


if __name__ == "__main__":
    main()
