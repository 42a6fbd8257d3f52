"""Benchmark: UMIs clustered/s (+ GCUPS) of the vsearch --cluster_fast drop-in on MI355X.

Workloads (BASELINE.json configs):
  --config 2 (default; the headline): one synthetic region bin of 2M dual-UMI reads per GPU (seed 1002 on
      rank 0, 1002*1_000_003 + rank on other ranks: weak scaling, one independent bin per GPU, no collective
      on the data path), --id 0.90, round-1 scoring (vsearch_umi_cluster.py:44-50).
  --config 3: 10M reads over 24 barcodes x 40 Zipf(1.1) region bins, LPT-sharded over the ranks (strong
      scaling: the node clusters the fixed 10M), round 1 (--id 0.93, run_config.json:16).
  --config 4: 70M reads, 24 barcodes x 40 Zipf bins, both rounds: round 1 on every bin, round 2 (default
      scoring, --id 0.97) on the round-1 consensus UMIs of every bin (tcr_consensus.py:190-267, :376-446).
  --config 5: the long-UMI high-error stress bin (300k ~96-nt UMIs, 15 % indels, >1k-member clusters).
A step = one full pass of the hot path over the rank's bins, the raw records staged in HBM beforehand
(umiclust_stage, untimed): vsearch's load-time work (umiclust_prepare: length filter and stable length sort, K1
DUST / 4-bit codes / unique 8-mers of both strands), greedy blocks of K2 prefilter + K3 walk alignment + host
resolution, K3T traceback for members, K4 consensus, and the result download.  Config 2 (N = 1) also runs the
file leg (`e2e`, on by default, --no-e2e skips it): the same bin written as a FASTA with 1,500-nt `seq=` reads,
then read FASTA -> cluster -> files written (umiclust_run_fasta, the reference's boundary:
vsearch_umi_cluster.py:17-56) and the fused drop-in (umiclust_run_fasta_parse); each writer is followed by a
replay of the same files (sizes, contiguous thread split, one streamed file; no formatting: tools/io_probe.c
io_probe_replay) as a reference point, write_replay_ratio = replay seconds / writer seconds.  It is NOT a bound:
the replay does not reissue the writer's exact system calls (open flags, directory order, chunking) and runs
against a filesystem the writer has just filled and emptied, so the ratio can exceed 1 (round 4: 1.10).

    python bench.py --gpus N --steps K --warmup W [--config 2|3|4|5] [--no-e2e]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...
--gpus N without a launcher (no WORLD_SIZE in the environment) starts N ranks itself through
torch.distributed.run before anything touches a GPU; under a launcher WORLD_SIZE must equal N.
"""
from __future__ import annotations

import argparse
import csv
import ctypes
import glob
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "ont-tcrconsensus_amd"))

METRIC = "UMIs clustered/sec + banded-NW GCUPS (whole node, 1/2/4/8 MI355X)"
HBM_PEAK_GBS = 8000.0      # MI355X_MICROARCH.md chip table (spec)
L2_GATHER_GBS = 18800.0    # MI355X_MICROARCH.md "Indexed rows: gather into LDS", L2-served rows, upper end
# integer VALU issue ceiling: 256 CUs x 4 SIMDs x 32 lanes per clock x 2.4 GHz (MI355X_MICROARCH.md
# "v_fma_f32 (wave64) 2 cyc (SIMD-32)"); lane-instructions per second
VALU_LANE_OPS = 256 * 4 * 32 * 2.4e9
# VALU lane-instructions per alignment cell of k_align_pk, measured: SQ_INSTS_VALU x 64 / cells computed
# (profiles/r03/pmc_align_valu.json, a rocprofv3 --pmc pass over the config-2 bench; round 2: 17.9)
def _align_valu_per_cell() -> float:
    p = os.path.join(ROOT, "profiles", "r03", "pmc_align_valu.json")
    return json.load(open(p))["valu_lane_instrs_per_computed_cell"] if os.path.exists(p) else 17.9


ALIGN_VALU_PER_CELL = _align_valu_per_cell()


def _prof(*names: str) -> str:
    """The newest committed measurement among profiles/<round>/<name> (round 6 first, then round 5)."""
    for rnd in ("r06", "r05"):
        for n in names:
            p = os.path.join(ROOT, "profiles", rnd, n)
            if os.path.exists(p):
                return p
    return os.path.join(ROOT, "profiles", "r05", names[-1])


def align_issue_ceiling() -> dict | None:
    """The aligner's ceiling at the measured issue cost of its own instruction mix: the column loop of
    k_align_pk<64> (tools/isa_mix.py -> profiles/r06/align_issue_mix_pk64.json: VOP2, packed VOP3P and other VOP3
    instructions per step of 64 cells per lane) priced with tools/valu_rate.hip's cycles per wave-instruction per
    SIMD at 4 waves per SIMD (profiles/r05/valu_rate.jsonl: 8-byte VOP3/VOP3P encodings issue ~1.5x slower than
    4-byte VOP2 ones), in the probe's own 2.4 GHz-nominal cycle units."""
    mp = _prof("align_issue_mix_pk64.json")
    rp = os.path.join(ROOT, "profiles", "r05", "valu_rate.jsonl")
    if not (os.path.exists(mp) and os.path.exists(rp)):
        return None
    mix = json.load(open(mp))
    rates = [json.loads(x) for x in open(rp) if x.strip()]
    cyc = lambda ops: sum(r["cycles_per_instr_at_2.4GHz"] for r in rates  # noqa: E731
                          if r["op"] in ops and r["chains"] == 8 and r["waves_per_simd"] == 4) / len(ops)
    c2 = cyc(["v_add_u32"])
    c3p = cyc(["v_pk_sub_i16", "v_pk_max_i16", "v_pk_ashrrev_i16", "v_pk_mad_u16"])
    c3 = cyc(["v_add3_u32", "v_and_or_b32", "v_bitop3_b32"])
    step = mix["vop2"] * c2 + mix["vop3p"] * c3p + mix["vop3"] * c3
    cells_per_step = 64 * 64  # 64 lanes x (32 packed rows = 64 cells)
    gcups = 1024 * 2.4e9 * cells_per_step / step / 1e9
    return dict(ceiling_gcups=gcups, cycles_per_step=step, cycles_vop2=c2, cycles_vop3p=c3p, cycles_vop3=c3,
                mix={k: mix[k] for k in ("vop2", "vop3p", "vop3")},
                source=[os.path.relpath(mp, ROOT), os.path.relpath(rp, ROOT)])


def cpu_baseline_bins(bins, identity: float, lens, budget_s: float = 20.0, preset: int = 1) -> dict:
    """The C oracle (oracle/) over whole bins on every host core the process may use (the reference runs one
    vsearch process per bin, utils.py:56-63): one thread per core pulls bins largest first until ~budget_s of
    wall time, each bin clustered whole; UMIs/s = the kept UMIs of the finished bins / wall time."""
    import concurrent.futures as cf
    import threading
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import orc
    cores = _host_cores()
    order = sorted(bins, key=lambda b: -b.umis.n)
    orc.cluster(orc.params(preset, identity, *lens), order[-1].umis.as_list())  # library load / tables
    lock = threading.Lock()
    state = dict(next=0, kept=0, reads=0, done=0)
    t0 = time.perf_counter()

    def worker(_):
        while True:
            with lock:
                if state["next"] >= len(order) or time.perf_counter() - t0 > budget_s:
                    return
                b = order[state["next"]]
                state["next"] += 1
            r = orc.cluster(orc.params(preset, identity, *lens), b.umis.as_list())
            with lock:
                state["kept"] += r["stats"]["kept"]
                state["reads"] += b.umis.n
                state["done"] += 1

    with cf.ThreadPoolExecutor(cores) as ex:
        list(ex.map(worker, range(cores)))
    t = time.perf_counter() - t0
    return dict(value=state["kept"] / t if t else 0.0, unit="UMIs/s", cores=cores, kind="port",
                sample=f"{state['done']} of {len(order)} whole bins, largest first ({state['reads']} reads), clustered "
                       f"by the C oracle restatement on {cores} threads (one bin per thread), {t:.1f} s wall; the "
                       f"largest bins are the slowest per UMI, so the full set runs faster per UMI on the CPU",
                seconds=t, n_kept=state["kept"])


def cpu_baseline_prefix(umis, n_sample: int, identity: float, lens, preset: int = 1) -> dict:
    """The C oracle (oracle/, 1 thread) on the first n_sample reads of the bin."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import orc
    seqs = umis.as_list()[:n_sample]
    t0 = time.perf_counter()
    r = orc.cluster(orc.params(preset, identity, *lens), seqs)
    dt = time.perf_counter() - t0
    return dict(value=r["stats"]["kept"] / dt, unit="UMIs/s", cores=1, kind="port",
                sample=f"first {n_sample} reads of the rank-0 bin ({r['stats']['kept']} kept, "
                       f"{r['n_clusters']} clusters) clustered by the C oracle restatement, 1 thread, "
                       f"{dt:.1f} s; CPU cost grows ~N*C, so the full bin is slower per UMI (full-bin oracle "
                       f"time: tests/golden/oracle_config2.json oracle_seconds)",
                seconds=dt, n_kept=r["stats"]["kept"])


def _host_cores() -> int:
    return min(16, len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1))


def cpu_baseline_threads(umis, n_sample: int, identity: float, lens, preset: int = 1, threads: int = 25) -> dict:
    """The C oracle in vsearch's multi-threaded mode (policy O4, cluster_core_parallel restated: rounds of
    `threads` queries searched against the index frozen at the round's start, then re-checked in order) with the
    round's searches on one OpenMP worker per host core (at most `threads`) -- how the reference runs vsearch
    (--threads >= 25, vsearch_umi_cluster.py:33-34, utils.py:56-63), the same policy as the GPU line -- on the
    first n_sample reads of the bin."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import orc
    cores = min(_host_cores(), threads)
    seqs = umis.as_list()[:n_sample]
    p = orc.params(preset, identity, *lens)
    p.threads, p.policy_threads = threads, 1
    old = os.environ.get("ORC_WORKERS")
    os.environ["ORC_WORKERS"] = str(cores)
    try:
        t0 = time.perf_counter()
        r = orc.cluster(p, seqs)
        dt = time.perf_counter() - t0
    finally:
        if old is None:
            os.environ.pop("ORC_WORKERS", None)
        else:
            os.environ["ORC_WORKERS"] = old
    return dict(value=r["stats"]["kept"] / dt, unit="UMIs/s", cores=cores, kind="port",
                sample=f"first {n_sample} reads of the rank-0 bin ({r['stats']['kept']} kept, {r['n_clusters']} "
                       f"clusters) clustered by the C oracle restatement in vsearch's --threads {threads} mode (policy "
                       f"O4: rounds of {threads} queries, the round's searches on {cores} OpenMP workers), {dt:.1f} s; "
                       f"CPU cost grows ~N*C, so the full bin is slower per UMI",
                seconds=dt, n_kept=r["stats"]["kept"])


def full_bin_cpu_reference(config: int, threads: int, identity: float) -> dict | None:
    """The oracle's measured wall time over the whole bin of `config` (tests/golden/make_oracle_golden.py), under the
    policy `threads` selects: O4 (vsearch --threads n, oracle_o4.json: the round's searches on `oracle_workers` OpenMP
    threads) or the sequential definition (oracle_config<N>.json, 1 thread)."""
    gold = os.path.join(ROOT, "tests", "golden")
    path = os.path.join(gold, "oracle_o4.json") if threads > 1 else os.path.join(gold, f"oracle_config{config}.json")
    if not os.path.exists(path):
        return None
    for name, g in sorted(json.load(open(path)).items()):
        if g.get("config") == config and g.get("scale") == 1.0 and "oracle_seconds" in g and "n_bins" not in g \
                and abs(g.get("identity", -1) - identity) < 1e-9 and g.get("preset") == 1:
            workers = g.get("oracle_workers", g.get("oracle_threads", 1))
            return dict(case=name, source=os.path.relpath(path, ROOT), seconds=g["oracle_seconds"],
                        umis_per_s=g["n_reads"] / g["oracle_seconds"], n_reads=g["n_reads"],
                        policy=policy_name(g.get("T", 1) if threads > 1 else 1),
                        workers=workers, host_cpu=g.get("host_cpu"),
                        note="the C oracle over the whole bin when it generated the golden (the builder's container, "
                             f"{workers} worker thread(s)), not this box")
    return None


def roofline(stats: list, config: int, traffic_json: str, tl_union: dict | None = None) -> tuple[dict, dict]:
    """The prefilter's counting kernel k_pf_count against the L2-served gather rate (its postings stay
    L2-resident: parts = XCDs), with the HBM fraction as a side figure; k_align against the integer VALU
    issue ceiling.  The kernel's launch time is its own HIP-event bracket on the stream it runs on
    (umiclust_stats.t_count_s / n_count_launches); the postings are every posting the prefilter streamed.
    With several lanes on the GPU (configs 3/4) the brackets of different lanes overlap, so `frac` charges each
    launch the time it shared; `device` divides by the union of the brackets over the timed steps
    (umiclust_timeline: the time some launch of the kernel held the device)."""
    t_cnt = sum(s.get("t_count_s", 0.0) for s in stats)
    n_cnt = sum(s.get("n_count_launches", 0) for s in stats)
    t_pf = sum(s["t_prefilter_s"] for s in stats)
    t_al = sum(s["t_align_s"] for s in stats)
    n_blocks = sum(s["n_blocks"] for s in stats)
    if n_cnt == 0:  # multi-segment bins only: the full kernel counts
        t_cnt, n_cnt = t_pf, n_blocks
    # algorithmic postings = every posting of the query-strands' k-mer lists (what vsearch's count touches, as
    # `cells` is the full rectangle however the kernel bands): the ones streamed + the deferred lists' (frequent
    # k-mers whose matches the kernel adds per surviving target: PrefilterArgs::fmask)
    streamed = sum(s["kmer_postings"] for s in stats)
    deferred = sum(s.get("kmer_postings_deferred", 0) for s in stats)
    pf_bytes = (streamed + deferred) * 2
    traffic = None
    if os.path.exists(traffic_json):
        try:
            tj = json.load(open(traffic_json))
            if tj.get("config", 2) == config and tj.get("kernel") == "k_pf_count":  # PMC traffic is per workload
                traffic = tj.get("prefilter_hbm_bytes_per_launch")
        except Exception:
            traffic = None
    # SURVEY 8d's prefilter bytes: postings x 4 B + C x 2 B of counter traffic per query-strand (C = centroids
    # indexed).  This build's postings are u16 (2 B) and its counters u8 in LDS, so `achieved` counts 2 B per posting
    # and no counter bytes; `survey` restates the same launches by SURVEY's formula against HBM's 8 TB/s.
    counter_cells = sum(s.get("counter_cells", 0) for s in stats)
    survey_bytes = streamed * 4 + counter_cells * 2
    achieved = pf_bytes / t_cnt / 1e9 if t_cnt > 0 else 0.0
    roof = dict(kernel="k_pf_count", bound="l2", achieved=achieved, peak=L2_GATHER_GBS, unit="GB/s",
                frac=achieved / L2_GATHER_GBS, traffic=traffic,
                hbm_frac=achieved / HBM_PEAK_GBS, hbm_peak=HBM_PEAK_GBS,
                bytes_per_launch=pf_bytes / max(1, n_cnt), launches=n_cnt,
                streamed_bytes_per_launch=2 * streamed / max(1, n_cnt),
                deferred_share=deferred / max(1, streamed + deferred),
                streamed_frac=(2 * streamed / t_cnt / 1e9 if t_cnt > 0 else 0.0) / L2_GATHER_GBS,
                avg_launch_ms=1e3 * t_cnt / max(1, n_cnt),
                prefilter_ms_per_block=1e3 * t_pf / max(1, n_blocks),
                note="2 B per u16 posting of the query-strands' k-mer lists (algorithmic: streamed + deferred, "
                     "the deferred lists' share in deferred_share; streamed_frac counts only what was streamed; "
                     "postings served from the XCD-partitioned L2; measured HBM "
                     "traffic is `traffic`); peak = L2-served gather rate, MI355X_MICROARCH.md (1,152-B rows). "
                     "What binds it is instruction issue, not bytes: VALU and LDS-atomic issue per posting "
                     "(profiles/r02/pmc_pf_count_c2.json)")
    # against the LDS atomic ceiling (what binds it: LDS array busy 0.69, 60 % of it bank-conflict replays): one
    # ds_add_u32 wave-instruction per 64 postings streamed, 4.32 cycles per wave-instruction per CU at best
    # (tools/pmc_calib.hip, conflict-free), at the clock measured during the kernel (GRBM_GUI_ACTIVE / 8 / duration of
    # its dispatches in a PMC run: tools/pmc_clock.py)
    cal_p = os.path.join(ROOT, "profiles", "r03", "pmc_calib.json")
    clk_p = _prof("pmc_clock_k_pf_count.json")
    if counter_cells and t_cnt > 0:
        roof["survey"] = dict(bytes_per_launch=survey_bytes / max(1, n_cnt), counter_cells=counter_cells,
                              achieved=survey_bytes / t_cnt / 1e9, frac_hbm=survey_bytes / t_cnt / 1e9 / HBM_PEAK_GBS,
                              note="SURVEY 8d: postings x 4 B + C x 2 B per query-strand, C = centroids indexed at the "
                                   "launch; the build stores u16 postings and u8 counters, so `achieved` uses 2 B; the "
                                   "counters live in LDS, so this rate exceeds HBM's 8 TB/s (frac_hbm > 1) by design")
    if os.path.exists(cal_p) and os.path.exists(clk_p) and n_cnt:
        cal, clk = json.load(open(cal_p)), json.load(open(clk_p))
        atom = streamed / 64.0 / n_cnt
        ghz = clk["clock_ghz"]
        ceil_ms = atom * cal["ds_add_u32_cycles_per_instr_per_cu"] / cal["cus"] / (ghz * 1e9) * 1e3
        roof["lds"] = dict(bound="lds-atomic issue", atomic_wave_instrs_per_launch=atom,
                           cycles_per_instr_per_cu=cal["ds_add_u32_cycles_per_instr_per_cu"], clock_ghz=ghz,
                           clock_source=os.path.relpath(clk_p, ROOT), ceiling_ms=ceil_ms,
                           frac=ceil_ms / roof["avg_launch_ms"], solo_launch_ms=clk.get("mean_us", 0) / 1e3 or None,
                           frac_solo=(ceil_ms / (clk["mean_us"] / 1e3)) if clk.get("mean_us") else None,
                           note="frac = the conflict-free atomic issue time of the launch's postings / its launch time "
                                "in the step (shared with the alignment chain); frac_solo against its duration alone "
                                "(PMC-serialised dispatches)")
    cells = sum(s["cells"] for s in stats)
    cells_c = sum(s["cells_computed"] for s in stats)
    g_alg = cells / t_al / 1e9 if t_al else 0.0
    g_cmp = cells_c / t_al / 1e9 if t_al else 0.0
    ceiling = VALU_LANE_OPS / ALIGN_VALU_PER_CELL / 1e9
    # against SURVEY §8d's nominal 12 int16 ops per affine cell with stats carry (not reachable with vsearch's path
    # statistics: DESIGN.md §6 "The aligner's instruction count" -- 15.4 VALU per cell in the ISA)
    ceiling12 = VALU_LANE_OPS / 12.0 / 1e9
    align = dict(kernel="k_align_pk", bound="valu", seconds_total=t_al, cells=cells, cells_computed=cells_c,
                 gcups_kernel=g_alg, gcups_computed=g_cmp, valu_per_cell=ALIGN_VALU_PER_CELL,
                 ceiling_gcups=ceiling, frac=g_alg / ceiling, frac_computed=g_cmp / ceiling,
                 ceiling_gcups_12ops=ceiling12, frac_12ops=g_alg / ceiling12,
                 speculative_ratio=cells_c / cells if cells else None)
    # the aligner alone: its kernels' durations in a PMC run (dispatches serialised, so nothing shares the CUs) of the
    # same workload, per bin, against this run's cells per bin (config 2: one bin per step)
    solo_p = _prof("rocprof_solo_kernel_stats_c2_r06.csv", "rocprof_solo_kernel_stats_c2_r05.csv")
    if config == 2 and os.path.exists(solo_p) and stats:
        t_solo = 0.0
        for r in csv.DictReader(open(solo_p, newline="")):
            nm = r["Name"].replace("void ", "").split("(")[0].split("::")[-1]
            if nm.startswith("k_align_pk") or nm.startswith("k_align_band"):
                t_solo += float(r["TotalDurationNs"]) * 1e-9
        bins_solo = 2  # tools/gpu_r05.sh `solo`: bench.py --steps 1 --warmup 1
        if t_solo > 0:
            align["gcups_solo"] = (cells / len(stats)) / (t_solo / bins_solo) / 1e9
            align["frac_solo"] = align["gcups_solo"] / ceiling
            align["solo_source"] = os.path.relpath(solo_p, ROOT)
    iss = align_issue_ceiling()
    if iss:
        iss["frac"] = g_alg / iss["ceiling_gcups"]
        if "gcups_solo" in align:
            iss["frac_solo"] = align["gcups_solo"] / iss["ceiling_gcups"]
        align["issue"] = iss
    if tl_union:
        tc, nc = tl_union.get("count", (0.0, 0))
        if tc > 0 and nc:
            a_dev = pf_bytes / tc / 1e9
            roof["device"] = dict(union_s=tc, brackets=nc, overlap=t_cnt / tc, ms_per_launch=1e3 * tc / nc,
                                  achieved=a_dev, frac=a_dev / L2_GATHER_GBS,
                                  note="the same bytes over the union of the counting launches' brackets across "
                                       "lanes (overlap = sum of brackets / union)")
        ta, na = tl_union.get("align", (0.0, 0))
        if ta > 0 and na:
            g_dev = cells / ta / 1e9
            align["device"] = dict(union_s=ta, brackets=na, overlap=t_al / ta, gcups=g_dev, frac=g_dev / ceiling,
                                   gcups_computed=cells_c / ta / 1e9, frac_computed=cells_c / ta / 1e9 / ceiling)
            if iss:
                align["device"]["frac_issue"] = g_dev / iss["ceiling_gcups"]
                align["device"]["frac_computed_issue"] = cells_c / ta / 1e9 / iss["ceiling_gcups"]
    return roof, align


def pmc_busy(kernel: str = "k_pf_count") -> dict | None:
    """Per-CU LDS-array and VALU busy of `kernel` (round 4: from the per-kernel PMC totals of
    profiles/r04/pmc_busy_c2_final.json, tools/pmc_agg.py; else round 3's CSV below)."""
    agg_path = _prof("pmc_busy_c2_r06.json", "pmc_busy_c2_r05.json")
    cal_path = os.path.join(ROOT, "profiles", "r03", "pmc_calib.json")
    if os.path.exists(agg_path) and os.path.exists(cal_path):
        agg = json.load(open(agg_path))
        k = next((x for x in agg if x.split("<")[0] == kernel and x.endswith(("<0, 4>", "<0>"))), None) or \
            next((x for x in agg if x.split("<")[0] == kernel), None)
        if k:
            cal = json.load(open(cal_path))
            n = agg[k]["dispatches"]
            per = {c: v / n for c, v in agg[k].items() if isinstance(v, float) and c not in ("mean_us",)}
            cyc = per["GRBM_GUI_ACTIVE"] / cal["xcds"]
            return dict(source=os.path.relpath(agg_path, ROOT), calibration=os.path.relpath(cal_path, ROOT),
                        dispatches=n, kernel_cycles=cyc, lds_insts_per_dispatch=per.get("SQ_INSTS_LDS"),
                        lds_array_busy_per_cu=per["SQ_LDS_IDX_ACTIVE"] * cal["lds_idx_active_cycles_per_unit"] / cal["cus"] / cyc,
                        valu_busy_per_simd=per["SQ_ACTIVE_INST_VALU"] * cal["active_inst_valu_cycles_per_unit"] / (cal["cus"] * 4) / cyc,
                        lds_bank_conflict_frac=per.get("SQ_LDS_BANK_CONFLICT", 0.0) / max(1.0, per["SQ_LDS_IDX_ACTIVE"]),
                        lds_array_cycles_per_instr=per["SQ_LDS_IDX_ACTIVE"] / max(1.0, per.get("SQ_INSTS_LDS", 0.0)),
                        valu_instrs_per_lds_instr=per["SQ_INSTS_VALU"] / max(1.0, per.get("SQ_INSTS_LDS", 0.0)))
    return _pmc_busy_csv(kernel)


def _pmc_busy_csv(kernel: str = "k_pf_count") -> dict | None:
    """Per-CU LDS-array and VALU busy of `kernel`, from the committed rocprofv3 PMC CSV
    (profiles/r03/pmc_busy_<kernel>.csv: SQ_LDS_IDX_ACTIVE, SQ_ACTIVE_INST_VALU, SQ_INSTS_LDS, SQ_INSTS_VALU,
    GRBM_GUI_ACTIVE, ...; one pass, step `busy` of tools/gpu_r03.sh) with the unit factors measured by the calibration
    kernels of tools/pmc_calib.hip (profiles/r03/pmc_calib.json): LDS busy = LDS-array cycles per CU / kernel
    cycles, VALU busy = VALU issue cycles per SIMD / kernel cycles, kernel cycles = GRBM_GUI_ACTIVE / XCDs."""
    csv_path = os.path.join(ROOT, "profiles", "r03", f"pmc_busy_{kernel}.csv")
    cal_path = os.path.join(ROOT, "profiles", "r03", "pmc_calib.json")
    if not (os.path.exists(csv_path) and os.path.exists(cal_path)):
        return None
    cal = json.load(open(cal_path))
    tot, disp = {}, set()
    for r in csv.DictReader(open(csv_path, newline="")):
        name = r["Kernel_Name"].replace("void ", "").split("(")[0].split("<")[0].split("::")[-1]
        if name != kernel:
            continue
        disp.add(r["Dispatch_Id"])
        tot[r["Counter_Name"]] = tot.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    if not disp:
        return None
    n = len(disp)
    per = {k: v / n for k, v in tot.items()}
    cyc = per["GRBM_GUI_ACTIVE"] / cal["xcds"]
    lds = per["SQ_LDS_IDX_ACTIVE"] * cal["lds_idx_active_cycles_per_unit"] / cal["cus"] / cyc
    valu = per["SQ_ACTIVE_INST_VALU"] * cal["active_inst_valu_cycles_per_unit"] / (cal["cus"] * 4) / cyc
    out = dict(source=os.path.relpath(csv_path, ROOT), calibration=os.path.relpath(cal_path, ROOT), dispatches=n,
               kernel_cycles=cyc, lds_array_busy_per_cu=lds, valu_busy_per_simd=valu,
               lds_bank_conflict_frac=per.get("SQ_LDS_BANK_CONFLICT", 0.0) / max(1.0, per["SQ_LDS_IDX_ACTIVE"]),
               lds_array_cycles_per_instr=per["SQ_LDS_IDX_ACTIVE"] / max(1.0, per.get("SQ_INSTS_LDS", 0.0)),
               valu_instrs_per_lds_instr=per["SQ_INSTS_VALU"] / max(1.0, per.get("SQ_INSTS_LDS", 0.0)))
    return out


def policy_name(threads: int) -> str:
    """which clustering definition a line measures."""
    return (f"O4: vsearch --threads {threads} (rounds of {threads} queries against the index frozen at the round's "
            "start, then re-checked in order)" if threads > 1 else "sequential: vsearch --threads 1")


def breakdown(stats: list) -> dict:
    k = ["t_total_s", "t_prefilter_s", "t_align_s", "t_consensus_s", "t_index_s", "t_host_s",
         "t_host_pass1_s", "t_sync_s", "t_merged_s"]
    return {x: sum(s[x] for s in stats) for x in k}


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", type=int, default=2, choices=(2, 3, 4, 5))
    ap.add_argument("--scale", type=float, default=1.0, help="fraction of the workload (testing only)")
    ap.add_argument("--identity", type=float, default=None,
                    help="default 0.90 (config 2), 0.93 (configs 3, 4 round 1), 0.75 (config 5)")
    ap.add_argument("--threads", type=int, default=int(os.environ.get("UMICLUST_BENCH_THREADS", "25")),
                    help="vsearch --threads of every bin: > 1 = policy O4 (rounds of that many queries, the mode the "
                         "reference runs: vsearch_umi_cluster.py:33-34, utils.py:56-63, n >= 25), 1 = the sequential "
                         "definition")
    ap.add_argument("--cpu-sample", type=int, default=40000,
                    help="reads of the sequential (--threads 1) CPU side figure's prefix")
    ap.add_argument("--cpu-sample-mt", type=int, default=200000,
                    help="reads of the CPU baseline's prefix in vsearch's --threads mode (the GPU line's policy)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-e2e", action="store_true", help="skip the file leg (config 2, N = 1)")
    ap.add_argument("--lanes", type=int, default=8,
                    help="configs 3/4: bins clustered concurrently per GPU (one device context per lane; 8 measured "
                         "best on config 3 with blocks across length changes: profiles/r03/mixlen_ab.json)")
    ap.add_argument("--pack-reads", type=int, default=int(os.environ.get("UMICLUST_PACK_READS", "200000")),
                    help="configs 3/4: cluster each lane's bins in packs of up to this many reads (umiclust_cluster_pack; "
                         "0: one bin per call; config 3: 100k and 200k equal on the whole set (7.60 / 7.61 M UMIs/s), "
                         "200k better on an 8-GPU share (45.6 vs 35.9 M node bound): profiles/r04/pack_ab_c3)")
    ap.add_argument("--shard-of", type=int, default=0,
                    help="configs 3/4, one GPU: cluster only the LPT share --shard of a --shard-of-GPU node (the bins that "
                         "rank would get); timing every share this way bounds the node's makespan")
    ap.add_argument("--shard", type=int, default=0)
    ap.add_argument("--largest-bin", action="store_true", help="configs 3/4: the largest bin alone")
    ap.add_argument("--bins", default="", help="configs 3/4: these bins alone (comma-separated indices)")
    ap.add_argument("--sweep-shares", default="",
                    help="--shard-sweep: only these share indices (comma-separated; no node value)")
    ap.add_argument("--shard-sweep", type=int, default=0,
                    help="configs 3/4, one GPU: time every LPT share of an N-GPU node one after another (plus the largest "
                         "bin alone) in one process; the largest share time is the measured N-GPU makespan bound")
    ap.add_argument("--no-confine", action="store_true",
                    help="--shard-sweep: do not confine the process to 1/N of the host CPUs")
    ap.add_argument("--e2e-files", action="store_true",
                    help="config 4 at the file boundary: per-bin FASTA inputs, round 1 through the fused drop-in "
                         "(clustering + parse outputs), round-2 FASTA from its consensus, round 2 to files, every bin "
                         "on `lanes` concurrent contexts (tcr_consensus.py:231-267, :411-446)")
    ap.add_argument("--read-len", type=int, default=800,
                    help="--e2e-files: length of the synthetic full read in each header's seq= field (production reads "
                         "are ~1,500 nt, SURVEY §8d; 800 is the longest whose 70M-record inputs and round-1 outputs fit "
                         "the GPU box's ~270 GiB host-memory cap on /dev/shm; 32 = SURVEY's --short-read)")
    ap.add_argument("--ranks-share-device", action="store_true",
                    help="testing only: every rank uses device 0 (rehearses the --gpus N path on a one-GPU box)")
    ap.add_argument("--digest-out", default="",
                    help="configs 3/4: each rank writes {bin index: digest} of its bins' last-step results to "
                         "<digest-out>.rank<r>.json (parity checks of the sharded path)")
    ap.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "traffic_latest.json"),
                    help="measured HBM bytes per prefilter launch (rocprofv3 PMC pass), if present")
    args = ap.parse_args()

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # one rank per GPU, started before anything here touches a GPU; exit with the launcher's status
        with socket.socket() as so:
            so.bind(("127.0.0.1", 0))
            port = so.getsockname()[1]
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
               "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
        raise SystemExit(subprocess.call(cmd))
    if int(os.environ.get("WORLD_SIZE", "1")) != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={os.environ.get('WORLD_SIZE', '1')} "
                         "(the launcher's rank count must equal --gpus)")
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    from umiclust import _lib, binset, shard, synth
    if args.shard_sweep:
        return shard_sweep(args)
    if args.e2e_files:
        return e2e_files(args)
    # multi-bin inputs are generated before anything touches the GPU (spawned workers)
    bins = None
    if args.config in (3, 4):
        all_bins = synth.config_bins(args.config, args.scale, workers=min(16, os.cpu_count() or 4))
        costs = [shard.bin_cost(b.umis.n) for b in all_bins]
        if args.bins:
            sel = [int(x) for x in args.bins.split(",")]
        elif args.largest_bin:
            sel = [max(range(len(costs)), key=lambda i: (costs[i], -i))]
        elif args.shard_of > 0:
            if world != 1 or not 0 <= args.shard < args.shard_of:
                raise SystemExit("--shard-of N --shard R: one process, 0 <= R < N")
            sel = shard.lpt_assign(costs, args.shard_of)[args.shard]
        else:
            sel = shard.lpt_assign(costs, world)[rank]
        bins = synth.concat_bins([all_bins[i] for i in sel])
        share_cost = sum(costs[i] for i in sel) / max(1e-9, sum(costs))
    import torch
    dist = None
    if world > 1:
        # the only cross-rank operations are a barrier and two host-scalar reductions (the bins shard with no data-path
        # collective): gloo over the host, so no RCCL communicator is ever initialised
        import torch.distributed as dist
        dist.init_process_group(backend="gloo")
    if not torch.cuda.is_available():
        raise SystemExit("bench.py needs a HIP device (there is no CPU backend)")
    ndev = torch.cuda.device_count()
    if args.ranks_share_device:
        local_rank = 0  # testing only: every rank on device 0 (a 1-GPU box rehearsing the N-rank path)
    elif local_rank >= ndev:
        raise SystemExit(f"bench.py: local rank {local_rank} but {ndev} visible device(s) (one rank per GPU)")
    torch.cuda.set_device(local_rank)

    if args.identity is None:
        args.identity = {2: 0.90, 3: 0.93, 4: 0.93, 5: 0.75}[args.config]
    lens = synth.CONFIG_LENGTHS[args.config]
    ctx = _lib.Context(local_rank)
    ctx2 = None
    umis = None
    if args.config == 2:
        seed = 1002 if rank == 0 else 1002 * 1_000_003 + rank
        umis = synth.make_umis(int(100_000 * args.scale), seed=seed, max_reads=int(2_000_000 * args.scale))
        workload = ("BASELINE config 2: synthetic 2M dual-UMI reads per GPU, one region bin, "
                    f"--id {args.identity:.2f}, round-1 scoring (match 10, mismatch -40, gapopen 0E/40I)")
    elif args.config == 5:
        seed = 1005 if rank == 0 else 1005 * 1_000_003 + rank
        umis = synth.make_umis(max(1, int(200 * args.scale)), seed=seed, mean_reads=1500.0, error_rate=0.15,
                               split=(0.0, 0.5, 0.5), max_edits=4, pattern_fwd=synth.UMI_FWD_LONG,
                               pattern_rev=synth.UMI_REV_LONG, max_reads=int(300_000 * args.scale))
        workload = ("BASELINE config 5 stress: synthetic 300k long (~96-nt) UMIs per GPU, 15% indels, deep "
                    f"clusters (NegBin mean 1500 reads/molecule), --id {args.identity:.2f}, "
                    f"--minseqlength {lens[0]} --maxseqlength {lens[1]}, round-1 scoring")
    elif args.config == 3:
        workload = (f"BASELINE config 3: synthetic {int(10_000_000 * args.scale)} reads over 24 barcodes x 40 "
                    f"Zipf(1.1) region bins, LPT-sharded over {world} GPU(s), round 1 --id {args.identity:.2f}")
    else:
        workload = (f"BASELINE config 4: synthetic {int(70_000_000 * args.scale)} reads over 24 barcodes x 40 "
                    f"Zipf(1.1) region bins, LPT-sharded over {world} GPU(s); round 1 --id {args.identity:.2f} "
                    "on every bin, round 2 (default scoring, --id 0.97) on the round-1 consensus UMIs of every "
                    "bin, consensus emitted")

    runners = []
    n_r1 = 0  # configs 3/4: units of round 1 at the head of a step's stats
    if umis is not None:
        params = _lib.params(_lib.PRESET_ROUND1, args.identity, *lens, threads=args.threads)
        ctx.stage(umis.seq, umis.off)  # the raw records resident in HBM (untimed)

        def step():
            t0 = time.perf_counter()
            ctx.prepare(params)  # A3: length filter, sort, DUST, codes, k-mers -- inside the step
            t_prep = time.perf_counter() - t0
            st = ctx.cluster()
            st["t_prepare_s"] = t_prep
            return [st]
    else:
        r1 = binset.BinRunner(ctx, bins, _lib.PRESET_ROUND1, args.identity, *lens, lanes=args.lanes, device=local_rank,
                              pack_reads=args.pack_reads, threads=args.threads)
        runners.append(r1)
        if args.config == 4:
            # round-2 inputs come from the round-1 results (deterministic): built once, resident like round 1
            r1.cluster_all()
            bins2 = binset.round2_binset(bins, r1.results())
            ctx2 = _lib.Context(local_rank)
            runners.append(binset.BinRunner(ctx2, bins2, binset.ROUND2["preset"], binset.ROUND2["identity"], *lens,
                                            lanes=args.lanes, device=local_rank, pack_reads=args.pack_reads,
                                            threads=args.threads))

        def step():
            nonlocal n_r1
            out = []
            for ri, r in enumerate(runners):
                t0 = time.perf_counter()
                r.prepare()  # A3 on every lane's staged bins -- inside the step
                t_prep = time.perf_counter() - t0
                st = r.cluster_all()
                if st:
                    st[0]["t_prepare_s"] = st[0].get("t_prepare_s", 0.0) + t_prep
                out += st
                if ri == 0:
                    n_r1 = len(out)
            return out

    def barrier():
        if dist is not None:
            dist.barrier()

    for _ in range(args.warmup):
        step()
    barrier()
    torch.cuda.synchronize()
    _lib.timeline(0, reset=True, device=local_rank)  # the kernels' device-time unions over the timed steps
    t0 = time.perf_counter()
    stats = []
    for _ in range(args.steps):
        stats.append(step())
    torch.cuda.synchronize()
    barrier()
    elapsed = time.perf_counter() - t0
    tl_union = {k: _lib.timeline(i) for i, k in enumerate(("count", "align"))}
    t_max = elapsed
    my_umis = sum(s["n_kept"] for s in stats[-1])
    tot_umis = my_umis
    if dist is not None:
        t = torch.tensor([elapsed, float(my_umis)], dtype=torch.float64)
        tm = t.clone()
        dist.all_reduce(tm, op=dist.ReduceOp.MAX)
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
        t_max = float(tm[0].item())
        tot_umis = int(t[1].item())
    total_umis = tot_umis * args.steps
    last = stats[-1]
    cells = sum(s["cells"] for s in last)
    value = total_umis / t_max
    gcups = cells * (world if args.config in (2, 5) else 1) * args.steps / t_max / 1e9

    if args.digest_out and runners:
        # every rank's bins (indices into the node's bin list) and their digests, per round
        dg = {"rank": rank, "world": world, "bins": [int(i) for i in sel], "rounds": []}
        for r in runners:
            dg["rounds"].append({str(int(sel[b])): binset.digest(x) for b, x in enumerate(r.results())})
        with open(f"{args.digest_out}.rank{rank}.json", "w") as fh:
            json.dump(dg, fh)
    if rank == 0:
        flat = [s for st in stats for s in st]
        roof, align = roofline(flat, args.config, args.traffic_json, tl_union)
        # per-step averages for the breakdown
        bd = {k: v / args.steps for k, v in breakdown(flat).items()}
        bd["t_prepare_s"] = sum(s.get("t_prepare_s", 0.0) for s in flat) / args.steps
        bd["wall"] = t_max / args.steps
        cfg = {"workload": workload, "parallelism": (f"{world} independent bins (1 per GPU), no data-path collective"
                                                      if args.config in (2, 5) else
                                                      f"LPT over {world} GPU(s) of the bins, no data-path collective"),
               "policy": policy_name(args.threads)}
        if umis is not None:
            cfg.update(reads_per_gpu=int(umis.n), umis_kept_per_gpu=int(last[0]["n_kept"]),
                       clusters=int(last[0]["n_clusters"]))
        else:
            cfg.update(bins_rank0=sum(r.nbins for r in runners), reads_rank0=int(sum(r.binset.n for r in runners)),
                       umis_kept_rank0=int(my_umis), clusters_rank0=int(sum(s["n_clusters"] for s in last)),
                       cost_share=share_cost)
            if args.largest_bin:
                cfg["selection"] = "the largest bin alone"
            elif args.shard_of > 0:
                cfg["selection"] = f"LPT share {args.shard} of {args.shard_of} (the bins rank {args.shard} of a {args.shard_of}-GPU run clusters)"
        out = {
            "metric": METRIC, "value": value, "unit": "UMIs/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": 1e3 * t_max / args.steps, "higher_is_better": True,
            "scaling": "weak" if args.config in (2, 5) else "strong", "vs_baseline": None, "dtype": "int16/int32",
            "data": "synthetic", "config": cfg, "gcups": gcups,
            "breakdown_s_per_step": bd,
            "merged_walks": sum(s["n_merged_walks"] for s in last), "deferred_queries": sum(s["n_deferred"] for s in last),
            "pairs_round_b": sum(s["pairs_round_b"] for s in last), "pairs_peer": sum(s["pairs_peer"] for s in last),
            "alignments_per_step": sum(s["n_alignments"] for s in last),
            "blocks": sum(s["n_blocks"] for s in last), "block_reruns": sum(s["n_reruns"] for s in last),
            "roofline": roof, "align": align,
        }
        if args.config == 2:
            busy = pmc_busy("k_pf_count")
            if busy:
                roof["pmc"] = busy
                lds = roof.get("lds")
                if lds and busy.get("lds_insts_per_dispatch"):
                    # SQ_INSTS_LDS of a PMC-serialised launch split into the counting atomics (one ds_add_u32
                    # wave-instruction per 64 streamed postings) and the rest: list-table reads/writes, counter
                    # zeroing, the threshold scan and the peer/candidate phases
                    tot = busy["lds_insts_per_dispatch"]
                    lds["insts_split"] = dict(lds_insts=tot, atomics=lds["atomic_wave_instrs_per_launch"],
                                              other=tot - lds["atomic_wave_instrs_per_launch"],
                                              atomic_share=lds["atomic_wave_instrs_per_launch"] / tot,
                                              source=busy["source"])
        if args.config in (3, 4):
            # per-bin wall times of the last step, measured while `lanes` bins share the GPU (so they do not
            # add up to the step): the largest bin bounds any split of these bins over GPUs
            per_bin = [s["t_total_s"] for s in last]
            out["largest_bin_s"] = max(per_bin) if per_bin else 0.0  # (the largest pack, with packing)
            if per_bin:
                w = max(last, key=lambda x: x["t_total_s"])
                out["slowest_unit"] = {k: w[k] for k in ("t_total_s", "n_kept", "n_clusters", "n_blocks", "n_reruns",
                                                         "n_alignments", "n_deferred", "t_host_s", "t_sync_s",
                                                         "t_prefilter_s", "t_align_s") if k in w}
                out["slowest_unit"]["bins"] = w.get("bins", [])[:8]
                out["slowest_unit"]["round"] = 1 if any(w is x for x in stats[-1][:n_r1]) else 2
            out["bins_timed"] = len(per_bin)
            out["pack_reads"] = args.pack_reads
            out["lanes"] = args.lanes
        cpu = None
        if not args.no_cpu_baseline and world == 1:
            if umis is not None:
                # the reference's operating mode (vsearch --threads on every core) is the baseline; the
                # 1-thread sequential definition on a smaller prefix rides along
                if args.threads > 1:  # the same policy as the GPU line
                    cpu = cpu_baseline_threads(umis, args.cpu_sample_mt, args.identity, lens, threads=args.threads)
                    cpu["serial_1thread"] = cpu_baseline_prefix(umis, args.cpu_sample, args.identity, lens)
                    cpu["serial_1thread"]["policy"] = policy_name(1)
                else:
                    cpu = cpu_baseline_prefix(umis, args.cpu_sample, args.identity, lens)
                cpu["policy"] = policy_name(args.threads)
                # the whole bin under the line's policy (tests/golden: the oracle's own wall time when it made the
                # golden), the other policy's whole-bin figure as a labelled side field
                full = full_bin_cpu_reference(args.config, args.threads, args.identity)
                if full:
                    cpu["full_bin_oracle"] = full
                other = full_bin_cpu_reference(args.config, 1 if args.threads > 1 else 25, args.identity)
                if other:
                    cpu["full_bin_oracle_other_policy"] = other
            else:
                cpu = cpu_baseline_bins(runners[0].binset.bins, args.identity, lens)
        out["cpu_baseline"] = cpu
        if not args.no_e2e and args.config == 2 and world == 1:
            out["e2e"] = e2e_leg(ctx, umis, args.identity, lens, threads=args.threads)
            # SURVEY §8d's UMIs/s (FASTA in -> files written) beside the HBM-resident value
            out["e2e_umis_per_s"] = out["e2e"]["umis_per_s"]
            out["e2e_fused_umis_per_s"] = out["e2e"]["fused_parse"]["umis_per_s"]
        print(json.dumps(out), flush=True)
    ctx.close()
    if ctx2 is not None:
        ctx2.close()
    if dist is not None:
        dist.destroy_process_group()


def _write_bin_fastas(job):
    """Worker (process pool): write the round's input FASTA of each (bin, path)."""
    from umiclust import synth
    out = []
    for b, path, read_len in job:
        synth.write_umi_fasta_fast(path, b.umis, seed=b.seed, read_len=read_len, chunk=16384)
        out.append(os.path.getsize(path))
    return out


def _read_consout(path: str) -> tuple[list, list]:
    """(consensus sequences, cluster sizes) of a consout FASTA (`>centroid=...;seqs=N;clusterid=K`), file order."""
    cons, sizes = [], []
    with open(path, "rb") as fh:
        hdr = None
        for line in fh:
            line = line.rstrip(b"\n")
            if line.startswith(b">"):
                hdr = line
                f = line.split(b";")
                sizes.append(int(next(x for x in reversed(f) if x.startswith(b"seqs="))[5:]))
                cons.append("")
            elif hdr is not None:
                cons[-1] += line.decode()
    return cons, sizes


def e2e_files(args) -> None:
    """BASELINE config 4 at the drop-in's file boundary on one GPU (the rank share of --shard-of/--shard, or every
    bin): round 1 = per bin `vsearch --cluster_fast` + parse_umi_clusters (tcr_consensus.py:231-267; here the fused
    drop-in umiclust_run_fasta_parse: consout + clusters_fa/ + smolecule_clusters.fa + stats), round 2 = per bin the
    consensus molecules' UMIs clustered to cluster<N> files + consout and parsed (:411-446).  Inputs (the per-bin
    FASTA region_split / extract_umis would leave; round 2's stands in for medaka + extract_umis on the consensus
    reads: synth.round2_bin) are written untimed; each round is timed from the first read to the last file written,
    its bins on `lanes` concurrent device contexts (one vsearch process per bin in the reference)."""
    import concurrent.futures as cf
    import shutil
    import tempfile
    import torch
    from umiclust import _lib, binset, shard, synth
    if args.config != 4:
        raise SystemExit("--e2e-files: config 4")
    lens = synth.CONFIG_LENGTHS[4]
    ident = args.identity if args.identity is not None else 0.93
    workers = min(16, os.cpu_count() or 4)
    all_bins = synth.config_bins(4, args.scale, workers=workers)
    costs = [shard.bin_cost(b.umis.n) for b in all_bins]
    sel = shard.lpt_assign(costs, args.shard_of)[args.shard] if args.shard_of > 0 else list(range(len(all_bins)))
    bins = [all_bins[i] for i in sel]
    base = os.environ.get("UMICLUST_E2E_DIR")
    if not base:
        try:
            st_ = os.statvfs("/dev/shm")
            base = "/dev/shm" if os.access("/dev/shm", os.W_OK) and st_.f_bavail * st_.f_frsize > (200 << 30) else None
        except OSError:
            base = None
    base = base or os.environ.get("TMPDIR", "/tmp")
    root = tempfile.mkdtemp(prefix="umiclust_c4e2e_", dir=base)
    try:
        dirs = [os.path.join(root, f"b{i:04d}") for i in range(len(bins))]
        for d in dirs:
            os.mkdir(d)
        t0 = time.perf_counter()

        def write_all(paths_bins):
            jobs = [[] for _ in range(workers)]
            order = sorted(range(len(paths_bins)), key=lambda i: -paths_bins[i][0].umis.n)
            load = [0] * workers
            for i in order:  # LPT over the writer processes
                w = min(range(workers), key=lambda k: load[k])
                jobs[w].append((paths_bins[i][0], paths_bins[i][1], args.read_len))
                load[w] += paths_bins[i][0].umis.n
            with cf.ProcessPoolExecutor(workers) as ex:
                return sum(sum(x) for x in ex.map(_write_bin_fastas, jobs))
        in1 = [os.path.join(d, "region_cluster_detected_umis.fasta") for d in dirs]
        bytes1 = write_all(list(zip(bins, in1)))
        t_gen1 = time.perf_counter() - t0
        _progress(f"e2e-files: {len(bins)} round-1 inputs written, {bytes1 / 1e9:.1f} GB in {t_gen1:.0f} s")
        torch.cuda.set_device(0)
        lanes = max(1, min(args.lanes, len(bins)))
        ctxs = [_lib.Context(0) for _ in range(lanes)]
        plan = shard.lpt_assign([shard.bin_cost(b.umis.n) for b in bins], lanes)
        p1 = _lib.params(_lib.PRESET_ROUND1, ident, *lens, threads=args.threads)
        p2 = _lib.params(binset.ROUND2["preset"], binset.ROUND2["identity"], *lens, threads=args.threads)
        pp1 = _lib.ParseParams(min_reads_per_cluster=4, max_reads_per_cluster=60, balance_strands=0, max_clusters=0)
        pp2 = _lib.ParseParams(min_reads_per_cluster=1, max_reads_per_cluster=60, balance_strands=0, max_clusters=0)
        # warm-up (untimed): one small bin through both paths, so allocations and code objects are not timed
        wi = min(range(len(bins)), key=lambda i: bins[i].umis.n)
        wd = os.path.join(root, "warm")
        os.mkdir(wd)
        ctxs[0].run_fasta_parse(p1, in1[wi], None, os.path.join(wd, "c.fa"), None, pp1, wd)
        shutil.rmtree(wd)

        def run_round(rnd):
            per = [None] * len(bins)

            def lane(li):
                for i in plan[li]:
                    d = os.path.join(dirs[i], f"round{rnd}")
                    os.mkdir(d)
                    t = time.perf_counter()
                    if rnd == 1:
                        st, pr = ctxs[li].run_fasta_parse(p1, in1[i], None, os.path.join(d, "umi_clusters_consensus.fasta"),
                                                          os.path.join(d, "vsearch_cluster.log"), pp1, d)
                    else:  # f2 in round 2 as well: the cluster<N> files only feed parse_umi_clusters (tcr_consensus.py:433-446)
                        st, pr = ctxs[li].run_fasta_parse(p2, in2[i], None,
                                                          os.path.join(d, "umi_clusters_consensus.fasta"),
                                                          os.path.join(d, "vsearch_cluster_consensus.log"), pp2, d)
                    per[i] = dict(seconds=time.perf_counter() - t, kept=st["n_kept"], clusters=st["n_clusters"],
                                  t_read_s=st["t_read_s"], t_cluster_s=st["t_total_s"], t_write_s=st["t_write_s"],
                                  written=pr["n_written"])
            t0_ = time.perf_counter()
            with cf.ThreadPoolExecutor(lanes) as ex:
                list(ex.map(lane, range(lanes)))
            wall = time.perf_counter() - t0_
            nf, nb = 0, 0
            for d in dirs:
                f, b = _tree_bytes(os.path.join(d, f"round{rnd}"))
                nf += f
                nb += b
            tot = lambda k: sum(x[k] for x in per)  # noqa: E731
            return dict(wall_s=wall, umis_kept=int(tot("kept")), umis_per_s=tot("kept") / wall, clusters=int(tot("clusters")),
                        clusters_written=int(tot("written")), sum_read_s=tot("t_read_s"), sum_cluster_s=tot("t_cluster_s"),
                        sum_write_s=tot("t_write_s"), largest_bin_s=max(x["seconds"] for x in per),
                        files_written=nf, bytes_written=nb), per
        r1, per1 = run_round(1)
        _progress(f"e2e-files: round 1 {r1['wall_s']:.1f} s, {r1['umis_per_s'] / 1e6:.2f} M UMIs/s")
        shm_peak = _fs_used(root)
        # round 1's clusters_fa/ and smolecule_clusters.fa go to medaka, not to round 2: freed (untimed) so that the
        # round-2 inputs fit beside the rest in RAM-backed storage
        for d in dirs:
            shutil.rmtree(os.path.join(d, "round1", "clusters_fa"), ignore_errors=True)
            try:
                os.remove(os.path.join(d, "round1", "smolecule_clusters.fa"))
            except OSError:
                pass
        # round-2 inputs from round 1's consout (untimed: medaka + extract_umis stand-in)
        t0 = time.perf_counter()
        b2 = []
        for i, b in enumerate(bins):
            cons, sizes = _read_consout(os.path.join(dirs[i], "round1", "umi_clusters_consensus.fasta"))
            b2.append(synth.round2_bin(b, cons, sizes))
        in2 = [os.path.join(d, "consensus_umis.fasta") for d in dirs]
        bytes2 = write_all(list(zip(b2, in2)))
        t_gen2 = time.perf_counter() - t0
        _progress(f"e2e-files: {len(bins)} round-2 inputs written, {bytes2 / 1e9:.1f} GB in {t_gen2:.0f} s")
        r2, _ = run_round(2)
        _progress(f"e2e-files: round 2 {r2['wall_s']:.1f} s, {r2['umis_per_s'] / 1e6:.2f} M UMIs/s")
        for c in ctxs:
            c.close()
        wall = r1["wall_s"] + r2["wall_s"]
        kept = r1["umis_kept"] + r2["umis_kept"]
        out = {"metric": METRIC, "value": kept / wall, "unit": "UMIs/s", "n_gpus": 1, "steps": 1, "warmup": 1,
               "ms_per_step": 1e3 * wall, "higher_is_better": True, "scaling": "strong", "vs_baseline": None,
               "dtype": "int16/int32", "data": "synthetic",
               "config": {"workload": f"BASELINE config 4 at the file boundary, scale {args.scale}: "
                                      f"{sum(b.umis.n for b in bins)} reads in {len(bins)} bins"
                                      + (f" (LPT share {args.shard} of {args.shard_of})" if args.shard_of else "")
                                      + f", both rounds, {args.read_len}-nt seq= reads",
                          "parallelism": f"one MI355X, {lanes} concurrent per-bin contexts", "output_dir": base},
               "round1": r1, "round2": r2, "input_bytes": [bytes1, bytes2], "input_write_s": [t_gen1, t_gen2],
               "storage_used_after_round1_bytes": shm_peak, "read_len": args.read_len,
               "note": "value = UMIs of both rounds / (round-1 wall + round-2 wall), each from its first FASTA read to "
                       "its last file; inputs written untimed; RAM-backed output_dir when /dev/shm has room"}
        print(json.dumps(out), flush=True)
    finally:
        shutil.rmtree(root, ignore_errors=True)


def shard_sweep(args) -> None:
    """8-GPU readiness measured on one GPU (configs 3/4): the node's bins are LPT-assigned to N ranks exactly as a
    `--gpus N` run assigns them (shard.lpt_assign), and each rank's share is clustered alone on this GPU, one after
    another, each timed over one full step (stage untimed; prepare + cluster of every round timed), after an untimed
    warm-up of the first share.  The largest share time is the makespan bound of an N-GPU node (each rank runs its
    share on its own GPU, no collective); the largest bin alone bounds any split of the bins."""
    from umiclust import _lib, binset, shard, synth
    if args.config not in (3, 4):
        raise SystemExit("--shard-sweep: configs 3 and 4")
    N = args.shard_sweep
    # host confinement, before anything touches the GPU: an N-GPU node gives each rank 1/N of the host's logical CPUs
    # (one process per GPU), so the share runs on 1/N of this process's affinity mask -- whole physical cores with
    # their SMT siblings, one NUMA node -- and the resolve pool is capped by that mask (driver.cpp pool_threads)
    confine = _confine_to_node_share(N) if not args.no_confine else None
    import torch
    ident = args.identity if args.identity is not None else 0.93
    lens = synth.CONFIG_LENGTHS[args.config]
    all_bins = synth.config_bins(args.config, args.scale, workers=min(16, os.cpu_count() or 4))
    costs = [shard.bin_cost(b.umis.n) for b in all_bins]
    plan = shard.lpt_assign(costs, N)
    largest = max(range(len(costs)), key=lambda i: (costs[i], -i))
    torch.cuda.set_device(0)
    ctx = _lib.Context(0)
    ctx2 = _lib.Context(0) if args.config == 4 else None

    def run(sel):
        bins = synth.concat_bins([all_bins[i] for i in sel])
        r1 = binset.BinRunner(ctx, bins, _lib.PRESET_ROUND1, ident, *lens, lanes=args.lanes, pack_reads=args.pack_reads,
                              threads=args.threads)
        runners = [r1]
        if args.config == 4:
            r1.cluster_all()
            b2 = binset.round2_binset(bins, r1.results())
            runners.append(binset.BinRunner(ctx2, b2, binset.ROUND2["preset"], binset.ROUND2["identity"], *lens,
                                            lanes=args.lanes, pack_reads=args.pack_reads, threads=args.threads))
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        st = []
        for r in runners:
            r.prepare()
            st += r.cluster_all()
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        kept = sum(x["n_kept"] for x in st)
        for r in runners:
            r.close()
        _progress(f"shard-sweep: {len(sel)} bins, {kept} UMIs in {dt:.2f} s")
        w = max(st, key=lambda x: x["t_total_s"]) if st else {}
        return dict(bins=len(sel), reads=int(bins.n), umis_kept=int(kept), seconds=dt, umis_per_s=kept / dt,
                    cost_share=sum(costs[i] for i in sel) / sum(costs),
                    largest_pack_s=max((x["t_total_s"] for x in st), default=0.0),
                    slowest_unit={k: w[k] for k in ("t_total_s", "n_kept", "n_blocks", "n_reruns", "n_deferred",
                                                    "t_host_s", "t_sync_s") if k in w} | {"bins": len(w.get("bins", [0]))},
                    long_units=[{k: x[k] for k in ("t_total_s", "n_kept", "n_blocks", "n_reruns") if k in x}
                                | {"bins": x.get("bins", [])[:4]} for x in st if x["t_total_s"] > 0.4 * dt])

    run(plan[0])  # warm-up (untimed): allocations, code objects
    pick = [int(x) for x in args.sweep_shares.split(",")] if args.sweep_shares else list(range(N))
    shares = [dict(run(plan[i]), share=i) for i in pick]
    big = run([largest])
    tmax = max(x["seconds"] for x in shares)
    node_umis = sum(x["umis_kept"] for x in shares)
    # measured on ONE GPU: `value` is this GPU's rate over the shares it ran; the N-GPU node figure is a model
    # (every share on its own GPU at the time measured here, host confined as above), reported apart
    tsum = sum(x["seconds"] for x in shares)
    out = {"metric": METRIC, "value": node_umis / tsum, "unit": "UMIs/s", "n_gpus": 1, "steps": 1, "warmup": 1,
           "ms_per_step": 1e3 * tsum, "higher_is_better": True, "scaling": "strong", "vs_baseline": None,
           "dtype": "int16/int32", "data": "synthetic",
           "config": {"workload": f"BASELINE config {args.config} at scale {args.scale}: every LPT share of an {N}-GPU "
                                  "node clustered alone on one MI355X, one after another",
                      "parallelism": f"{N} shares (shard.lpt_assign), each timed alone on one GPU",
                      "policy": policy_name(args.threads), "lanes": args.lanes, "pack_reads": args.pack_reads,
                      "host_confinement": confine},
           "node_bound_model": {"n_gpus": N, "value": node_umis / tmax, "unit": "UMIs/s", "makespan_s": tmax,
                                "note": f"a model, not a measurement: the node's UMIs / the largest share's time, as if "
                                        f"{N} GPUs ran their shares at once, each rank on 1/{N} of the host "
                                        "(host_confinement); no N-GPU run was made"},
           "shares": shares, "makespan_s": tmax, "sum_s": tsum,
           "largest_bin": dict(big, bin=largest), "measured_on": "one GPU"}
    if len(pick) < N:  # a subset of the shares: no node figure
        out.update(partial_shares=pick)
        out["node_bound_model"]["value"] = None
    print(json.dumps(out), flush=True)
    ctx.close()
    if ctx2 is not None:
        ctx2.close()


def _confine_to_node_share(n: int) -> dict:
    """Restrict this process (and the threads it starts later) to 1/n of its affinity mask: whole physical cores with
    their SMT siblings, taken from one NUMA node (sysfs topology), so that a one-GPU run sees the host share one rank
    of an n-GPU node gets.  Returns what was applied."""
    mask = sorted(os.sched_getaffinity(0))
    want = max(1, len(mask) // n)

    def sib(c):
        try:
            txt = open(f"/sys/devices/system/cpu/cpu{c}/topology/thread_siblings_list").read().strip()
            out = set()
            for part in txt.split(","):
                a, _, b = part.partition("-")
                out.update(range(int(a), int(b or a) + 1))
            return out
        except OSError:
            return {c}

    def node(c):
        for d in glob.glob(f"/sys/devices/system/cpu/cpu{c}/node*"):
            return os.path.basename(d)
        return "node0"

    first = node(mask[0])
    pick = []
    for c in mask:
        if len(pick) >= want:
            break
        if c in pick or node(c) != first:
            continue
        pick += [x for x in sorted(sib(c)) if x in mask and x not in pick]
    pick = pick[:want]
    os.sched_setaffinity(0, pick)
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()
        quota = None if q == "max" else int(q) / int(per)
    except (OSError, ValueError):
        pass
    return dict(share=f"1/{n}", cpus=len(pick), cpu_list=pick, of_mask=len(mask), numa=first, cgroup_cpu_quota=quota)


def _progress(msg: str) -> None:
    print(f"[bench {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


def _fs_used(path: str) -> int:
    st = os.statvfs(path)
    return (st.f_blocks - st.f_bfree) * st.f_frsize


def _tree_bytes(d: str) -> tuple[int, int]:
    n = b = 0
    for root, _, files in os.walk(d):
        for f in files:
            n += 1
            b += os.path.getsize(os.path.join(root, f))
    return n, b


def _numbered_sizes(d: str, prefix: str, suffix: str = "") -> list:
    """Sizes of d/<prefix><N><suffix> in N order."""
    out = []
    for f in os.listdir(d):
        if f.startswith(prefix) and f.endswith(suffix) and f[len(prefix):len(f) - len(suffix)].isdigit():
            out.append((int(f[len(prefix):len(f) - len(suffix)]), os.path.getsize(os.path.join(d, f))))
    return [sz for _, sz in sorted(out)]


def replay_probe(d: str, sizes: list, one_bytes: int, threads: int) -> dict:
    """tools/io_probe.c io_probe_replay: the writer's own create / write / close sequence (the same file sizes, the
    same contiguous split over `threads`, one_bytes streamed into one more file as the fused writer streams
    smolecule_clusters.fa) with no formatting: a reference point for the writer's time, not a bound (it does not
    reissue the writer's exact system calls)."""
    import numpy as np
    lib = ctypes.CDLL(os.path.join(ROOT, "tools", "libioprobe.so"))
    lib.io_probe_replay.restype = ctypes.c_double
    lib.io_probe_replay.argtypes = [ctypes.c_char_p, ctypes.c_int64, ctypes.POINTER(ctypes.c_int64), ctypes.c_int,
                                    ctypes.c_int64]
    pd = os.path.join(d, "replay")
    os.mkdir(pd)
    sz = np.ascontiguousarray(sizes, np.int64)
    t = lib.io_probe_replay(pd.encode(), len(sz), sz.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)), threads,
                            int(one_bytes))
    os.rmdir(pd)
    if t < 0:
        raise RuntimeError("io_probe_replay failed")
    tot = int(sz.sum()) + int(one_bytes)
    return dict(files=len(sz) + (1 if one_bytes else 0), bytes=tot, threads=threads, seconds=t,
                gbps=tot / t / 1e9 if t > 0 else None)


def e2e_leg(ctx, umis, identity: float, lens, read_len: int = 1500, threads: int = 25) -> dict:
    """§8d's UMIs/s at the drop-in's file boundary (vsearch_umi_cluster.py:17-56: FASTA in, cluster<N> files +
    consout out; umiclust_run_fasta) and for the fused drop-in (umiclust_run_fasta_parse:
    clustering + parse_umi_clusters' outputs, no cluster<N> files), on the same bin written with 1,500-nt `seq=`
    reads.  Each writer is followed by a replay of its files (same sizes and thread split, no formatting);
    write_replay_ratio = replay seconds / writer seconds (a reference point, not a bound)."""
    import shutil
    import tempfile
    from umiclust import _lib, synth
    io_t = max(1, min(16, len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)))
    # RAM-backed (/dev/shm) when it has room: on the GPU box's disk-backed overlay every create / delete cycle of
    # ~10^5 files leaves the next one slower (the same replay: 2.0 s fresh, 7.6 s after one delete, 25 s after three:
    # profiles/r04/io_order_probe.txt), so later writers would be timed against the filesystem's history
    base = os.environ.get("UMICLUST_E2E_DIR")
    if not base:
        try:
            st_ = os.statvfs("/dev/shm")
            base = "/dev/shm" if os.access("/dev/shm", os.W_OK) and st_.f_bavail * st_.f_frsize > (64 << 30) else None
        except OSError:
            base = None
    base = base or os.environ.get("TMPDIR", "/tmp")
    d = tempfile.mkdtemp(prefix="umiclust_e2e_", dir=base)
    try:
        fa = os.path.join(d, "region_cluster0_detected_umis.fasta")
        t0 = time.perf_counter()
        synth.write_umi_fasta_fast(fa, umis, read_len=read_len)
        t_gen = time.perf_counter() - t0
        size = os.path.getsize(fa)
        # every timed write below starts with no dirty pages of an earlier phase still draining (untimed sync)
        os.sync()
        out = os.path.join(d, "out")
        os.mkdir(out)
        p = _lib.params(_lib.PRESET_ROUND1, identity, *lens, threads=threads)
        t0 = time.perf_counter()
        st = ctx.run_fasta(p, fa, os.path.join(out, "cluster"), os.path.join(out, "umi_clusters_consensus.fasta"),
                           os.path.join(out, "vsearch_cluster.log"))
        t_run = time.perf_counter() - t0
        t0 = time.perf_counter()
        ctx.wait_host()  # the input's release, which the call leaves on a thread of the context
        t_rel = time.perf_counter() - t0
        nf, nb = _tree_bytes(out)
        sizes = _numbered_sizes(out, "cluster")
        cons_bytes = os.path.getsize(os.path.join(out, "umi_clusters_consensus.fasta"))
        shutil.rmtree(out, ignore_errors=True)
        os.sync()
        bound = replay_probe(d, sizes, cons_bytes, io_t)
        os.sync()
        # the fused drop-in (run_config.json:17-19 defaults: >= 4 reads, <= 60 per cluster, no strand balancing)
        work = os.path.join(d, "work")
        os.mkdir(work)
        pp = _lib.ParseParams(min_reads_per_cluster=4, max_reads_per_cluster=60, balance_strands=0, max_clusters=0)
        t0 = time.perf_counter()
        st2, pr = ctx.run_fasta_parse(p, fa, None, os.path.join(work, "umi_clusters_consensus.fasta"),
                                      os.path.join(work, "vsearch_cluster.log"), pp, work)
        t_fused = time.perf_counter() - t0
        t0 = time.perf_counter()
        ctx.wait_host()
        t_rel2 = time.perf_counter() - t0
        nf2, nb2 = _tree_bytes(os.path.join(work, "clusters_fa"))
        sizes2 = _numbered_sizes(os.path.join(work, "clusters_fa"), "cluster", ".fasta")
        smol = os.path.getsize(os.path.join(work, "smolecule_clusters.fa"))
        _, nb_all = _tree_bytes(work)
        shutil.rmtree(work, ignore_errors=True)
        os.sync()
        bound_f = replay_probe(d, sizes2, smol, io_t)
        return dict(
            umis_per_s=st["n_kept"] / t_run, seconds=t_run, fasta_bytes=size, n_kept=st["n_kept"],
            # the call returns once every output is written; its input's release (unmapping the FASTA) runs on after
            # it, on a thread of the context (umiclust_wait_host): counted here as well
            input_release_s=t_rel, umis_per_s_incl_release=st["n_kept"] / (t_run + t_rel),
            clusters=st["n_clusters"], t_read_s=st.get("t_read_s"), t_cluster_s=st["t_total_s"],
            t_write_s=st.get("t_write_s"), files_written=nf, bytes_written=nb,
            write_gbps=nb / st["t_write_s"] / 1e9 if st.get("t_write_s") else None,
            write_replay=bound,
            write_replay_ratio=bound["seconds"] / st["t_write_s"] if st.get("t_write_s") else None,
            fasta_write_s=t_gen,
            fused_parse=dict(umis_per_s=st2["n_kept"] / t_fused, seconds=t_fused, t_read_s=st2.get("t_read_s"),
                             input_release_s=t_rel2, umis_per_s_incl_release=st2["n_kept"] / (t_fused + t_rel2),
                             t_cluster_s=st2["t_total_s"], t_write_s=st2.get("t_write_s"),
                             clusters_written=pr["n_written"], cluster_files=nf2, cluster_file_bytes=nb2,
                             smolecule_bytes=smol, bytes_written=nb_all,
                             write_gbps=nb_all / st2["t_write_s"] / 1e9 if st2.get("t_write_s") else None,
                             write_replay=bound_f,
                             write_replay_ratio=bound_f["seconds"] / st2["t_write_s"] if st2.get("t_write_s") else None),
            output_dir=base,
            note="page-cache-warm input; outputs under output_dir (RAM-backed /dev/shm when it has room); every timed write (writers and "
                 "replays) starts after an untimed sync; write_replay = io_probe_replay of the writer's files "
                 "(sizes, contiguous thread split, the one streamed file) with no formatting; write_replay_ratio = "
                 "write_replay seconds / the writer's seconds -- a reference point, not a bound")
    finally:
        shutil.rmtree(d, ignore_errors=True)


if __name__ == "__main__":
    main()
