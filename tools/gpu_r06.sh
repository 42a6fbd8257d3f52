#!/bin/bash
# GPU session steps (round 6).  Every GPU step has its own time limit; the first failure ends the call.
# Usage: bash tools/gpu_r06.sh <tag> <steps...>
#   steps: tests | smoke | bench | seq | trace | solo | busy | busy2 | fetch | write | pfprof | c3 | c4 | c5 | c5trace
#          | sweep3 | sweep4 (SHARES=) | c4e2e (SCALE=, READLEN=) | resdump | default | tracefull | pf1ab | bandab
#          | regrowab | valu | c3trace
# The default bench line is config 2 under --threads 25 (policy O4, the reference's mode); `seq` is --threads 1.
# (The round-5 script's c3lazy / predab / prab / pf2ab / hqab steps drove switches that no longer exist: removed.)
set -o pipefail
tag=${1:-r06}
shift
out=gpurun_out/$tag
mkdir -p "$out"
export TMPDIR=/tmp
B="bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-e2e"
SQ="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_VALU GRBM_GUI_ACTIVE GRBM_COUNT"
SQ2="SQ_WAVES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_SMEM GRBM_GUI_ACTIVE GRBM_COUNT"
rc=0
for st in "$@"; do
  echo "== $st $(date +%T)"
  case $st in
    tests) timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
             > "$out/tests.log" 2>&1; rc=$?; tail -3 "$out/tests.log" ;;
    smoke) timeout -k 10 300 python3 -u -c 'import __graft_entry__ as g; g.smoke()' > "$out/smoke.log" 2>&1; rc=$? ;;
    bench) timeout -k 10 900 python3 -u bench.py --steps 5 --warmup 1 > "$out/bench.json" 2> "$out/bench.err"; rc=$? ;;
    seq) timeout -k 10 300 python3 -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-e2e --threads 1 \
           > "$out/seq.json" 2> "$out/seq.err"; rc=$? ;;
    trace) timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d "$out/trace" -o run -- \
             python3 $B > "$out/trace.log" 2>&1; rc=$?
           [ $rc = 0 ] && python3 tools/kstats.py "$out/trace/run_kernel_stats.csv" 6 > "$out/trace_kstats.txt" 2>&1 && python3 tools/gpu_idle.py "$out/trace" > "$out/trace_idle.txt" 2>&1 ;;
    solo) # PMC collection serialises the dispatches: the kernel trace of this run holds every kernel's solo duration
          timeout -s KILL 400 rocprofv3 --pmc GRBM_GUI_ACTIVE --kernel-trace --stats --output-format csv -d "$out/solo" -o run -- \
             python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-e2e > "$out/solo.log" 2>&1; rc=$?
          [ $rc = 0 ] && python3 tools/pmc_clock.py "$out/solo/run_counter_collection.csv" "k_pf_count<0, 4>" "$out/pmc_clock_k_pf_count.json"
          rm -f "$out/solo/run_kernel_trace.csv" "$out/solo/run_counter_collection.csv" ;;
    busy|busy2) # per-kernel totals only (the full counter CSV exceeds what a call may bring back)
          [ "$st" = busy ] && CT="$SQ" || CT="$SQ2"
          timeout -s KILL 300 rocprofv3 --pmc $CT --output-format csv -d "$out/$st" -o run -- python3 $B \
             > "$out/$st.log" 2>&1; rc=$?
          if [ $rc = 0 ]; then python3 tools/pmc_agg.py "$out/$st/run_counter_collection.csv" "$out/${st}_agg.json"; rc=$?; fi
          rm -f "$out/$st/run_counter_collection.csv" ;;
    fetch|write) # one counter per pass; per-kernel totals only
          [ "$st" = fetch ] && CT=FETCH_SIZE || CT=WRITE_SIZE
          timeout -s KILL 300 rocprofv3 --pmc $CT --output-format csv -d "$out/$st" -o run -- python3 $B \
             > "$out/$st.log" 2>&1; rc=$?
          if [ $rc = 0 ]; then python3 tools/pmc_agg.py "$out/$st/run_counter_collection.csv" "$out/${st}_agg.json"; rc=$?; fi
          rm -f "$out/$st/run_counter_collection.csv" ;;
    pfprof) UMICLUST_PFPROF=1 timeout -k 10 300 python3 -u $B > "$out/pfprof.json" 2> "$out/pfprof.err"; rc=$? ;;
    c3) timeout -k 10 500 python3 -u bench.py --config 3 --steps 2 --warmup 1 --no-cpu-baseline > "$out/c3.json" 2> "$out/c3.err"; rc=$? ;;
    c4) timeout -k 10 600 python3 -u bench.py --config 4 --steps 1 --warmup 0 --no-cpu-baseline > "$out/c4.json" 2> "$out/c4.err"; rc=$? ;;
    c5) timeout -k 10 400 python3 -u bench.py --config 5 --steps 3 --warmup 1 --no-cpu-baseline > "$out/c5.json" 2> "$out/c5.err"; rc=$? ;;
    c5trace) timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/c5trace" -o run -- \
             python3 bench.py --config 5 --steps 2 --warmup 1 --no-cpu-baseline --no-e2e > "$out/c5trace.log" 2>&1; rc=$?
             rm -f "$out/c5trace/run_kernel_trace.csv" ;;
    sweep3) timeout -k 10 900 python3 -u bench.py --config 3 --shard-sweep 8 > "$out/sweep3.json" 2> "$out/sweep3.err"; rc=$? ;;
    sweep4) timeout -k 10 1000 python3 -u bench.py --config 4 --shard-sweep 8 --sweep-shares "${SHARES:-}" > "$out/sweep4.json" 2> "$out/sweep4.err"; rc=$? ;;
    c4e2e) timeout -k 10 1100 python3 -u bench.py --config 4 --e2e-files --scale "${SCALE:-1.0}" --read-len "${READLEN:-1500}" \
             > "$out/c4e2e.json" 2> "$out/c4e2e.err"; rc=$? ;;
    valu) timeout -k 10 120 ./tools/valu_rate > "$out/valu_rate.jsonl" 2>&1; rc=$? ;;
    default) timeout -k 10 700 python3 -u bench.py > "$out/bench_default.json" 2> "$out/bench_default.err"; rc=$? ;;
    pf1ab) for v in ${PF1S:-10240 0}; do for c in ${PCFGS:-3 5 2}; do
              UMICLUST_PF1=$v timeout -k 10 400 python3 -u bench.py --config $c --steps 2 --warmup 1 --no-cpu-baseline --no-e2e \
                > "$out/pf1_${v}_c$c.json" 2> "$out/pf1_${v}_c$c.err" || { rc=$?; break 2; }; rc=0; done; done ;;
    c3trace) timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/c3trace" -o run -- \
             python3 bench.py --config 3 --steps 1 --warmup 1 --no-cpu-baseline --no-e2e > "$out/c3trace.log" 2>&1; rc=$?
             [ $rc = 0 ] && python3 tools/kstats.py "$out/c3trace/run_kernel_stats.csv" 2 > "$out/c3trace_kstats.txt" 2>&1 \
               && python3 tools/gpu_idle.py "$out/c3trace" > "$out/c3trace_idle.txt" 2>&1
             rm -f "$out/c3trace/run_kernel_trace.csv" ;;
    bandab) for v in ${BANDS:-140000 0 20000}; do for c in ${PCFGS:-3 5}; do
              UMICLUST_BAND=$v timeout -k 10 400 python3 -u bench.py --config $c --steps 2 --warmup 1 --no-cpu-baseline --no-e2e \
                > "$out/band${v}_c$c.json" 2> "$out/band${v}_c$c.err" || { rc=$?; break 2; }; rc=0; done; done ;;
    tracefull) # the default bench command itself under the kernel tracer (the roofline's rocprof cross-check)
          timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/tracefull" -o run -- \
             python3 bench.py > "$out/tracefull.out" 2> "$out/tracefull.err"; rc=$?
          [ $rc = 0 ] && python3 tools/kstats.py "$out/tracefull/run_kernel_stats.csv" 6 > "$out/tracefull_kstats.txt" 2>&1
          rm -f "$out/tracefull/run_kernel_trace.csv" ;;
    regrowab) for v in ${REGS:-0 16 4}; do for c in ${PCFGS:-5 4}; do
              UMICLUST_REGROW=$v timeout -k 10 400 python3 -u bench.py --config $c --steps 1 --warmup 1 --no-cpu-baseline --no-e2e \
                > "$out/rg${v}_c$c.json" 2> "$out/rg${v}_c$c.err" || { rc=$?; break 2; }; rc=0; done; done ;;
    e2eprobe) timeout -k 10 400 python3 -u tools/e2e_probe.py "$out/e2e_probe.json" > "$out/e2e_probe.log" 2>&1; rc=$? ;;
    arrab) for v in ${ARRS:-0 3 1 0 3}; do for c in ${PCFGS:-2 3 5}; do
              UMICLUST_ARRANGE=$v timeout -k 10 400 python3 -u bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline --no-e2e \
                > "$out/arr${v}_c${c}_$RANDOM.json" 2> /dev/null || { rc=$?; break 2; }; rc=0; done; done ;;
    rdab) for v in ${RDS:-32 48 64 96 32}; do for c in ${PCFGS:-5 4}; do
              UMICLUST_REGROW_DEPTH=$v timeout -k 10 500 python3 -u bench.py --config $c --steps 2 --warmup 1 --no-cpu-baseline --no-e2e \
                > "$out/rd${v}_c${c}_$RANDOM.json" 2> /dev/null || { rc=$?; break 2; }; rc=0; done; done ;;
    c2dbg) UMICLUST_DEBUG=1 timeout -k 10 300 python3 -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-e2e \
             > "$out/c2dbg.json" 2> "$out/c2dbg.err"; rc=$? ;;
    rbprio) for v in ${RBP:-1 0 1 0}; do for c in ${PCFGS:-5}; do
              UMICLUST_RB_PRIO=$v timeout -k 10 300 python3 -u bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline --no-e2e \
                > "$out/rbp${v}_c${c}_$RANDOM.json" 2> /dev/null || { rc=$?; break 2; }; rc=0; done; done ;;
    wprio) for v in ${WPS:-1 0 1 0}; do for c in ${PCFGS:-5}; do
              UMICLUST_RB_WPRIO=$v timeout -k 10 300 python3 -u bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline --no-e2e \
                > "$out/wp${v}_c${c}_$RANDOM.json" 2> /dev/null || { rc=$?; break 2; }; rc=0; done; done ;;
    bwprio) for v in ${WPS:-1 0 1 0}; do for c in ${PCFGS:-5}; do
              UMICLUST_BAND_WPRIO=$v timeout -k 10 300 python3 -u bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline --no-e2e \
                > "$out/bwp${v}_c${c}_$RANDOM.json" 2> /dev/null || { rc=$?; break 2; }; rc=0; done; done ;;
    recab) for v in ${RECS:-1 0 1 0 1 0}; do for c in ${PCFGS:-2}; do
              UMICLUST_REC_DIRECT=$v timeout -k 10 300 python3 -u bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline --no-e2e \
                > "$out/rec${v}_c${c}_$RANDOM.json" 2> /dev/null || { rc=$?; break 2; }; rc=0; done; done ;;
    rtab) for v in ${RTS:-8 12 16 8 12 16}; do for c in ${PCFGS:-2 5}; do
              UMICLUST_RESOLVE_THREADS=$v timeout -k 10 300 python3 -u bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline --no-e2e \
                > "$out/rt${v}_c${c}_$RANDOM.json" 2> /dev/null || { rc=$?; break 2; }; rc=0; done; done ;;
    rbab) for v in ${RBS:-4096 0 4096 0}; do for c in ${PCFGS:-5}; do
              UMICLUST_RB_DIRECT=$v timeout -k 10 300 python3 -u bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline --no-e2e \
                > "$out/rb${v}_c${c}_$RANDOM.json" 2> /dev/null || { rc=$?; break 2; }; rc=0; done; done ;;
    dbg2) for c in ${PCFGS:-2 5}; do UMICLUST_DEBUG=2 timeout -k 10 300 python3 -u bench.py --config $c --steps 2 --warmup 1 \
             --no-cpu-baseline --no-e2e > "$out/dbg2_c$c.json" 2> "$out/dbg2_c$c.err" || { rc=$?; break; }; rc=0; done ;;
    c5dbg) UMICLUST_DEBUG=1 timeout -k 10 300 python3 -u bench.py --config 5 --steps 1 --warmup 1 --no-cpu-baseline \
             > "$out/c5dbg.json" 2> "$out/c5dbg.err"; rc=$? ;;
    lazyab) for v in ${LAZYS:-5 0 5 0}; do for c in ${PCFGS:-5 2 3 4}; do
              UMICLUST_LAZY=$v timeout -k 10 500 python3 -u bench.py --config $c --steps 2 --warmup 1 --no-cpu-baseline --no-e2e \
                > "$out/lz${v}_c${c}_$RANDOM.json" 2> /dev/null || { rc=$?; break 2; }; rc=0; done; done ;;
    ldsprobe) timeout -k 10 120 ./tools/lds_atom_probe 2.4 > "$out/lds_atom_probe.jsonl" 2>&1; rc=$? ;;
    arrcheck) timeout -k 10 120 ./tools/arrange_check > "$out/arrange_check.json" 2>&1; rc=$? ;;
    alignt) timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "align or golden or o4" \
             > "$out/alignt.log" 2>&1; rc=$?; tail -3 "$out/alignt.log" ;;
    ptab) for v in ${PTS:-1 0 1 0 1 0}; do for c in ${PCFGS:-2 3 5}; do
              UMICLUST_PT_SIDE=$v timeout -k 10 500 python3 -u bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline --no-e2e \
                > "$out/pt${v}_c${c}_$RANDOM.json" 2> /dev/null || { rc=$?; break 2; }; rc=0; done; done ;;
    resdump) # the recorded resolve passes of the ThreadSanitizer replay (tests/golden/resolve/)
          timeout -k 10 300 python3 -u tests/golden/make_resolve_dumps.py "$out/resolve" > "$out/resdump.log" 2>&1; rc=$? ;;
    *) echo "unknown step $st"; rc=2 ;;
  esac
  echo "== $st rc=$rc $(date +%T)"
  [ $rc != 0 ] && exit $rc
done
exit 0
