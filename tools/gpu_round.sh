#!/bin/bash
# GPU-box session: parity tests, then bench legs; every step under its own time limit, chained with &&
# so the first failure (or fault / timeout) ends the call.
# Usage: bash tools/gpu_round.sh <tag> <steps...>   steps: tests | c2 | c3 | c4 | c5 | e2e | trace
set -o pipefail
tag=${1:-run}
shift
out=gpurun_out/$tag
mkdir -p "$out"
export TMPDIR=/tmp
rc=0
for st in "$@"; do
  echo "== $st $(date +%T)"
  case $st in
    tests) timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
             > "$out/tests.log" 2>&1; rc=$?; tail -3 "$out/tests.log" ;;
    c2) timeout -k 10 300 python3 -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > "$out/c2.json" 2> "$out/c2.err"; rc=$? ;;
    c3cpu) timeout -k 10 500 python3 -u bench.py --config 3 --steps 1 --warmup 1 > "$out/c3cpu.json" 2> "$out/c3cpu.err"; rc=$? ;;
    c2cpu) timeout -k 10 300 python3 -u bench.py --steps 2 --warmup 1 > "$out/c2cpu.json" 2> "$out/c2cpu.err"; rc=$? ;;
    c3) timeout -k 10 400 python3 -u bench.py --config 3 --steps 2 --warmup 1 --no-cpu-baseline > "$out/c3.json" 2> "$out/c3.err"; rc=$? ;;
    c4) timeout -k 10 600 python3 -u bench.py --config 4 --steps 1 --warmup 0 --no-cpu-baseline > "$out/c4.json" 2> "$out/c4.err"; rc=$? ;;
    c5) timeout -k 10 300 python3 -u bench.py --config 5 --steps 2 --warmup 1 --no-cpu-baseline > "$out/c5.json" 2> "$out/c5.err"; rc=$? ;;
    e2e) timeout -k 10 400 python3 -u bench.py --steps 1 --warmup 1 --no-cpu-baseline --e2e > "$out/e2e.json" 2> "$out/e2e.err"; rc=$? ;;
    trace) timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/trace" -o run -- \
             python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline > "$out/trace.log" 2>&1; rc=$? ;;
    pmc_fetch|pmc_write|pmc_sq|pmc_valu|pmc_l2|pmc_inst)
       case $st in
         pmc_inst) ctr="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_BRANCH SQ_INSTS_VMEM_WR" ;;
         pmc_l2) ctr="TCC_REQ_sum TCC_HIT_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum" ;;
         pmc_fetch) ctr="FETCH_SIZE" ;;
         pmc_write) ctr="WRITE_SIZE" ;;
         pmc_sq) ctr="SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE" ;;
         pmc_valu) ctr="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY" ;;
       esac
       timeout -s KILL 300 rocprofv3 --pmc $ctr --output-format csv -d "$out/$st" -o run -- \
         python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline > "$out/$st.log" 2>&1; rc=$? ;;
    trace3) timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/trace3" -o run -- \
             python3 bench.py --config 3 --lanes 1 --steps 1 --warmup 0 --no-cpu-baseline > "$out/trace3.log" 2>&1; rc=$? ;;
    *) echo "unknown step $st"; rc=2 ;;
  esac
  echo "== $st rc=$rc $(date +%T)"
  [ $rc -ne 0 ] && break
done
for f in "$out"/*.json; do [ -f "$f" ] && { echo "--- $f"; cut -c1-600 "$f"; }; done
exit $rc
