#!/bin/bash
# Round-2 profiling session (config 2): GPU tests, bench, kernel trace, PMC passes (FETCH, WRITE, SQ).
set -o pipefail
out=gpurun_out/${1:-prof}
mkdir -p "$out"
export TMPDIR=/tmp
B="bench.py --steps 1 --warmup 0 --no-cpu-baseline"
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$out/tests.log" 2>&1 &&
timeout -k 10 300 python3 -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > "$out/c2.json" 2> "$out/c2.err" &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/trace" -o run -- python3 $B > "$out/trace.log" 2>&1 &&
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$out/pmc_fetch" -o run -- python3 $B > "$out/pmc_fetch.log" 2>&1 &&
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$out/pmc_write" -o run -- python3 $B > "$out/pmc_write.log" 2>&1 &&
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE \
  --output-format csv -d "$out/pmc_sq" -o run -- python3 $B > "$out/pmc_sq.log" 2>&1 &&
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS SQ_INSTS_BRANCH \
  --output-format csv -d "$out/pmc_sq2" -o run -- python3 $B > "$out/pmc_sq2.log" 2>&1
rc=$?
tail -2 "$out/tests.log"
cut -c1-300 "$out/c2.json"
exit $rc
