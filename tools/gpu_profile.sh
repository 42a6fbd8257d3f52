#!/bin/bash
# One GPU-box profiling session (run through gpurun from the repo root):
#   bench (JSON line), rocprofv3 kernel-trace stats, and separate PMC passes (FETCH_SIZE, WRITE_SIZE,
#   SQ/TCC counters) over a 1-step bench; every step under its own time limit, chained with &&.
# Usage: bash tools/gpu_profile.sh <tag> [bench args...]
set -o pipefail
tag=${1:-run}
shift
out=gpurun_out/$tag
mkdir -p "$out"
export TMPDIR=/tmp
B="bench.py --steps 1 --warmup 0 --no-cpu-baseline $*"
timeout -k 10 300 python3 -u bench.py --steps 3 --warmup 1 "$@" > "$out/bench.json" 2> "$out/bench.err" &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/trace" -o run -- python3 $B \
    > "$out/trace.log" 2>&1 &&
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$out/pmc_fetch" -o run -- python3 $B \
    > "$out/pmc_fetch.log" 2>&1 &&
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$out/pmc_write" -o run -- python3 $B \
    > "$out/pmc_write.log" 2>&1 &&
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE TCC_HIT_sum TCC_MISS_sum \
    --output-format csv -d "$out/pmc_sq" -o run -- python3 $B > "$out/pmc_sq.log" 2>&1
rc=$?
find "$out" -name '*.csv' | head -50
exit $rc
