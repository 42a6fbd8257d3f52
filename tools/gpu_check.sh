#!/bin/bash
# GPU-box check: parity tests, then one bench line (no CPU baseline) and a kernel-trace summary.
# Usage: bash tools/gpu_check.sh <tag> [bench args...]
set -o pipefail
tag=${1:-run}
shift
out=gpurun_out/$tag
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$out/tests.log" 2>&1 &&
timeout -k 10 300 python3 -u bench.py --steps 3 --warmup 1 --no-cpu-baseline "$@" > "$out/bench.json" 2> "$out/bench.err" &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/trace" -o run -- \
    python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline "$@" > "$out/trace.log" 2>&1
rc=$?
tail -3 "$out/tests.log"
cat "$out/bench.json"
exit $rc
