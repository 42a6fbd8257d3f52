#!/bin/bash
# Round-2 last check (default pinning): GPU tests, smoke, default bench, config 5.
set -o pipefail
o=gpurun_out/fin2
mkdir -p $o
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $o/gpu_tests.log 2>&1 || exit $?
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.log 2>&1 || exit $?
timeout -k 10 400 python -u bench.py > $o/bench_c2.json 2> $o/bench_c2.err || exit $?
timeout -k 10 400 python -u bench.py --config 5 --steps 3 --warmup 1 --no-cpu-baseline > $o/bench_c5.json 2> $o/bench_c5.err || exit $?
