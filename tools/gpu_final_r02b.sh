#!/bin/bash
# Round-2 closing run (after the banded aligner): GPU tests, smoke, benches of configs 2-5, kernel stats.
set -o pipefail
o=gpurun_out/fin
mkdir -p $o
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $o/gpu_tests.log 2>&1 || exit $?
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.log 2>&1 || exit $?
timeout -k 10 400 python -u bench.py > $o/bench_c2.json 2> $o/bench_c2.err || exit $?
for c in 5 3 4; do
  timeout -k 10 600 python -u bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline > $o/bench_c$c.json 2> $o/bench_c$c.err || exit $?
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $o/prof -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > $o/bench_c2_prof.json 2> $o/prof.err || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $o/prof5 -o run -- python3 bench.py --config 5 --steps 3 --warmup 1 --no-cpu-baseline > $o/bench_c5_prof.json 2> $o/prof5.err || exit $?
