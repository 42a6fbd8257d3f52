#!/bin/bash
# A/B of environment variants on one config, interleaved and repeated: bash tools/ab_env.sh <tag> <config> <steps> <reps> "<ENV=..>" ...
set -o pipefail
out=gpurun_out/$1; cfg=$2; steps=$3; reps=$4; shift 4
mkdir -p "$out"
export TMPDIR=/tmp
for r in $(seq 1 $reps); do
  i=0
  for v in "$@"; do
    i=$((i+1))
    env $v timeout -k 10 400 python3 -u bench.py --config $cfg --steps $steps --warmup 1 --no-cpu-baseline \
      > "$out/v${i}_r$r.json" 2> "$out/v${i}_r$r.err" || exit $?
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read()); print(sys.argv[2], round(d['value']), round(d['ms_per_step'],1))" "$out/v${i}_r$r.json" "$v"
  done
done
