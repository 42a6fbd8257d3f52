#!/bin/bash
# A/B of split passes (UMICLUST_SPLIT=1, default) against whole passes (0) on configs 2, 3, 5; one line each.
set -o pipefail
out=gpurun_out/${1:-ab}
mkdir -p "$out"
export TMPDIR=/tmp
for cfg in 2 5 3; do
  for sp in 1 0; do
    st=2; [ $cfg = 3 ] && st=1
    UMICLUST_SPLIT=$sp timeout -k 10 400 python3 -u bench.py --config $cfg --steps $st --warmup 1 --no-cpu-baseline \
      > "$out/c${cfg}_s$sp.json" 2> "$out/c${cfg}_s$sp.err" || exit $?
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read()); print(sys.argv[1], round(d['value']), round(d['ms_per_step'],1))" "$out/c${cfg}_s$sp.json"
  done
done
