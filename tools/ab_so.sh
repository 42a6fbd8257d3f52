#!/bin/bash
# Same-box A/B of two builds of libumiclust.so: ab_base/libumiclust.so (A) against the in-tree build (B).
# Usage: bash tools/ab_so.sh <tag> <configs...>   (each config: A, B, A, B; bench.py short lines)
set -o pipefail
tag=${1:-ab}; shift
out=gpurun_out/$tag; mkdir -p "$out"
L=ont-tcrconsensus_amd/umiclust/libumiclust.so
cp $L "$out/.new.so" || exit 1
rc=0
for c in "$@"; do
  for v in A B A B; do
    if [ $v = A ]; then cp ont-tcrconsensus_amd/ab_base/libumiclust.so $L; else cp "$out/.new.so" $L; fi
    timeout -k 10 400 python3 -u bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline --no-e2e \
      > "$out/c${c}_$v$RANDOM.json" 2>> "$out/err.log" || { rc=$?; break 2; }
  done
done
cp "$out/.new.so" $L; rm -f "$out/.new.so"
exit $rc
