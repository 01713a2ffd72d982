#!/bin/bash
# Box: what coordinator partitions cost a single shard apiserver (each partition brings its own executor, so
# the shard serves C watch streams per kind): N=1 with C=1/2/4 forced, in alternation.
set -o pipefail
out=${1:-gpurun_out/c_on_one_shard}
mkdir -p "$out"
for i in 1 2; do
  for c in 1 2 4; do
    timeout -k 10 300 python bench.py --steps 20 --warmup 5 \
      --extra-env NEXUS__COORDINATOR_PARTITIONS=$c > $out/c${c}_$i.json 2> $out/c${c}_$i.err || exit $?
    python scripts/box/summarize.py $out/c${c}_$i.json
  done
done
