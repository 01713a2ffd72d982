#!/bin/bash
# Box: eight shards on one rank with coordinator partitions C=1/2/4 in alternation.
set -o pipefail
out=${1:-gpurun_out/spr8_c}
mkdir -p "$out"
for i in 1 2; do
  for c in 1 2 4; do
    timeout -k 10 300 python bench.py --shards-per-rank 8 --steps 20 --warmup 5 \
      --extra-env NEXUS__COORDINATOR_PARTITIONS=$c > $out/c${c}_$i.json 2> $out/c${c}_$i.err || exit $?
    python scripts/box/summarize.py $out/c${c}_$i.json
  done
done
