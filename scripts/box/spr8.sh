#!/bin/bash
# Box: eight shard apiservers on one rank (experiment shape; the driver's N=8 is one shard per GPU on a node)
set -o pipefail
out=${1:-gpurun_out/spr8}
mkdir -p "$out"
b() {
  local name=$1; shift
  timeout -k 10 300 python bench.py "$@" > $out/$name.json 2> $out/$name.err || exit $?
  python scripts/box/summarize.py $out/$name.json
}
b spr8_auto --shards-per-rank 8 --steps 20 --warmup 5
b spr8_c4 --shards-per-rank 8 --steps 20 --warmup 5 --extra-env NEXUS__COORDINATOR_PARTITIONS=4
b spr4_auto --shards-per-rank 4 --steps 20 --warmup 5
