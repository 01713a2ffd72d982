#!/bin/bash
# Box run: bench.py in the three modes (native / compat-unthrottled / compat) and the 8-shards-per-rank
# topology with coordinator partitions forced to C=4.  usage: bash scripts/box/baselines.sh <outdir>
set -o pipefail
out=${1:-gpurun_out/baselines}
mkdir -p "$out"
b() {  # name, args...
  local name=$1; shift
  timeout -k 10 300 python bench.py "$@" > $out/$name.json 2> $out/$name.err || exit $?
  python scripts/box/summarize.py $out/$name.json
}
b native_t100 --templates 100 --steps 5 --warmup 2
b unthrottled_t100 --mode compat-unthrottled --templates 100 --steps 5 --warmup 2
b unthrottled_t1000 --mode compat-unthrottled --steps 3 --warmup 1
b compat_t100 --mode compat --templates 100 --steps 2 --warmup 1 --timeout 200
b spr8_c1 --shards-per-rank 8 --steps 10 --warmup 3
b spr8_c4 --shards-per-rank 8 --steps 10 --warmup 3 --extra-env NEXUS__COORDINATOR_PARTITIONS=4
