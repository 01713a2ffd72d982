#!/bin/bash
# Box: cProfile of the parent coordinator with 8 shards on one rank and C=4 (its own share of the per-template
# work is a quarter; what is left is relaying and report routing for every key).
set -o pipefail
out=${1:-gpurun_out/prof8_parent}
mkdir -p "$out"
timeout -k 10 300 python bench.py --shards-per-rank 8 --steps 20 --warmup 5 \
  --extra-env NEXUS__COORDINATOR_PARTITIONS=4 --extra-env NCC_PROFILE=$PWD/$out/coord.prof > $out/prof.json 2> $out/prof.err || exit $?
python scripts/box/summarize.py $out/prof.json
python -c "
import pstats
p = pstats.Stats('$out/coord.prof')
p.sort_stats('tottime').print_stats(40)
p.sort_stats('cumtime').print_stats(50)" > $out/parent_profile.txt
