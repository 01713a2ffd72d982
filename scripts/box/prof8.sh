#!/bin/bash
# Box: cProfile of the coordinator with 8 shards on one rank (C=1), plus a plain run for reference.
set -o pipefail
out=${1:-gpurun_out/prof8}
mkdir -p "$out"
timeout -k 10 300 python bench.py --shards-per-rank 8 --steps 20 --warmup 5 > $out/plain.json 2> $out/plain.err || exit $?
python scripts/box/summarize.py $out/plain.json
timeout -k 10 300 python bench.py --shards-per-rank 8 --steps 20 --warmup 5 \
  --extra-env NCC_PROFILE=$PWD/$out/coord.prof > $out/prof.json 2> $out/prof.err || exit $?
python scripts/box/summarize.py $out/prof.json
python -c "
import pstats
p = pstats.Stats('$out/coord.prof')
p.sort_stats('tottime').print_stats(45)
p.sort_stats('cumtime').print_stats(60)" > $out/coord_profile.txt
