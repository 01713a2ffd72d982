#!/bin/bash
# Box: per-wave timeline (NCC_BENCH_DEBUG) and a cProfile of the coordinator over a bench run.
set -o pipefail
out=${1:-gpurun_out/timeline}
mkdir -p "$out"
NCC_BENCH_DEBUG=1 timeout -k 10 240 python bench.py --steps 8 --warmup 2 > $out/debug.json 2> $out/debug.err || exit $?
python scripts/box/summarize.py $out/debug.json
timeout -k 10 240 python bench.py --steps 20 --warmup 5 --extra-env NCC_PROFILE=$PWD/$out/coord.prof > $out/prof.json 2> $out/prof.err || exit $?
python scripts/box/summarize.py $out/prof.json
python -c "import pstats; pstats.Stats('$out/coord.prof').sort_stats('tottime').print_stats(40)" > $out/coord_tottime.txt
python -c "import pstats; pstats.Stats('$out/coord.prof').sort_stats('cumtime').print_stats(60)" > $out/coord_cumtime.txt
for i in 1 2 3; do
  timeout -k 10 240 python bench.py --steps 20 --warmup 5 > $out/default_$i.json 2> $out/default_$i.err || exit $?
  python scripts/box/summarize.py $out/default_$i.json
done
