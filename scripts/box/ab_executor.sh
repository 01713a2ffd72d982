#!/bin/bash
# Box A/B in alternation: ab_prev/ncc-executor (A) vs the tree's ncc/bin/ncc-executor (B), driver shape.
# usage: bash scripts/box/ab_executor.sh <outdir> [pairs]
set -o pipefail
out=${1:-gpurun_out/ab_exec}
pairs=${2:-3}
mkdir -p "$out"
for i in $(seq 1 $pairs); do
  for v in prev cur; do
    if [ $v = prev ]; then export NCC_EXECUTOR_BINARY=$PWD/ab_prev/ncc-executor; else unset NCC_EXECUTOR_BINARY; fi
    timeout -k 10 240 python bench.py --steps 20 --warmup 5 > $out/${v}_$i.json 2> $out/${v}_$i.err || exit $?
    python scripts/box/summarize.py $out/${v}_$i.json
  done
done
