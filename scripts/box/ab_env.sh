#!/bin/bash
# Box A/B in alternation of one controller environment override: A = bench with --extra-env "$AB_ENV",
# B = the tree's defaults; driver shape.  usage: AB_ENV=KEY=VAL bash scripts/box/ab_env.sh <outdir> [pairs]
set -o pipefail
out=${1:-gpurun_out/ab_env}
pairs=${2:-3}
mkdir -p "$out"
for i in $(seq 1 $pairs); do
  timeout -k 10 240 python bench.py --steps 20 --warmup 5 --extra-env "$AB_ENV" > $out/prev_$i.json 2> $out/prev_$i.err || exit $?
  python scripts/box/summarize.py $out/prev_$i.json
  timeout -k 10 240 python bench.py --steps 20 --warmup 5 > $out/cur_$i.json 2> $out/cur_$i.err || exit $?
  python scripts/box/summarize.py $out/cur_$i.json
done
