#!/bin/bash
# Box A/B in alternation of one controller environment override with extra bench arguments: A = bench with
# --extra-env "$AB_ENV", B = the tree's defaults.  usage: AB_ENV=KEY=VAL bash scripts/box/ab_env_args.sh <outdir> <pairs> [bench args...]
set -o pipefail
out=${1:-gpurun_out/ab_env}
pairs=${2:-3}
shift 2
mkdir -p "$out"
for i in $(seq 1 $pairs); do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --extra-env "$AB_ENV" "$@" > $out/prev_$i.json 2> $out/prev_$i.err || exit $?
  python scripts/box/summarize.py $out/prev_$i.json
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 "$@" > $out/cur_$i.json 2> $out/cur_$i.err || exit $?
  python scripts/box/summarize.py $out/cur_$i.json
done
