#!/bin/bash
# Box A/B of two trees in alternation: abtree_prev/ (A: an earlier commit, built in-tree) vs this tree (B).
# usage: bash scripts/box/ab_tree.sh <outdir> <pairs> [bench args...]
set -o pipefail
out=${1:-gpurun_out/ab_tree}
pairs=${2:-3}
shift 2
mkdir -p "$out"
root=$PWD
for i in $(seq 1 $pairs); do
  (cd abtree_prev && timeout -k 10 300 python bench.py --steps 20 --warmup 5 "$@") > $out/prev_$i.json 2> $out/prev_$i.err || exit $?
  python scripts/box/summarize.py $out/prev_$i.json
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 "$@" > $out/cur_$i.json 2> $out/cur_$i.err || exit $?
  python scripts/box/summarize.py $out/cur_$i.json
done
