#!/bin/bash
# Box: the driver's exact N=1 command repeated, to characterise run-to-run spread on the final tree.
set -o pipefail
out=${1:-gpurun_out/repeat}
n=${2:-8}
mkdir -p "$out"
for i in $(seq 1 $n); do
  timeout -k 10 240 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $out/n1_$i.json 2> $out/n1_$i.err || exit $?
  python scripts/box/summarize.py $out/n1_$i.json
done
