#!/bin/bash
# Box A/B in alternation: bench_prev.py (A) vs bench.py (B), driver shape (--steps 20 --warmup 5).
set -o pipefail
out=${1:-gpurun_out/ab}
mkdir -p "$out"
for i in 1 2 3; do
  for v in prev cur; do
    f=bench.py; [ $v = prev ] && f=bench_prev.py
    timeout -k 10 240 python $f --steps 20 --warmup 5 > $out/${v}_$i.json 2> $out/${v}_$i.err || exit $?
    python scripts/box/summarize.py $out/${v}_$i.json
  done
done
