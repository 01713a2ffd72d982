#!/bin/bash
# Box: latency configs 1-3 in both modes, then two driver-shape bench runs.
set -o pipefail
out=${1:-gpurun_out/suite_small}
mkdir -p "$out"
timeout -k 10 300 python -u bench/suite.py --configs 1,2,3 --modes native,compat-unthrottled --churn-seconds 15 \
  --timeout 120 --out $out/suite.json > $out/suite.log 2>&1 || exit $?
for i in 1 2; do
  timeout -k 10 240 python bench.py --steps 20 --warmup 5 > $out/bench_$i.json 2> $out/bench_$i.err || exit $?
  python scripts/box/summarize.py $out/bench_$i.json
done
