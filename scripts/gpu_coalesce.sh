#!/bin/bash
# Coalesce-window sweep on the box: suite config 1 (single-object latency) and bench N=1 (burst throughput).
mkdir -p gpurun_out
fatal() { case "$1" in 124|134|137|139) echo "fatal status $1 in $2; stopping"; exit "$1";; esac; }
python native/build.py > gpurun_out/build.log 2>&1 || exit 1
for r in 1 2; do
for w in 0.005 0.002 0.001; do
  NCC_OPT_COALESCE_WINDOW=$w timeout -k 10 120 python bench/suite.py --configs 1 --modes native --out gpurun_out/co_s1_${w}_$r.json > /dev/null 2>&1; s=$?; fatal $s s1
  timeout -k 10 300 python bench.py --extra-env NCC_OPT_COALESCE_WINDOW=$w > gpurun_out/co_b_${w}_$r.json 2>/dev/null; s=$?; fatal $s b
  python -c "
import json; s=json.load(open('gpurun_out/co_s1_${w}_$r.json'))[0]['waves']; b=json.loads(open('gpurun_out/co_b_${w}_$r.json').read().strip().splitlines()[-1])
print('w=$w', 'cfg1 p50', s['p50_ms'], 'p99', s['p99_ms'], '| bench', b['value'], 'p50', b['p50_latency_ms'])"
done; done
