#!/bin/bash
# Box: config 2 (2 shards, 100 templates x 2 dependents, 10 waves) three times per mode, per-wave max latency.
set -o pipefail
out=${1:-gpurun_out/cfg2}
mkdir -p "$out"
for i in 1 2 3; do
  timeout -k 10 200 python -u bench/suite.py --configs 2 --modes native,compat-unthrottled --timeout 60 \
    --out $out/cfg2_$i.json > $out/cfg2_$i.log 2>&1 || exit $?
  python -c "import json
for r in json.load(open('$out/cfg2_$i.json')): print(r['mode'], r['waves']['p50_ms'], r['waves']['p99_ms'], r['waves']['max_ms_per_wave'])"
done
