#!/bin/bash
# GC freeze policy A/B: round-2 "5,1" vs the new default "1,none", ABBA at 1000 templates, then a pair at 20 000.
# Usage: bash scripts/gpu_r3_gc.sh <dir>
set -o pipefail
out=gpurun_out/$1
mkdir -p $out
i=0
for g in 5,1 1,none 1,none 5,1; do
  i=$((i + 1)); name=g${g/,/_}_$i
  timeout -k 10 150 python3 bench.py --gpus 1 --steps 20 --warmup 5 --extra-env NCC_GC_FREEZE=$g > $out/$name.json 2> $out/$name.err || exit 1
  python3 -c "import json;d=json.loads(open('$out/$name.json').read().strip().splitlines()[-1]);print('$name',d['value'],d['p50_latency_ms'],d['p99_latency_ms'],d['controller_cpu_us_per_object_split'],d['rss_mib']['coordinator'],flush=True)"
done
for g in 5,1 1,none; do
  name=t20k_g${g/,/_}
  timeout -k 10 500 python3 bench.py --templates 20000 --steps 5 --warmup 4 --extra-env NCC_GC_FREEZE=$g > $out/$name.json 2> $out/$name.err || exit 1
  python3 -c "import json;d=json.loads(open('$out/$name.json').read().strip().splitlines()[-1]);print('$name',d['value'],d['p50_latency_ms'],d['p99_latency_ms'],d['controller_cpu_us_per_object_split'],d['rss_mib']['coordinator'],flush=True)"
done
