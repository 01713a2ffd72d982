#!/bin/bash
# Template-count scale runs (20k, 50k templates on one shard).  Usage: bash scripts/gpu_r3_scale.sh <dir>
set -o pipefail
out=gpurun_out/$1
mkdir -p $out
for T in 20000 50000; do
  timeout -k 10 500 python3 bench.py --templates $T --steps 5 --warmup 4 > $out/t$T.json 2> $out/t$T.err || exit 1
  python3 -c "import json;d=json.loads(open('$out/t$T.json').read().strip().splitlines()[-1]);print($T,d['value'],d['p50_latency_ms'],d['p99_latency_ms'],d['controller_cpu_us_per_object_split'],d['rss_mib'],d['cold_start_s'],flush=True)"
done
