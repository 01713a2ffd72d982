#!/bin/bash
# 1k vs 20k templates in ABBA order (per-object CPU at scale, same session).  Usage: bash scripts/gpu_r3_scale2.sh <dir>
set -o pipefail
out=gpurun_out/$1
mkdir -p $out
i=0
for T in 1000 20000 20000 1000; do
  i=$((i + 1))
  steps=20; warm=5; [ "$T" = 20000 ] && steps=5 && warm=4
  timeout -k 10 500 python3 bench.py --templates $T --steps $steps --warmup $warm > $out/t${T}_$i.json 2> $out/t${T}_$i.err || exit 1
  python3 -c "import json;d=json.loads(open('$out/t${T}_$i.json').read().strip().splitlines()[-1]);print('t${T}_$i',d['value'],d['p50_latency_ms'],d['p99_latency_ms'],d['controller_cpu_us_per_object_split'],d['cpu_cores_busy'],flush=True)"
done
