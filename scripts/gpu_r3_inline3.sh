#!/bin/bash
# NCC_INLINE_BATCH 256 vs 16 in ABBA order (cancels a box that drifts within the call).  Usage: bash scripts/gpu_r3_inline3.sh <dir>
set -o pipefail
out=gpurun_out/$1
mkdir -p $out
i=0
for b in 256 16 16 256 256 16 16 256; do
  i=$((i + 1))
  name=b${b}_$i
  timeout -k 10 150 python3 bench.py --gpus 1 --steps 20 --warmup 5 --stages --extra-env NCC_INLINE_BATCH=$b > $out/$name.json 2> $out/$name.err || exit 1
  python3 -c "
import json;d=json.loads(open('$out/$name.json').read().strip().splitlines()[-1]);s=d.get('stages') or {}
print('$name',d['value'],d['p50_latency_ms'],d['p99_latency_ms'],d['controller_cpu_us_per_object'],{k:(v['p50_ms'],v['p99_ms']) for k,v in s.items() if isinstance(v,dict) and 'p50_ms' in v},flush=True)"
done
