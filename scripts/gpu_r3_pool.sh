#!/bin/bash
# connections per shard (NCC_POOL_SIZE) A/B in alternation at 0 ms and 5 ms.  Usage: bash scripts/gpu_r3_pool.sh <dir>
set -o pipefail
out=gpurun_out/$1
mkdir -p $out
for i in 1 2; do
  for ps in 256 64 32; do
    for lat in 0 5; do
      name=p${ps}_l${lat}_$i
      timeout -k 10 150 python3 bench.py --gpus 1 --steps 20 --warmup 5 --shard-latency-ms $lat --extra-env NCC_POOL_SIZE=$ps > $out/$name.json 2> $out/$name.err || exit 1
      python3 -c "import json;d=json.loads(open('$out/$name.json').read().strip().splitlines()[-1]);print('$name',d['value'],d['p50_latency_ms'],d['p99_latency_ms'],d['controller_cpu_us_per_object_split'],flush=True)"
    done
  done
done
