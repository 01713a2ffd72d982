#!/bin/bash
# N=4 re-check: lat 0 and 5 ms, twice each, alternating.  Usage: bash scripts/gpu_r3_n4.sh <out dir name> [extra bench args]
set -o pipefail
out=gpurun_out/$1
shift
mkdir -p $out
port=29810
for i in 1 2; do
  for lat in 0 5; do
    port=$((port + 1))
    name=n4_lat${lat}_$i
    timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 \
      --master-port $port bench.py --gpus 4 --steps 20 --warmup 5 --shard-latency-ms $lat "$@" > $out/$name.json 2> $out/$name.err || exit $?
    python3 -c "import json;d=json.loads([l for l in open('$out/$name.json').read().splitlines() if l.startswith('{')][-1]);print('$name',d['value'],d['p50_latency_ms'],d['p99_latency_ms'],d['controller_cpu_us_per_object'],d['controller_cpu_us_per_object_split'],d['cpu_cores_busy'],flush=True)"
  done
done
