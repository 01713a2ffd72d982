#!/bin/bash
# event-repeat-window 1s vs 10s: ABBA at 1000 templates, then one pair at 20 000.  Usage: bash scripts/gpu_r3_rw.sh <dir>
set -o pipefail
out=gpurun_out/$1
mkdir -p $out
i=0
for w in 1s 10s 10s 1s; do
  i=$((i + 1)); name=w${w}_$i
  timeout -k 10 150 python3 bench.py --gpus 1 --steps 20 --warmup 5 --extra-env NEXUS__EVENT_REPEAT_WINDOW=$w > $out/$name.json 2> $out/$name.err || exit 1
  python3 -c "import json;d=json.loads(open('$out/$name.json').read().strip().splitlines()[-1]);print('$name',d['value'],d['p50_latency_ms'],d['p99_latency_ms'],d['controller_cpu_us_per_object_split'],d['cpu_cores_busy']['controller-apiserver'],flush=True)"
done
for w in 1s 10s; do
  name=t20k_w${w}
  timeout -k 10 500 python3 bench.py --templates 20000 --steps 5 --warmup 4 --extra-env NEXUS__EVENT_REPEAT_WINDOW=$w > $out/$name.json 2> $out/$name.err || exit 1
  python3 -c "import json;d=json.loads(open('$out/$name.json').read().strip().splitlines()[-1]);print('$name',d['value'],d['p50_latency_ms'],d['p99_latency_ms'],d['controller_cpu_us_per_object_split'],d['cpu_cores_busy']['controller-apiserver'],flush=True)"
done
