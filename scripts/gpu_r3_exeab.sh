#!/bin/bash
# Executor binary A/B (ncc/bin/ncc-executor-old vs the current build), ABBA order.  Usage: bash scripts/gpu_r3_exeab.sh <dir>
set -o pipefail
out=gpurun_out/$1
mkdir -p $out
i=0
for v in old new new old old new new old; do
  i=$((i + 1))
  bin=$PWD/ncc/bin/ncc-executor; [ "$v" = old ] && bin=$PWD/ncc/bin/ncc-executor-old
  name=${v}_$i
  timeout -k 10 150 python3 bench.py --gpus 1 --steps 20 --warmup 5 --extra-env NCC_EXECUTOR_BINARY=$bin > $out/$name.json 2> $out/$name.err || exit 1
  python3 -c "import json;d=json.loads(open('$out/$name.json').read().strip().splitlines()[-1]);print('$name',d['value'],d['p50_latency_ms'],d['p99_latency_ms'],d['controller_cpu_us_per_object_split'],flush=True)"
done
