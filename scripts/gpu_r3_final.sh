#!/bin/bash
# Round-3 final box check: the GPU test tier, smoke, then the driver's bench shape twice.
# Usage: bash scripts/gpu_r3_final.sh <out dir name>
set -o pipefail
out=gpurun_out/$1
mkdir -p $out
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $out/pytest_gpu.log 2>&1 || exit $?
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || exit $?
for i in 1 2; do
  timeout -k 10 150 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $out/bench_$i.json 2> $out/bench_$i.err || exit $?
  python3 -c "import json;d=json.loads(open('$out/bench_$i.json').read().strip().splitlines()[-1]);print('bench_$i',d['value'],d['p50_latency_ms'],d['p99_latency_ms'],d['controller_cpu_us_per_object_split'],d['cpu_cores_busy']['coordinator'],flush=True)"
done
tail -1 $out/pytest_gpu.log
tail -1 $out/smoke.log
