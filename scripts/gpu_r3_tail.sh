#!/bin/bash
# Late round-3 box check: GPU tier, smoke, the driver's bench shape three times, then the five BASELINE
# configurations (native).  Usage: bash scripts/gpu_r3_tail.sh <out dir name>
set -o pipefail
out=gpurun_out/$1
mkdir -p $out
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $out/pytest_gpu.log 2>&1 || exit $?
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || exit $?
for i in 1 2 3; do
  timeout -k 10 150 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $out/bench_$i.json 2> $out/bench_$i.err || exit $?
  python3 -c "import json;d=json.loads(open('$out/bench_$i.json').read().strip().splitlines()[-1]);print('bench_$i',d['value'],d['p50_latency_ms'],d['p99_latency_ms'],d['controller_cpu_us_per_object_split'],d['cpu_cores_busy']['coordinator'],flush=True)"
done
timeout -k 10 600 python3 bench/suite.py --modes native --out $out/suite.json > $out/suite.log 2>&1 || exit $?
tail -1 $out/pytest_gpu.log
tail -1 $out/smoke.log
cut -c 1-300 $out/suite.log | tail -12
