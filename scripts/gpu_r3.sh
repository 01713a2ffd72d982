#!/bin/bash
# Round-3 box check: N=1 bench x3 (driver shape) and the 8-shard one-rank topology x2, with per-stage latency.
mkdir -p gpurun_out/$1
fatal() { case "$1" in 124|134|137|139) echo "fatal status $1 in $2; stopping"; exit "$1";; esac; }
for i in 1 2 3; do
  timeout -k 10 150 python3 bench.py --gpus 1 --steps 20 --warmup 5 --stages > gpurun_out/$1/n1_$i.json 2> gpurun_out/$1/n1_$i.err; s=$?; fatal $s n1_$i
done
for i in 1 2; do
  timeout -k 10 200 python3 bench.py --gpus 1 --steps 20 --warmup 5 --shards-per-rank 8 > gpurun_out/$1/s8_$i.json 2> gpurun_out/$1/s8_$i.err; s=$?; fatal $s s8_$i
done
for f in gpurun_out/$1/*.json; do python3 -c "
import json; d=json.loads(open('$f').read().strip().splitlines()[-1]); c=d['cpu_cores_busy']; ms=d['ms_per_step']; n=d['config']['shards']
print('$f', d['value'], d['p50_latency_ms'], d['p99_latency_ms'], d['controller_cpu_us_per_object_split'], {k: v for k, v in c.items()}, (d.get('stages') or {}).get('p99_owner'))"; done
