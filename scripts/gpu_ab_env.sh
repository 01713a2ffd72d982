#!/bin/bash
# A/B of one controller environment override on the same tree, interleaved: gpu_ab_env.sh <dir> <KEY=VAL> <reps> [bench args...]
d=$1; kv=$2; reps=$3; shift 3
mkdir -p gpurun_out/$d
fatal() { case "$1" in 124|134|137|139) echo "fatal status $1 in $2; stopping"; exit "$1";; esac; }
for i in $(seq 1 $reps); do
  timeout -k 10 200 python3 bench.py "$@" > gpurun_out/$d/a_$i.json 2>/dev/null; s=$?; fatal $s a$i
  timeout -k 10 200 python3 bench.py "$@" --extra-env "$kv" > gpurun_out/$d/b_$i.json 2>/dev/null; s=$?; fatal $s b$i
done
for f in gpurun_out/$d/a_*.json gpurun_out/$d/b_*.json; do python3 -c "
import json; d=json.loads(open('$f').read().strip().splitlines()[-1]); c=d['cpu_cores_busy']
print('$f', d['value'], d['p50_latency_ms'], d['p99_latency_ms'], d['controller_cpu_us_per_object_split'], {k: v for k, v in c.items()})"; done
