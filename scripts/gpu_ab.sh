#!/bin/bash
# A/B: ab_old/ (previous tree) vs the current tree, alternating N=1 bench runs.
mkdir -p gpurun_out
fatal() { case "$1" in 124|134|137|139) echo "fatal status $1 in $2; stopping"; exit "$1";; esac; }
python native/build.py > gpurun_out/build.log 2>&1 || exit 1
(cd ab_old && python native/build.py > ../gpurun_out/build_old.log 2>&1) || exit 1
for i in $(seq 1 ${AB_REPS:-3}); do
  (cd ab_old && timeout -k 10 300 python bench.py "$@" > ../gpurun_out/ab_old_$i.json 2>/dev/null); s=$?; fatal $s old$i
  timeout -k 10 300 python bench.py "$@" > gpurun_out/ab_new_$i.json 2>/dev/null; s=$?; fatal $s new$i
done
for f in gpurun_out/ab_old_*.json gpurun_out/ab_new_*.json; do python -c "
import json,sys; d=json.loads(open('$f').read().strip().splitlines()[-1]); c=d['cpu_cores_busy']; ms=d['ms_per_step']
print('$f', d['value'], d['p50_latency_ms'], {k: round(v*ms*1000/3000/d['n_gpus'],1) for k,v in c.items()})"; done
