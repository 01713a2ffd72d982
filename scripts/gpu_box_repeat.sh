#!/bin/bash
# Repeated N=1/2/4 bench runs (variance estimate): usage gpu_box_repeat.sh REPEATS
mkdir -p gpurun_out
fatal() { case "$1" in 124|134|137|139) echo "fatal status $1 in $2; stopping"; exit "$1";; esac; }
python native/build.py > gpurun_out/build.log 2>&1 || exit 1
for r in $(seq 1 ${1:-2}); do
  timeout -k 10 300 python bench.py > gpurun_out/rep${r}_n1.json 2>/dev/null; s=$?; fatal $s n1; echo "rep $r n1: $s"
  for n in 2 4; do
    timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 \
      --master-port 2970$n bench.py --gpus $n > gpurun_out/rep${r}_n$n.json 2>/dev/null; s=$?; fatal $s n$n; echo "rep $r n$n: $s"
  done
done
for f in gpurun_out/rep*_n*.json; do python -c "
import json; d=json.loads(open('$f').read().strip().splitlines()[-1]); print('$f', d['value'], d['ms_per_step'], d['p50_latency_ms'], d['p99_latency_ms'], d['cold_start_s'])"; done
