#!/bin/bash
# A/B at N=1 (ab_old vs current, AB_REPS alternations), then N=2 and N=4 runs of the current tree.
mkdir -p gpurun_out
fatal() { case "$1" in 124|134|137|139) echo "fatal status $1 in $2; stopping"; exit "$1";; esac; }
bash scripts/gpu_ab.sh "$@" || exit $?
for n in 2 4; do
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 \
    --master-port 2980$n bench.py --gpus $n "$@" > gpurun_out/scale_n$n.json 2>/dev/null; s=$?; fatal $s n$n
  python -c "
import json; d=json.loads(open('gpurun_out/scale_n$n.json').read().strip().splitlines()[-1])
print('N=$n', d['value'], d['p50_latency_ms'], d['cpu_cores_busy'])"
done
