#!/bin/bash
# Worker-count sweep at N=2 and N=4 (16 vs 32 per executor).
mkdir -p gpurun_out
fatal() { case "$1" in 124|134|137|139) echo "fatal status $1 in $2; stopping"; exit "$1";; esac; }
python native/build.py > gpurun_out/build.log 2>&1 || exit 1
for r in 1 2; do for n in 2 4; do for w in 16 32; do
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 \
    --master-port 299$n$((w % 10)) bench.py --gpus $n --workers $w > gpurun_out/wkn${n}_${w}_$r.json 2>/dev/null; s=$?; fatal $s n${n}w$w
  python -c "
import json; d=json.loads(open('gpurun_out/wkn${n}_${w}_$r.json').read().strip().splitlines()[-1])
print('N=$n workers=$w', d['value'], d['p50_latency_ms'], d['cpu_cores_busy']['executors'], d['cpu_cores_busy']['coordinator'])"
done; done; done
