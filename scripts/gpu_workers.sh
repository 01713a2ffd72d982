#!/bin/bash
# Worker-count sweep on the box (bench N=1, then N=4 for the two best candidates).
mkdir -p gpurun_out
fatal() { case "$1" in 124|134|137|139) echo "fatal status $1 in $2; stopping"; exit "$1";; esac; }
python native/build.py > gpurun_out/build.log 2>&1 || exit 1
for r in 1 2; do
for w in 8 16 32 64; do
  timeout -k 10 300 python bench.py --workers $w > gpurun_out/wk_${w}_$r.json 2>/dev/null; s=$?; fatal $s w$w
  python -c "
import json; d=json.loads(open('gpurun_out/wk_${w}_$r.json').read().strip().splitlines()[-1]); c=d['cpu_cores_busy']; ms=d['ms_per_step']
print('workers=$w', d['value'], d['p50_latency_ms'], {k: round(v*ms*1000/3000,1) for k,v in c.items() if k!='shard-apiserver-max'})"
done; done
for w in 16 64; do
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 \
    --master-port 2990$((w % 10)) bench.py --gpus 4 --workers $w > gpurun_out/wk4_${w}.json 2>/dev/null; s=$?; fatal $s n4w$w
  python -c "
import json; d=json.loads(open('gpurun_out/wk4_${w}.json').read().strip().splitlines()[-1])
print('N=4 workers=$w', d['value'], d['p50_latency_ms'], d['cpu_cores_busy'])"
done
