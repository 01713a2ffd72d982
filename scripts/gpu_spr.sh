#!/bin/bash
# Many shards on the 1-GPU box: one rank hosting S shard apiservers (coordinator load at 4 and 8 shards).
mkdir -p gpurun_out
fatal() { case "$1" in 124|134|137|139) echo "fatal status $1 in $2; stopping"; exit "$1";; esac; }
python native/build.py > gpurun_out/build.log 2>&1 || exit 1
for S in 4 8; do
  timeout -k 10 300 python bench.py --shards-per-rank $S > gpurun_out/spr_$S.json 2>gpurun_out/spr_$S.err; s=$?; fatal $s spr$S
  python -c "
import json; d=json.loads(open('gpurun_out/spr_$S.json').read().strip().splitlines()[-1]); c=d['cpu_cores_busy']; ms=d['ms_per_step']
print('S=$S', d['value'], d['p50_latency_ms'], c, 'coordinator us/template-pass', round(c['coordinator']*ms*1000/1000,1))"
done
