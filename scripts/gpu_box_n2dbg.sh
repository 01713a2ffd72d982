#!/bin/bash
mkdir -p gpurun_out
fatal() { case "$1" in 124|134|137|139) echo "fatal status $1 in $2; stopping"; exit "$1";; esac; }
python native/build.py > gpurun_out/build.log 2>&1 || exit 1
for r in 1 2 3 4; do
  NCC_BENCH_DEBUG=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 2990$r bench.py --gpus 2 --keep --extra-env NCC_CPU_REPORT=1 --extra-env NEXUS__LOG_LEVEL=INFO > gpurun_out/n2dbg_$r.json 2> gpurun_out/n2dbg_$r.err
  s=$?; fatal $s r$r
  python -c "
import json; d=json.loads(open('gpurun_out/n2dbg_$r.json').read().strip().splitlines()[-1]); print('r=$r', d['value'], d['p50_latency_ms'], d['p99_latency_ms'])"
  cp /tmp/ncc-bench-r0-*/controller.log gpurun_out/n2dbg_${r}_controller.log 2>/dev/null; rm -rf /tmp/ncc-bench-r*
done
