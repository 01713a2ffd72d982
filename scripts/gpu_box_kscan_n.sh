#!/bin/bash
# executors-per-shard scan at N ranks: usage gpu_box_kscan_n.sh N k1 k2 ...
mkdir -p gpurun_out
fatal() { case "$1" in 124|134|137|139) echo "fatal status $1 in $2; stopping"; exit "$1";; esac; }
python native/build.py > gpurun_out/build.log 2>&1 || exit 1
n=$1; shift
for k in "$@"; do
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 \
    --master-port 2980$k bench.py --gpus $n --extra-env NEXUS__EXECUTORS_PER_SHARD=$k > gpurun_out/kscan_n${n}_k$k.json 2>/dev/null
  s=$?; fatal $s k$k; echo "n=$n k=$k: $s"
done
for k in "$@"; do python -c "
import json; d=json.loads(open('gpurun_out/kscan_n${n}_k$k.json').read().strip().splitlines()[-1]); print('k=$k', d['value'], d['ms_per_step'], d['p50_latency_ms'], d['cpu_cores_busy'])"; done
