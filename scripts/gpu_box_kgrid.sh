#!/bin/bash
# repeated executors-per-shard grid: usage gpu_box_kgrid.sh "Ns" "ks" repeats
mkdir -p gpurun_out
fatal() { case "$1" in 124|134|137|139) echo "fatal status $1 in $2; stopping"; exit "$1";; esac; }
python native/build.py > gpurun_out/build.log 2>&1 || exit 1
for r in $(seq 1 $3); do for n in $1; do for k in $2; do
  if [ "$n" = 1 ]; then
    timeout -k 10 300 python bench.py --extra-env NEXUS__EXECUTORS_PER_SHARD=$k > gpurun_out/kg_n${n}_k${k}_r$r.json 2>/dev/null
  else
    timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 \
      --master-port 29$n$k$r bench.py --gpus $n --extra-env NEXUS__EXECUTORS_PER_SHARD=$k > gpurun_out/kg_n${n}_k${k}_r$r.json 2>/dev/null
  fi
  s=$?; fatal $s n${n}k$k; python -c "
import json; d=json.loads(open('gpurun_out/kg_n${n}_k${k}_r$r.json').read().strip().splitlines()[-1]); print('n=$n k=$k r=$r', d['value'], d['p50_latency_ms'], round(d['cpu_cores_busy']['executors'],2))"
done; done; done
