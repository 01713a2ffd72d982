#!/bin/bash
# Round-3 profiles of the final tree: rocprofv3 kernel trace + stats over a bench run (no GPU dispatches
# expected: the workload is a control plane), then the C++ executor's own sampling profile over the driver's
# bench shape.  Usage: bash scripts/gpu_r3_prof.sh <out dir name>
set -o pipefail
out=gpurun_out/$1
mkdir -p $out
bash scripts/box/rocprof.sh $out/rocprof > $out/rocprof.log 2>&1 || exit $?
timeout -k 10 150 python3 bench.py --gpus 1 --steps 20 --warmup 5 --extra-env NCC_SAMPLE_PROFILE=$PWD/$out/samples \
  > $out/sampled_bench.json 2> $out/sampled_bench.err || exit $?
python3 scripts/executor_profile.py $out/samples --top 25 > $out/executor_profile.txt 2>&1 || exit $?
cat $out/rocprof.log | tail -5
head -40 $out/executor_profile.txt
