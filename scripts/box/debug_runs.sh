#!/bin/bash
# Box: several driver-shape runs with per-wave timings (NCC_BENCH_DEBUG) to study run-to-run variance.
# usage: bash scripts/box/debug_runs.sh <outdir> [runs]
set -o pipefail
out=${1:-gpurun_out/debug_runs}
runs=${2:-4}
mkdir -p "$out"
for i in $(seq 1 $runs); do
  NCC_BENCH_DEBUG=1 timeout -k 10 240 python bench.py --steps 20 --warmup 5 --extra-env NCC_CPU_REPORT=1 \
    > $out/run_$i.json 2> $out/run_$i.err || exit $?
  python scripts/box/summarize.py $out/run_$i.json
done
