#!/bin/bash
# Box: rocprofv3 kernel trace over a bench run (this control plane dispatches no GPU kernels; the trace
# records that), kept to a short run.
set -o pipefail
out=${1:-gpurun_out/rocprof}
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$out/trace" -o run -- python3 bench.py --steps 5 --warmup 2 \
  > "$out/bench.json" 2> "$out/rocprof.err" || exit $?
python scripts/box/summarize.py "$out/bench.json"
if [ -d "$out/trace" ]; then find "$out/trace" -type f; else echo "no trace files: no kernel dispatches were recorded"; fi
