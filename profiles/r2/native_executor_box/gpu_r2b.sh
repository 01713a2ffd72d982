#!/bin/bash
# round-2 box check of the native executor: GPU tier, smoke, bench A/B (native vs python executors),
# executors-per-shard, injected shard latency
set -o pipefail
out=gpurun_out/r2b
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $out/pytest.log 2>&1 || exit $?
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || exit $?
run() {  # name, args...
  local name=$1; shift
  timeout -k 10 240 python bench.py --steps 20 --warmup 5 "$@" > $out/$name.json 2> $out/$name.err || exit $?
  python -c "import json;d=json.loads(open('$out/$name.json').read().strip().splitlines()[-1]);print('$name',d['value'],d['p50_latency_ms'],d['controller_cpu_us_per_object'],d['controller_cpu_us_per_object_split'])"
}
run native_default
run python_default --extra-env NCC_EXECUTOR_IMPL=python
run native_k1 --extra-env NEXUS__EXECUTORS_PER_SHARD=1
run native_k2 --extra-env NEXUS__EXECUTORS_PER_SHARD=2
run native_lat5 --shard-latency-ms 5
run native_lat20 --shard-latency-ms 20
run native_default_2
