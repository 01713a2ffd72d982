#!/bin/bash
# round-2 (session 4) box check of HEAD: GPU tier, smoke, driver-shape bench x3, 5 ms shard latency
set -o pipefail
out=gpurun_out/r2d
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $out/pytest.log 2>&1 || exit $?
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || exit $?
run() {  # name, args...
  local name=$1; shift
  timeout -k 10 240 python bench.py --steps 20 --warmup 5 "$@" > $out/$name.json 2> $out/$name.err || exit $?
  python -c "import json;d=json.loads(open('$out/$name.json').read().strip().splitlines()[-1]);print('$name',d['value'],d['p50_latency_ms'],d['controller_cpu_us_per_object'],d['controller_cpu_us_per_object_split'],d['controller_sizing'])"
}
run default_1
run default_2
run default_3
run lat5 --shard-latency-ms 5
