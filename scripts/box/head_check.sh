#!/bin/bash
# Box check of the tree: GPU tier, smoke, driver-shape bench x3, 5 ms shard latency.
# usage: bash scripts/box/head_check.sh <outdir>
set -o pipefail
out=${1:-gpurun_out/head}
mkdir -p $out
echo "ulimit -n: $(ulimit -n) / hard $(ulimit -Hn); nproc $(nproc)"
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $out/pytest.log 2>&1 || exit $?
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || exit $?
tail -1 $out/smoke.log
run() {  # name, args...
  local name=$1; shift
  timeout -k 10 240 python bench.py --steps 20 --warmup 5 "$@" > $out/$name.json 2> $out/$name.err || exit $?
  python scripts/box/summarize.py $out/$name.json
}
run default_1
run default_2
run default_3
run lat5 --shard-latency-ms 5
