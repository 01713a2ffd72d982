#!/bin/bash
# Box: sustained load — 100 timed waves (300k objects at N=1) — for throughput drift and controller memory.
set -o pipefail
out=${1:-gpurun_out/sustained}
mkdir -p "$out"
timeout -k 10 600 python bench.py --steps 100 --warmup 5 > $out/long_100.json 2> $out/long_100.err || exit $?
python scripts/box/summarize.py $out/long_100.json
python -c "import json;d=json.loads(open('$out/long_100.json').read().strip().splitlines()[-1]);print('rss', d['rss_mib'], 'children', d['controller_children'])"
