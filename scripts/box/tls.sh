#!/bin/bash
# Box: plain HTTP vs mutual TLS in alternation (driver shape), N=1.
set -o pipefail
out=${1:-gpurun_out/tls}
mkdir -p "$out"
for i in 1 2 3; do
  timeout -k 10 240 python bench.py --steps 20 --warmup 5 > $out/http_$i.json 2> $out/http_$i.err || exit $?
  python scripts/box/summarize.py $out/http_$i.json
  timeout -k 10 240 python bench.py --steps 20 --warmup 5 --tls > $out/tls_$i.json 2> $out/tls_$i.err || exit $?
  python scripts/box/summarize.py $out/tls_$i.json
done
