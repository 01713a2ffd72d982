"""One summary line per bench.py JSON file (the last JSON line in each)."""
import json
import sys

for path in sys.argv[1:]:
    with open(path) as f:
        d = json.loads([ln for ln in f.read().splitlines() if ln.startswith("{")][-1])
    c = d["config"]
    print(f"{path}: N={d['n_gpus']} lat={c.get('shard_latency_ms')} {d['value']:.0f} obj/s "
          f"ms/step={d['ms_per_step']} p50={d['p50_latency_ms']} p99={d['p99_latency_ms']} "
          f"us/obj={d.get('controller_cpu_us_per_object')} {d.get('controller_cpu_us_per_object_split')} "
          f"busy={d.get('cpu_cores_busy')}", flush=True)
