"""Deployment-target tier, run by the driver on the MI355X box (`pytest -m gpu`).

The controller has no GPU kernels (the workload is control-plane I/O; see README.md), so these
tests exercise what must hold on the box the framework ships to: the in-tree C++ extension
loads (no silent Python fallback), the flagship end-to-end sync works, and the benchmark
harness produces a valid result line.
"""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

pytestmark = pytest.mark.gpu


def test_native_extension_loaded():
    from ncc import native
    m = native.load(required=True)
    q = m.RateLimitingQueue(0.03, 5.0, 50.0, 300)
    assert q.add("template/nexus/a") and not q.add("template/nexus/a")
    assert q.try_get() == "template/nexus/a"
    from ncc.api import fingerprint as fp
    assert fp.IMPL == "native"


def test_smoke_on_box():
    sys.path.insert(0, ROOT)
    import __graft_entry__ as g
    g.smoke()


def test_bench_contract_single_shard():
    # 300 templates × 3 steps: enough CPU in every process for its 10 ms clock ticks to register
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--templates", "300", "--steps", "3",
                        "--warmup", "1"], capture_output=True, text=True, timeout=300, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    line = [l for l in r.stdout.splitlines() if l.startswith("{")][-1]
    res = json.loads(line)
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config"):
        assert k in res
    assert res["n_gpus"] == 1 and res["value"] > 0 and res["controller_alive"]
    # the data plane that ran is the C++ shard executor, not the Python fallback
    assert res["controller_sizing"]["executor_impl"] == "native", res["controller_sizing"]
    assert res["controller_to_substrate"] is not None and res["host"]["calibration"].get("cpp_ctl_scan_ns"), \
        (res["controller_cpu_us_per_object"], res["substrate_us_per_object"], res["host"])
    # the production transport beside the headline: TLS on every apiserver, HTTP/2 by ALPN, product defaults
    assert res["tls_value"] > 0 and res["tls_config"]["shard_transport"] == "http2" and \
        res["tls_config"]["controller_transport"] == "h2" and res["tls_config"]["cpu_affinity"] == "none", res
    assert res["bench_settings"]["NEXUS__CLIENT_HTTP2"] == "on"
