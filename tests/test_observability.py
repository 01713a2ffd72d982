"""Ops endpoints, structured logging, coordinator↔executor framing, fake-apiserver control plane,
and executor supervision (restart after a crash)."""
import asyncio
import io
import json
import logging
import os
import signal
import socket
import threading
from http.server import BaseHTTPRequestHandler, HTTPServer

import aiohttp
import pytest

from ncc.api import resources as R
from ncc.controller.ipc import Channel
from ncc.fakeapi.server import FakeApiServer
from ncc.kube import errors as E
from ncc.kube.kubeconfig import ClusterConfig
from ncc.kube.rest import RestClient
from ncc.telemetry.logging import DatadogHandler, JsonFormatter, configure_logging
from ncc.testing.env import FakeEnvironment
from ncc.testing.workload import make_configmap, make_secret, make_template

NS = "nexus"


async def test_ops_server_endpoints():
    pytest.importorskip("prometheus_client")
    from ncc.telemetry.http import OpsServer, PrometheusMetrics
    prom = PrometheusMetrics("nexus_configuration_controller")
    prom.gauge("reconcile_latency", 12.5)
    prom.gauge("workqueue_length", 3, {"queue": "templates"})
    prom.count("reconciles", 2)
    prom.histogram("shard_write_ms", 4.0)
    state = {"ready": False}
    ops = OpsServer(ready=lambda: state["ready"], prometheus=prom, extra=lambda: {"queue": {"depth": 3}})
    port = await ops.start("127.0.0.1:0")
    base = f"http://127.0.0.1:{port}"
    try:
        async with aiohttp.ClientSession() as s:
            async with s.get(base + "/healthz") as r:
                assert r.status == 200
            async with s.get(base + "/readyz") as r:
                assert r.status == 503
            state["ready"] = True
            async with s.get(base + "/readyz") as r:
                assert r.status == 200
            async with s.get(base + "/metrics") as r:
                text = await r.text()
                assert "nexus_configuration_controller_reconcile_latency 12.5" in text
                assert 'nexus_configuration_controller_workqueue_length{queue="templates"} 3.0' in text
                assert "nexus_configuration_controller_reconciles_total 2.0" in text
                assert "nexus_configuration_controller_shard_write_ms_count 1.0" in text
            async with s.get(base + "/debug/state") as r:
                assert (await r.json()) == {"queue": {"depth": 3}}
    finally:
        await ops.stop()


def test_json_logging_and_text_format():
    buf = io.StringIO()
    configure_logging("debug", "json", stream=buf)
    logging.getLogger("ncc.test").info("hello %s", "world", extra={"shard": "s0", "n": 3})
    rec = json.loads(buf.getvalue().strip().splitlines()[-1])
    assert rec["msg"] == "hello world" and rec["level"] == "INFO" and rec["shard"] == "s0" and rec["n"] == 3
    assert rec["time"].endswith("Z")
    try:
        raise ValueError("boom")
    except ValueError:
        logging.getLogger("ncc.test").exception("failed")
    rec = json.loads(buf.getvalue().strip().splitlines()[-1])
    assert "ValueError: boom" in rec["error"]
    buf2 = io.StringIO()
    configure_logging("WARN", "text", stream=buf2)
    logging.getLogger("ncc.test").info("hidden")
    logging.getLogger("ncc.test").warning("shown")
    assert "hidden" not in buf2.getvalue() and "WARNING ncc.test shown" in buf2.getvalue()
    configure_logging("INFO", "json", stream=io.StringIO())
    assert isinstance(logging.getLogger().handlers[0].formatter, JsonFormatter)


def test_datadog_handler_ships_batches():
    got = []

    class H(BaseHTTPRequestHandler):
        def do_POST(self):  # noqa: N802
            body = self.rfile.read(int(self.headers["Content-Length"]))
            got.append((self.path, self.headers.get("DD-API-KEY"), json.loads(body)))
            self.send_response(202)
            self.end_headers()

        def log_message(self, *a):
            pass

    srv = HTTPServer(("127.0.0.1", 0), H)
    threading.Thread(target=srv.serve_forever, daemon=True).start()
    try:
        h = DatadogHandler("k3y", f"http://127.0.0.1:{srv.server_port}", "ncc", "pod-1", batch=2, flush_interval=0.2)
        lg = logging.getLogger("ncc.dd")
        lg.addHandler(h)
        lg.setLevel(logging.INFO)
        lg.propagate = False
        for i in range(3):
            lg.info("m%d", i)
        import time
        end = time.monotonic() + 5
        while sum(len(b) for _, _, b in got) < 3 and time.monotonic() < end:
            time.sleep(0.05)
        lg.removeHandler(h)
        assert got and got[0][0] == "/api/v2/logs" and got[0][1] == "k3y"
        items = [i for _, _, b in got for i in b]
        assert [i["msg"] for i in items] == ["m0", "m1", "m2"]
        assert items[0]["service"] == "ncc" and items[0]["hostname"] == "pod-1" and items[0]["status"] == "INFO"
    finally:
        srv.shutdown()


async def test_ipc_channel_single_batched_and_eof():
    a, b = socket.socketpair()
    ra, wa = await asyncio.open_connection(sock=a)
    rb, wb = await asyncio.open_connection(sock=b)
    ca, cb = Channel(ra, wa), Channel(rb, wb)
    ca.send({"t": "ready", "i": 0})
    await ca.drain()
    assert await cb.recv() == [{"t": "ready", "i": 0}]
    for i in range(5):  # sent within one loop iteration → one batched frame
        ca.send({"t": "report", "k": f"template/{NS}/t{i}", "r": {"s0": None}})
    await asyncio.sleep(0)
    await ca.drain()
    got = await cb.recv()
    assert [m["k"] for m in got] == [f"template/{NS}/t{i}" for i in range(5)]
    assert ca.sent == 2 and cb.received == 2
    ca.close()
    assert await cb.recv() is None
    cb.close()


async def test_fakeapi_control_endpoints():
    srv = FakeApiServer(name="ctl")
    srv.markers.add_spec("secrets", "data.version")
    url = await srv.start()
    client = RestClient(ClusterConfig(server=url), max_retries=0)
    try:
        async with aiohttp.ClientSession() as s:
            items = [make_secret(f"s{i}", NS, version=1) for i in range(5)] + [make_template(0, NS)]
            async with s.post(url + "/_fake/apply", json={"items": items, "yield_every": 2}) as r:
                a = await r.json()
            assert a["applied"] == 6 and a["t1_ns"] >= a["t0_ns"]
            want = [{"plural": "secrets", "value": "MQ==", "count": 5}]
            async with s.post(url + "/_fake/markers/wait", json={"want": want, "timeout": 2, "times": True,
                                                                 "keyed": True}) as r:
                w = await r.json()
            assert w["ok"] and sorted(w["times"]["secrets=MQ=="]) == [f"{NS}/s{i}" for i in range(5)]
            async with s.post(url + "/_fake/markers/wait", json={"want": [dict(want[0], value="Mg==")],
                                                                 "timeout": 0.1}) as r:
                assert (await r.json())["ok"] is False
            # apply again with a new version updates in place (same UID, new RV)
            uid = srv.state.get(R.SECRETS, NS, "s0")["metadata"]["uid"]
            async with s.post(url + "/_fake/apply", json={"items": [make_secret("s0", NS, version=2)]}) as r:
                await r.json()
            assert srv.state.get(R.SECRETS, NS, "s0")["metadata"]["uid"] == uid
            # seed a dependent owned by a live template
            cm = make_configmap("c0", NS)
            cm["__owner_template__"] = "algo-00000"
            async with s.post(url + "/_fake/objects", json={"items": [cm]}) as r:
                assert (await r.json())["created"] == 1
            ref = srv.state.get(R.CONFIGMAPS, NS, "c0")["metadata"]["ownerReferences"][0]
            assert ref["uid"] == srv.state.get(R.TEMPLATES, NS, "algo-00000")["metadata"]["uid"]
            async with s.get(url + "/_fake/stats") as r:
                st = await r.json()
            assert st["objects"] and st["state"]["create"] >= 7
            async with s.post(url + "/_fake/markers", json={"specs": {"configmaps": "data.version"}}) as r:
                assert (await r.json())["specs"] == {"secrets": "data.version", "configmaps": "data.version"}
            # fault injection: every request fails with 503, then recovery
            async with s.post(url + "/_fake/faults", json={"error_rate": 1.0, "error_code": 503,
                                                          "write_only": False}) as r:
                assert (await r.json())["error_rate"] == 1.0
            with pytest.raises(E.ApiError) as ei:
                await client.get(R.SECRETS, NS, "s0")
            assert ei.value.code == 503
            async with s.post(url + "/_fake/faults", json={"error_rate": 0.0}) as r:
                await r.json()
            assert (await client.get(R.SECRETS, NS, "s0"))["metadata"]["name"] == "s0"
    finally:
        await client.close()
        await srv.stop()


async def test_executor_restarts_after_crash(tmp_path):
    """The coordinator supervises executor processes: a killed executor is respawned and syncing resumes."""
    from ncc.app import App
    env = await FakeEnvironment(1, str(tmp_path)).start()
    cc, sc = env.controller_client(), env.shard_client(0)
    stop = asyncio.Event()
    app = App(env.app_config(mode="native", executors_per_shard=1))
    try:
        await app.build()
        task = asyncio.ensure_future(app.run(stop))
        await asyncio.wait_for(app.controller.ready.wait(), 15)
        h = app.pool.handles[0]
        os.kill(h.proc.pid, signal.SIGKILL)
        loop = asyncio.get_running_loop()
        end = loop.time() + 15
        while (h.restarts < 1 or not h.ready.is_set()) and loop.time() < end:
            await asyncio.sleep(0.05)
        assert h.restarts == 1 and h.ready.is_set()
        await cc.create(R.TEMPLATES, NS, make_template(3, NS, secrets=[], configmaps=[]))
        while loop.time() < end:
            try:
                await sc.get(R.TEMPLATES, NS, "algo-00003")
                break
            except E.NotFound:
                await asyncio.sleep(0.05)
        assert (await sc.get(R.TEMPLATES, NS, "algo-00003"))["metadata"]["name"] == "algo-00003"
        assert app.debug_state()["executors"][0]["restarts"] == 1
        stop.set()
        await asyncio.wait_for(task, 15)
    finally:
        stop.set()
        await cc.close()
        await sc.close()
        await env.stop()


async def test_executor_protocol_in_process(tmp_path, monkeypatch):
    """`executor_main` driven in-process over a socketpair: synced → ready → per-shard report → clean exit
    on EOF."""
    from ncc.config import config_to_env
    from ncc.controller.executor import executor_main
    env = await FakeEnvironment(1, str(tmp_path), subprocesses=True, token="t0k").start()
    for k, v in config_to_env(env.app_config(mode="native")).items():
        monkeypatch.setenv(k, v)
    cc = env.controller_client()
    parent, child = socket.socketpair()
    try:
        await cc.create(R.TEMPLATES, NS, make_template(1, NS, secrets=[], configmaps=[]))
        task = asyncio.ensure_future(executor_main(child.fileno(), 0, ["shard-0"], (0, 1)))
        r, w = await asyncio.open_connection(sock=parent)
        ch = Channel(r, w)
        msgs = []
        loop = asyncio.get_running_loop()
        end = loop.time() + 15
        while loop.time() < end and not any(m.get("t") == "report" for m in msgs):
            batch = await asyncio.wait_for(ch.recv(), 15)
            msgs.extend(batch or [])
        status = [m for m in msgs if m.get("t") == "status"]  # periodic, from the start (shape: status_view)
        assert status and set(status[0]["s"]) == {"shard-0"}
        msgs = [m for m in msgs if m.get("t") != "status"]
        assert msgs[:2] == [{"t": "synced", "i": 0}, {"t": "ready", "i": 0}]
        rep = next(m for m in msgs if m.get("t") == "report")
        assert rep["k"] == f"template/{NS}/algo-00001" and rep["r"] == {"shard-0": None} and rep["w"] is True
        ch.close()  # the coordinator going away ends the executor
        assert await asyncio.wait_for(task, 15) == 0
    finally:
        await cc.close()
        await env.stop()
