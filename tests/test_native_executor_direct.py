"""The C++ shard executor (`ncc/bin/ncc-executor`) driven directly over its socketpair protocol
(native/executor/executor.cpp header comment): no coordinator, the test plays it.

* An idle executor whose shard is unreachable sleeps: it waits for the shard caches with a timed Event
  wait (loop.hpp `Event::wait_for`), not a polling loop, so it makes no periodic wake-ups.
* A pass over a template reports one typed failure per shard (ncc/controller/failures.py): a rogue shard
  Secret comes back as {c: RogueResourceError, k: Secret, n: <name>, h: 0, m: <reference message>}.
"""
import asyncio
import json
import os
import re
import socket
import sys

import pytest

from ncc.api import resources as R
from ncc.controller.ipc import Channel
from ncc.controller.native_executor import binary_path
from ncc.fakeapi.server import FakeApiServer
from ncc.testing.workload import make_secret, make_template

pytestmark = pytest.mark.skipif(binary_path() is None, reason="ncc/bin/ncc-executor is not built")
NS = "nexus"


def cfg(shards: list, **kw) -> dict:
    doc = {"namespace": NS, "alias": "controller-cluster", "workers": 8, "pool_size": 8, "request_timeout": 5.0,
           "coalesce_window": 0.0, "failure_base_delay": 0.05, "failure_max_delay": 0.2, "rate_limit_qps": 50,
           "rate_limit_burst": 300, "shard_sync_timeout": 30.0, "full_resync_period": 0, "log_level": 30,
           "shards": shards}
    doc.update(kw)
    return {"t": "cfg", "c": json.dumps(doc)}


def line(obj: dict) -> bytes:
    return json.dumps({"type": "ADDED", "object": obj}).encode()


class Executor:
    def __init__(self, config: dict, env: dict | None = None):
        self.config, self.env = config, env
        self.pending: list = []  # messages received but not yet returned by next_message

    async def __aenter__(self):
        parent, child = socket.socketpair(socket.AF_UNIX, socket.SOCK_STREAM)
        env = dict(os.environ, **(self.env or {}))
        self.proc = await asyncio.create_subprocess_exec(
            binary_path(), "--fd", str(child.fileno()), "--index", "0", "--part", "0/1", pass_fds=(child.fileno(),),
            env=env, stderr=asyncio.subprocess.PIPE)
        child.close()
        reader, writer = await asyncio.open_connection(sock=parent)
        self.ch = Channel(reader, writer)
        self.ch.send(self.config)
        return self

    def snapshot(self, kind: int, objs: list) -> None:
        self.ch.send({"t": "s", "k": kind, "l": [line(o) for o in objs]})

    async def next_message(self, t: str, timeout: float = 10.0) -> dict:
        """The next message of type `t`.  A batch holds several messages (reports travel in batches): the ones
        after the match stay buffered for the next call, instead of being dropped (driving
        the executor with the first-match-only version under-counted 50 reports as 13–46)."""
        async def go():
            while True:
                for i, m in enumerate(self.pending):
                    if m.get("t") == t:
                        del self.pending[:i + 1]  # earlier messages of other types are consumed, as before
                        return m
                self.pending.clear()
                batch = await self.ch.recv()
                assert batch is not None, "executor closed the channel"
                self.pending.extend(batch)
        return await asyncio.wait_for(go(), timeout)

    async def close(self) -> str:
        self.ch.close()
        _, err = await asyncio.wait_for(self.proc.communicate(), 10)
        return err.decode(errors="replace")

    async def __aexit__(self, *exc):
        if self.proc.returncode is None:
            self.proc.kill()
            await self.proc.wait()


async def test_idle_executor_with_unreachable_shard_does_not_poll():
    with socket.socket() as s:  # a port nothing listens on
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    shard = {"name": "dead", "server": f"http://127.0.0.1:{port}"}
    async with Executor(cfg([shard]), env={"NCC_CPU_REPORT": "1", "NCC_STATUS_S": "5"}) as ex:
        for k in range(4):
            ex.snapshot(k, [])
        # the controller side is synced; the executor now waits (up to 30 s) for the dead shard's caches
        await asyncio.sleep(2.0)
        assert ex.proc.returncode is None
        err = await ex.close()
    m = re.search(r"loop_wakeups=(\d+)", err)
    assert m, err[-2000:]
    # a 10 ms polling wait would have woken ~200 times in 2 s, the request-deadline sweep 4 times (it runs
    # only while a connection is in use); the reflectors' reconnect backoff (0.8 s, 1.6 s... for 4
    # informers) and their failed connects account for about a dozen
    print(m.group(0))
    assert int(m.group(1)) < 30, m.group(0)


async def test_rogue_dependent_report_is_typed():
    srv = FakeApiServer(name="shard-0")
    url = await srv.start()
    try:
        rogue = make_secret("s0", NS, version=3)
        srv.state.create(R.SECRETS, NS, rogue)
        tpl = make_template(0, NS, secrets=["s0"])
        tpl["metadata"].update(uid="u-0", resourceVersion="10", generation=1)
        sec = make_secret("s0", NS)
        sec["metadata"].update(uid="u-s", resourceVersion="11")
        async with Executor(cfg([{"name": "shard-0", "server": url}])) as ex:
            for k, objs in ((0, [tpl]), (1, []), (2, [sec]), (3, [])):
                ex.snapshot(k, objs)
            await ex.next_message("ready")
            rep = await ex.next_message("report")
            assert rep["k"] == "template/nexus/algo-00000" and rep["u"] == "u-0" and rep["g"] == 1
            f = rep["r"]["shard-0"]
            assert f == {"c": "RogueResourceError", "k": "Secret", "n": "s0", "h": 0,
                         "m": 'Resource "s0" already exists and is not managed by any Machine Learning Algorithm'}
            assert srv.state.get(R.SECRETS, NS, "s0")["data"] == rogue["data"]  # refused, not overwritten
            # the shard template itself was written: only the dependent failed
            assert srv.state.get(R.TEMPLATES, NS, "algo-00000")["spec"] == tpl["spec"]
            await ex.close()
    finally:
        await srv.stop()


async def test_sampling_profile_is_written_and_symbolized(tmp_path):
    """NCC_SAMPLE_PROFILE: the executor samples its own CPU (SIGPROF) and writes the executable mappings and
    the sampled addresses on exit; scripts/executor_profile.py maps them to functions."""
    import importlib.util
    spec = importlib.util.spec_from_file_location(
        "executor_profile", os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "scripts",
                                         "executor_profile.py"))
    prof = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(prof)
    srv = FakeApiServer(name="shard-0")
    url = await srv.start()
    try:
        tpl = make_template(0, NS, secrets=["s0"])
        tpl["metadata"].update(uid="u-0", resourceVersion="10", generation=1)
        sec = make_secret("s0", NS)
        sec["metadata"].update(uid="u-s", resourceVersion="11")
        async with Executor(cfg([{"name": "shard-0", "server": url}]),
                            env={"NCC_SAMPLE_PROFILE": str(tmp_path), "NCC_SAMPLE_US": "50"}) as ex:
            for k, objs in ((0, [tpl]), (1, []), (2, [sec]), (3, [])):
                ex.snapshot(k, objs)
            await ex.next_message("report")
            await ex.close()
    finally:
        await srv.stop()
    files = list(tmp_path.glob("executor-0-*.samples"))
    assert len(files) == 1
    text = files[0].read_text()
    assert "# map " in text and "ncc-executor" in text
    counts = prof.load_samples([str(tmp_path)])
    out = prof.report(counts, binary_path(), 10)
    assert out.split()[0].isdigit() and "== self" in out if counts else out == "no samples"


async def test_frame_pointer_build_records_call_stacks(tmp_path, monkeypatch):
    """The profile flavor (native/build.py: frame pointers, NCC_FRAME_POINTERS) adds the return addresses up the
    rbp chain to each sample, and the report gains call sites and an inclusive view."""
    import importlib.util
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(root, "native"))
    import build
    try:
        fp_bin = build.build_executor(profile=True)
    except Exception as e:  # noqa: BLE001 — no compiler here
        pytest.skip(f"the profiling executor is not buildable here: {e}")
    monkeypatch.setenv("NCC_EXECUTOR_BINARY", fp_bin)
    spec = importlib.util.spec_from_file_location("executor_profile", os.path.join(root, "scripts", "executor_profile.py"))
    prof = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(prof)
    srv = FakeApiServer(name="shard-0")
    url = await srv.start()
    try:
        tpls, secs = [], []
        for i in range(200):
            t = make_template(i, NS, secrets=[f"s{i}"])
            t["metadata"].update(uid=f"u-{i}", resourceVersion=str(10 + i), generation=1)
            sec = make_secret(f"s{i}", NS, payload=4096)
            sec["metadata"].update(uid=f"u-s{i}", resourceVersion=str(1000 + i))
            tpls.append(t)
            secs.append(sec)
        async with Executor(cfg([{"name": "shard-0", "server": url}]),
                            env={"NCC_SAMPLE_PROFILE": str(tmp_path), "NCC_SAMPLE_US": "50"}) as ex:
            for k, objs in ((0, tpls), (1, []), (2, secs), (3, [])):
                ex.snapshot(k, objs)
            for _ in range(200):
                await ex.next_message("report")
            await ex.close()
    finally:
        await srv.stop()
    files = list(tmp_path.glob("executor-0-*.samples"))
    assert len(files) == 1
    rows = [ln.split() for ln in files[0].read_text().splitlines() if ln and not ln.startswith("#")]
    if not rows:
        pytest.skip("no CPU sample taken on this host")
    assert any(len(r) > 2 for r in rows), rows[:5]  # return addresses up the frame-pointer chain
    out = prof.report(prof.load_samples([str(tmp_path)]), fp_bin, 10)
    assert "== inclusive" in out and "no call stacks" not in out


async def test_every_report_of_a_batch_is_seen():
    """50 templates in one snapshot: the executor reports on each, several reports to a frame; the helper keeps
    the rest of a batch for its next call, so all 50 are counted (the first-match version saw 13–46)."""
    srv = FakeApiServer(name="shard-0")
    url = await srv.start()
    try:
        ts = []
        for i in range(50):
            t = make_template(i, NS)
            t["metadata"].update(uid=f"u-{i}", resourceVersion=str(10 + i), generation=1)
            ts.append(t)
        async with Executor(cfg([{"name": "shard-0", "server": url}])) as ex:
            for k, objs in ((0, ts), (1, []), (2, []), (3, [])):
                ex.snapshot(k, objs)
            seen = set()
            while len(seen) < 50:
                seen.add((await ex.next_message("report", timeout=20))["k"])
            assert seen == {f"template/{NS}/algo-{i:05d}" for i in range(50)}
    finally:
        await srv.stop()


async def test_unreadable_relayed_line_costs_only_itself():
    """A relayed watch batch with an unreadable line: the executor logs it and applies the rest of the batch
    (the template after it is still synced and reported)."""
    srv = FakeApiServer(name="shard-0")
    url = await srv.start()
    try:
        t0 = make_template(0, NS)
        t0["metadata"].update(uid="u-0", resourceVersion="10", generation=1)
        t1 = make_template(1, NS)
        t1["metadata"].update(uid="u-1", resourceVersion="11", generation=1)
        async with Executor(cfg([{"name": "shard-0", "server": url}])) as ex:
            for k, objs in ((0, [t0]), (1, []), (2, []), (3, [])):
                ex.snapshot(k, objs)
            assert (await ex.next_message("report"))["k"] == "template/nexus/algo-00000"
            ex.ch.send({"t": "w", "k": 0, "l": [b'{"type":"ADDED","object":{"metadata":{"name":"x"},"spec":{,}}}',
                                                 line(t1)]})
            rep = await ex.next_message("report")
            assert rep["k"] == "template/nexus/algo-00001" and rep["r"]["shard-0"] is None
            assert srv.state.get(R.TEMPLATES, NS, "algo-00001") is not None
            err = await ex.close()
        assert "unreadable relayed line" in err
    finally:
        await srv.stop()


@pytest.mark.parametrize("code,reason", [(400, ""), (401, ""), (403, ""), (405, ""), (422, "Invalid"), (429, ""),
                                         (500, ""), (502, ""), (503, ""), (504, ""), (418, ""), (500, "Forbidden")])
async def test_failure_class_matches_the_python_client(code, reason):
    """A shard answering a write with an error status: the C++ executor's report names the failure with the
    class the Python client (ncc/kube/errors.py `from_status`) gives the same response, so status messages
    and Events read the same under either executor."""
    from ncc.kube import errors as E
    srv = FakeApiServer(name="shard-0")
    url = await srv.start()
    try:
        srv.faults.update({"rules": [{"method": m, "resource": "nexusalgorithmtemplates", "code": code,
                                      "reason": reason, "count": 1} for m in ("POST", "PUT", "PATCH")]})
        tpl = make_template(0, NS)
        tpl["metadata"].update(uid="u-0", resourceVersion="10", generation=1)
        async with Executor(cfg([{"name": "shard-0", "server": url}])) as ex:
            for k, objs in ((0, [tpl]), (1, []), (2, []), (3, [])):
                ex.snapshot(k, objs)
            rep = await ex.next_message("report")
            await ex.close()
    finally:
        await srv.stop()
    wire = E.from_status(code, {"reason": reason, "message": "injected fault"})  # what the fake server sends
    want = type(E.from_status(code, {"reason": wire.reason, "message": str(wire)})).__name__
    f = rep["r"]["shard-0"]
    assert f["c"] == want and f["h"] == code, f


@pytest.mark.skipif(__import__("shutil").which("openssl") is None, reason="openssl CLI needed to mint test certificates")
@pytest.mark.parametrize("case", ["ok", "wrong-ca", "no-client-cert", "insecure-skip", "server-name-ok",
                                  "server-name-wrong"])
async def test_tls_shard_connections(tmp_path, case):
    """The C++ executor's OpenSSL client against a mutual-TLS shard apiserver (the Python client's twin is
    tests/test_tls.py): verification against the kubeconfig CA, the client certificate, insecure-skip-tls-verify
    and tls-server-name.  A refused handshake is a TransportError failure in the report, not a crash."""
    from ncc.testing.env import FakeEnvironment
    from ncc.testing.pki import make_pki
    env = await FakeEnvironment(1, str(tmp_path), tls=True).start()
    try:
        pki = env.pki
        shard = {"name": "shard-0", "server": env.shard_urls[0], "ca_pem": pki.ca_data.decode(),
                 "cert_pem": pki.client_cert_data.decode(), "key_pem": pki.client_key_data.decode()}
        other = make_pki(str(tmp_path / "other")) if case in ("wrong-ca", "insecure-skip") else None
        if case == "wrong-ca":
            shard["ca_pem"] = other.ca_data.decode()
        elif case == "no-client-cert":
            shard["cert_pem"] = shard["key_pem"] = ""
        elif case == "insecure-skip":
            shard.update(ca_pem=other.ca_data.decode(), insecure=True)
        elif case == "server-name-ok":
            shard["tls_server_name"] = "kube.test"
        elif case == "server-name-wrong":
            shard["tls_server_name"] = "not-in-the-cert.example"
        tpl = make_template(0, NS)
        tpl["metadata"].update(uid="u-0", resourceVersion="10", generation=1)
        ok = case in ("ok", "insecure-skip", "server-name-ok")
        async with Executor(cfg([shard], shard_sync_timeout=1.0)) as ex:
            for k, objs in ((0, [tpl]), (1, []), (2, []), (3, [])):
                ex.snapshot(k, objs)
            rep = await ex.next_message("report", timeout=15)
            err = await ex.close()
        f = rep["r"]["shard-0"]
        if ok:
            assert f is None, (f, err[-2000:])
            assert env.shard_servers[0].state.get(R.TEMPLATES, NS, "algo-00000") is not None
        else:
            assert f is not None and f["c"] in ("TransportError", "ShardNotReadyError"), f
    finally:
        await env.stop()


async def test_retry_after_is_honoured():
    """A 429 with Retry-After: the C++ client waits and sends the request again (at most 5 times, ≤ 10 s
    each); the pass succeeds and no failure is reported."""
    srv = FakeApiServer(name="shard-0")
    url = await srv.start()
    try:
        srv.faults.update({"rules": [{"method": "POST", "resource": "nexusalgorithmtemplates", "code": 429,
                                      "retry_after": 1, "count": 2}]})
        tpl = make_template(0, NS)
        tpl["metadata"].update(uid="u-0", resourceVersion="10", generation=1)
        async with Executor(cfg([{"name": "shard-0", "server": url}])) as ex:
            for k, objs in ((0, [tpl]), (1, []), (2, []), (3, [])):
                ex.snapshot(k, objs)
            t0 = asyncio.get_running_loop().time()
            rep = await ex.next_message("report", timeout=20)
            waited = asyncio.get_running_loop().time() - t0
            await ex.close()
        assert rep["r"]["shard-0"] is None and waited >= 1.9
        assert srv.state.get(R.TEMPLATES, NS, "algo-00000") is not None
        assert srv.faults.rules[0]["count"] == 0
    finally:
        await srv.stop()


async def test_token_file_is_reread_on_401(tmp_path):
    """A rotated bound service-account token: the shard starts answering 401 to the old token; the client
    re-reads its token file once and retries with the new token (no failure reported)."""
    srv = FakeApiServer(name="shard-0", token="t1")
    url = await srv.start()
    tok = tmp_path / "token"
    tok.write_text("t1\n")
    try:
        t0 = make_template(0, NS)
        t0["metadata"].update(uid="u-0", resourceVersion="10", generation=1)
        t1 = make_template(1, NS)
        t1["metadata"].update(uid="u-1", resourceVersion="11", generation=1)
        async with Executor(cfg([{"name": "shard-0", "server": url, "token_file": str(tok)}])) as ex:
            for k, objs in ((0, [t0]), (1, []), (2, []), (3, [])):
                ex.snapshot(k, objs)
            assert (await ex.next_message("report"))["r"]["shard-0"] is None
            srv.token = "t2"  # rotation: the server now wants the new token, which the file holds
            tok.write_text("t2\n")
            ex.ch.send({"t": "w", "k": 0, "l": [line(t1)]})
            rep = await ex.next_message("report", timeout=15)
            await ex.close()
        assert rep["k"] == "template/nexus/algo-00001" and rep["r"]["shard-0"] is None, rep
        assert srv.state.get(R.TEMPLATES, NS, "algo-00001") is not None
    finally:
        await srv.stop()


async def test_answered_write_ends_the_reflectors_outage_backoff():
    """The C++ reflectors back off up to 30 s after a shard outage (client-go's schedule).  A write the shard
    answers again wakes them at once (`Shard::answering`), so shard-side drift right after the outage is
    repaired without waiting out the backoff."""
    srv = FakeApiServer(name="shard-0")
    url = await srv.start()
    try:
        t0 = make_template(0, NS)
        t0["metadata"].update(uid="u-0", resourceVersion="10", generation=1)
        async with Executor(cfg([{"name": "shard-0", "server": url}])) as ex:
            for k, objs in ((0, [t0]), (1, []), (2, []), (3, [])):
                ex.snapshot(k, objs)
            assert (await ex.next_message("report"))["r"]["shard-0"] is None
            srv.faults.update({"down": True, "write_only": False})
            srv.drop_watches()
            await asyncio.sleep(3.5)  # reflector failures at ~0, 0.8, 2.4 s: the current wait is ~3.2-6.4 s
            srv.faults.update({"down": False})
            t1 = make_template(1, NS)
            t1["metadata"].update(uid="u-1", resourceVersion="11", generation=1)
            ex.ch.send({"t": "w", "k": 0, "l": [line(t1)]})
            assert (await ex.next_message("report", timeout=15))["r"]["shard-0"] is None
            await asyncio.sleep(0.3)  # the woken reflectors relist and watch again
            from ncc.kube.kubeconfig import ClusterConfig
            from ncc.kube.rest import RestClient
            client = RestClient(ClusterConfig(server=url))  # through the API: the watch streams see it
            live = await client.get(R.TEMPLATES, NS, "algo-00000")
            live["spec"]["container"]["versionTag"] = "drift"
            await client.update(R.TEMPLATES, NS, live)
            await client.close()
            loop = asyncio.get_running_loop()
            end = loop.time() + 1.5
            while loop.time() < end:
                if srv.state.get(R.TEMPLATES, NS, "algo-00000")["spec"]["container"]["versionTag"] != "drift":
                    break
                await asyncio.sleep(0.02)
            assert srv.state.get(R.TEMPLATES, NS, "algo-00000")["spec"] == t0["spec"], "drift not repaired"
            await ex.close()
    finally:
        await srv.stop()


def test_profile_report_maps_another_machines_paths():
    """A profile taken on the GPU box names the box's copy of this tree; the report maps it to this checkout by
    the longest path tail that exists here (scripts/executor_profile.py `local_path`)."""
    import importlib.util
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    spec = importlib.util.spec_from_file_location("executor_profile", os.path.join(root, "scripts", "executor_profile.py"))
    prof = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(prof)
    here = os.path.join(root, "scripts", "executor_profile.py")
    assert prof.local_path("/tmp/code/Some__repo/repo/scripts/executor_profile.py") == here
    assert prof.local_path(here) == here
    assert prof.local_path("/no/such/dir/file.so") == "/no/such/dir/file.so"
    assert prof.local_path("[vdso]") == "[vdso]"
