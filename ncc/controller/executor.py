"""Shard executors: one OS process per group of shards, supervised by the coordinator.

The reference reconciles every shard from one process, sequentially (controller.go:790).  A
Python control plane is CPU-bound per request, so native mode splits the work the way a
multi-GPU trainer splits ranks — one process per shard (MI355X node) — while keeping a single
writer for the controller cluster:

* **coordinator** (the `python -m ncc` process): controller-cluster informers, status
  conditions, adoption of referenced Secrets/ConfigMaps, Events; aggregates per-shard results.
* **executors** (`python -m ncc.executor`, spawned here): each watches the controller cluster
  read-only (desired state) plus its own shards, and reconciles desired → shard with its own
  queue and workers.  After every pass it reports `(key, generation, {shard: error|None}, wrote)`
  to the coordinator over a socketpair (msgpack frames, `ncc.controller.ipc`).

Executors never write to the controller cluster, so the coordinator stays the only writer of
status and ownerRefs and no cross-process write races are introduced.  A crashed executor is
restarted with exponential backoff; its shards are level-triggered, so the restart resyncs them.
"""
from __future__ import annotations

import asyncio
import logging
import os
import socket
import sys
import time
import zlib

from .ipc import Channel, RawChannel
from .relay import deliver
from ..aio import wait_timeout

log = logging.getLogger("ncc.executor")

EXIT_GRACE_S = 10.0  # how long a child may take to exit once its channel has closed


def partition(names: list[str], n: int) -> list[list[str]]:
    """Round-robin shard → executor assignment (stable for a given shard list)."""
    n = max(1, min(n, len(names)))
    parts: list[list[str]] = [[] for _ in range(n)]
    for i, s in enumerate(names):
        parts[i % n].append(s)
    return parts


def key_part(key: str, parts: int) -> int:
    """Stable key → partition (crc32 of "ns/name"; a template's and its delete's keys agree)."""
    _, _, nsname = key.partition("/")
    return zlib.crc32(nsname.encode()) % parts


def partition_filter(part: int, parts: int):
    """Informer key filter for partition `part` of `parts` (agrees with `key_part`)."""
    crc = zlib.crc32

    def keep(ns: str, name: str) -> bool:
        return crc(f"{ns}/{name}".encode()) % parts == part
    keep.part, keep.parts = part, parts  # lets informers test the partition natively (scan_event_part)
    return keep


def partition_owner_filter(part: int, parts: int, referenced=None):
    """Dependent filter for partition `part` of `parts`: keep unowned objects (rogue detection and not yet
    adopted references need them), objects with at least one owner template in this partition, and —
    with `referenced(ns, name)` — objects a template of this partition references; drop the rest (owned
    only by other partitions' templates) before they are decoded."""
    crc = zlib.crc32

    def keep(ns: str, name: str, owners: tuple) -> bool:
        if not owners:
            return True
        for o in owners:
            if crc(f"{ns}/{o}".encode()) % parts == part:
                return True
        return referenced is not None and referenced(ns, name)
    keep.part, keep.parts, keep.referenced = part, parts, referenced
    return keep


class ExecutorHandle:
    def __init__(self, index: int, shards: list[str], on_message, env: dict | None = None,
                 part: int = 0, parts: int = 1, argv: list | None = None, what: str = "executor"):
        self.argv = argv  # child command after `python`; default: the shard executor
        self.what = what
        self.index = index
        self.shards = shards
        self.part = part
        self.parts = parts
        self.on_message = on_message
        # coordinator: callable(index, buffer, start) -> (other messages, end) folding the raw frame stream
        # (reports) natively
        self.on_stream = None
        self.env = env
        self.proc: asyncio.subprocess.Process | None = None
        self.channel: Channel | None = None
        self.ready = asyncio.Event()  # workers running
        self.synced = asyncio.Event()  # caches synced (a gated child reports this before it may run)
        self.restarts = 0
        self.status: dict | None = None  # the executor's last {"t": "status"} (status_view), for /debug/state
        self.gated = False  # spawned for a warm standby: workers wait for {"t": "go"}
        self.gate_open = False
        self.on_spawn = None  # callable(handle) once the channel to a (re)started child is up (watch relay)
        self.on_exit = None  # callable(handle) when that child has gone
        self.on_need = None  # callable(handle, msg): the child asks for a controller object (watch relay)
        # native shard executor (ncc/bin/ncc-executor): `config` renders its first message ({"t": "cfg"})
        self.native = False
        self.binary: str | None = None
        self.config = None
        self._task: asyncio.Task | None = None
        self._stopping = False

    async def _spawn(self) -> None:
        parent, child = socket.socketpair(socket.AF_UNIX, socket.SOCK_STREAM)
        root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        env = dict(self.env or os.environ)
        env["PYTHONPATH"] = root + os.pathsep + env.get("PYTHONPATH", "")
        first = None
        if self.native:
            program = self.binary
            args = ["--fd", str(child.fileno()), "--index", str(self.index), "--part", f"{self.part}/{self.parts}"]
            first = {"t": "cfg", "c": await self.config.render(self)}
        elif self.argv is not None:
            program = sys.executable
            args = [*self.argv, "--control-fd", str(child.fileno())]
        else:
            program = sys.executable
            args = ["-m", "ncc.executor", "--fd", str(child.fileno()), "--index", str(self.index),
                    "--shards", ",".join(self.shards), "--part", f"{self.part}/{self.parts}"]
        gated = self.gated and not self.gate_open
        if gated:
            env["NCC_GATED"] = "1"
        else:
            env.pop("NCC_GATED", None)
        self.proc = await asyncio.create_subprocess_exec(program, *args, pass_fds=(child.fileno(),), env=env)
        child.close()
        if self.on_stream is not None:
            # reports are folded natively straight off the socket (no stream reader, no task wake-up per frame)
            self._eof = asyncio.Event()
            self.channel = RawChannel(parent, self._fold, self._dispatch, self._eof.set)
        else:
            reader, writer = await asyncio.open_connection(sock=parent)
            self.channel = Channel(reader, writer)
        if first is not None:
            self.channel.send(first)
        if gated and self.gate_open:  # the gate opened while this child was being spawned
            self.channel.send({"t": "go"})
        if self.on_spawn is not None:
            self.on_spawn(self)

    def open_gate(self) -> None:
        """This replica leads now: let the (already running, caches synced) child start its workers."""
        if self.gate_open:
            return
        self.gate_open = True
        if self.channel is not None:
            self.channel.send({"t": "go"})

    def kill(self) -> None:
        """Leadership lost: stop the child at once (SIGKILL), without letting it drain its writes."""
        self._stopping = True
        if self.proc is not None and self.proc.returncode is None:
            try:
                self.proc.kill()
            except ProcessLookupError:
                pass

    async def _run(self) -> None:
        backoff = 1.0
        while not self._stopping:
            self.ready.clear()
            self.synced.clear()
            await self._spawn()
            if isinstance(self.channel, RawChannel):
                await self._eof.wait()  # messages are dispatched from the channel's read callback
            else:
                while True:
                    batch = await self.channel.recv()
                    if batch is None:
                        break
                    self._dispatch(batch)
            if self.on_exit is not None:
                self.on_exit(self)
            try:  # the channel is gone: a child that does not exit on its own (wedged) is killed
                rc = await asyncio.wait_for(self.proc.wait(), EXIT_GRACE_S)
            except asyncio.TimeoutError:
                log.error("%s %d (shards %s) did not exit after its channel closed; killing it", self.what,
                          self.index, self.shards)
                self.proc.kill()
                rc = await self.proc.wait()
            self.channel.close()
            if self._stopping:
                return
            self.restarts += 1
            log.error("%s %d (shards %s) exited with %s; restarting in %.1fs", self.what, self.index, self.shards,
                      rc, backoff)
            await asyncio.sleep(backoff)
            backoff = min(backoff * 2, 30.0)

    def _dispatch(self, batch: list) -> None:
        for msg in batch:
            if not isinstance(msg, dict):
                continue
            t = msg.get("t")
            if t == "ready":
                self.ready.set()
                self.synced.set()
            elif t == "synced":
                self.synced.set()
            elif t == "need":
                if self.on_need is not None:
                    self.on_need(self, msg)
                continue
            elif t == "status":
                self.status = status_view(msg)
                continue
            self.on_message(self.index, msg)

    def _fold(self, buf, start: int):
        return self.on_stream(self.index, buf, start)

    def start(self) -> None:
        self._task = asyncio.ensure_future(self._run())

    async def stop(self, timeout: float = 10.0) -> None:
        self._stopping = True
        if self.proc is not None and self.proc.returncode is None:
            try:
                self.proc.terminate()
                await wait_timeout(self.proc.wait(), timeout)
            except (ProcessLookupError, asyncio.TimeoutError):
                try:
                    self.proc.kill()
                except ProcessLookupError:
                    pass
        if self._task is not None:
            self._task.cancel()
            try:
                await self._task
            except (asyncio.CancelledError, Exception):  # noqa: BLE001
                pass


class ExecutorPool:
    """`n` shard groups × `per_shard` key partitions.  Every executor of a group watches the same shards;
    each reconciles only the keys of its partition (`key_part`), so one busy shard can use several cores."""

    def __init__(self, shard_names: list[str], n: int, on_message, env: dict | None = None, per_shard: int = 1,
                 part_base: int = 0, part_stride: int = 1, gated: bool = False, relay=None,
                 native_config=None, on_stream=None):
        """With partitioned coordinators (`part_stride` = C > 1, this coordinator owning keys ≡ `part_base`
        mod C), executor j of a group takes the global key partition part_base + C·j of C·per_shard, so its
        keys are exactly a share of this coordinator's."""
        self.per_shard = max(1, per_shard)
        self.part_base = part_base
        self.part_stride = max(1, part_stride)
        self.on_message = on_message
        self.on_stream = on_stream  # raw-stream report folding (Controller.on_executor_stream)
        self.env = env
        self.relay = relay  # coordinator's WatchRelay: executors get the controller cluster from it
        self.native_config = native_config  # NativeExecutorConfig: run ncc/bin/ncc-executor instead of Python
        self.gated = gated
        self.gate_open = not gated
        self._next_index = 0
        self.handles: list[ExecutorHandle] = []
        for group in partition(shard_names, n):
            self._new_group(group)

    def _new_group(self, shards: list[str]) -> list[ExecutorHandle]:
        hs = [ExecutorHandle(self._next_index + j, list(shards), self.on_message, self.env,
                             self.part_base + self.part_stride * j, self.part_stride * self.per_shard)
              for j in range(self.per_shard)]
        for h in hs:
            h.gated, h.gate_open = self.gated, self.gate_open
            h.on_stream = self.on_stream
            if self.relay is not None:
                h.on_spawn, h.on_exit, h.on_need = self.relay.attach, self.relay.detach, self.relay.on_need
            if self.native_config is not None:
                from .native_executor import binary_path
                h.native, h.binary, h.config = True, binary_path(), self.native_config
        self._next_index += self.per_shard
        self.handles.extend(hs)
        return hs

    def resync_partition(self, part: int, parts: int) -> None:
        """Every executor passes over the keys of coordinator partition `part` of `parts` again (that
        partition's process came up and holds no report state)."""
        for h in self.handles:
            if h.channel is not None:
                h.channel.send({"t": "resync", "p": part, "n": parts})

    def add_shards(self, names: list[str]) -> None:
        """Hot-add: one new executor group per added shard (started immediately)."""
        for n in names:
            for h in self._new_group([n]):
                h.start()

    async def remove_shards(self, names: list[str]) -> None:
        """Hot-remove: stop every group that serves a removed shard; respawn it for its remaining shards."""
        gone = set(names)
        hit = [h for h in self.handles if gone & set(h.shards)]
        groups = {tuple(h.shards) for h in hit}
        await asyncio.gather(*(h.stop() for h in hit))
        self.handles = [h for h in self.handles if h not in hit]
        for g in groups:
            rest = [s for s in g if s not in gone]
            if rest:
                for h in self._new_group(rest):
                    h.start()

    def shards(self) -> list[str]:
        return sorted({s for h in self.handles for s in h.shards})

    def start(self) -> None:
        for h in self.handles:
            h.start()

    async def wait_ready(self, timeout: float | None = None) -> bool:
        try:
            await wait_timeout(asyncio.gather(*(h.ready.wait() for h in self.handles)), timeout)
            return True
        except asyncio.TimeoutError:
            return False

    async def stop(self) -> None:
        await asyncio.gather(*(h.stop() for h in self.handles))

    def open_gate(self) -> None:
        self.gate_open = True
        for h in self.handles:
            h.open_gate()

    def all_synced(self) -> bool:
        return all(h.synced.is_set() for h in self.handles)

    def kill(self) -> None:
        for h in self.handles:
            h.kill()

    def stats(self) -> dict:
        return {h.index: {"shards": h.shards, "part": f"{h.part}/{h.parts}", "restarts": h.restarts,
                          "impl": "native" if h.native else "python",
                          "alive": h.proc is not None and h.proc.returncode is None, "status": h.status}
                for h in self.handles}


class CoordinatorPartitions:
    """Child coordinator processes for key partitions 1..C-1 (partition 0 is the parent itself).

    Each child is a native-mode coordinator (`python -m ncc`) restricted to the template keys ≡ p mod C: it
    watches the controller cluster with that key filter, adopts, writes status and Events for its keys.  It
    runs no executors: the parent's executors serve every key, and the parent's report table hands the
    reports on the child's keys to `forward`, which relays them raw over the child's control channel.  The
    parent holds the leader Lease and the ops endpoints; children exit when that channel closes."""

    def __init__(self, parts: int, env: dict, gated: bool = False, on_child_ready=None):
        self.parts = parts
        self.handles = []
        self.on_child_ready = on_child_ready  # callable(p): child p is up (again) and needs every report
        self.forwarded = 0
        for p in range(1, parts):
            e = dict(env)
            e.update({"NCC_COORDINATOR_PART": f"{p}/{parts}", "NEXUS__LEADER_ELECT": "False",
                      "NEXUS__METRICS_BIND_ADDRESS": "", "NEXUS__HEALTH_BIND_ADDRESS": ""})
            h = ExecutorHandle(p, [], self._on_child_message, e, p, parts, argv=["-m", "ncc"],
                               what="coordinator partition")
            h.gated = gated
            self.handles.append(h)

    def _on_child_message(self, index: int, msg) -> None:
        if isinstance(msg, dict) and msg.get("t") == "ready" and self.on_child_ready is not None:
            self.on_child_ready(index)

    def forward(self, part: int, msgs: list) -> None:
        """Executor reports (raw msgpack messages) on partition `part`'s keys, to its process."""
        if not 1 <= part < self.parts:
            return
        ch = self.handles[part - 1].channel
        if ch is None:
            return  # restarting: it is resynced once it reports ready
        for m in msgs:
            ch.send_packed(m)
        self.forwarded += len(msgs)

    def start(self) -> None:
        for h in self.handles:
            h.start()

    def ready(self) -> bool:
        return all(h.ready.is_set() for h in self.handles)

    def open_gate(self) -> None:
        for h in self.handles:
            h.open_gate()

    def kill(self) -> None:
        for h in self.handles:
            h.kill()

    async def stop(self) -> None:
        await asyncio.gather(*(h.stop() for h in self.handles))

    def stats(self) -> dict:
        return {h.index: {"part": f"{h.part}/{h.parts}", "restarts": h.restarts, "ready": h.ready.is_set(),
                          "alive": h.proc is not None and h.proc.returncode is None} for h in self.handles}


# per shard in a C++ executor's status: its client's adaptive concurrency limit and what drove it
# (native/executor/http.hpp `Client::finish`)
FLOW_FIELDS = ("limit", "inflight", "max_inflight", "rejected_429", "overload_signals", "cuts", "gated",
               "qps_wait_ms", "connections", "write_batches", "requests", "slow_start_exits", "increases_held",
               "loop_wakeups", "loop_coalesced", "http2", "h2_streams", "h2_refused", "h2_goaways", "h2_dead",
               "h2_goaway_errors", "h2_downgraded", "h2_calm", "cap")


def status_view(msg: dict) -> dict:
    """An executor's periodic status message ({"t": "status", "s": {shard: {plural: [synced, watching,
    events, relists, last error]}}, "q", "r", "w", "e"}) as /debug/state shows it."""
    shards, flow = {}, {}
    for shard, kinds in (msg.get("s") or {}).items():
        shards[shard] = {plural: {"synced": bool(v[0]), "watching": bool(v[1]), "events": v[2], "relists": v[3],
                                  "last_error": v[4] or None}
                         for plural, v in (kinds or {}).items()
                         if plural != "flow" and isinstance(v, (list, tuple)) and len(v) >= 5}
        fl = (kinds or {}).get("flow")
        if isinstance(fl, (list, tuple)) and len(fl) >= 8:  # the C++ executor's client-side flow control
            flow[shard] = dict(zip(FLOW_FIELDS, fl))
    out = {"shards": shards, "queued": msg.get("q"), "passes": msg.get("r"), "writes": msg.get("w"),
           "errors": msg.get("e"), "at": time.time()}
    if flow:
        out["flow"] = flow
    if isinstance(msg.get("gc"), dict):  # the Python executor's collector passes (ncc/gctune.py)
        out["gc"] = msg["gc"]
    return out


def status_message(index: int, shards: list, stats: dict) -> dict:
    """The Python executor's status message, the same shape as the C++ executor's (`send_status`)."""
    out = {}
    for sh in shards:
        kinds = {}
        for inf in sh.factory.informers():
            err = inf.last_error if not inf.watching else None
            kinds[inf.rt.plural] = [inf.has_synced(), inf.watching, inf.events, inf.relists,
                                    repr(err)[:300] if err is not None else ""]
        out[sh.name] = kinds
    from .. import gctune
    return {"t": "status", "i": index, "s": out, "q": stats.get("queued"), "r": stats.get("reconciles"),
            "w": stats.get("writes"), "e": stats.get("errors"), "gc": dict(gctune.STATS)}


# ---------------------------------------------------------------------------------------- executor side
async def executor_main(fd: int, index: int, shards: list[str], part: tuple = (0, 1)) -> int:
    from ..app import App, setup_signal_handler
    from ..config import load_config

    cfg = load_config()
    sock = socket.socket(fileno=fd)
    reader, writer = await asyncio.open_connection(sock=sock)
    channel = Channel(reader, writer)
    stop = asyncio.Event()
    setup_signal_handler(stop)
    app = App(cfg, role="executor", shard_filter=set(shards))
    if part[1] > 1:
        app.options.partition = part
    await app.build()
    ctl = app.controller
    ctl.reporter = channel.send
    ctl.on_ready = lambda: channel.send({"t": "ready", "i": index})
    ctl.on_synced = lambda: channel.send({"t": "synced", "i": index})
    feeds = app.relay_feeds  # controller informers fed by the coordinator's watch relay (or None)
    if feeds is not None:
        asked: dict = {}

        def need(kind: int, key: str) -> None:  # at most once a second per object, like the C++ executor
            now = asyncio.get_running_loop().time()
            if now - asked.get(key, -1e9) >= 1.0:
                if len(asked) > 4096:
                    _prune()
                asked[key] = now
                channel.send({"t": "need", "k": kind, "n": key})
        ctl.need = need

        def _prune():  # keep the memo small: forget requests older than a minute
            now = asyncio.get_running_loop().time()
            for k in [k for k, t in asked.items() if now - t > 60.0]:
                del asked[k]

    async def watch_parent():
        # {"t": "go"} opens the gate of an executor pre-spawned by a warm standby; the coordinator closing
        # its end (or dying) ends this executor — and so does a channel it cannot read any more (a malformed
        # or oversized frame): an executor cut off from the relay would reconcile from a stale cache, so it
        # exits and the coordinator respawns it with a fresh snapshot
        try:
            await _watch_parent()
        except Exception:  # noqa: BLE001
            log.exception("executor %d: channel to the coordinator failed; exiting", index)
            exit_code[0] = 1
        stop.set()

    exit_code = [0]

    async def _watch_parent():
        while True:
            batch = await channel.recv()
            if batch is None:
                return
            for msg in batch:
                if not isinstance(msg, dict):
                    continue
                if feeds is not None and deliver(feeds, msg):
                    continue
                if msg.get("t") == "go":
                    app.open_gate()
                elif msg.get("t") == "resync" and app.controller is not None:
                    app.controller.enqueue_all(part=(int(msg.get("p", 0)), int(msg.get("n", 1))))

    async def send_status():
        period = float(os.environ.get("NCC_STATUS_S", "5"))
        while True:
            c = app.controller
            st = dict(c.stats) if c is not None else {}
            if c is not None:
                st["queued"] = len(c.queue)
            channel.send(status_message(index, app.shards, st))
            await asyncio.sleep(period)

    wp = asyncio.ensure_future(watch_parent())
    sp = asyncio.ensure_future(send_status())
    try:
        await app.run(stop)
    finally:
        wp.cancel()
        sp.cancel()
        try:
            await channel.drain()
        except Exception:  # noqa: BLE001
            pass
        channel.close()
    return exit_code[0]


def main(argv=None) -> int:
    from ..proclimits import raise_nofile_limit
    raise_nofile_limit()
    import argparse

    from ..config import load_config
    from ..telemetry.logging import configure_logging

    p = argparse.ArgumentParser(prog="python -m ncc.executor")
    p.add_argument("--fd", type=int, required=True)
    p.add_argument("--index", type=int, default=0)
    p.add_argument("--shards", default="")
    p.add_argument("--part", default="0/1", help="key partition p/k of this executor within its shard group")
    a = p.parse_args(argv)
    pi, _, pk = a.part.partition("/")
    part = (int(pi), int(pk or 1))
    cfg = load_config()
    configure_logging(cfg.log_level, cfg.log_format)
    logging.getLogger().handlers[0].addFilter(lambda r: setattr(r, "executor", a.index) or True)
    from .. import sampler
    sampler.start(f"executor{a.index}")
    prof_path = os.environ.get("NCC_PROFILE")
    if prof_path:
        import cProfile
        prof = cProfile.Profile()
        prof.enable()
        try:
            return asyncio.run(executor_main(a.fd, a.index, [s for s in a.shards.split(",") if s], part))
        finally:
            prof.disable()
            prof.dump_stats(f"{prof_path}.executor{a.index}")
    return asyncio.run(executor_main(a.fd, a.index, [s for s in a.shards.split(",") if s], part))
