"""The coordinator's fold of shard-executor reports.

Every executor pass over a template (or workgroup) ends in one report to the coordinator:
`{"t": "report", "k": key, "u": uid, "g": generation, "r": {shard: error | None}, "w": wrote}`.  The coordinator
keeps, per object key and shard, the last reported (uid, generation, error) and derives the status condition
once *every* shard has reported on the current version (`readiness`).  This is the native mode's version of
the reference's sequential shard loop outcome (`/root/reference/controller.go:790-831`, one error aborts the
loop; here each shard's error is kept and listed).

`ReportTable` is the specification and the fallback; `ncc._native.ReportTable` (native/ncc_native.cpp) is
the implementation the coordinator uses.  Both are fed raw IPC frames (`ipc.Channel.recv_raw`: one msgpack
message, or an array of them), so at 8 shards the 8 reports per template and wave are folded without
materialising a dict per report.  tests/test_reports.py drives the two in lock-step.

`feed(body, batch)` returns `(complete, wrote, errors, others, reports, pending)`:
- `complete`: keys whose report leaves a complete set for the reported version, when the report changed a
  per-shard result or wrote (a repeat of an already complete set with nothing new is not a completion: at 8
  shards each executor's second, dependent-triggered pass would otherwise re-evaluate the template ~5 times
  per wave);
- `wrote`: keys of reports whose pass wrote something (the next status pass records the `Synced` Event);
- `errors`: the failing shard of every failed per-shard result (a metric count each);
- `others`: every non-report message, decoded;
- `reports` / `pending`: reports folded, and how many of them left the set incomplete.
"""
from __future__ import annotations

import zlib

import msgpack

from .. import native
from .ipc import _HDR, MAX_FRAME


class ReportTable:
    def __init__(self) -> None:
        self._shards: list[str] = []
        self._state: dict[str, dict[str, tuple]] = {}
        self._part, self._parts = 0, 1
        self._forwards: dict[int, list] = {}

    def set_partition(self, part: int, parts: int) -> None:
        """This coordinator owns the keys of partition `part` of `parts` (executor.key_part); reports on other
        keys are not folded but kept, as msgpack messages, for `take_forwards` (the parent coordinator relays
        them to the partition's process)."""
        if parts < 1 or not 0 <= part < parts:
            raise ValueError("set_partition: 0 <= part < parts")
        self._part, self._parts = part, parts

    def take_forwards(self) -> dict:
        out, self._forwards = self._forwards, {}
        return out

    def set_shards(self, shards) -> None:
        self._shards = list(shards)

    def shards(self) -> list[str]:
        return list(self._shards)

    def __len__(self) -> int:
        return len(self._state)

    def pop(self, key: str) -> None:
        self._state.pop(key, None)

    def drop_shards(self, names) -> None:
        for st in self._state.values():
            for n in names:
                st.pop(n, None)

    def feed(self, body: bytes, batch: bool) -> tuple:
        msgs = msgpack.unpackb(body, raw=False)
        if not batch:
            msgs = [msgs]
        elif not isinstance(msgs, list):
            raise ValueError("msgpack: malformed frame")
        complete, wrote, errors, others = [], [], [], []
        reports = pending = 0
        for msg in msgs:
            if not isinstance(msg, dict) or msg.get("t") != "report":
                others.append(msg)
                continue
            key, uid, gen = msg["k"], msg.get("u", ""), int(msg.get("g") or 0)
            if self._parts > 1:
                p = zlib.crc32(key.partition("/")[2].encode()) % self._parts
                if p != self._part:
                    self._forwards.setdefault(p, []).append(msgpack.packb(msg, use_bin_type=True))
                    continue
            reports += 1
            st = self._state.setdefault(key, {})
            changed = False
            for shard, err in msg["r"].items():
                e = (uid, gen, err or None)
                changed = changed or st.get(shard) != e
                st[shard] = e
                if err:
                    errors.append(shard)
            if msg.get("w"):
                wrote.append(key)
            for s in self._shards:
                e = st.get(s)
                if e is None or e[0] != uid or e[1] < gen:
                    pending += 1
                    break
            else:
                if changed or msg.get("w"):
                    complete.append(key)
        return complete, wrote, errors, others, reports, pending

    def feed_stream(self, buffer, start: int) -> tuple:
        """Every complete frame of `buffer[start:]` (ipc.py framing) folded: feed()'s tuple + the offset of the
        first byte not consumed."""
        complete, wrote, errors, others = [], [], [], []
        reports = pending = 0
        pos, end = start, len(buffer)
        while end - pos >= 4:
            (n,) = _HDR.unpack_from(buffer, pos)
            batch = bool(n & 0x80000000)
            n &= 0x7FFFFFFF
            if n > MAX_FRAME:
                raise ValueError(f"frame too large: {n}")
            if end - pos - 4 < n:
                break
            r = self.feed(bytes(buffer[pos + 4:pos + 4 + n]), batch)
            complete += r[0]
            wrote += r[1]
            errors += r[2]
            others += r[3]
            reports += r[4]
            pending += r[5]
            pos += 4 + n
        return complete, wrote, errors, others, reports, pending, pos

    def readiness(self, key: str, uid: str, generation: int):
        st = self._state.get(key)
        if st is None:
            return None
        out = {}
        for s in self._shards:
            e = st.get(s)
            if e is None or e[0] != uid or e[1] < generation:
                return None
            out[s] = e[2]
        return out


    def ready_ok(self, key: str, uid: str, generation: int):
        """None while some shard has not reported on this version, else whether every shard succeeded."""
        r = self.readiness(key, uid, generation)
        return None if r is None else not any(r.values())


def make_report_table():
    """The native table when the extension is loaded, else the Python one."""
    m = native.load()
    if m is not None and hasattr(m, "ReportTable"):
        return m.ReportTable()
    return ReportTable()
