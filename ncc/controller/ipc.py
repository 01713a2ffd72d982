"""Length-prefixed msgpack framing between the coordinator and its shard-executor processes."""
from __future__ import annotations

import asyncio
import collections
import logging
import os
import struct

import msgpack

_HDR = struct.Struct(">I")
log = logging.getLogger("ncc.ipc")

MAX_FRAME = 64 * 1024 * 1024
FRAME_BUDGET = 16 * 1024 * 1024  # coalesce queued messages into frames of about this size at most
# A peer that stops reading (an executor wedged or stopped) must not grow the coordinator's memory without
# bound: past this many unsent bytes the channel is closed as if the peer had gone (it is respawned with a
# fresh snapshot), as an apiserver terminates a watcher that cannot keep up.
MAX_BACKLOG = int(os.environ.get("NCC_IPC_MAX_BACKLOG", str(512 << 20)))


def frames(msgs: list):
    """Encoded messages → framed bytes: one frame per FRAME_BUDGET bytes of messages (a msgpack array when it
    holds several), so a frame never approaches the MAX_FRAME cap."""
    group, size = [], 0
    for m in msgs:
        if group and size + len(m) > FRAME_BUDGET:
            yield _frame(group)
            group, size = [], 0
        group.append(m)
        size += len(m)
    if group:
        yield _frame(group)


def _frame(msgs: list) -> bytes:
    n = len(msgs)
    batch = n > 1
    if batch:  # a msgpack array of the queued messages
        head = bytes((0x90 | n,)) if n < 16 else (b"\xdc" + n.to_bytes(2, "big") if n < 65536
                                                 else b"\xdd" + n.to_bytes(4, "big"))
        body = head + b"".join(msgs)
    else:
        body = msgs[0]
    if len(body) > MAX_FRAME:
        raise ValueError(f"message too large for one frame: {len(body)} bytes")
    return _HDR.pack(len(body) | (0x80000000 if batch else 0)) + body


class RawChannel:
    """The coordinator's end of an executor socketpair, without asyncio streams.

    Executors report after every pass; at 8 shards the coordinator takes in tens of thousands of small
    frames per second.  Through a StreamReader each read costs a protocol callback, a buffer copy, a reader
    task wake-up and a resume.  Here the socket's readability callback reads what has arrived and hands it
    straight to `fold(buffer, start) -> (other messages, end)` (the native report table parses the framing
    and folds the reports in place); `on_messages(list)` gets whatever it did not fold, `on_eof()` the end
    of the stream.  Writes use the same frames as `Channel`, sent from the loop directly (the relay's lines,
    `go`/`resync`/`cred`), buffered only while the socket is full."""

    def __init__(self, sock, fold, on_messages, on_eof):
        sock.setblocking(False)
        self.sock = sock
        self._fd = sock.fileno()
        self._loop = asyncio.get_running_loop()
        self._fold, self._on_messages, self._on_eof = fold, on_messages, on_eof
        self._rbuf = bytearray()
        self._rpos = 0
        self._pending: list = []
        self._flush_handle: asyncio.Handle | None = None
        self._out = bytearray()
        self._writing = False
        self._drained: asyncio.Future | None = None
        self._closed = False
        self.sent = 0
        self.received = 0
        self._loop.add_reader(self._fd, self._on_readable)

    # ------------------------------------------------------------------ read side
    def _on_readable(self) -> None:
        try:
            data = self.sock.recv(1 << 18)
        except (BlockingIOError, InterruptedError):
            return
        except OSError:
            data = b""
        if not data:
            self._eof()
            return
        self.received += 1
        if self._rpos < len(self._rbuf):  # a partial frame is waiting
            self._rbuf += data
            src, start = self._rbuf, self._rpos
        else:
            src, start = data, 0
        try:
            msgs, end = self._fold(src, start)
        except Exception:  # noqa: BLE001 — a corrupt stream: drop the executor (the handle restarts it)
            import logging
            logging.getLogger("ncc.ipc").exception("bad frame from a shard executor; closing its channel")
            self._eof()
            return
        if end >= len(src):
            self._rbuf, self._rpos = bytearray(), 0
        elif src is data:
            self._rbuf, self._rpos = bytearray(data[end:]), 0
        elif end > (1 << 16):
            del self._rbuf[:end]
            self._rpos = 0
        else:
            self._rpos = end
        if msgs:
            self._on_messages(msgs)

    def _eof(self) -> None:
        if self._closed:
            return
        self.close()
        self._on_eof()

    # ------------------------------------------------------------------ write side
    def send(self, msg) -> None:
        self.send_packed(msgpack.packb(msg, use_bin_type=True))

    def send_packed(self, packed: bytes) -> None:
        if self._closed:
            return
        self._pending.append(packed)
        if self._flush_handle is None:
            self._flush_handle = self._loop.call_soon(self._flush)

    def _flush(self) -> None:
        self._flush_handle = None
        if self._closed or not self._pending:
            self._pending.clear()
            return
        pending, self._pending = self._pending, []
        for frame in frames(pending):
            self._out += frame
            self.sent += 1
        self._write()
        if len(self._out) > MAX_BACKLOG and not self._closed:
            log.error("peer is not reading (%d MiB unsent): closing the channel", len(self._out) >> 20)
            self._out.clear()
            self._eof()

    def _write(self) -> None:
        while self._out:
            try:
                n = self.sock.send(self._out)
            except (BlockingIOError, InterruptedError):
                break
            except OSError:
                self._out.clear()
                self._eof()
                return
            del self._out[:n]
        if self._out and not self._writing:
            self._writing = True
            self._loop.add_writer(self._fd, self._on_writable)
        elif not self._out:
            if self._writing:
                self._writing = False
                self._loop.remove_writer(self._fd)
            if self._drained is not None and not self._drained.done():
                self._drained.set_result(None)

    def _on_writable(self) -> None:
        self._write()

    async def drain(self) -> None:
        self._flush()
        if self._out and not self._closed:
            self._drained = self._loop.create_future()
            await self._drained

    def close(self) -> None:
        if self._closed:
            return
        self._closed = True
        if self._flush_handle is not None:
            self._flush_handle.cancel()
            self._flush_handle = None
        try:
            self._loop.remove_reader(self._fd)
            if self._writing:
                self._loop.remove_writer(self._fd)
        except (ValueError, OSError):
            pass
        if self._drained is not None and not self._drained.done():
            self._drained.set_result(None)
        try:
            self.sock.close()
        except OSError:
            pass


class Channel:
    def __init__(self, reader: asyncio.StreamReader, writer: asyncio.StreamWriter):
        self.reader = reader
        self.writer = writer
        self._pending: list = []
        self._flush_handle: asyncio.Handle | None = None
        self.sent = 0
        self.received = 0
        self._rbuf = bytearray()  # bytes read but not yet framed
        self._rpos = 0
        self._frames: collections.deque = collections.deque()  # framed, not yet handed out (recv_raw)

    def send(self, msg) -> None:
        """Queue a message; frames are coalesced and written on the next loop iteration."""
        self.send_packed(msgpack.packb(msg, use_bin_type=True))

    def send_packed(self, packed: bytes) -> None:
        """Queue an already msgpack-encoded message (the watch relay encodes a batch once for every
        executor it goes to)."""
        self._pending.append(packed)
        if self._flush_handle is None:
            self._flush_handle = asyncio.get_running_loop().call_soon(self._flush)

    def _flush(self) -> None:
        self._flush_handle = None
        if not self._pending or self.writer.is_closing():
            self._pending.clear()
            return
        pending, self._pending = self._pending, []
        for frame in frames(pending):
            self.writer.write(frame)
            self.sent += 1

    async def drain(self) -> None:
        self._flush()
        await self.writer.drain()

    async def recv(self) -> list | None:
        """Next batch of messages (list), or None at EOF."""
        raw = await self.recv_raw()
        if raw is None:
            return None
        body, batch = raw
        msg = msgpack.unpackb(body, raw=False)
        return msg if batch else [msg]

    async def recv_raw(self) -> tuple[bytes, bool] | None:
        """Next frame undecoded: (msgpack body, whether it is an array of messages), or None at EOF."""
        if not self._frames:
            frames = await self.recv_frames()
            if frames is None:
                return None
            self._frames.extend(frames)
        return self._frames.popleft()

    async def recv_frames(self) -> list | None:
        """Every complete frame that has arrived, undecoded ([(body, batch), ...], at least one), or None at
        EOF.  One read per call instead of two awaited `readexactly` per frame: a coordinator at 8 shards
        receives ~70k small report frames per 8 waves."""
        if self._frames:
            out = list(self._frames)
            self._frames.clear()
            return out
        buf = self._rbuf
        while True:
            out = []
            pos, end = self._rpos, len(buf)
            with memoryview(buf) as mv:  # released before the buffer is resized below
                while end - pos >= 4:
                    (n,) = _HDR.unpack_from(buf, pos)
                    batch = bool(n & 0x80000000)
                    n &= 0x7FFFFFFF
                    if n > MAX_FRAME:
                        raise ValueError(f"frame too large: {n}")
                    if end - pos - 4 < n:
                        break
                    out.append((bytes(mv[pos + 4:pos + 4 + n]), batch))
                    pos += 4 + n
            if pos == end:
                buf.clear()
                pos = 0
            elif pos > (1 << 16):
                del buf[:pos]
                pos = 0
            self._rpos = pos
            if out:
                self.received += len(out)
                return out
            try:
                data = await self.reader.read(1 << 18)
            except ConnectionError:
                data = b""
            if not data:
                return None
            buf += data

    async def recv_folded(self, fold) -> list | None:
        """Read what has arrived and fold it in place: `fold(buffer, start) -> (messages, end)` consumes the
        complete frames of `buffer[start:]` (the coordinator's native report table parses the framing itself)
        and returns the messages it did not fold.  Returns them after each read (possibly none), or None at
        EOF.  Not to be mixed with recv/recv_raw on one channel."""
        try:
            data = await self.reader.read(1 << 18)
        except ConnectionError:
            data = b""
        if not data:
            return None
        if self._rpos < len(self._rbuf):  # a partial frame is waiting
            self._rbuf += data
            src, start = self._rbuf, self._rpos
        else:
            src, start = data, 0
        msgs, end = fold(src, start)
        if end >= len(src):
            self._rbuf, self._rpos = bytearray(), 0
        elif src is data:
            self._rbuf, self._rpos = bytearray(data[end:]), 0
        elif end > (1 << 16):
            del self._rbuf[:end]
            self._rpos = 0
        else:
            self._rpos = end
        return msgs

    def close(self) -> None:
        try:
            self.writer.close()
        except Exception:  # noqa: BLE001
            pass
