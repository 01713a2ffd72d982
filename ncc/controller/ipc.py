"""Length-prefixed msgpack framing between the coordinator and its shard-executor processes."""
from __future__ import annotations

import asyncio
import collections
import struct

import msgpack

_HDR = struct.Struct(">I")
MAX_FRAME = 64 * 1024 * 1024
FRAME_BUDGET = 16 * 1024 * 1024  # coalesce queued messages into frames of about this size at most


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
        group, size = [], 0
        for m in pending:  # one frame per FRAME_BUDGET bytes: a frame never approaches the MAX_FRAME cap
            if group and size + len(m) > FRAME_BUDGET:
                self._write_frame(group)
                group, size = [], 0
            group.append(m)
            size += len(m)
        self._write_frame(group)

    def _write_frame(self, msgs: list) -> None:
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
        self.writer.write(_HDR.pack(len(body) | (0x80000000 if batch else 0)) + body)
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
