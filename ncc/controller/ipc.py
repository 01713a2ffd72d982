"""Length-prefixed msgpack framing between the coordinator and its shard-executor processes."""
from __future__ import annotations

import asyncio
import struct

import msgpack

_HDR = struct.Struct(">I")
MAX_FRAME = 64 * 1024 * 1024


class Channel:
    def __init__(self, reader: asyncio.StreamReader, writer: asyncio.StreamWriter):
        self.reader = reader
        self.writer = writer
        self._pending: list = []
        self._flush_handle: asyncio.Handle | None = None
        self.sent = 0
        self.received = 0

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
        n = len(self._pending)
        batch = n > 1
        if batch:  # a msgpack array of the queued messages
            head = bytes((0x90 | n,)) if n < 16 else (b"\xdc" + n.to_bytes(2, "big") if n < 65536
                                                     else b"\xdd" + n.to_bytes(4, "big"))
            body = head + b"".join(self._pending)
        else:
            body = self._pending[0]
        self._pending = []
        self.writer.write(_HDR.pack(len(body) | (0x80000000 if batch else 0)) + body)
        self.sent += 1

    async def drain(self) -> None:
        self._flush()
        await self.writer.drain()

    async def recv(self) -> list | None:
        """Next batch of messages (list), or None at EOF."""
        try:
            hdr = await self.reader.readexactly(_HDR.size)
        except (asyncio.IncompleteReadError, ConnectionError):
            return None
        (n,) = _HDR.unpack(hdr)
        batch = bool(n & 0x80000000)
        n &= 0x7FFFFFFF
        if n > MAX_FRAME:
            raise ValueError(f"frame too large: {n}")
        try:
            body = await self.reader.readexactly(n)
        except (asyncio.IncompleteReadError, ConnectionError):
            return None
        self.received += 1
        msg = msgpack.unpackb(body, raw=False)
        return msg if batch else [msg]

    def close(self) -> None:
        try:
            self.writer.close()
        except Exception:  # noqa: BLE001
            pass
