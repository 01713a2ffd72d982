"""HTTP proxies for the API clients, as client-go's transport uses them.

client-go takes a cluster's proxy from the kubeconfig's `proxy-url` (`rest.Config.Proxy`), and otherwise from
the environment through Go's `http.ProxyFromEnvironment`: `HTTPS_PROXY` for https:// servers, `HTTP_PROXY` for
http://, `NO_PROXY` exempting hosts, and requests to localhost / loopback addresses never proxied.  A
kube-apiserver is reached through the proxy with an HTTP CONNECT tunnel, and TLS (and HTTP/2) run inside it.

`proxy_for` picks the proxy for a server URL by those rules; `open_tunnel` opens the CONNECT tunnel and hands
back the connected socket, which the connection pools then wrap (`ncc/kube/transport.py`, `h2client.py`).
The C++ shard executor is given the same proxy URL by the coordinator and opens the same tunnel
(`native/executor/http.hpp` `Conn::connect`).  `socks5://` (and `socks5h://`) proxies are supported as Go's
transport supports them (RFC 1928, username/password authentication RFC 1929): the target's IP address when it
is one, its name for the proxy to resolve otherwise.
"""
from __future__ import annotations

import asyncio
import base64
import ipaddress
import os
import socket
from urllib.parse import unquote, urlsplit

from ..aio import wait_timeout
from . import errors as E


def _is_loopback(host: str) -> bool:
    try:
        return ipaddress.ip_address(host.strip("[]")).is_loopback
    except ValueError:
        return False


def _bypassed(host: str, port: int, no_proxy: str) -> bool:
    """Go's NO_PROXY matching (golang.org/x/net/http/httpproxy): `*` matches everything; an IP or CIDR matches
    addresses; a domain matches itself and its subdomains, a leading dot only the subdomains; an entry may
    carry a port, which must then match too."""
    for raw in no_proxy.split(","):
        e = raw.strip().lower()
        if not e:
            continue
        if e == "*":
            return True
        e_port = None
        if e.count(":") == 1 or (e.startswith("[") and "]:" in e):
            e, _, p = e.rpartition(":")
            e_port = int(p) if p.isdigit() else None
        e = e.strip("[]")
        if e_port is not None and e_port != port:
            continue
        try:
            net = ipaddress.ip_network(e, strict=False)
            try:
                if ipaddress.ip_address(host.strip("[]")) in net:
                    return True
            except ValueError:
                pass
            continue
        except ValueError:
            pass
        if e.startswith("*."):  # Go's parseNoProxy: "*.example.com" is ".example.com" (subdomains only)
            e = e[1:]
        if e.startswith("."):
            if host.endswith(e):
                return True
        elif host == e or host.endswith("." + e):
            return True
    return False


def proxy_for(server: str, explicit: str | None = None, environ=None) -> str | None:
    """The proxy URL a client of `server` goes through, or None for a direct connection."""
    if explicit:
        return explicit if "://" in explicit else "http://" + explicit
    env = os.environ if environ is None else environ
    u = urlsplit(server)
    host = (u.hostname or "").lower()
    if host == "localhost" or _is_loopback(host):
        return None
    https = u.scheme == "https"
    proxy = (env.get("HTTPS_PROXY") or env.get("https_proxy")) if https else \
        (env.get("HTTP_PROXY") or env.get("http_proxy"))
    if not proxy:
        return None
    port = u.port or (443 if https else 80)
    if _bypassed(host, port, env.get("NO_PROXY") or env.get("no_proxy") or ""):
        return None
    return proxy if "://" in proxy else "http://" + proxy


def connect_request(proxy: str, host: str, port: int) -> bytes:
    """The CONNECT request for `host:port` through `proxy` (with Basic proxy credentials from its userinfo)."""
    p = urlsplit(proxy)
    target = f"[{host}]:{port}" if ":" in host else f"{host}:{port}"
    head = f"CONNECT {target} HTTP/1.1\r\nHost: {target}\r\n"
    if p.username is not None:
        cred = f"{unquote(p.username)}:{unquote(p.password or '')}".encode()
        head += "Proxy-Authorization: Basic " + base64.b64encode(cred).decode() + "\r\n"
    return (head + "\r\n").encode("latin-1")


def socks5_connect_request(host: str, port: int) -> bytes:
    """RFC 1928 CONNECT: an IPv4/IPv6 address as such, a name as a domain (the proxy resolves it)."""
    h = host.strip("[]")
    try:
        ip = ipaddress.ip_address(h)
        addr = (b"\x01" if ip.version == 4 else b"\x04") + ip.packed
    except ValueError:
        name = h.encode("idna")
        if len(name) > 255:
            raise E.TransportError(f"socks5: host name too long: {h[:64]}...")
        addr = b"\x03" + bytes([len(name)]) + name
    return b"\x05\x01\x00" + addr + port.to_bytes(2, "big")


async def _socks5_handshake(loop, sock, p, host: str, port: int, timeout: float) -> None:
    where = f"socks5 proxy {p.hostname}:{p.port or 1080}"

    async def exactly(n: int) -> bytes:
        out = b""
        while len(out) < n:
            chunk = await wait_timeout(loop.sock_recv(sock, n - len(out)), timeout)
            if not chunk:
                raise E.TransportError(f"{where} closed the connection during the handshake")
            out += chunk
        return out

    user = unquote(p.username) if p.username is not None else None
    await wait_timeout(loop.sock_sendall(sock, b"\x05\x02\x00\x02" if user is not None else b"\x05\x01\x00"),
                       timeout)
    ver, method = await exactly(2)
    if ver != 5 or method == 0xFF or (method == 2 and user is None) or method not in (0, 2):
        raise E.TransportError(f"{where} refused every authentication method offered (chose {method:#x})")
    if method == 2:
        u, pw = user.encode(), unquote(p.password or "").encode()
        if len(u) > 255 or len(pw) > 255:
            raise E.TransportError(f"{where}: credentials longer than 255 bytes")
        await wait_timeout(loop.sock_sendall(sock, b"\x01" + bytes([len(u)]) + u + bytes([len(pw)]) + pw), timeout)
        if (await exactly(2))[1] != 0:
            raise E.TransportError(f"{where} rejected the username/password")
    await wait_timeout(loop.sock_sendall(sock, socks5_connect_request(host, port)), timeout)
    ver, rep, _, atyp = await exactly(4)
    if ver != 5 or rep != 0:
        raise E.TransportError(f"{where} refused CONNECT {host}:{port}: reply {rep:#x}")
    alen = {1: 4, 4: 16}.get(atyp)
    if alen is None:
        alen = (await exactly(1))[0]
    await exactly(alen + 2)  # the bound address and port: unused


async def open_tunnel(proxy: str, host: str, port: int, timeout: float) -> socket.socket:
    """A socket connected through `proxy` to `host:port` (CONNECT answered 200, or the SOCKS5 handshake done),
    ready for TLS or HTTP."""
    p = urlsplit(proxy)
    socks = p.scheme in ("socks5", "socks5h")
    if p.scheme not in ("http", "") and not socks:
        raise E.TransportError(f"proxy {proxy}: only http:// (CONNECT) and socks5:// proxies are supported")
    phost, pport = p.hostname or "", p.port or (1080 if socks else 80)
    loop = asyncio.get_running_loop()
    try:
        infos = await wait_timeout(loop.getaddrinfo(phost, pport, type=socket.SOCK_STREAM), timeout)
    except (OSError, asyncio.TimeoutError) as e:
        raise E.TransportError(f"proxy {phost}:{pport}: {type(e).__name__}: {e}") from e
    family, _, _, _, addr = infos[0]
    sock = socket.socket(family, socket.SOCK_STREAM)
    sock.setblocking(False)
    try:
        await wait_timeout(loop.sock_connect(sock, addr), timeout)
        if socks:
            await _socks5_handshake(loop, sock, p, host, port, timeout)
            return sock
        await wait_timeout(loop.sock_sendall(sock, connect_request(proxy, host, port)), timeout)
        buf = b""
        while b"\r\n\r\n" not in buf:
            chunk = await wait_timeout(loop.sock_recv(sock, 4096), timeout)
            if not chunk:
                raise E.TransportError(f"proxy {phost}:{pport} closed the connection during CONNECT")
            buf += chunk
            if len(buf) > 65536:
                raise E.TransportError(f"proxy {phost}:{pport}: CONNECT answer too large")
        head, _, rest = buf.partition(b"\r\n\r\n")
        line = head.split(b"\r\n", 1)[0]
        parts = line.split(b" ", 2)
        if len(parts) < 2 or parts[1] != b"200":
            raise E.TransportError(f"proxy {phost}:{pport} refused CONNECT {host}:{port}: "
                                   f"{line.decode('latin-1', 'replace')[:120]}")
        if rest:
            raise E.TransportError(f"proxy {phost}:{pport} sent data before the tunnel was used")
        return sock
    except BaseException as e:
        sock.close()
        if isinstance(e, (OSError, asyncio.TimeoutError)):
            raise E.TransportError(f"proxy {phost}:{pport}: {type(e).__name__}: {e}") from e
        raise
