"""Small asyncio ASGI server: HTTP/1.1 (keep-alive, Content-Length and chunked bodies, streamed responses) and
RFC 6455 WebSockets, plus the ASGI lifespan protocol.

The reference serves Django through ``manage.py runserver`` plus a Channels/Daphne layer for its two
websockets (``core/kubeops.py:127-140``, ``kubeoperator/routing.py:9-18``). uvicorn is present in this image but
its websocket support needs the ``websockets``/``wsproto`` packages, which are not, so the control plane
carries its own server (stdlib only). It is not meant to face the internet directly -- the compose topology
puts nginx in front, as the reference does (``docker/nginx/f2o.conf``).
"""
from __future__ import annotations

import asyncio
import base64
import hashlib
import logging
import os
import signal
import struct
from urllib.parse import unquote

log = logging.getLogger("kubeoperator.server")
WS_GUID = b"258EAFA5-E914-47DA-95CA-C5AB0DC85B11"
MAX_HEADER = 64 * 1024
MAX_BODY = 512 * 1024 * 1024
REASONS = {101: "Switching Protocols", 200: "OK", 201: "Created", 204: "No Content", 301: "Moved Permanently",
           302: "Found", 304: "Not Modified", 307: "Temporary Redirect", 400: "Bad Request", 401: "Unauthorized",
           403: "Forbidden", 404: "Not Found", 405: "Method Not Allowed", 409: "Conflict", 413: "Payload Too Large",
           422: "Unprocessable Entity", 500: "Internal Server Error", 502: "Bad Gateway", 503: "Service Unavailable"}


class _Closed(Exception):
    pass


async def _read_head(reader: asyncio.StreamReader) -> bytes | None:
    try:
        data = await reader.readuntil(b"\r\n\r\n")
    except asyncio.IncompleteReadError as e:
        if not e.partial:
            return None
        raise _Closed() from e
    except asyncio.LimitOverrunError as e:
        raise _Closed("header too large") from e
    if len(data) > MAX_HEADER:
        raise _Closed("header too large")
    return data


async def _read_body(reader, headers: dict) -> bytes:
    if headers.get(b"transfer-encoding", b"").lower() == b"chunked":
        out = bytearray()
        while True:
            line = await reader.readline()
            size = int(line.split(b";")[0].strip() or b"0", 16)
            if size == 0:
                await reader.readline()
                return bytes(out)
            out += await reader.readexactly(size)
            await reader.readexactly(2)
            if len(out) > MAX_BODY:
                raise _Closed("body too large")
    n = int(headers.get(b"content-length", b"0") or 0)
    if n > MAX_BODY:
        raise _Closed("body too large")
    return await reader.readexactly(n) if n else b""


class Server:
    def __init__(self, app, host: str = "0.0.0.0", port: int = 8000):
        self.app, self.host, self.port = app, host, port
        self._server = None
        self._lifespan_queue: asyncio.Queue | None = None
        self._lifespan_task = None

    # ---------------------------------------------------------------------------------------- lifespan
    async def _lifespan(self, kind: str) -> None:
        if self._lifespan_queue is None:
            self._lifespan_queue = asyncio.Queue()
            done = asyncio.Queue()
            self._lifespan_done = done

            async def receive():
                return await self._lifespan_queue.get()

            async def send(msg):
                await done.put(msg)

            async def run():
                try:
                    await self.app({"type": "lifespan", "asgi": {"version": "3.0"}, "state": {}}, receive, send)
                except Exception:  # noqa: BLE001 -- apps without lifespan support
                    await done.put({"type": "lifespan.unsupported"})

            self._lifespan_task = asyncio.ensure_future(run())
        await self._lifespan_queue.put({"type": f"lifespan.{kind}"})
        msg = await self._lifespan_done.get()
        if msg["type"].endswith(".failed"):
            raise RuntimeError(msg.get("message", f"lifespan {kind} failed"))

    # ---------------------------------------------------------------------------------------- connections
    async def _handle(self, reader: asyncio.StreamReader, writer: asyncio.StreamWriter) -> None:
        peer = writer.get_extra_info("peername") or ("", 0)
        try:
            while True:
                head = await _read_head(reader)
                if head is None:
                    break
                lines = head.decode("latin-1").split("\r\n")
                method, target, version = lines[0].split(" ", 2)
                headers = []
                hmap = {}
                for ln in lines[1:]:
                    if not ln:
                        continue
                    k, _, v = ln.partition(":")
                    kb, vb = k.strip().lower().encode("latin-1"), v.strip().encode("latin-1")
                    headers.append((kb, vb))
                    hmap[kb] = vb
                path, _, qs = target.partition("?")
                scope_base = {"asgi": {"version": "3.0"}, "http_version": version.split("/")[-1],
                              "path": unquote(path), "raw_path": path.encode(), "query_string": qs.encode(),
                              "root_path": "", "headers": headers, "client": tuple(peer[:2]),
                              "server": (self.host, self.port)}
                if hmap.get(b"upgrade", b"").lower() == b"websocket":
                    await self._websocket(reader, writer, dict(scope_base, type="websocket", scheme="ws",
                                                               subprotocols=[]), hmap)
                    break
                body = await _read_body(reader, hmap)
                keep = await self._http(writer, dict(scope_base, type="http", method=method, scheme="http"), body,
                                        hmap, version)
                if not keep:
                    break
        except (_Closed, ConnectionError, asyncio.IncompleteReadError, ValueError):
            pass
        except Exception:  # noqa: BLE001
            log.exception("connection error")
        finally:
            try:
                writer.close()
                await writer.wait_closed()
            except Exception:  # noqa: BLE001
                pass

    async def _http(self, writer, scope, body: bytes, hmap: dict, version: str) -> bool:
        sent_body = False
        state = {"started": False, "chunked": False, "status": 500}
        keep_alive = version == "HTTP/1.1" and hmap.get(b"connection", b"").lower() != b"close"

        async def receive():
            nonlocal sent_body
            if not sent_body:
                sent_body = True
                return {"type": "http.request", "body": body, "more_body": False}
            await asyncio.sleep(3600)
            return {"type": "http.disconnect"}

        async def send(msg):
            if msg["type"] == "http.response.start":
                state["status"] = msg["status"]
                hdrs = list(msg.get("headers", []))
                names = {k.lower() for k, _ in hdrs}
                if b"content-length" not in names:
                    hdrs.append((b"transfer-encoding", b"chunked"))
                    state["chunked"] = True
                hdrs.append((b"connection", b"keep-alive" if keep_alive else b"close"))
                out = [f"HTTP/1.1 {msg['status']} {REASONS.get(msg['status'], 'Status')}\r\n".encode()]
                out += [k + b": " + v + b"\r\n" for k, v in hdrs]
                writer.write(b"".join(out) + b"\r\n")
                state["started"] = True
            elif msg["type"] == "http.response.body":
                data = msg.get("body", b"")
                more = msg.get("more_body", False)
                if state["chunked"]:
                    if data:
                        writer.write(f"{len(data):x}\r\n".encode() + data + b"\r\n")
                    if not more:
                        writer.write(b"0\r\n\r\n")
                else:
                    writer.write(data)
                await writer.drain()

        try:
            await self.app(scope, receive, send)
        except Exception:  # noqa: BLE001
            log.exception("ASGI app error")
            if not state["started"]:
                writer.write(b"HTTP/1.1 500 Internal Server Error\r\ncontent-length: 0\r\nconnection: close\r\n\r\n")
            return False
        log.info('%s "%s %s" %s', scope["client"][0] if scope["client"] else "-", scope["method"], scope["path"],
                 state["status"])
        return keep_alive

    # ---------------------------------------------------------------------------------------- websockets
    async def _websocket(self, reader, writer, scope, hmap: dict) -> None:
        key = hmap.get(b"sec-websocket-key", b"")
        accept = base64.b64encode(hashlib.sha1(key + WS_GUID).digest())
        state = {"accepted": False, "closed": False, "connect_sent": False}
        write_lock = asyncio.Lock()

        async def send_frame(op: int, payload: bytes = b""):
            n = len(payload)
            if n < 126:
                hdr = struct.pack("!BB", 0x80 | op, n)
            elif n < 65536:
                hdr = struct.pack("!BBH", 0x80 | op, 126, n)
            else:
                hdr = struct.pack("!BBQ", 0x80 | op, 127, n)
            async with write_lock:
                writer.write(hdr + payload)
                await writer.drain()

        async def read_frame():
            b1, b2 = await reader.readexactly(2)
            fin, op = b1 & 0x80, b1 & 0x0F
            n = b2 & 0x7F
            if n == 126:
                n = struct.unpack("!H", await reader.readexactly(2))[0]
            elif n == 127:
                n = struct.unpack("!Q", await reader.readexactly(8))[0]
            if n > MAX_BODY:
                raise _Closed("frame too large")
            mask = await reader.readexactly(4) if b2 & 0x80 else None
            data = await reader.readexactly(n)
            if mask:
                data = bytes(b ^ mask[i & 3] for i, b in enumerate(data))
            return bool(fin), op, data

        async def receive():
            if not state["connect_sent"]:
                state["connect_sent"] = True
                return {"type": "websocket.connect"}
            buf, first_op = bytearray(), None
            while True:
                try:
                    fin, op, data = await read_frame()
                except (asyncio.IncompleteReadError, ConnectionError, _Closed):
                    state["closed"] = True
                    return {"type": "websocket.disconnect", "code": 1006}
                if op == 0x8:
                    code = struct.unpack("!H", data[:2])[0] if len(data) >= 2 else 1000
                    if not state["closed"]:
                        state["closed"] = True
                        try:
                            await send_frame(0x8, data[:2])
                        except ConnectionError:
                            pass
                    return {"type": "websocket.disconnect", "code": code}
                if op == 0x9:
                    await send_frame(0xA, data)
                    continue
                if op == 0xA:
                    continue
                if op in (0x1, 0x2):
                    first_op, buf = op, bytearray(data)
                elif op == 0x0:
                    buf += data
                if fin:
                    if first_op == 0x1:
                        return {"type": "websocket.receive", "text": buf.decode()}
                    return {"type": "websocket.receive", "bytes": bytes(buf)}

        async def send(msg):
            t = msg["type"]
            if t == "websocket.accept":
                hdrs = [b"HTTP/1.1 101 Switching Protocols", b"upgrade: websocket", b"connection: Upgrade",
                        b"sec-websocket-accept: " + accept]
                if msg.get("subprotocol"):
                    hdrs.append(b"sec-websocket-protocol: " + msg["subprotocol"].encode())
                writer.write(b"\r\n".join(hdrs) + b"\r\n\r\n")
                await writer.drain()
                state["accepted"] = True
            elif t == "websocket.send":
                if state["closed"]:
                    raise ConnectionError("websocket closed")
                if msg.get("text") is not None:
                    await send_frame(0x1, msg["text"].encode())
                else:
                    await send_frame(0x2, msg.get("bytes") or b"")
            elif t == "websocket.close":
                if not state["accepted"]:
                    writer.write(b"HTTP/1.1 403 Forbidden\r\ncontent-length: 0\r\n\r\n")
                    await writer.drain()
                elif not state["closed"]:
                    state["closed"] = True
                    await send_frame(0x8, struct.pack("!H", msg.get("code", 1000)))

        try:
            await self.app(scope, receive, send)
        except (ConnectionError, _Closed):
            pass
        except Exception:  # noqa: BLE001
            log.exception("websocket app error")

    # ---------------------------------------------------------------------------------------- run
    async def start(self) -> None:
        await self._lifespan("startup")
        self._server = await asyncio.start_server(self._handle, self.host, self.port, limit=MAX_HEADER + 1024)
        sock = self._server.sockets[0].getsockname()
        self.port = sock[1]
        log.info("listening on http://%s:%s", self.host, self.port)

    async def stop(self) -> None:
        if self._server is not None:
            self._server.close()
            await self._server.wait_closed()
        try:
            await asyncio.wait_for(self._lifespan("shutdown"), 5)
        except Exception:  # noqa: BLE001
            pass

    async def serve_forever(self) -> None:
        await self.start()
        stop = asyncio.Event()
        loop = asyncio.get_running_loop()
        for sig in (signal.SIGINT, signal.SIGTERM):
            try:
                loop.add_signal_handler(sig, stop.set)
            except (NotImplementedError, RuntimeError):
                pass
        await stop.wait()
        await self.stop()


def run(app, host: str = "0.0.0.0", port: int = 8000) -> None:
    logging.basicConfig(level=os.environ.get("LOG_LEVEL", "INFO"),
                        format="%(asctime)s %(levelname)s %(name)s: %(message)s")
    asyncio.run(Server(app, host, port).serve_forever())
