"""A small LDAPv3 client (RFC 4511): simple bind, subtree search with RFC 4515 string filters, unbind.

The reference authenticates and syncs users with ``django-auth-ldap`` / ``ldap3`` (``users/authentication/
ldap.py:14-121``, ``users/sync/ldap.py:9-75``). Neither is installed on the controller image, so the control
plane speaks the protocol itself: BER encoding of the few messages it needs over a plain or TLS socket
(``ldap://`` / ``ldaps://``). ``ldap3`` is still used when it is importable.
"""
from __future__ import annotations

import re
import socket
import ssl
from urllib.parse import urlparse


class LDAPError(Exception):
    def __init__(self, code: int, message: str = ""):
        super().__init__(f"LDAP result {code}: {message}" if message else f"LDAP result {code}")
        self.code = code


# ------------------------------------------------------------------------------------------------- BER
def _len(n: int) -> bytes:
    if n < 0x80:
        return bytes([n])
    b = n.to_bytes((n.bit_length() + 7) // 8, "big")
    return bytes([0x80 | len(b)]) + b


def tlv(tag: int, payload: bytes) -> bytes:
    return bytes([tag]) + _len(len(payload)) + payload


def ber_int(v: int, tag: int = 0x02) -> bytes:
    n = max(1, (v.bit_length() + 8) // 8)
    return tlv(tag, v.to_bytes(n, "big", signed=True))


def ber_str(v, tag: int = 0x04) -> bytes:
    return tlv(tag, v.encode() if isinstance(v, str) else bytes(v))


def ber_bool(v: bool) -> bytes:
    return tlv(0x01, b"\xff" if v else b"\x00")


def seq(*items: bytes, tag: int = 0x30) -> bytes:
    return tlv(tag, b"".join(items))


def decode(data: bytes, pos: int = 0):
    """One TLV at ``pos`` -> (tag, value bytes, next position)."""
    tag = data[pos]
    n = data[pos + 1]
    pos += 2
    if n & 0x80:
        k = n & 0x7F
        n = int.from_bytes(data[pos:pos + k], "big")
        pos += k
    return tag, data[pos:pos + n], pos + n


def children(value: bytes) -> list:
    out, pos = [], 0
    while pos < len(value):
        tag, v, pos = decode(value, pos)
        out.append((tag, v))
    return out


def as_int(v: bytes) -> int:
    return int.from_bytes(v, "big", signed=True) if v else 0


# --------------------------------------------------------------------------------------- RFC 4515 filter
def _unescape(s: str) -> bytes:
    return re.sub(rb"\\([0-9a-fA-F]{2})", lambda m: bytes([int(m.group(1), 16)]), s.encode())


def escape_filter_value(v: str) -> str:
    """RFC 4515 escaping of a value put into a filter (user names must not inject filter syntax)."""
    return "".join(f"\\{ord(c):02x}" if c in "*()\\\x00" else c for c in v)


def encode_filter(f: str) -> bytes:
    f = f.strip()
    if not (f.startswith("(") and f.endswith(")")):
        f = f"({f})"
    node, rest = _parse(f, 0)
    if rest != len(f):
        raise ValueError(f"trailing characters in filter {f!r}")
    return node


def _parse(f: str, i: int):
    if f[i] != "(":
        raise ValueError(f"bad filter at {i}: {f!r}")
    i += 1
    op = f[i]
    if op in "&|":
        items = []
        i += 1
        while f[i] == "(":
            n, i = _parse(f, i)
            items.append(n)
        if f[i] != ")":
            raise ValueError(f"unbalanced filter {f!r}")
        return seq(*items, tag=0xA0 if op == "&" else 0xA1), i + 1
    if op == "!":
        n, i = _parse(f, i + 1)
        if f[i] != ")":
            raise ValueError(f"unbalanced filter {f!r}")
        return tlv(0xA2, n), i + 1
    j = f.index(")", i)
    item = f[i:j]
    m = re.match(r"^([A-Za-z0-9.;-]+)(~=|>=|<=|=)(.*)$", item, re.S)
    if not m:
        raise ValueError(f"bad filter item {item!r}")
    attr, cmp_, val = m.groups()
    if cmp_ == "=" and val == "*":
        return ber_str(attr, 0x87), j + 1  # present
    if cmp_ == "=" and "*" in val:
        parts = val.split("*")
        subs = []
        if parts[0]:
            subs.append(ber_str(_unescape(parts[0]), 0x80))
        for p in parts[1:-1]:
            if p:
                subs.append(ber_str(_unescape(p), 0x81))
        if parts[-1]:
            subs.append(ber_str(_unescape(parts[-1]), 0x82))
        return seq(ber_str(attr), seq(*subs), tag=0xA4), j + 1
    tag = {"=": 0xA3, ">=": 0xA5, "<=": 0xA6, "~=": 0xA8}[cmp_]
    return seq(ber_str(attr), ber_str(_unescape(val)), tag=tag), j + 1


# ------------------------------------------------------------------------------------------------ client
class LDAPConnection:
    def __init__(self, uri: str, timeout: float = 10.0):
        u = urlparse(uri)
        tls = u.scheme == "ldaps"
        port = u.port or (636 if tls else 389)
        sock = socket.create_connection((u.hostname, port), timeout=timeout)
        if tls:
            ctx = ssl.create_default_context()
            ctx.check_hostname = False
            ctx.verify_mode = ssl.CERT_NONE
            sock = ctx.wrap_socket(sock, server_hostname=u.hostname)
        self.sock = sock
        self.msgid = 0
        self.buf = b""

    def _send(self, op: bytes) -> int:
        self.msgid += 1
        self.sock.sendall(seq(ber_int(self.msgid), op))
        return self.msgid

    def _recv(self):
        """Next LDAPMessage -> (message id, op tag, op value)."""
        while True:
            if len(self.buf) >= 2:
                try:
                    tag, value, end = decode(self.buf)
                    if end <= len(self.buf):
                        self.buf = self.buf[end:]
                        (_, mid), (optag, opval) = children(value)[:2]
                        return as_int(mid), optag, opval
                except IndexError:
                    pass
            chunk = self.sock.recv(65536)
            if not chunk:
                raise LDAPError(-1, "connection closed")
            self.buf += chunk

    @staticmethod
    def _result(opval: bytes) -> None:
        parts = children(opval)
        code = as_int(parts[0][1])
        if code != 0:
            raise LDAPError(code, parts[2][1].decode(errors="replace") if len(parts) > 2 else "")

    def bind(self, dn: str, password: str) -> None:
        if not password:
            raise LDAPError(49, "empty password (unauthenticated bind refused)")
        self._send(seq(ber_int(3), ber_str(dn), ber_str(password, 0x80), tag=0x60))
        _, optag, opval = self._recv()
        if optag != 0x61:
            raise LDAPError(-1, f"unexpected response tag {optag:#x} to bind")
        self._result(opval)

    def search(self, base: str, filt: str, attributes: list[str] | None = None, size_limit: int = 0) -> list[dict]:
        """Subtree search -> [{"dn": ..., "attrs": {name: [str, ...]}}]."""
        req = seq(ber_str(base), ber_int(2, 0x0A), ber_int(0, 0x0A), ber_int(size_limit), ber_int(0),
                  ber_bool(False), encode_filter(filt), seq(*[ber_str(a) for a in (attributes or [])]), tag=0x63)
        mid = self._send(req)
        out = []
        while True:
            rid, optag, opval = self._recv()
            if rid != mid:
                continue
            if optag == 0x64:  # SearchResultEntry
                dn, attrs = children(opval)[:2]
                entry = {"dn": dn[1].decode(), "attrs": {}}
                for _, a in children(attrs[1]):
                    name, vals = children(a)[:2]
                    entry["attrs"][name[1].decode()] = [v.decode(errors="replace") for _, v in children(vals[1])]
                out.append(entry)
            elif optag == 0x65:  # SearchResultDone
                self._result(opval)
                return out

    def unbind(self) -> None:
        try:
            self._send(tlv(0x42, b""))
        finally:
            self.sock.close()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.unbind()
