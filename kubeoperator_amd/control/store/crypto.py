"""Secret-at-rest encryption and password hashing for the control plane (stdlib only).

The reference only *signs* secrets (itsdangerous JWS with SECRET_KEY, common/models.py:46-56): anyone
with DB read access recovers every host password. Here secrets are encrypted: HMAC-SHA256 used as a PRF
in counter mode produces the keystream (key = HKDF-style derivation of SECRET_KEY, 16-byte random
nonce per value), and an HMAC-SHA256 tag over nonce||ciphertext authenticates it (encrypt-then-MAC).
Passwords of console users are PBKDF2-SHA256 hashed (600k iterations).
"""
from __future__ import annotations

import base64
import hashlib
import hmac
import os

PREFIX = "enc1:"


def _keys(secret: str) -> tuple[bytes, bytes]:
    root = hashlib.sha256(secret.encode()).digest()
    enc = hmac.new(root, b"kubeoperator-amd/enc", hashlib.sha256).digest()
    mac = hmac.new(root, b"kubeoperator-amd/mac", hashlib.sha256).digest()
    return enc, mac


def _stream(key: bytes, nonce: bytes, n: int) -> bytes:
    out = bytearray()
    ctr = 0
    while len(out) < n:
        out += hmac.new(key, nonce + ctr.to_bytes(8, "big"), hashlib.sha256).digest()
        ctr += 1
    return bytes(out[:n])


def encrypt(plain: str, secret: str) -> str:
    if plain is None or plain == "":
        return ""
    if isinstance(plain, str) and plain.startswith(PREFIX):
        return plain
    enc, mac = _keys(secret)
    nonce = os.urandom(16)
    data = plain.encode()
    ct = bytes(a ^ b for a, b in zip(data, _stream(enc, nonce, len(data))))
    tag = hmac.new(mac, nonce + ct, hashlib.sha256).digest()[:16]
    return PREFIX + base64.urlsafe_b64encode(nonce + tag + ct).decode()


def decrypt(token: str, secret: str) -> str:
    if not token:
        return ""
    if not token.startswith(PREFIX):
        return token  # plaintext legacy value
    raw = base64.urlsafe_b64decode(token[len(PREFIX):].encode())
    nonce, tag, ct = raw[:16], raw[16:32], raw[32:]
    enc, mac = _keys(secret)
    if not hmac.compare_digest(tag, hmac.new(mac, nonce + ct, hashlib.sha256).digest()[:16]):
        raise ValueError("secret failed authentication (wrong SECRET_KEY or tampered value)")
    return bytes(a ^ b for a, b in zip(ct, _stream(enc, nonce, len(ct)))).decode()


def hash_password(password: str, iterations: int | None = None) -> str:
    iterations = iterations or int(os.environ.get("KOP_PBKDF2_ITERS", "600000"))
    salt = os.urandom(16)
    dk = hashlib.pbkdf2_hmac("sha256", password.encode(), salt, iterations)
    return f"pbkdf2_sha256${iterations}${base64.b64encode(salt).decode()}${base64.b64encode(dk).decode()}"


def verify_password(password: str, encoded: str) -> bool:
    try:
        algo, it, salt, h = encoded.split("$")
        if algo != "pbkdf2_sha256":
            return False
        dk = hashlib.pbkdf2_hmac("sha256", password.encode(), base64.b64decode(salt), int(it))
        return hmac.compare_digest(dk, base64.b64decode(h))
    except Exception:
        return False
