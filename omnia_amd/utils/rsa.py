"""Minimal RSA for service-account auth: PKCS#1 / PKCS#8 PEM private keys,
RSASSA-PKCS1-v1_5 SHA-256 signatures (RS256), and key generation for tests.

The image ships no ``cryptography`` package; GCS service-account credentials
(``private_key`` in the JSON key file) need RS256 to mint the OAuth2 JWT
assertion, so the handful of primitives live here.  Verification is
``omnia_amd.facade.auth.rsa_verify_pkcs1_sha256``.
"""
from __future__ import annotations

import base64
import hashlib
import secrets
from dataclasses import dataclass

_SHA256_DI = bytes.fromhex("3031300d060960864801650304020105000420")
_RSA_OID = bytes.fromhex("06092a864886f70d0101010500")  # rsaEncryption + NULL


@dataclass
class PrivateKey:
    n: int
    e: int
    d: int
    p: int = 0
    q: int = 0

    @property
    def size(self) -> int:
        return (self.n.bit_length() + 7) // 8


# ------------------------------------------------------------------ DER
def _read_tlv(b: bytes, i: int) -> tuple[int, bytes, int]:
    tag = b[i]
    ln = b[i + 1]
    i += 2
    if ln & 0x80:
        nb = ln & 0x7F
        ln = int.from_bytes(b[i:i + nb], "big")
        i += nb
    return tag, b[i:i + ln], i + ln


def _seq_items(body: bytes) -> list[tuple[int, bytes]]:
    out, i = [], 0
    while i < len(body):
        tag, val, i = _read_tlv(body, i)
        out.append((tag, val))
    return out


def _enc_len(n: int) -> bytes:
    if n < 0x80:
        return bytes([n])
    b = n.to_bytes((n.bit_length() + 7) // 8, "big")
    return bytes([0x80 | len(b)]) + b


def _tlv(tag: int, val: bytes) -> bytes:
    return bytes([tag]) + _enc_len(len(val)) + val


def _int(v: int) -> bytes:
    b = v.to_bytes(max(1, (v.bit_length() + 8) // 8), "big")  # leading 0 keeps it positive
    return _tlv(0x02, b)


# ------------------------------------------------------------------ PEM
def load_private_key(pem: str | bytes) -> PrivateKey:
    if isinstance(pem, bytes):
        pem = pem.decode()
    lines = [ln for ln in pem.strip().splitlines() if ln and not ln.startswith("-----")]
    der = base64.b64decode("".join(lines))
    tag, body, _ = _read_tlv(der, 0)
    if tag != 0x30:
        raise ValueError("private key is not a DER SEQUENCE")
    items = _seq_items(body)
    if len(items) >= 3 and items[1][0] == 0x30 and items[2][0] == 0x04:  # PKCS#8
        _, body, _ = _read_tlv(items[2][1], 0)
        items = _seq_items(body)
    ints = [int.from_bytes(v, "big") for t, v in items if t == 0x02]
    if len(ints) < 4:
        raise ValueError("not an RSA private key")
    _, n, e, d = ints[:4]
    p, q = (ints[4], ints[5]) if len(ints) >= 6 else (0, 0)
    return PrivateKey(n, e, d, p, q)


def dump_private_key_pkcs8(k: PrivateKey) -> str:
    dp, dq = k.d % (k.p - 1), k.d % (k.q - 1)
    qinv = pow(k.q, -1, k.p)
    rsa = _tlv(0x30, b"".join(_int(v) for v in (0, k.n, k.e, k.d, k.p, k.q, dp, dq, qinv)))
    der = _tlv(0x30, _int(0) + _tlv(0x30, _RSA_OID) + _tlv(0x04, rsa))
    b64 = base64.b64encode(der).decode()
    body = "\n".join(b64[i:i + 64] for i in range(0, len(b64), 64))
    return f"-----BEGIN PRIVATE KEY-----\n{body}\n-----END PRIVATE KEY-----\n"


# ------------------------------------------------------------------ sign
def sign_pkcs1_sha256(k: PrivateKey, msg: bytes) -> bytes:
    t = _SHA256_DI + hashlib.sha256(msg).digest()
    if k.size < len(t) + 11:
        raise ValueError("key too small for SHA-256 PKCS#1 v1.5")
    em = b"\x00\x01" + b"\xff" * (k.size - len(t) - 3) + b"\x00" + t
    m = int.from_bytes(em, "big")
    if k.p and k.q:  # CRT
        dp, dq = k.d % (k.p - 1), k.d % (k.q - 1)
        m1, m2 = pow(m, dp, k.p), pow(m, dq, k.q)
        h = (pow(k.q, -1, k.p) * (m1 - m2)) % k.p
        s = m2 + h * k.q
    else:
        s = pow(m, k.d, k.n)
    return s.to_bytes(k.size, "big")


# ------------------------------------------------------------------ keygen (tests)
def _probable_prime(bits: int) -> int:
    small = [p for p in range(3, 2000, 2) if all(p % q for q in range(3, int(p ** 0.5) + 1, 2))]
    while True:
        c = secrets.randbits(bits) | (1 << (bits - 1)) | (1 << (bits - 2)) | 1
        if any(c % p == 0 for p in small):
            continue
        d, r = c - 1, 0
        while d % 2 == 0:
            d //= 2
            r += 1
        for _ in range(24):
            a = secrets.randbelow(c - 3) + 2
            x = pow(a, d, c)
            if x in (1, c - 1):
                continue
            for _ in range(r - 1):
                x = pow(x, 2, c)
                if x == c - 1:
                    break
            else:
                break
        else:
            return c


def generate_private_key(bits: int = 2048, e: int = 65537) -> PrivateKey:
    while True:
        p, q = _probable_prime(bits // 2), _probable_prime(bits // 2)
        phi = (p - 1) * (q - 1)
        if p != q and phi % e:
            return PrivateKey(p * q, e, pow(e, -1, phi), p, q)
