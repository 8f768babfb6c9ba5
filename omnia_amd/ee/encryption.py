"""Envelope encryption of session data at rest (``ee/pkg/encryption``).

* AES-256-GCM primitive: native AES-NI/PCLMUL (``omnia_amd/native/csrc/aes_gcm.cpp``).
* :class:`LocalKMS` -- key-encryption keys (KEKs) kept locally, versioned,
  rotatable; each ``encrypt`` draws a fresh data key (DEK), seals the data with
  it and wraps the DEK with the current KEK version (envelope encryption).
* :class:`VaultTransitKMS` -- HashiCorp Vault transit engine over HTTP
  (``ee/pkg/encryption/vault_transit.go``): DEK wrapped by ``/transit/encrypt``.
  AWS KMS / GCP KMS / Azure Key Vault need their vendor SDKs, absent here;
  selecting them raises ``ProviderUnavailable``.
* :class:`Encryptor` -- field-level message / tool-call / runtime-event
  encryption with the ``_encryption`` metadata record (``encryptor.go:76-157``,
  ``envelope.go``), and :class:`ReEncryptor` for KEK rotation
  (``reencryptor.go``).

Ciphertext blob layout (binary, base64 in JSON):
``b"OE1" | kid_len u8 | kid | ver_len u8 | ver | edk_len u16 | edk | iv 12 | ct||tag``.
"""
from __future__ import annotations

import base64
import json
import os
import struct
import threading
import time
from dataclasses import dataclass, field

from ..native import native

ALGORITHM = "AES-256-GCM"
META_KEY = "_encryption"
PAYLOAD_KEY = "_payload"
MAGIC = b"OE1"


class ProviderUnavailable(RuntimeError):
    pass


@dataclass
class EncryptOutput:
    ciphertext: bytes
    key_id: str
    key_version: str
    algorithm: str = ALGORITHM


@dataclass
class KeyMetadata:
    key_id: str
    key_version: str
    algorithm: str = ALGORITHM
    created_at: float = 0.0
    enabled: bool = True


def seal(key: bytes, plaintext: bytes, aad: bytes = b"") -> bytes:
    iv = os.urandom(12)
    return iv + native().aes_gcm_encrypt(key, iv, plaintext, aad)


def open_(key: bytes, blob: bytes, aad: bytes = b"") -> bytes:
    return native().aes_gcm_decrypt(key, blob[:12], blob[12:], aad)


def _pack(kid: str, ver: str, edk: bytes, body: bytes) -> bytes:
    k, v = kid.encode(), ver.encode()
    return MAGIC + bytes([len(k)]) + k + bytes([len(v)]) + v + struct.pack(">H", len(edk)) + \
        edk + body


def _unpack(blob: bytes):
    if blob[:3] != MAGIC:
        raise ValueError("not an omnia envelope")
    o = 3
    kl = blob[o]
    kid = blob[o + 1:o + 1 + kl].decode()
    o += 1 + kl
    vl = blob[o]
    ver = blob[o + 1:o + 1 + vl].decode()
    o += 1 + vl
    (el,) = struct.unpack(">H", blob[o:o + 2])
    edk = blob[o + 2:o + 2 + el]
    return kid, ver, edk, blob[o + 2 + el:]


class LocalKMS:
    """Versioned local KEKs (a key file or an in-memory ring)."""

    def __init__(self, key_id: str = "local", keys: dict[str, bytes] | None = None,
                 current: str | None = None, path: str | None = None):
        self.key_id = key_id
        self.path = path
        self._lock = threading.Lock()
        if path and os.path.exists(path):
            d = json.loads(open(path).read())
            keys = {v: base64.b64decode(k) for v, k in d["keys"].items()}
            current = d["current"]
        self.keys = dict(keys or {"1": os.urandom(32)})
        self.current = current or max(self.keys, key=int)
        self.created = {v: time.time() for v in self.keys}
        self._save()

    def _save(self):
        if self.path:
            tmp = self.path + ".tmp"
            with open(tmp, "w") as f:
                json.dump({"current": self.current,
                           "keys": {v: base64.b64encode(k).decode() for v, k in
                                    self.keys.items()}}, f)
            os.chmod(tmp, 0o600)
            os.replace(tmp, self.path)

    def encrypt(self, plaintext: bytes) -> EncryptOutput:
        dek = os.urandom(32)
        with self._lock:
            ver, kek = self.current, self.keys[self.current]
        aad = f"{self.key_id}:{ver}".encode()
        edk = seal(kek, dek, aad)
        body = seal(dek, plaintext)
        return EncryptOutput(_pack(self.key_id, ver, edk, body), self.key_id, ver)

    def decrypt(self, blob: bytes) -> bytes:
        kid, ver, edk, body = _unpack(blob)
        if kid != self.key_id:
            raise ValueError(f"envelope sealed under key {kid!r}, not {self.key_id!r}")
        kek = self.keys.get(ver)
        if kek is None:
            raise ValueError(f"unknown key version {ver}")
        dek = open_(kek, edk, f"{kid}:{ver}".encode())
        return open_(dek, body)

    def key_metadata(self) -> KeyMetadata:
        return KeyMetadata(self.key_id, self.current, created_at=self.created[self.current])

    def rotate(self) -> tuple[str, str]:
        with self._lock:
            prev = self.current
            nv = str(max(int(v) for v in self.keys) + 1)
            self.keys[nv] = os.urandom(32)
            self.created[nv] = time.time()
            self.current = nv
            self._save()
        return prev, nv

    def close(self):
        pass


class VaultTransitKMS:
    """DEK wrapping through Vault's transit engine (HTTP, token auth)."""

    def __init__(self, addr: str, key_name: str, token: str, mount: str = "transit",
                 timeout: float = 10.0):
        self.addr, self.key, self.token, self.mount = addr.rstrip("/"), key_name, token, mount
        self.timeout = timeout
        self.key_id = f"vault:{key_name}"

    def _call(self, path: str, body: dict | None = None) -> dict:
        import requests

        url = f"{self.addr}/v1/{self.mount}/{path}"
        h = {"X-Vault-Token": self.token}
        r = (requests.post(url, json=body, headers=h, timeout=self.timeout) if body is not None
             else requests.get(url, headers=h, timeout=self.timeout))
        if r.status_code >= 400:
            raise RuntimeError(f"vault {path}: HTTP {r.status_code} {r.text[:200]}")
        return r.json().get("data", {}) if r.text else {}

    def encrypt(self, plaintext: bytes) -> EncryptOutput:
        dek = os.urandom(32)
        d = self._call(f"encrypt/{self.key}", {"plaintext": base64.b64encode(dek).decode()})
        wrapped = d["ciphertext"]  # vault:v<N>:...
        ver = wrapped.split(":")[1].lstrip("v") if wrapped.startswith("vault:") else "1"
        return EncryptOutput(_pack(self.key_id, ver, wrapped.encode(), seal(dek, plaintext)),
                             self.key_id, ver)

    def decrypt(self, blob: bytes) -> bytes:
        _kid, _ver, edk, body = _unpack(blob)
        d = self._call(f"decrypt/{self.key}", {"ciphertext": edk.decode()})
        return open_(base64.b64decode(d["plaintext"]), body)

    def key_metadata(self) -> KeyMetadata:
        d = self._call(f"keys/{self.key}")
        return KeyMetadata(self.key_id, str(d.get("latest_version", 1)))

    def rotate(self) -> tuple[str, str]:
        prev = self.key_metadata().key_version
        self._call(f"keys/{self.key}/rotate", {})
        return prev, self.key_metadata().key_version

    def close(self):
        pass


def build_provider(cfg: dict):
    """``ProviderConfig``-shaped dict -> provider (``config.go``)."""
    t = (cfg.get("type") or cfg.get("providerType") or "local").lower()
    if t in ("local", "static"):
        return LocalKMS(cfg.get("keyID", "local"), path=cfg.get("keyFile"))
    if t in ("vault", "vault-transit", "vaulttransit"):
        return VaultTransitKMS(cfg["address"], cfg.get("keyName", "omnia"),
                               cfg.get("token") or os.environ.get("VAULT_TOKEN", ""),
                               cfg.get("mount", "transit"))
    if t in ("aws-kms", "awskms", "gcp-kms", "gcpkms", "azure-keyvault", "azurekeyvault"):
        raise ProviderUnavailable(f"{t} needs its vendor SDK, which is not installed")
    raise ValueError(f"unknown KMS provider type {t!r}")


@dataclass
class EncryptionEvent:
    field: str
    key_id: str
    key_version: str
    algorithm: str = ALGORITHM


class Encryptor:
    """Field-level encryption of session records."""

    def __init__(self, provider):
        self.p = provider

    def _enc(self, s: str) -> EncryptOutput:
        return self.p.encrypt(s.encode())

    def encrypt_message(self, msg: dict) -> tuple[dict, list[EncryptionEvent]]:
        """msg: {"content": str, "metadata": {str: str}, ...} -> encrypted copy."""
        out = dict(msg)
        meta = dict(msg.get("metadata") or {})
        events, fields, last = [], [], None
        if out.get("content"):
            o = self._enc(out["content"])
            out["content"] = base64.b64encode(o.ciphertext).decode()
            events.append(EncryptionEvent("content", o.key_id, o.key_version))
            fields.append("content")
            last = o
        for k, v in list(meta.items()):
            if k == META_KEY or not v:
                continue
            o = self._enc(str(v))
            meta[k] = base64.b64encode(o.ciphertext).decode()
            events.append(EncryptionEvent("metadata." + k, o.key_id, o.key_version))
            fields.append("metadata." + k)
            last = o
        if last is not None:
            meta[META_KEY] = json.dumps({"keyID": last.key_id, "keyVersion": last.key_version,
                                         "algorithm": last.algorithm, "fields": fields})
        out["metadata"] = meta
        return out, events

    def decrypt_message(self, msg: dict) -> dict:
        meta = dict(msg.get("metadata") or {})
        rec = meta.pop(META_KEY, None)
        if rec is None:
            return msg
        fields = json.loads(rec).get("fields", [])
        out = dict(msg)
        for f in fields:
            if f == "content":
                out["content"] = self.p.decrypt(base64.b64decode(out["content"])).decode()
            elif f.startswith("metadata."):
                k = f[len("metadata."):]
                meta[k] = self.p.decrypt(base64.b64decode(meta[k])).decode()
        out["metadata"] = meta
        return out

    def encrypt_envelope(self, value) -> dict:
        o = self.p.encrypt(json.dumps(value).encode())
        return {META_KEY: {"keyID": o.key_id, "keyVersion": o.key_version,
                           "algorithm": o.algorithm},
                PAYLOAD_KEY: base64.b64encode(o.ciphertext).decode()}

    @staticmethod
    def is_envelope(v) -> bool:
        return isinstance(v, dict) and META_KEY in v and PAYLOAD_KEY in v

    def decrypt_envelope(self, env: dict):
        return json.loads(self.p.decrypt(base64.b64decode(env[PAYLOAD_KEY])))

    def encrypt_tool_call(self, tc: dict) -> dict:
        out = dict(tc)
        for k in ("arguments", "result"):
            if out.get(k) not in (None, "", {}):
                out[k] = self.encrypt_envelope(out[k])
        if out.get("errorMessage"):
            out["errorMessage"] = json.dumps(self.encrypt_envelope(out["errorMessage"]))
        return out

    def decrypt_tool_call(self, tc: dict) -> dict:
        out = dict(tc)
        for k in ("arguments", "result"):
            if self.is_envelope(out.get(k)):
                out[k] = self.decrypt_envelope(out[k])
        em = out.get("errorMessage")
        if isinstance(em, str) and em.startswith("{"):
            try:
                env = json.loads(em)
                if self.is_envelope(env):
                    out["errorMessage"] = self.decrypt_envelope(env)
            except json.JSONDecodeError:
                pass
        return out


@dataclass
class ReEncryptor:
    """Re-wrap stored ciphertexts under the provider's current key version."""

    provider: object
    stats: dict = field(default_factory=lambda: {"scanned": 0, "rewrapped": 0, "skipped": 0})

    def rewrap(self, blob: bytes) -> bytes:
        self.stats["scanned"] += 1
        _kid, ver, _edk, _body = _unpack(blob)
        if ver == self.provider.key_metadata().key_version:
            self.stats["skipped"] += 1
            return blob
        out = self.provider.encrypt(self.provider.decrypt(blob)).ciphertext
        self.stats["rewrapped"] += 1
        return out

    def rewrap_b64(self, s: str) -> str:
        return base64.b64encode(self.rewrap(base64.b64decode(s))).decode()
