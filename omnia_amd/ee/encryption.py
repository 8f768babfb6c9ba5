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
        self._mtime = 0.0
        if path and os.path.exists(path):
            keys, current = self._read()
        self.keys = dict(keys or {"1": os.urandom(32)})
        self.current = current or max(self.keys, key=int)
        self.created = {v: time.time() for v in self.keys}
        self._save()

    def _read(self):
        with open(self.path) as f:
            d = json.loads(f.read())
        self._mtime = os.stat(self.path).st_mtime
        return {v: base64.b64decode(k) for v, k in d["keys"].items()}, d["current"]

    def _maybe_reload(self):
        """Another process (the key-rotation controller) rotated the shared key
        file: pick up the new current version and keep every old one."""
        if not self.path or not os.path.exists(self.path):
            return
        if os.stat(self.path).st_mtime == self._mtime:
            return
        with self._lock:
            keys, current = self._read()
            for v in keys:
                self.created.setdefault(v, time.time())
            self.keys.update(keys)
            self.current = current

    def _save(self):
        if self.path:
            tmp = self.path + ".tmp"
            with open(tmp, "w") as f:
                json.dump({"current": self.current,
                           "keys": {v: base64.b64encode(k).decode() for v, k in
                                    self.keys.items()}}, f)
            os.chmod(tmp, 0o600)
            os.replace(tmp, self.path)
            self._mtime = os.stat(self.path).st_mtime

    def encrypt(self, plaintext: bytes) -> EncryptOutput:
        self._maybe_reload()
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
            self._maybe_reload()
            kek = self.keys.get(ver)
        if kek is None:
            raise ValueError(f"unknown key version {ver}")
        dek = open_(kek, edk, f"{kid}:{ver}".encode())
        return open_(dek, body)

    def key_metadata(self) -> KeyMetadata:
        self._maybe_reload()
        return KeyMetadata(self.key_id, self.current, created_at=self.created[self.current])

    def rotate(self) -> tuple[str, str]:
        self._maybe_reload()
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


# ------------------------------------------------------------------ cloud KMS (REST, no SDKs)
def sigv4_headers(method: str, url: str, body: bytes, region: str, service: str,
                  access_key: str, secret_key: str, session_token: str = "",
                  extra: dict | None = None, now=None) -> dict:
    """AWS Signature V4 Authorization header for a request (header form)."""
    import datetime as dt
    import hashlib
    import hmac
    import urllib.parse

    u = urllib.parse.urlsplit(url)
    t = now or dt.datetime.now(dt.timezone.utc)
    amz_date, day = t.strftime("%Y%m%dT%H%M%SZ"), t.strftime("%Y%m%d")
    hdrs = {"host": u.netloc, "x-amz-date": amz_date, **{k.lower(): v for k, v in
                                                         (extra or {}).items()}}
    if session_token:
        hdrs["x-amz-security-token"] = session_token
    signed = ";".join(sorted(hdrs))
    canon_h = "".join(f"{k}:{hdrs[k].strip()}\n" for k in sorted(hdrs))
    creq = "\n".join([method, u.path or "/", u.query, canon_h, signed,
                      hashlib.sha256(body).hexdigest()])
    scope = f"{day}/{region}/{service}/aws4_request"
    sts = "\n".join(["AWS4-HMAC-SHA256", amz_date, scope,
                     hashlib.sha256(creq.encode()).hexdigest()])

    def h(k, m):
        return hmac.new(k, m.encode(), hashlib.sha256).digest()

    k = h(h(h(h(("AWS4" + secret_key).encode(), day), region), service), "aws4_request")
    sig = hmac.new(k, sts.encode(), hashlib.sha256).hexdigest()
    out = {k2: v for k2, v in hdrs.items() if k2 != "host"}
    out["Authorization"] = (f"AWS4-HMAC-SHA256 Credential={access_key}/{scope}, "
                            f"SignedHeaders={signed}, Signature={sig}")
    return out


class _WrappingKMS:
    """Common envelope logic: a fresh DEK per record, wrapped by the cloud key."""

    key_id = "kms"

    def _wrap(self, dek: bytes) -> tuple[bytes, str]:  # pragma: no cover - interface
        raise NotImplementedError

    def _unwrap(self, edk: bytes) -> bytes:  # pragma: no cover - interface
        raise NotImplementedError

    def encrypt(self, plaintext: bytes) -> EncryptOutput:
        dek = os.urandom(32)
        edk, ver = self._wrap(dek)
        return EncryptOutput(_pack(self.key_id, ver, edk, seal(dek, plaintext)), self.key_id,
                             ver)

    def decrypt(self, blob: bytes) -> bytes:
        kid, _ver, edk, body = _unpack(blob)
        if kid != self.key_id:
            raise ValueError(f"envelope sealed under key {kid!r}, not {self.key_id!r}")
        return open_(self._unwrap(edk), body)

    def close(self):
        pass

    @staticmethod
    def _post(url: str, body: dict, headers: dict, timeout: float = 10.0) -> dict:
        import requests

        r = requests.post(url, data=json.dumps(body).encode(), headers=headers, timeout=timeout)
        if r.status_code >= 400:
            raise RuntimeError(f"KMS {url}: HTTP {r.status_code} {r.text[:200]}")
        return r.json() if r.text else {}


class AWSKMS(_WrappingKMS):
    """AWS KMS ``TrentService`` JSON API (Encrypt / Decrypt / DescribeKey /
    RotateKeyOnDemand), SigV4-signed; credentials from the env like the SDK."""

    def __init__(self, key_id: str, region: str, access_key: str = "", secret_key: str = "",
                 session_token: str = "", endpoint: str = ""):
        self.arn, self.region = key_id, region
        self.ak = access_key or os.environ.get("AWS_ACCESS_KEY_ID", "")
        self.sk = secret_key or os.environ.get("AWS_SECRET_ACCESS_KEY", "")
        self.st = session_token or os.environ.get("AWS_SESSION_TOKEN", "")
        self.url = endpoint or f"https://kms.{region}.amazonaws.com/"
        self.key_id = f"aws-kms:{key_id}"

    def _call(self, op: str, body: dict) -> dict:
        raw = json.dumps(body).encode()
        extra = {"content-type": "application/x-amz-json-1.1",
                 "x-amz-target": f"TrentService.{op}"}
        h = sigv4_headers("POST", self.url, raw, self.region, "kms", self.ak, self.sk, self.st,
                          extra)
        h.update({"Content-Type": extra["content-type"], "X-Amz-Target": extra["x-amz-target"]})
        return self._post(self.url, body, h)

    def _wrap(self, dek):
        d = self._call("Encrypt", {"KeyId": self.arn, "Plaintext": base64.b64encode(dek).decode()})
        return base64.b64decode(d["CiphertextBlob"]), "aws"

    def _unwrap(self, edk):
        d = self._call("Decrypt", {"KeyId": self.arn,
                                   "CiphertextBlob": base64.b64encode(edk).decode()})
        return base64.b64decode(d["Plaintext"])

    def key_metadata(self) -> KeyMetadata:
        d = self._call("DescribeKey", {"KeyId": self.arn}).get("KeyMetadata", {})
        return KeyMetadata(self.key_id, "aws", created_at=float(d.get("CreationDate") or 0))

    def rotate(self) -> tuple[str, str]:
        self._call("RotateKeyOnDemand", {"KeyId": self.arn})
        return "aws", "aws"  # AWS keeps backing-key versions internal; blobs self-describe


class GCPKMS(_WrappingKMS):
    """Cloud KMS REST (``:encrypt`` / ``:decrypt`` on a CryptoKey); OAuth bearer
    from ``GOOGLE_OAUTH_ACCESS_TOKEN`` or the metadata server."""

    def __init__(self, key_name: str, token: str = "",
                 endpoint: str = "https://cloudkms.googleapis.com"):
        self.name, self.base = key_name, endpoint.rstrip("/")
        self.token = token
        self.key_id = f"gcp-kms:{key_name.rsplit('/', 1)[-1]}"

    def _bearer(self) -> str:
        if self.token or os.environ.get("GOOGLE_OAUTH_ACCESS_TOKEN"):
            return self.token or os.environ["GOOGLE_OAUTH_ACCESS_TOKEN"]
        import requests

        r = requests.get("http://metadata.google.internal/computeMetadata/v1/instance/"
                         "service-accounts/default/token", headers={"Metadata-Flavor": "Google"},
                         timeout=5)
        r.raise_for_status()
        return r.json()["access_token"]

    def _call(self, verb: str, body: dict) -> dict:
        return self._post(f"{self.base}/v1/{self.name}:{verb}", body,
                          {"Authorization": f"Bearer {self._bearer()}",
                           "Content-Type": "application/json"})

    def _wrap(self, dek):
        d = self._call("encrypt", {"plaintext": base64.b64encode(dek).decode()})
        return base64.b64decode(d["ciphertext"]), d.get("name", "").rsplit("/", 1)[-1] or "1"

    def _unwrap(self, edk):
        d = self._call("decrypt", {"ciphertext": base64.b64encode(edk).decode()})
        return base64.b64decode(d["plaintext"])

    def key_metadata(self) -> KeyMetadata:
        return KeyMetadata(self.key_id, "primary")

    def rotate(self) -> tuple[str, str]:
        return "primary", "primary"  # rotation is a CryptoKey schedule on the GCP side


class AzureKeyVaultKMS(_WrappingKMS):
    """Key Vault ``wrapkey`` / ``unwrapkey`` (RSA-OAEP-256) REST; bearer from
    ``AZURE_ACCESS_TOKEN`` or the instance metadata service (workload identity)."""

    def __init__(self, vault_url: str, key_name: str, key_version: str = "", token: str = "",
                 api_version: str = "7.4"):
        self.vault, self.name, self.ver = vault_url.rstrip("/"), key_name, key_version
        self.token, self.api = token, api_version
        self.key_id = f"azure-kv:{key_name}"

    def _bearer(self) -> str:
        if self.token or os.environ.get("AZURE_ACCESS_TOKEN"):
            return self.token or os.environ["AZURE_ACCESS_TOKEN"]
        import requests

        r = requests.get("http://169.254.169.254/metadata/identity/oauth2/token",
                         params={"api-version": "2018-02-01",
                                 "resource": "https://vault.azure.net"},
                         headers={"Metadata": "true"}, timeout=5)
        r.raise_for_status()
        return r.json()["access_token"]

    def _call(self, path: str, body: dict) -> dict:
        return self._post(f"{self.vault}/keys/{path}?api-version={self.api}", body,
                          {"Authorization": f"Bearer {self._bearer()}",
                           "Content-Type": "application/json"})

    def _wrap(self, dek):
        path = f"{self.name}/{self.ver}/wrapkey" if self.ver else f"{self.name}/wrapkey"
        d = self._call(path, {"alg": "RSA-OAEP-256", "value": base64.urlsafe_b64encode(
            dek).rstrip(b"=").decode()})
        kver = d.get("kid", "").rstrip("/").rsplit("/", 1)[-1] or self.ver or "current"
        return (kver.encode() + b"|" + base64.urlsafe_b64decode(d["value"] + "=" * (
            -len(d["value"]) % 4))), kver

    def _unwrap(self, edk):
        kver, wrapped = edk.split(b"|", 1)
        d = self._call(f"{self.name}/{kver.decode()}/unwrapkey",
                       {"alg": "RSA-OAEP-256",
                        "value": base64.urlsafe_b64encode(wrapped).rstrip(b"=").decode()})
        return base64.urlsafe_b64decode(d["value"] + "=" * (-len(d["value"]) % 4))

    def key_metadata(self) -> KeyMetadata:
        return KeyMetadata(self.key_id, self.ver or "current")

    def rotate(self) -> tuple[str, str]:
        return self.ver or "current", self.ver or "current"  # versions are created in Azure


def build_provider(cfg: dict):
    """``ProviderConfig``-shaped dict -> provider (``config.go``)."""
    t = (cfg.get("type") or cfg.get("providerType") or "local").lower()
    if t in ("local", "static"):
        return LocalKMS(cfg.get("keyID", "local"), path=cfg.get("keyFile"))
    if t in ("vault", "vault-transit", "vaulttransit"):
        return VaultTransitKMS(cfg["address"], cfg.get("keyName", "omnia"),
                               cfg.get("token") or os.environ.get("VAULT_TOKEN", ""),
                               cfg.get("mount", "transit"))
    if t in ("aws-kms", "awskms"):
        return AWSKMS(cfg["keyID"], cfg.get("region", os.environ.get("AWS_REGION", "us-east-1")),
                      endpoint=cfg.get("endpoint", ""))
    if t in ("gcp-kms", "gcpkms"):
        return GCPKMS(cfg["keyID"], endpoint=cfg.get("endpoint",
                                                     "https://cloudkms.googleapis.com"))
    if t in ("azure-keyvault", "azurekeyvault"):
        return AzureKeyVaultKMS(cfg["vaultURL"], cfg.get("keyName") or cfg["keyID"],
                                cfg.get("keyVersion", ""))
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
