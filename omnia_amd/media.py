"""Media storage for multimodal turns (``internal/media``).

Storage references look like ``omnia://sessions/<session>/media/<id>``.

* :class:`LocalMediaStorage` -- proxy uploads through the facade
  (``/media/upload/<id>``), files under a root dir with JSON sidecars, TTL expiry,
  size cap and MIME allowlist (``local.go``).
* :class:`S3MediaStorage` / :class:`GCSMediaStorage` -- direct uploads to object
  storage with presigned URLs (AWS SigV4 query signing / GCS V4 HMAC signing;
  pure HMAC-SHA256, no SDK) and ``confirm-upload`` (``s3.go``, ``gcs.go``).
* :class:`AzureBlobMediaStorage` -- service SAS tokens (HMAC-SHA256) (``azure.go``).
* :func:`mount_media` -- the facade's HTTP routes (``handler.go:117-140``), plus the
  WebSocket hooks the facade calls: ``upload_url`` (``upload_request`` frames) and
  ``put_frame`` (binary OMNI media chunks assembled into one object).
"""
from __future__ import annotations

import base64
import datetime as dt
import hashlib
import hmac
import json
import time
import urllib.parse
import uuid
from dataclasses import asdict, dataclass, field
from pathlib import Path

REF_PREFIX = "omnia://"
DEFAULT_MAX_BYTES = 100 * 2**20
DEFAULT_TTL_S = 24 * 3600
DEFAULT_MIME = ("image/", "audio/", "video/", "application/pdf", "text/plain")


def make_ref(session_id: str, media_id: str) -> str:
    return f"{REF_PREFIX}sessions/{session_id}/media/{media_id}"


def parse_ref(ref: str) -> tuple[str, str]:
    if not ref.startswith(REF_PREFIX + "sessions/"):
        raise ValueError(f"bad storage ref {ref!r}")
    parts = ref[len(REF_PREFIX):].split("/")
    if len(parts) != 4 or parts[2] != "media" or not parts[1] or not parts[3]:
        raise ValueError(f"bad storage ref {ref!r}")
    if any(p in (".", "..") or "/" in p or "\\" in p for p in (parts[1], parts[3])):
        raise ValueError("path traversal in storage ref")
    return parts[1], parts[3]


@dataclass
class MediaInfo:
    storage_ref: str
    filename: str = ""
    mime_type: str = "application/octet-stream"
    size_bytes: int = 0
    created_at: float = field(default_factory=time.time)
    expires_at: float = 0.0

    def expired(self, now=None) -> bool:
        return bool(self.expires_at) and (now or time.time()) > self.expires_at


class MediaError(ValueError):
    pass


class _Base:
    def __init__(self, max_bytes: int = DEFAULT_MAX_BYTES, ttl_s: float = DEFAULT_TTL_S,
                 allowed_mime=DEFAULT_MIME):
        self.max_bytes, self.ttl_s, self.allowed = max_bytes, ttl_s, tuple(allowed_mime or ())
        self.pending: dict[str, dict] = {}
        self.frames: dict[str, dict] = {}

    def _check(self, req: dict):
        size = int(req.get("size_bytes") or 0)
        if size > self.max_bytes:
            raise MediaError(f"media larger than {self.max_bytes} bytes")
        mt = req.get("mime_type") or "application/octet-stream"
        if self.allowed and not any(mt.startswith(a) for a in self.allowed):
            raise MediaError(f"mime type {mt} not allowed")
        return size, mt


class LocalMediaStorage(_Base):
    proxy = True

    def __init__(self, root: str, base_url: str = "", **kw):
        super().__init__(**kw)
        self.root = Path(root)
        self.root.mkdir(parents=True, exist_ok=True)
        self.base_url = base_url.rstrip("/")

    def _path(self, ref: str) -> Path:
        sid, mid = parse_ref(ref)
        return self.root / "sessions" / sid / mid

    async def upload_url(self, session_id: str, req: dict) -> dict:
        size, mt = self._check(req)
        uid = uuid.uuid4().hex
        ref = make_ref(session_id, uid)
        self.pending[uid] = {"ref": ref, "filename": req.get("filename", ""), "mime": mt,
                             "size": size, "expires": time.time() + 900}
        return {"upload_id": uid, "url": f"{self.base_url}/media/upload/{uid}",
                "storage_ref": ref, "method": "PUT", "expires_at": time.time() + 900,
                "headers": {"Content-Type": mt}}

    def write_upload(self, upload_id: str, data: bytes) -> MediaInfo:
        p = self.pending.pop(upload_id, None)
        if p is None or p["expires"] < time.time():
            raise MediaError("unknown or expired upload id")
        if len(data) > self.max_bytes:
            raise MediaError("upload exceeds size cap")
        return self._store(p["ref"], data, p["filename"], p["mime"])

    def _store(self, ref, data, filename, mime) -> MediaInfo:
        path = self._path(ref)
        path.parent.mkdir(parents=True, exist_ok=True)
        path.write_bytes(data)
        info = MediaInfo(ref, filename, mime, len(data),
                         expires_at=time.time() + self.ttl_s if self.ttl_s else 0.0)
        path.with_suffix(".json").write_text(json.dumps(asdict(info)))
        return info

    async def info(self, ref: str) -> MediaInfo:
        p = self._path(ref).with_suffix(".json")
        if not p.exists():
            raise FileNotFoundError(ref)
        info = MediaInfo(**json.loads(p.read_text()))
        if info.expired():
            await self.delete(ref)
            raise FileNotFoundError(ref)
        return info

    async def read(self, ref: str) -> bytes:
        await self.info(ref)
        return self._path(ref).read_bytes()

    async def download_url(self, ref: str) -> str:
        sid, mid = parse_ref(ref)
        return f"{self.base_url}/media/download/{sid}/{mid}"

    async def delete(self, ref: str):
        p = self._path(ref)
        for q in (p, p.with_suffix(".json")):
            if q.exists():
                q.unlink()

    def sweep(self) -> int:
        """Delete expired media (TTL)."""
        n = 0
        for j in self.root.glob("sessions/*/*.json"):
            try:
                info = MediaInfo(**json.loads(j.read_text()))
            except (ValueError, TypeError):
                continue
            if info.expired():
                j.with_suffix("").unlink(missing_ok=True)
                j.unlink(missing_ok=True)
                n += 1
        return n

    async def put_frame(self, session_id: str, frame: dict) -> dict | None:
        """Assemble binary OMNI media frames (``facade/protocol.py``): chunks of one
        ``media_id`` arrive with increasing ``seq``; FLAG_LAST (or an unchunked
        frame) completes the object."""
        from .facade.protocol import FLAG_CHUNKED, FLAG_LAST

        meta = frame.get("meta") or {}
        payload = frame.get("payload", b"")
        mid_b = frame.get("media_id") or b""
        mid = (mid_b.decode(errors="ignore") if isinstance(mid_b, bytes) else str(mid_b)) or \
            meta.get("media_id") or uuid.uuid4().hex
        if any(c in mid for c in "/\\") or mid in (".", ".."):
            raise MediaError("bad media id")
        key = f"{session_id}/{mid}"
        st = self.frames.setdefault(key, {"chunks": {}, "size": 0, "meta": meta})
        st["chunks"][int(frame.get("seq", len(st["chunks"])))] = payload
        st["size"] += len(payload)
        if st["size"] > self.max_bytes:
            self.frames.pop(key, None)
            raise MediaError("media stream exceeds size cap")
        flags = int(frame.get("flags", 0))
        if flags & FLAG_CHUNKED and not flags & FLAG_LAST:
            return None
        self.frames.pop(key, None)
        data = b"".join(st["chunks"][k] for k in sorted(st["chunks"]))
        m = {**st["meta"], **meta}
        info = self._store(make_ref(session_id, mid), data, m.get("filename", ""),
                           m.get("mime_type", "application/octet-stream"))
        return {"storage_ref": info.storage_ref, "size_bytes": info.size_bytes,
                "mime_type": info.mime_type}


# ------------------------------------------------------------------ signing helpers
def _hmac(key: bytes, msg: str) -> bytes:
    return hmac.new(key, msg.encode(), hashlib.sha256).digest()


def sigv4_presign(method: str, host: str, path: str, region: str, service: str,
                  access_key: str, secret_key: str, expires_s: int = 900, now=None,
                  algo: str = "AWS4-HMAC-SHA256", prefix: str = "AWS4",
                  req_type: str = "aws4_request", header_prefix: str = "X-Amz",
                  scheme: str = "https") -> str:
    """Query-string presigned URL (AWS SigV4; GCS V4 HMAC uses the same scheme with
    the ``GOOG4`` names)."""
    t = now or dt.datetime.now(dt.timezone.utc)
    amz_date, datestamp = t.strftime("%Y%m%dT%H%M%SZ"), t.strftime("%Y%m%d")
    scope = f"{datestamp}/{region}/{service}/{req_type}"
    q = {f"{header_prefix}-Algorithm": algo,
         f"{header_prefix}-Credential": f"{access_key}/{scope}",
         f"{header_prefix}-Date": amz_date, f"{header_prefix}-Expires": str(expires_s),
         f"{header_prefix}-SignedHeaders": "host"}
    canon_q = "&".join(f"{urllib.parse.quote(k, safe='-_.~')}="
                       f"{urllib.parse.quote(v, safe='-_.~')}" for k, v in sorted(q.items()))
    canon_path = urllib.parse.quote(path, safe="/-_.~")
    creq = "\n".join([method, canon_path, canon_q, f"host:{host}\n", "host",
                      "UNSIGNED-PAYLOAD"])
    sts = "\n".join([algo, amz_date, scope, hashlib.sha256(creq.encode()).hexdigest()])
    k = _hmac((prefix + secret_key).encode(), datestamp)
    k = _hmac(k, region)
    k = _hmac(k, service)
    k = _hmac(k, req_type)
    sig = hmac.new(k, sts.encode(), hashlib.sha256).hexdigest()
    return f"{scheme}://{host}{canon_path}?{canon_q}&{header_prefix}-Signature={sig}"


class S3MediaStorage(_Base):
    proxy = False

    def __init__(self, bucket: str, region: str, access_key: str, secret_key: str,
                 endpoint: str = "", prefix: str = "omnia", **kw):
        super().__init__(**kw)
        self.bucket, self.region = bucket, region
        self.ak, self.sk = access_key, secret_key
        self.host = endpoint or f"{bucket}.s3.{region}.amazonaws.com"
        self.prefix = prefix
        self.index: dict[str, MediaInfo] = {}

    def _key(self, ref):
        sid, mid = parse_ref(ref)
        return f"/{self.prefix}/sessions/{sid}/{mid}"

    def _sign(self, method, ref, expires=900):
        return sigv4_presign(method, self.host, self._key(ref), self.region, "s3", self.ak,
                             self.sk, expires)

    async def upload_url(self, session_id: str, req: dict) -> dict:
        size, mt = self._check(req)
        uid = uuid.uuid4().hex
        ref = make_ref(session_id, uid)
        self.pending[uid] = {"ref": ref, "filename": req.get("filename", ""), "mime": mt,
                             "size": size}
        return {"upload_id": uid, "url": self._sign("PUT", ref), "storage_ref": ref,
                "method": "PUT", "expires_at": time.time() + 900}

    async def confirm(self, upload_id: str) -> MediaInfo:
        p = self.pending.pop(upload_id, None)
        if p is None:
            raise MediaError("unknown upload id")
        info = MediaInfo(p["ref"], p["filename"], p["mime"], p["size"],
                         expires_at=time.time() + self.ttl_s if self.ttl_s else 0.0)
        self.index[p["ref"]] = info
        return info

    async def info(self, ref):
        if ref not in self.index:
            raise FileNotFoundError(ref)
        return self.index[ref]

    async def download_url(self, ref: str) -> str:
        return self._sign("GET", ref)

    async def delete(self, ref):
        self.index.pop(ref, None)

    async def put_frame(self, session_id, frame):
        raise MediaError("streamed media frames need proxy (local) storage")


class GCSMediaStorage(S3MediaStorage):
    """GCS XML API with HMAC interoperability keys (V4 ``GOOG4-HMAC-SHA256``)."""

    def __init__(self, bucket: str, access_id: str, secret: str, **kw):
        super().__init__(bucket, "auto", access_id, secret,
                         endpoint="storage.googleapis.com", **kw)

    def _key(self, ref):
        return f"/{self.bucket}" + super()._key(ref)

    def _sign(self, method, ref, expires=900):
        return sigv4_presign(method, self.host, self._key(ref), "auto", "storage", self.ak,
                             self.sk, expires, algo="GOOG4-HMAC-SHA256", prefix="GOOG4",
                             req_type="goog4_request", header_prefix="X-Goog")


class AzureBlobMediaStorage(S3MediaStorage):
    """Azure Blob service SAS (HMAC-SHA256 over the string-to-sign, sv=2020-12-06)."""

    def __init__(self, account: str, container: str, account_key_b64: str, **kw):
        super().__init__(container, "", account, account_key_b64,
                         endpoint=f"{account}.blob.core.windows.net", **kw)
        self.account, self.container = account, container
        self.key = base64.b64decode(account_key_b64)

    def _sign(self, method, ref, expires=900):
        sid, mid = parse_ref(ref)
        blob = f"{self.prefix}/sessions/{sid}/{mid}"
        perms = "cw" if method == "PUT" else "r"
        se = (dt.datetime.now(dt.timezone.utc) + dt.timedelta(seconds=expires)).strftime(
            "%Y-%m-%dT%H:%M:%SZ")
        sv = "2020-12-06"
        canon = f"/blob/{self.account}/{self.container}/{blob}"
        sts = "\n".join([perms, "", se, canon, "", "", "https", sv, "b", "", "", "", "", "",
                         "", ""])
        sig = base64.b64encode(hmac.new(self.key, sts.encode(), hashlib.sha256).digest())
        q = urllib.parse.urlencode({"sp": perms, "se": se, "spr": "https", "sv": sv,
                                    "sr": "b", "sig": sig.decode()})
        return f"https://{self.host}/{self.container}/{blob}?{q}"


def build_media_storage(env: dict):
    """``internal/media/env.go``: OMNIA_MEDIA_STORAGE=local|s3|gcs|azure."""
    kind = (env.get("OMNIA_MEDIA_STORAGE") or "").lower()
    kw = {"max_bytes": int(env.get("OMNIA_MEDIA_MAX_BYTES", DEFAULT_MAX_BYTES)),
          "ttl_s": float(env.get("OMNIA_MEDIA_TTL_S", DEFAULT_TTL_S))}
    if kind == "local":
        return LocalMediaStorage(env.get("OMNIA_MEDIA_ROOT", "/var/lib/omnia/media"),
                                 env.get("OMNIA_MEDIA_BASE_URL", ""), **kw)
    if kind == "s3":
        return S3MediaStorage(env["OMNIA_MEDIA_BUCKET"], env.get("AWS_REGION", "us-east-1"),
                              env.get("AWS_ACCESS_KEY_ID", ""),
                              env.get("AWS_SECRET_ACCESS_KEY", ""),
                              env.get("OMNIA_MEDIA_ENDPOINT", ""), **kw)
    if kind == "gcs":
        return GCSMediaStorage(env["OMNIA_MEDIA_BUCKET"], env.get("GCS_HMAC_ACCESS_ID", ""),
                               env.get("GCS_HMAC_SECRET", ""), **kw)
    if kind == "azure":
        return AzureBlobMediaStorage(env["AZURE_STORAGE_ACCOUNT"], env["OMNIA_MEDIA_BUCKET"],
                                     env["AZURE_STORAGE_KEY"], **kw)
    return None


def mount_media(app, storage):
    """HTTP routes on the facade app (aiohttp)."""
    from aiohttp import web

    async def request_upload(request):
        d = await request.json()
        try:
            return web.json_response(await storage.upload_url(d.get("session_id", ""), d))
        except MediaError as e:
            return web.json_response({"error": str(e)}, status=400)

    async def upload(request):
        if not getattr(storage, "proxy", False):
            return web.json_response({"error": "direct-upload storage"}, status=400)
        data = await request.read()
        try:
            info = storage.write_upload(request.match_info["id"], data)
        except MediaError as e:
            return web.json_response({"error": str(e)}, status=400)
        return web.json_response(asdict(info), status=201)

    async def confirm(request):
        try:
            info = await storage.confirm(request.match_info["id"])
        except MediaError as e:
            return web.json_response({"error": str(e)}, status=400)
        return web.json_response(asdict(info))

    async def download(request):
        ref = make_ref(request.match_info["sid"], request.match_info["mid"])
        try:
            info = await storage.info(ref)
        except (FileNotFoundError, ValueError):
            return web.json_response({"error": "not found"}, status=404)
        if getattr(storage, "proxy", False):
            return web.Response(body=await storage.read(ref), content_type=info.mime_type)
        raise web.HTTPFound(await storage.download_url(ref))

    async def info(request):
        ref = make_ref(request.match_info["sid"], request.match_info["mid"])
        try:
            return web.json_response(asdict(await storage.info(ref)))
        except (FileNotFoundError, ValueError):
            return web.json_response({"error": "not found"}, status=404)

    app.router.add_post("/media/request-upload", request_upload)
    app.router.add_put("/media/upload/{id}", upload)
    app.router.add_post("/media/upload/{id}", upload)
    app.router.add_post("/media/confirm-upload/{id}", confirm)
    app.router.add_get("/media/download/{sid}/{mid}", download)
    app.router.add_get("/media/info/{sid}/{mid}", info)
    return app


