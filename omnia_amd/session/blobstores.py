"""Cold-tier object stores: S3 (and S3-compatible), GCS and Azure Blob, over
their REST APIs with request signing done here.

Reference: ``internal/session/providers/cold/blobstore.go`` (Put / Get / Delete
/ List / Exists / Ping), ``blobstore_s3.go`` (region, custom endpoint, path
style for MinIO, static keys), ``blobstore_gcs.go`` (service-account JSON),
``blobstore_azure.go`` (account name + shared key), ``config.go`` (prefix
``sessions/``), wiring ``cmd/session-api/main.go:809-830`` (``--cold-backend``,
``--cold-bucket``, ``--cold-region``, ``--cold-endpoint``).  The reference
links the vendor SDKs; none are importable here, so each store speaks the
service's HTTP API directly with the standard library:

* S3: SigV4 header signing (``AWS4-HMAC-SHA256``, ``x-amz-content-sha256``),
  virtual-host or path-style URLs, ListObjectsV2 pagination;
* GCS: the JSON API with an OAuth2 access token minted from the service
  account key (RS256 JWT bearer grant, :mod:`omnia_amd.utils.rsa`), or the XML
  API with HMAC interoperability keys (SigV4 under the ``GOOG4`` names), or no
  auth against an emulator (``STORAGE_EMULATOR_HOST``);
* Azure: Shared Key authorization (``SharedKey account:sig`` over the Blob
  service string-to-sign), BlockBlob puts, marker-paginated container listing;
  an emulator endpoint uses the path-style ``/<account>/<container>`` layout.

The stores are synchronous (the cold archive runs off the request path) and
the object interface matches :class:`omnia_amd.session.store.LocalBlobStore`,
so :class:`~omnia_amd.session.store.ColdArchive` works on any of them.
"""
from __future__ import annotations

import base64
import datetime as dt
import hashlib
import hmac
import json
import os
import time
import urllib.error
import urllib.parse
import urllib.request
import xml.etree.ElementTree as ET

EMPTY_SHA256 = hashlib.sha256(b"").hexdigest()


class BlobError(RuntimeError):
    def __init__(self, msg: str, status: int = 0):
        super().__init__(msg)
        self.status = status


def _http(method: str, url: str, headers: dict, body: bytes | None, timeout: float):
    req = urllib.request.Request(url, data=body, method=method, headers=headers)
    try:
        with urllib.request.urlopen(req, timeout=timeout) as r:  # noqa: S310 - configured URL
            return r.status, dict(r.headers), r.read()
    except urllib.error.HTTPError as e:
        return e.code, dict(e.headers or {}), e.read()
    except (urllib.error.URLError, OSError) as e:
        raise BlobError(f"{method} {url}: {e}") from e


def _uri_encode(s: str, safe: str = "-_.~") -> str:
    return urllib.parse.quote(s, safe=safe)


# ------------------------------------------------------------------ SigV4
def sigv4_authorization(method: str, url: str, headers: dict, payload_hash: str, region: str,
                        service: str, access_key: str, secret_key: str, now=None,
                        algo: str = "AWS4-HMAC-SHA256", prefix: str = "AWS4",
                        req_type: str = "aws4_request", date_header: str = "x-amz-date") -> dict:
    """Sign a request in place (SigV4, Authorization header form).  ``headers``
    gains ``host`` and the date header; returns it."""
    t = now or dt.datetime.now(dt.timezone.utc)
    amz_date, datestamp = t.strftime("%Y%m%dT%H%M%SZ"), t.strftime("%Y%m%d")
    u = urllib.parse.urlsplit(url)
    headers.setdefault("host", u.netloc)
    headers[date_header] = amz_date
    canon_uri = _uri_encode(urllib.parse.unquote(u.path) or "/", safe="/-_.~")
    pairs = urllib.parse.parse_qsl(u.query, keep_blank_values=True)
    canon_q = "&".join(f"{_uri_encode(k)}={_uri_encode(v)}" for k, v in sorted(pairs))
    lower = {k.lower(): " ".join(str(v).strip().split()) for k, v in headers.items()}
    signed = ";".join(sorted(lower))
    canon_h = "".join(f"{k}:{lower[k]}\n" for k in sorted(lower))
    creq = "\n".join([method, canon_uri, canon_q, canon_h, signed, payload_hash])
    scope = f"{datestamp}/{region}/{service}/{req_type}"
    sts = "\n".join([algo, amz_date, scope, hashlib.sha256(creq.encode()).hexdigest()])
    k = hmac.new((prefix + secret_key).encode(), datestamp.encode(), hashlib.sha256).digest()
    for part in (region, service, req_type):
        k = hmac.new(k, part.encode(), hashlib.sha256).digest()
    sig = hmac.new(k, sts.encode(), hashlib.sha256).hexdigest()
    headers["Authorization"] = (f"{algo} Credential={access_key}/{scope}, "
                                f"SignedHeaders={signed}, Signature={sig}")
    return headers


class _Base:
    def __init__(self, prefix: str = "sessions/", timeout: float = 30.0):
        self.prefix = prefix
        self.timeout = timeout

    def _k(self, key: str) -> str:
        return self.prefix + key

    def _unk(self, key: str) -> str:
        return key[len(self.prefix):] if key.startswith(self.prefix) else key


# ------------------------------------------------------------------ S3
class S3BlobStore(_Base):
    service = "s3"
    algo, key_prefix, req_type, date_header = "AWS4-HMAC-SHA256", "AWS4", "aws4_request", \
        "x-amz-date"
    hash_header = "x-amz-content-sha256"
    token_header = "x-amz-security-token"

    def __init__(self, bucket: str, region: str = "us-east-1", endpoint: str = "",
                 access_key: str = "", secret_key: str = "", session_token: str = "",
                 use_path_style: bool = False, prefix: str = "sessions/", timeout: float = 30.0):
        super().__init__(prefix, timeout)
        self.bucket, self.region = bucket, region or "us-east-1"
        self.ak, self.sk, self.token = access_key, secret_key, session_token
        self.path_style = use_path_style
        if endpoint and "://" not in endpoint:
            endpoint = "https://" + endpoint
        self.endpoint = endpoint.rstrip("/")

    def _base(self) -> str:
        if self.endpoint:
            if self.path_style:
                return f"{self.endpoint}/{self.bucket}"
            u = urllib.parse.urlsplit(self.endpoint)
            return f"{u.scheme}://{self.bucket}.{u.netloc}"
        return f"https://{self.bucket}.s3.{self.region}.amazonaws.com"

    def _url(self, key: str = "", query: dict | None = None) -> str:
        u = self._base() + "/" + _uri_encode(key, safe="/-_.~")
        if query:
            u += "?" + urllib.parse.urlencode(sorted(query.items()), quote_via=urllib.parse.quote)
        return u

    def _req(self, method: str, url: str, body: bytes = b"", extra: dict | None = None):
        headers = dict(extra or {})
        ph = hashlib.sha256(body).hexdigest() if body else EMPTY_SHA256
        if self.hash_header:
            headers[self.hash_header] = ph
        if self.token:
            headers[self.token_header] = self.token
        if self.ak and self.sk:
            sigv4_authorization(method, url, headers, ph, self.region, self.service, self.ak,
                                self.sk, algo=self.algo, prefix=self.key_prefix,
                                req_type=self.req_type, date_header=self.date_header)
        return _http(method, url, headers, body if method in ("PUT", "POST") else None,
                     self.timeout)

    def put(self, key: str, data: bytes, content_type: str = "application/octet-stream"):
        st, _, body = self._req("PUT", self._url(self._k(key)), bytes(data),
                                {"Content-Type": content_type})
        if st >= 300:
            raise BlobError(f"put {key}: HTTP {st} {body[:200]!r}", st)

    def get(self, key: str) -> bytes | None:
        st, _, body = self._req("GET", self._url(self._k(key)))
        if st == 404:
            return None
        if st >= 300:
            raise BlobError(f"get {key}: HTTP {st}", st)
        return body

    def delete(self, key: str):
        st, _, _ = self._req("DELETE", self._url(self._k(key)))
        if st >= 300 and st != 404:
            raise BlobError(f"delete {key}: HTTP {st}", st)

    def exists(self, key: str) -> bool:
        st, _, _ = self._req("HEAD", self._url(self._k(key)))
        if st >= 300 and st != 404:
            raise BlobError(f"head {key}: HTTP {st}", st)
        return st < 300

    def list(self, prefix: str = "") -> list[str]:
        out, token = [], None
        while True:
            q = {"list-type": "2", "prefix": self._k(prefix)}
            if token:
                q["continuation-token"] = token
            st, _, body = self._req("GET", self._url("", q))
            if st >= 300:
                raise BlobError(f"list {prefix}: HTTP {st}", st)
            root = ET.fromstring(body)
            ns = root.tag[:root.tag.index("}") + 1] if root.tag.startswith("{") else ""
            out += [self._unk(c.findtext(f"{ns}Key")) for c in root.iter(f"{ns}Contents")]
            if (root.findtext(f"{ns}IsTruncated") or "false").lower() != "true":
                return sorted(out)
            token = root.findtext(f"{ns}NextContinuationToken")

    def ping(self):
        st, _, _ = self._req("HEAD", self._url(""))
        if st >= 300:
            raise BlobError(f"bucket {self.bucket}: HTTP {st}", st)


class GCSHMACBlobStore(S3BlobStore):
    """GCS XML API with HMAC interoperability keys (SigV4 under GOOG4 names)."""
    service = "storage"
    algo, key_prefix, req_type, date_header = "GOOG4-HMAC-SHA256", "GOOG4", "goog4_request", \
        "x-goog-date"
    hash_header = "x-goog-content-sha256"

    def __init__(self, bucket: str, access_id: str, secret: str,
                 endpoint: str = "https://storage.googleapis.com", **kw):
        super().__init__(bucket, "auto", endpoint, access_id, secret, use_path_style=True, **kw)


# ------------------------------------------------------------------ GCS (JSON API)
GCS_SCOPE = "https://www.googleapis.com/auth/devstorage.read_write"


class GCSBlobStore(_Base):
    def __init__(self, bucket: str, credentials: dict | None = None,
                 endpoint: str = "https://storage.googleapis.com", prefix: str = "sessions/",
                 timeout: float = 30.0, clock=time.time):
        super().__init__(prefix, timeout)
        self.bucket = bucket
        self.creds = credentials
        self.endpoint = endpoint.rstrip("/")
        self.clock = clock
        self._token: tuple[str, float] | None = None
        self._key = None

    def _bearer(self) -> dict:
        if not self.creds:
            return {}  # emulator / anonymous
        now = self.clock()
        if self._token is None or self._token[1] - 60 <= now:
            from ..utils import rsa

            if self._key is None:
                self._key = rsa.load_private_key(self.creds["private_key"])
            uri = self.creds.get("token_uri") or "https://oauth2.googleapis.com/token"

            def b64(d) -> str:
                raw = d if isinstance(d, bytes) else json.dumps(d, separators=(",", ":")).encode()
                return base64.urlsafe_b64encode(raw).rstrip(b"=").decode()

            head = {"alg": "RS256", "typ": "JWT"}
            if self.creds.get("private_key_id"):
                head["kid"] = self.creds["private_key_id"]
            claims = {"iss": self.creds["client_email"], "scope": GCS_SCOPE, "aud": uri,
                      "iat": int(now), "exp": int(now) + 3600}
            signing = f"{b64(head)}.{b64(claims)}"
            jwt = signing + "." + b64(rsa.sign_pkcs1_sha256(self._key, signing.encode()))
            form = urllib.parse.urlencode({
                "grant_type": "urn:ietf:params:oauth:grant-type:jwt-bearer",
                "assertion": jwt}).encode()
            st, _, body = _http("POST", uri, {"Content-Type":
                                              "application/x-www-form-urlencoded"}, form,
                                self.timeout)
            if st >= 300:
                raise BlobError(f"gcs token exchange: HTTP {st} {body[:200]!r}", st)
            tok = json.loads(body)
            self._token = (tok["access_token"], now + float(tok.get("expires_in", 3600)))
        return {"Authorization": f"Bearer {self._token[0]}"}

    def _obj(self, key: str) -> str:
        return (f"{self.endpoint}/storage/v1/b/{_uri_encode(self.bucket)}/o/"
                f"{_uri_encode(self._k(key), safe='')}")

    def put(self, key: str, data: bytes, content_type: str = "application/octet-stream"):
        url = (f"{self.endpoint}/upload/storage/v1/b/{_uri_encode(self.bucket)}/o?"
               + urllib.parse.urlencode({"uploadType": "media", "name": self._k(key)}))
        st, _, body = _http("POST", url, {**self._bearer(), "Content-Type": content_type},
                            bytes(data), self.timeout)
        if st >= 300:
            raise BlobError(f"put {key}: HTTP {st} {body[:200]!r}", st)

    def get(self, key: str) -> bytes | None:
        st, _, body = _http("GET", self._obj(key) + "?alt=media", self._bearer(), None,
                            self.timeout)
        if st == 404:
            return None
        if st >= 300:
            raise BlobError(f"get {key}: HTTP {st}", st)
        return body

    def delete(self, key: str):
        st, _, _ = _http("DELETE", self._obj(key), self._bearer(), None, self.timeout)
        if st >= 300 and st != 404:
            raise BlobError(f"delete {key}: HTTP {st}", st)

    def exists(self, key: str) -> bool:
        st, _, _ = _http("GET", self._obj(key), self._bearer(), None, self.timeout)
        if st >= 300 and st != 404:
            raise BlobError(f"stat {key}: HTTP {st}", st)
        return st < 300

    def list(self, prefix: str = "") -> list[str]:
        out, page = [], None
        while True:
            q = {"prefix": self._k(prefix)}
            if page:
                q["pageToken"] = page
            url = (f"{self.endpoint}/storage/v1/b/{_uri_encode(self.bucket)}/o?"
                   + urllib.parse.urlencode(q))
            st, _, body = _http("GET", url, self._bearer(), None, self.timeout)
            if st >= 300:
                raise BlobError(f"list {prefix}: HTTP {st}", st)
            d = json.loads(body or b"{}")
            out += [self._unk(it["name"]) for it in d.get("items", [])]
            page = d.get("nextPageToken")
            if not page:
                return sorted(out)

    def ping(self):
        st, _, _ = _http("GET", f"{self.endpoint}/storage/v1/b/{_uri_encode(self.bucket)}",
                         self._bearer(), None, self.timeout)
        if st >= 300:
            raise BlobError(f"bucket {self.bucket}: HTTP {st}", st)


# ------------------------------------------------------------------ Azure Blob
AZURE_VERSION = "2021-08-06"


def azure_shared_key(account: str, key: bytes, method: str, url: str, headers: dict) -> str:
    """``SharedKey`` signature over the Blob service string-to-sign."""
    h = {k.lower(): str(v) for k, v in headers.items()}
    cl = h.get("content-length", "")
    std = [method, h.get("content-encoding", ""), h.get("content-language", ""),
           "" if cl == "0" else cl, h.get("content-md5", ""), h.get("content-type", ""),
           h.get("date", ""), h.get("if-modified-since", ""), h.get("if-match", ""),
           h.get("if-none-match", ""), h.get("if-unmodified-since", ""), h.get("range", "")]
    canon_h = "".join(f"{k}:{' '.join(h[k].split())}\n" for k in sorted(h)
                      if k.startswith("x-ms-"))
    u = urllib.parse.urlsplit(url)
    res = f"/{account}{u.path or '/'}"
    q: dict[str, list] = {}
    for k, v in urllib.parse.parse_qsl(u.query, keep_blank_values=True):
        q.setdefault(k.lower(), []).append(v)
    for k in sorted(q):
        res += f"\n{k}:{','.join(sorted(q[k]))}"
    sts = "\n".join(std) + "\n" + canon_h + res
    return base64.b64encode(hmac.new(key, sts.encode(), hashlib.sha256).digest()).decode()


class AzureBlobStore(_Base):
    def __init__(self, account: str, container: str, account_key_b64: str = "",
                 endpoint: str = "", prefix: str = "sessions/", timeout: float = 30.0):
        super().__init__(prefix, timeout)
        self.account, self.container = account, container
        self.key = base64.b64decode(account_key_b64) if account_key_b64 else b""
        self.base = (endpoint.rstrip("/") if endpoint
                     else f"https://{account}.blob.core.windows.net")

    def _req(self, method: str, url: str, body: bytes = b"", extra: dict | None = None):
        headers = {"x-ms-date": dt.datetime.now(dt.timezone.utc).strftime(
            "%a, %d %b %Y %H:%M:%S GMT"), "x-ms-version": AZURE_VERSION, **(extra or {})}
        if method in ("PUT", "POST"):
            headers["Content-Length"] = str(len(body))
        if self.key:
            headers["Authorization"] = (f"SharedKey {self.account}:"
                                        + azure_shared_key(self.account, self.key, method, url,
                                                           headers))
        return _http(method, url, headers, body if method in ("PUT", "POST") else None,
                     self.timeout)

    def _url(self, key: str) -> str:
        return f"{self.base}/{self.container}/{_uri_encode(self._k(key), safe='/-_.~')}"

    def put(self, key: str, data: bytes, content_type: str = "application/octet-stream"):
        st, _, body = self._req("PUT", self._url(key), bytes(data),
                                {"x-ms-blob-type": "BlockBlob", "Content-Type": content_type})
        if st >= 300:
            raise BlobError(f"put {key}: HTTP {st} {body[:200]!r}", st)

    def get(self, key: str) -> bytes | None:
        st, _, body = self._req("GET", self._url(key))
        if st == 404:
            return None
        if st >= 300:
            raise BlobError(f"get {key}: HTTP {st}", st)
        return body

    def delete(self, key: str):
        st, _, _ = self._req("DELETE", self._url(key))
        if st >= 300 and st != 404:
            raise BlobError(f"delete {key}: HTTP {st}", st)

    def exists(self, key: str) -> bool:
        st, _, _ = self._req("HEAD", self._url(key))
        if st >= 300 and st != 404:
            raise BlobError(f"head {key}: HTTP {st}", st)
        return st < 300

    def list(self, prefix: str = "") -> list[str]:
        out, marker = [], ""
        while True:
            q = {"restype": "container", "comp": "list", "prefix": self._k(prefix)}
            if marker:
                q["marker"] = marker
            url = f"{self.base}/{self.container}?" + urllib.parse.urlencode(q)
            st, _, body = self._req("GET", url)
            if st >= 300:
                raise BlobError(f"list {prefix}: HTTP {st}", st)
            root = ET.fromstring(body)
            out += [self._unk(b.findtext("Name")) for b in root.iter("Blob")]
            marker = root.findtext("NextMarker") or ""
            if not marker:
                return sorted(out)

    def ping(self):
        st, _, _ = self._req("GET", f"{self.base}/{self.container}?restype=container")
        if st >= 300:
            raise BlobError(f"container {self.container}: HTTP {st}", st)


# ------------------------------------------------------------------ factory
def build_cold_blobstore(backend: str, bucket: str, region: str = "", endpoint: str = "",
                         prefix: str = "sessions/", env: dict | None = None):
    """``--cold-backend s3|gcs|azure`` with the vendors' standard credential env:
    AWS_ACCESS_KEY_ID / AWS_SECRET_ACCESS_KEY / AWS_SESSION_TOKEN (+
    COLD_S3_PATH_STYLE), GOOGLE_APPLICATION_CREDENTIALS (service-account JSON) or
    GCS_HMAC_ACCESS_ID / GCS_HMAC_SECRET, STORAGE_EMULATOR_HOST, and
    AZURE_STORAGE_ACCOUNT / AZURE_STORAGE_KEY."""
    env = os.environ if env is None else env
    b = (backend or "").lower()
    if b == "s3":
        return S3BlobStore(bucket, region or env.get("AWS_REGION", "us-east-1"), endpoint,
                           env.get("AWS_ACCESS_KEY_ID", ""), env.get("AWS_SECRET_ACCESS_KEY", ""),
                           env.get("AWS_SESSION_TOKEN", ""),
                           use_path_style=env.get("COLD_S3_PATH_STYLE", "").lower() == "true"
                           or bool(endpoint), prefix=prefix)
    if b == "gcs":
        if env.get("GCS_HMAC_ACCESS_ID"):
            return GCSHMACBlobStore(bucket, env["GCS_HMAC_ACCESS_ID"],
                                    env.get("GCS_HMAC_SECRET", ""),
                                    endpoint=endpoint or "https://storage.googleapis.com",
                                    prefix=prefix)
        creds = None
        if env.get("GOOGLE_APPLICATION_CREDENTIALS"):
            with open(env["GOOGLE_APPLICATION_CREDENTIALS"]) as f:
                creds = json.load(f)
        emu = env.get("STORAGE_EMULATOR_HOST", "")
        ep = endpoint or (("http://" + emu if "://" not in emu else emu) if emu
                          else "https://storage.googleapis.com")
        return GCSBlobStore(bucket, None if emu and not creds else creds, ep, prefix=prefix)
    if b == "azure":
        return AzureBlobStore(env.get("AZURE_STORAGE_ACCOUNT", ""), bucket,
                              env.get("AZURE_STORAGE_KEY", ""), endpoint, prefix=prefix)
    raise ValueError(f"unknown cold backend {backend!r} (s3, gcs, azure)")
