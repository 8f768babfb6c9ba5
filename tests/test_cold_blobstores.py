"""Cold-tier object stores against in-repo fakes of the S3, GCS (JSON API +
OAuth2 token endpoint) and Azure Blob REST APIs.  Each fake re-derives the
request signature independently (SigV4 canonical request, RS256 JWT over the
service-account public key, Azure Shared Key string-to-sign) and rejects a
mismatch, lists in small pages to exercise pagination, and the cold archive
(Parquet batches + manifest) round-trips sessions through every backend
(reference ``internal/session/providers/cold/blobstore_*.go``)."""
import asyncio
import base64
import datetime as dt
import hashlib
import hmac
import json
import threading
import urllib.parse

import pytest
from aiohttp import web

from omnia_amd.facade.auth import rsa_verify_pkcs1_sha256
from omnia_amd.session.blobstores import (AzureBlobStore, BlobError, GCSBlobStore,
                                          GCSHMACBlobStore, S3BlobStore, build_cold_blobstore,
                                          sigv4_authorization)
from omnia_amd.session.model import Message, Session
from omnia_amd.session.store import ColdArchive
from omnia_amd.utils import rsa


class ThreadServer:
    def __init__(self, app):
        self.app = app
        self.loop = asyncio.new_event_loop()
        self.ready = threading.Event()
        self.t = threading.Thread(target=self._run, daemon=True)
        self.t.start()
        self.ready.wait(10)

    def _run(self):
        asyncio.set_event_loop(self.loop)

        async def start():
            self.runner = web.AppRunner(self.app)
            await self.runner.setup()
            site = web.TCPSite(self.runner, "127.0.0.1", 0)
            await site.start()
            self.port = site._server.sockets[0].getsockname()[1]

        self.loop.run_until_complete(start())
        self.ready.set()
        self.loop.run_forever()

    @property
    def url(self):
        return f"http://127.0.0.1:{self.port}"

    def close(self):
        async def stop():
            await self.runner.cleanup()

        asyncio.run_coroutine_threadsafe(stop(), self.loop).result(10)
        self.loop.call_soon_threadsafe(self.loop.stop)
        self.t.join(10)


# ------------------------------------------------------------------ SigV4
def test_sigv4_matches_the_aws_get_vanilla_vector():
    """AWS SigV4 test suite 'get-vanilla' (AKIDEXAMPLE, 20150830T123600Z,
    us-east-1/service)."""
    h = sigv4_authorization("GET", "https://example.amazonaws.com/", {},
                            hashlib.sha256(b"").hexdigest(), "us-east-1", "service",
                            "AKIDEXAMPLE", "wJalrXUtnFEMI/K7MDENG+bPxRfiCYEXAMPLEKEY",
                            now=dt.datetime(2015, 8, 30, 12, 36, tzinfo=dt.timezone.utc))
    assert h["Authorization"] == (
        "AWS4-HMAC-SHA256 Credential=AKIDEXAMPLE/20150830/us-east-1/service/aws4_request, "
        "SignedHeaders=host;x-amz-date, "
        "Signature=5fa00fa31553b73ebf1942676e86291e8372ff2a2260956d9b8aae1d763fbf31")


def _verify_sigv4(request, body: bytes, secret: str, algo="AWS4-HMAC-SHA256", pre="AWS4",
                  rtype="aws4_request", date_h="x-amz-date", hash_h="x-amz-content-sha256"):
    """Independent SigV4 check of a received request."""
    auth = request.headers.get("Authorization", "")
    parts = dict(p.strip().split("=", 1) for p in auth[len(algo) + 1:].split(","))
    cred, signed, sig = parts["Credential"], parts["SignedHeaders"], parts["Signature"]
    _, date, region, service, _ = cred.split("/")
    assert request.headers[hash_h] == hashlib.sha256(body).hexdigest()
    q = sorted(urllib.parse.parse_qsl(request.query_string, keep_blank_values=True))
    cq = "&".join(f"{urllib.parse.quote(k, safe='-_.~')}={urllib.parse.quote(v, safe='-_.~')}"
                  for k, v in q)
    ch = "".join(f"{k}:{request.headers[k].strip()}\n" for k in signed.split(";"))
    path = urllib.parse.quote(urllib.parse.unquote(request.raw_path.split("?")[0]),
                              safe="/-_.~")
    creq = "\n".join([request.method, path, cq, ch, signed, request.headers[hash_h]])
    sts = "\n".join([algo, request.headers[date_h], f"{date}/{region}/{service}/{rtype}",
                     hashlib.sha256(creq.encode()).hexdigest()])
    k = (pre + secret).encode()
    for part in (date, region, service, rtype):
        k = hmac.new(k, part.encode(), hashlib.sha256).digest()
    return hmac.compare_digest(sig, hmac.new(k, sts.encode(), hashlib.sha256).hexdigest())


def s3_fake(secret: str, page: int = 2, **kw):
    objs: dict[str, bytes] = {}
    seen = {"requests": 0}

    async def handle(request):
        body = await request.read()
        if not _verify_sigv4(request, body, secret, **kw):
            return web.Response(status=403, text="SignatureDoesNotMatch")
        seen["requests"] += 1
        path = urllib.parse.unquote(request.path)
        bucket, _, key = path.lstrip("/").partition("/")
        if bucket != "bkt":
            return web.Response(status=404)
        if request.method == "PUT":
            objs[key] = body
            return web.Response(status=200)
        if request.method in ("GET", "HEAD") and key:
            if key not in objs:
                return web.Response(status=404)
            return web.Response(body=objs[key] if request.method == "GET" else b"")
        if request.method == "DELETE":
            objs.pop(key, None)
            return web.Response(status=204)
        if request.method == "HEAD":
            return web.Response(status=200)
        q = request.query
        keys = sorted(k for k in objs if k.startswith(q.get("prefix", "")))
        start = int(q.get("continuation-token", "0"))
        chunk = keys[start:start + page]
        more = start + page < len(keys)
        xml = ('<?xml version="1.0"?><ListBucketResult '
               'xmlns="http://s3.amazonaws.com/doc/2006-03-01/">'
               + "".join(f"<Contents><Key>{k}</Key></Contents>" for k in chunk)
               + f"<IsTruncated>{'true' if more else 'false'}</IsTruncated>"
               + (f"<NextContinuationToken>{start + page}</NextContinuationToken>" if more
                  else "") + "</ListBucketResult>")
        return web.Response(text=xml, content_type="application/xml")

    app = web.Application(client_max_size=64 * 2**20)
    app.router.add_route("*", "/{tail:.*}", handle)
    return app, objs, seen


def _archive_roundtrip(store):
    arch = ColdArchive(store)
    items = [(Session(id=f"s{i}", agent_name="a", namespace="ns"),
              [Message(role="user", content=f"hello {i}"),
               Message(role="assistant", content=f"hi {i}")]) for i in range(3)]
    key = arch.archive(items)
    assert store.exists(key) and store.exists("manifest.json")
    again = ColdArchive(store)  # a new process reads the manifest back
    s, msgs = again.get("s1")
    assert s.agent_name == "a" and [m.content for m in msgs] == ["hello 1", "hi 1"]
    return key


def test_s3_store_signed_crud_pagination_and_archive():
    app, objs, seen = s3_fake("SECRET")
    srv = ThreadServer(app)
    try:
        st = S3BlobStore("bkt", "eu-west-1", srv.url, "AKID", "SECRET", use_path_style=True)
        for i in range(5):
            st.put(f"batches/{i}.parquet", f"data{i}".encode())
        assert st.get("batches/3.parquet") == b"data3"
        assert st.get("missing") is None and not st.exists("missing")
        assert st.list("batches/") == [f"batches/{i}.parquet" for i in range(5)]  # 3 pages
        assert set(objs) == {f"sessions/batches/{i}.parquet" for i in range(5)}  # prefix
        st.delete("batches/0.parquet")
        assert not st.exists("batches/0.parquet")
        key = _archive_roundtrip(st)
        assert f"sessions/{key}" in objs
        bad = S3BlobStore("bkt", "eu-west-1", srv.url, "AKID", "WRONG", use_path_style=True)
        with pytest.raises(BlobError) as e:
            bad.put("x", b"y")
        assert e.value.status == 403
    finally:
        srv.close()


def test_gcs_hmac_xml_api_uses_goog4_signing():
    app, objs, _ = s3_fake("GSECRET", algo="GOOG4-HMAC-SHA256", pre="GOOG4",
                           rtype="goog4_request", date_h="x-goog-date",
                           hash_h="x-goog-content-sha256")
    srv = ThreadServer(app)
    try:
        st = GCSHMACBlobStore("bkt", "GOOGID", "GSECRET", endpoint=srv.url)
        st.put("a/b.bin", b"\x00\x01")
        assert st.get("a/b.bin") == b"\x00\x01" and st.list("a/") == ["a/b.bin"]
    finally:
        srv.close()


# ------------------------------------------------------------------ GCS (JSON API)
@pytest.fixture(scope="module")
def sa_key():
    return rsa.generate_private_key(1024)


def gcs_fake(key, page=2):
    objs: dict[str, bytes] = {}
    state = {"tokens": 0}

    async def token(request):
        form = await request.post()
        assert form["grant_type"] == "urn:ietf:params:oauth:grant-type:jwt-bearer"
        h, c, s = form["assertion"].split(".")
        pad = lambda x: base64.urlsafe_b64decode(x + "=" * (-len(x) % 4))  # noqa: E731
        if not rsa_verify_pkcs1_sha256(key.n, key.e, f"{h}.{c}".encode(), pad(s)):
            return web.json_response({"error": "invalid_grant"}, status=400)
        claims = json.loads(pad(c))
        assert claims["iss"] == "svc@proj.iam.gserviceaccount.com"
        assert claims["scope"].endswith("devstorage.read_write")
        assert claims["exp"] - claims["iat"] == 3600
        assert json.loads(pad(h))["kid"] == "k1"
        state["tokens"] += 1
        return web.json_response({"access_token": f"tok{state['tokens']}",
                                  "expires_in": 3600})

    def authed(request):
        return request.headers.get("Authorization", "").startswith("Bearer tok")

    async def upload(request):
        if not authed(request):
            return web.Response(status=401)
        assert request.query["uploadType"] == "media"
        objs[request.query["name"]] = await request.read()
        return web.json_response({"name": request.query["name"]})

    async def obj(request):
        if not authed(request):
            return web.Response(status=401)
        name = urllib.parse.unquote(request.match_info["name"])
        if name not in objs:
            return web.Response(status=404)
        if request.method == "DELETE":
            del objs[name]
            return web.Response(status=204)
        if request.query.get("alt") == "media":
            return web.Response(body=objs[name])
        return web.json_response({"name": name, "size": str(len(objs[name]))})

    async def listing(request):
        if not authed(request):
            return web.Response(status=401)
        keys = sorted(k for k in objs if k.startswith(request.query.get("prefix", "")))
        start = int(request.query.get("pageToken", "0"))
        out = {"items": [{"name": k} for k in keys[start:start + page]]}
        if start + page < len(keys):
            out["nextPageToken"] = str(start + page)
        return web.json_response(out)

    async def bucket(request):
        return web.json_response({"name": "bkt"}) if authed(request) else web.Response(status=401)

    app = web.Application(client_max_size=64 * 2**20)
    app.router.add_post("/token", token)
    app.router.add_post("/upload/storage/v1/b/bkt/o", upload)
    app.router.add_get("/storage/v1/b/bkt/o", listing)
    app.router.add_get("/storage/v1/b/bkt", bucket)
    app.router.add_route("*", "/storage/v1/b/bkt/o/{name:.+}", obj)
    return app, objs, state


def test_gcs_service_account_json_api(sa_key):
    app, objs, state = gcs_fake(sa_key)
    srv = ThreadServer(app)
    clock = [1_000_000.0]
    try:
        creds = {"type": "service_account", "client_email": "svc@proj.iam.gserviceaccount.com",
                 "private_key_id": "k1", "private_key": rsa.dump_private_key_pkcs8(sa_key),
                 "token_uri": srv.url + "/token"}
        st = GCSBlobStore("bkt", creds, endpoint=srv.url, clock=lambda: clock[0])
        st.ping()
        for i in range(3):
            st.put(f"b/{i}", bytes([i]) * 10)
        assert st.get("b/2") == b"\x02" * 10 and st.get("nope") is None
        assert st.list("b/") == ["b/0", "b/1", "b/2"]
        assert "sessions/b/1" in objs
        st.delete("b/1")
        assert not st.exists("b/1")
        _archive_roundtrip(st)
        assert state["tokens"] == 1  # cached
        clock[0] += 3600  # expired: re-minted
        st.get("b/0")
        assert state["tokens"] == 2
    finally:
        srv.close()


def test_rsa_pkcs8_roundtrip_and_signature(sa_key):
    k2 = rsa.load_private_key(rsa.dump_private_key_pkcs8(sa_key))
    assert (k2.n, k2.e, k2.d) == (sa_key.n, sa_key.e, sa_key.d)
    sig = rsa.sign_pkcs1_sha256(k2, b"msg")
    assert rsa_verify_pkcs1_sha256(sa_key.n, sa_key.e, b"msg", sig)
    assert not rsa_verify_pkcs1_sha256(sa_key.n, sa_key.e, b"msh", sig)
    # CRT and plain exponentiation agree
    plain = rsa.PrivateKey(k2.n, k2.e, k2.d)
    assert rsa.sign_pkcs1_sha256(plain, b"msg") == sig


# ------------------------------------------------------------------ Azure
ACCOUNT, AKEY = "devacct", base64.b64encode(b"k" * 32).decode()


def _azure_expected(request, body):
    """Independent Shared Key string-to-sign for the Blob service."""
    h = {k.lower(): v for k, v in request.headers.items()}
    cl = h.get("content-length", "")
    lines = [request.method, h.get("content-encoding", ""), h.get("content-language", ""),
             "" if cl in ("0", "") else cl, h.get("content-md5", ""), h.get("content-type", ""),
             h.get("date", ""), h.get("if-modified-since", ""), h.get("if-match", ""),
             h.get("if-none-match", ""), h.get("if-unmodified-since", ""), h.get("range", "")]
    xms = "".join(f"{k}:{h[k]}\n" for k in sorted(h) if k.startswith("x-ms-"))
    res = f"/{ACCOUNT}{request.raw_path.split('?')[0]}"
    params = {}
    for k, v in urllib.parse.parse_qsl(request.query_string, keep_blank_values=True):
        params.setdefault(k.lower(), []).append(v)
    res += "".join(f"\n{k}:{','.join(sorted(params[k]))}" for k in sorted(params))
    sts = "\n".join(lines) + "\n" + xms + res
    sig = base64.b64encode(hmac.new(base64.b64decode(AKEY), sts.encode(),
                                    hashlib.sha256).digest()).decode()
    return f"SharedKey {ACCOUNT}:{sig}"


def azure_fake(page=2):
    objs: dict[str, bytes] = {}

    async def handle(request):
        body = await request.read()
        if request.headers.get("Authorization") != _azure_expected(request, body):
            return web.Response(status=403, text="AuthenticationFailed")
        assert request.headers["x-ms-version"]
        name = urllib.parse.unquote(request.path.lstrip("/").partition("/")[2])
        if request.query.get("comp") == "list":
            keys = sorted(k for k in objs if k.startswith(request.query.get("prefix", "")))
            start = int(request.query.get("marker") or 0)
            nxt = str(start + page) if start + page < len(keys) else ""
            xml = ("<EnumerationResults><Blobs>"
                   + "".join(f"<Blob><Name>{k}</Name></Blob>" for k in keys[start:start + page])
                   + f"</Blobs><NextMarker>{nxt}</NextMarker></EnumerationResults>")
            return web.Response(text=xml, content_type="application/xml")
        if request.query.get("restype") == "container":
            return web.Response(status=200)
        if request.method == "PUT":
            assert request.headers["x-ms-blob-type"] == "BlockBlob"
            objs[name] = body
            return web.Response(status=201)
        if name not in objs:
            return web.Response(status=404)
        if request.method == "DELETE":
            del objs[name]
            return web.Response(status=202)
        return web.Response(body=objs[name] if request.method == "GET" else b"")

    app = web.Application(client_max_size=64 * 2**20)
    app.router.add_route("*", "/{tail:.*}", handle)
    return app, objs


def test_azure_shared_key_store():
    app, objs = azure_fake()
    srv = ThreadServer(app)
    try:
        st = AzureBlobStore(ACCOUNT, "cont", AKEY, endpoint=srv.url)
        st.ping()
        for i in range(5):
            st.put(f"x/{i}", b"v%d" % i)
        assert st.get("x/4") == b"v4" and st.get("none") is None
        assert st.list("x/") == [f"x/{i}" for i in range(5)]
        assert "sessions/x/0" in objs
        st.delete("x/0")
        assert not st.exists("x/0")
        _archive_roundtrip(st)
        bad = AzureBlobStore(ACCOUNT, "cont", base64.b64encode(b"z" * 32).decode(),
                             endpoint=srv.url)
        with pytest.raises(BlobError):
            bad.put("y", b"1")
    finally:
        srv.close()


def test_factory_reads_vendor_env(tmp_path):
    s3 = build_cold_blobstore("s3", "b", "us-west-2", "http://minio:9000", env={
        "AWS_ACCESS_KEY_ID": "A", "AWS_SECRET_ACCESS_KEY": "S"})
    assert isinstance(s3, S3BlobStore) and s3.path_style and s3.ak == "A"
    assert s3._url("k") == "http://minio:9000/b/k"
    assert S3BlobStore("b", "eu-west-1")._url("k") == "https://b.s3.eu-west-1.amazonaws.com/k"
    g = build_cold_blobstore("gcs", "b", env={"STORAGE_EMULATOR_HOST": "localhost:4443"})
    assert isinstance(g, GCSBlobStore) and g.creds is None and \
        g.endpoint == "http://localhost:4443"
    gh = build_cold_blobstore("gcs", "b", env={"GCS_HMAC_ACCESS_ID": "i", "GCS_HMAC_SECRET": "s"})
    assert isinstance(gh, GCSHMACBlobStore)
    az = build_cold_blobstore("azure", "c", env={"AZURE_STORAGE_ACCOUNT": "acc",
                                                 "AZURE_STORAGE_KEY": AKEY})
    assert isinstance(az, AzureBlobStore) and az.base == "https://acc.blob.core.windows.net"
    with pytest.raises(ValueError):
        build_cold_blobstore("ftp", "b", env={})
