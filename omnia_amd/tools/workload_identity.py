"""``workloadIdentity`` tool auth: a bearer token for the tool's audience under
the pod's ambient Azure identity (reference ``internal/runtime/tools/auth.go:26-50``
``resolveWorkloadIdentityHeader`` and ``azure_token.go``, which go through the
Azure SDK's DefaultAzureCredential).

There is no Azure SDK here, so the exchange is done directly: the Azure
workload-identity webhook projects a Kubernetes service-account token into the
pod and sets ``AZURE_CLIENT_ID`` / ``AZURE_TENANT_ID`` /
``AZURE_FEDERATED_TOKEN_FILE`` (+ ``AZURE_AUTHORITY_HOST``); the acquirer trades
that federated token for an Entra ID access token with a client-credentials
grant whose client assertion is the projected token (scope ``<audience>/.default``).
The file is re-read on every exchange (the kubelet rotates it), and tokens are
cached per audience until five minutes before they expire.

Only ``cloud: azure`` is supported; any other cloud, or no acquirer, fails the
call loudly rather than sending an unauthenticated request.
"""
from __future__ import annotations

import asyncio
import os
import time

CLOUD_AZURE = "azure"
DEFAULT_HEADER = "Authorization"
DEFAULT_AUTHORITY = "https://login.microsoftonline.com/"
ASSERTION_TYPE = "urn:ietf:params:oauth:client-assertion-type:jwt-bearer"
REFRESH_MARGIN_S = 300.0


class WorkloadIdentityError(Exception):
    pass


class AzureTokenAcquirer:
    """Entra ID tokens from the projected federated token (per-audience cache).

    ``post(url, form) -> (status, json)`` is injectable for tests; the default
    posts with aiohttp."""

    def __init__(self, env=None, post=None, now=time.time):
        env = os.environ if env is None else env
        self.tenant = env.get("AZURE_TENANT_ID", "")
        self.client_id = env.get("AZURE_CLIENT_ID", "")
        self.token_file = env.get("AZURE_FEDERATED_TOKEN_FILE", "")
        self.authority = env.get("AZURE_AUTHORITY_HOST") or DEFAULT_AUTHORITY
        self.post = post or _aiohttp_post
        self.now = now
        self.cache: dict[str, tuple[str, float]] = {}
        self._lock = None
        self.exchanges = 0

    def configured(self) -> bool:
        return bool(self.tenant and self.client_id and self.token_file)

    async def token(self, audience: str) -> str:
        if not audience:
            raise WorkloadIdentityError("workloadIdentity: audience is required")
        loop = asyncio.get_running_loop()
        if self._lock is None or self._lock[0] is not loop:  # a lock serves one loop
            self._lock = (loop, asyncio.Lock())
        async with self._lock[1]:  # low contention: one lock over cache + exchange
            hit = self.cache.get(audience)
            if hit is not None and self.now() < hit[1] - REFRESH_MARGIN_S:
                return hit[0]
            if not self.configured():
                raise WorkloadIdentityError(
                    "workloadIdentity: AZURE_TENANT_ID / AZURE_CLIENT_ID / "
                    "AZURE_FEDERATED_TOKEN_FILE not set (is the pod's identity federated?)")
            try:
                with open(self.token_file) as f:
                    assertion = f.read().strip()
            except OSError as e:
                raise WorkloadIdentityError(f"workloadIdentity: federated token: {e}") from None
            scope = audience.rstrip("/") + "/.default"
            url = f"{self.authority.rstrip('/')}/{self.tenant}/oauth2/v2.0/token"
            self.exchanges += 1
            status, body = await self.post(url, {
                "client_id": self.client_id, "scope": scope, "grant_type": "client_credentials",
                "client_assertion_type": ASSERTION_TYPE, "client_assertion": assertion})
            if status != 200 or not isinstance(body, dict) or "access_token" not in body:
                err = (body or {}).get("error_description") or (body or {}).get("error") \
                    if isinstance(body, dict) else body
                raise WorkloadIdentityError(
                    f"acquire azure token for {audience!r}: HTTP {status}: {str(err)[:200]}")
            tok = body["access_token"]
            self.cache[audience] = (tok, self.now() + float(body.get("expires_in", 3600)))
            return tok


async def _aiohttp_post(url: str, form: dict):
    import aiohttp

    async with aiohttp.ClientSession(timeout=aiohttp.ClientTimeout(total=30)) as s:
        async with s.post(url, data=form) as r:
            try:
                body = await r.json(content_type=None)
            except Exception:  # noqa: BLE001 - non-JSON error page
                body = await r.text()
            return r.status, body


_default: AzureTokenAcquirer | None = None


def default_acquirer() -> AzureTokenAcquirer:
    """The process's acquirer (the pod has one ambient identity)."""
    global _default
    if _default is None:
        _default = AzureTokenAcquirer()
    return _default


def wif_config(entry: dict, cfg: dict) -> dict | None:
    """The handler's workloadIdentity settings, or None: the CRD's handler-level
    ``auth: {type: workloadIdentity, workloadIdentity: {cloud, audience, header}}``
    or the flattened runtime form ``authType/authCloud/authAudience/authHeader``."""
    auth = entry.get("auth") or {}
    if auth.get("type") == "workloadIdentity":
        w = auth.get("workloadIdentity") or {}
        return {"cloud": w.get("cloud", ""), "audience": w.get("audience", ""),
                "header": w.get("header") or DEFAULT_HEADER}
    if (cfg.get("authType") or "") == "workloadIdentity":
        return {"cloud": cfg.get("authCloud", ""), "audience": cfg.get("authAudience", ""),
                "header": cfg.get("authHeader") or DEFAULT_HEADER}
    return None


async def resolve_header(acq, wif: dict) -> tuple[str, str]:
    """(header name, "Bearer <token>") for a workloadIdentity handler."""
    if wif.get("cloud") != CLOUD_AZURE:
        raise WorkloadIdentityError(
            f"workloadIdentity cloud {wif.get('cloud')!r} not supported (only 'azure')")
    if acq is None:
        raise WorkloadIdentityError("workloadIdentity: no token acquirer configured")
    tok = await acq.token(wif.get("audience", ""))
    return wif.get("header") or DEFAULT_HEADER, "Bearer " + tok
