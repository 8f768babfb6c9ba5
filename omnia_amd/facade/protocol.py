"""WebSocket facade wire protocol (JSON + binary OMNI frames).

JSON shapes mirror ``internal/facade/protocol.go:93-362``: client types
``message | upload_request | tool_result | tool_call_ack | tool_call_nack |
hangup``; server types ``connected | chunk | done | tool_call | tool_result |
error | upload_ready | upload_complete | media_chunk | interrupt |
session_config``; every server message carries an RFC3339 ``timestamp``.

Binary frames (``internal/facade/binary.go:26-139``): 32-byte big-endian header
``"OMNI" | version u8 | flags u8 | type u8 | reserved u8 | metaLen u32 |
payloadLen u32 | sequence u32 | mediaID[12]`` followed by JSON metadata and the
payload.  Flags: compressed 0x01, chunked 0x02, last 0x04.  Payloads above
1 MiB are split into 64 KiB chunks.
"""
from __future__ import annotations

import datetime as _dt
import json as _json
import time as _time
import json
import struct

PROTOCOL_VERSION = 1

# client -> server
MESSAGE = "message"
UPLOAD_REQUEST = "upload_request"
TOOL_RESULT = "tool_result"
TOOL_CALL_ACK = "tool_call_ack"
TOOL_CALL_NACK = "tool_call_nack"
HANGUP = "hangup"
CLIENT_TYPES = {MESSAGE, UPLOAD_REQUEST, TOOL_RESULT, TOOL_CALL_ACK, TOOL_CALL_NACK, HANGUP}

# server -> client
CONNECTED = "connected"
CHUNK = "chunk"
DONE = "done"
TOOL_CALL = "tool_call"
ERROR = "error"
UPLOAD_READY = "upload_ready"
UPLOAD_COMPLETE = "upload_complete"
MEDIA_CHUNK = "media_chunk"
INTERRUPT = "interrupt"
SESSION_CONFIG = "session_config"

# error codes
E_INVALID_MESSAGE = "INVALID_MESSAGE"
E_SESSION_NOT_FOUND = "SESSION_NOT_FOUND"
E_SESSION_EXPIRED = "SESSION_EXPIRED"
E_INTERNAL = "INTERNAL_ERROR"
E_AGENT_UNAVAILABLE = "AGENT_UNAVAILABLE"
E_TOOL_FAILED = "TOOL_FAILED"
E_UPLOAD_FAILED = "UPLOAD_FAILED"
E_MEDIA_NOT_ENABLED = "MEDIA_NOT_ENABLED"
E_RATE_LIMITED = "RATE_LIMITED"
E_UNSATISFIABLE_FORMAT = "UNSATISFIABLE_FORMAT"


_TS = [-1, ""]  # (whole second, "YYYY-MM-DDTHH:MM:SS") of the last stamp


def now_rfc3339() -> str:
    """UTC RFC 3339 with microseconds (``datetime.isoformat`` + ``Z``); the
    date/time prefix is formatted once per second -- it is stamped on every
    streamed frame."""
    t = _time.time()
    sec = int(t)
    if sec != _TS[0]:
        _TS[0] = sec
        _TS[1] = _dt.datetime.fromtimestamp(sec, _dt.timezone.utc).strftime("%Y-%m-%dT%H:%M:%S")
    us = int((t - sec) * 1e6)
    return f"{_TS[1]}.{us:06d}Z" if us else _TS[1] + "Z"


_enc = _json.encoder.encode_basestring_ascii  # what json.dumps uses for str


def chunk_text(session_json: str, content: str, role: str = "") -> str:
    """The serialized ``chunk`` frame -- byte-identical to
    ``json.dumps(chunk(...), separators=(",", ":"))`` -- without building the
    dict (the hot path: one frame per streamed token).  ``session_json`` is the
    JSON-encoded session id (``""`` when there is none)."""
    head = '{"type":"chunk"' + (',"session_id":' + session_json if session_json else "")
    body = (',"content":' + _enc(content) if content else "") + \
        (',"role":' + _enc(role) if role else "")
    return head + body + ',"timestamp":"' + now_rfc3339() + '"}'


def server_msg(mtype: str, session_id: str = "", **fields) -> dict:
    m = {"type": mtype}
    if session_id:
        m["session_id"] = session_id
    for k, v in fields.items():
        if v is not None and v != "" and v != [] and v != {}:
            m[k] = v
    m["timestamp"] = now_rfc3339()
    return m


def connected(session_id: str, binary: bool, max_payload: int, resumed: bool = False) -> dict:
    return server_msg(CONNECTED, session_id, connected={
        "capabilities": {"binary_frames": binary, "max_payload_size": max_payload,
                         "protocol_version": PROTOCOL_VERSION},
        **({"resumed": True} if resumed else {})})


def chunk(session_id: str, content: str, role: str = "") -> dict:
    return server_msg(CHUNK, session_id, content=content, role=role)


def done(session_id: str, content: str, parts=None, usage: dict | None = None) -> dict:
    return server_msg(DONE, session_id, content=content, parts=parts, usage=usage)


def error(session_id: str, code: str, message: str, details: dict | None = None) -> dict:
    return server_msg(ERROR, session_id, error={"code": code, "message": message,
                                                **({"details": details} if details else {})})


def tool_call(session_id: str, call_id: str, name: str, arguments: dict,
              consent_message: str = "", categories=None) -> dict:
    tc = {"id": call_id, "name": name}
    if arguments:
        tc["arguments"] = arguments
    if consent_message:
        tc["consent_message"] = consent_message
    if categories:
        tc["categories"] = list(categories)
    return server_msg(TOOL_CALL, session_id, tool_call=tc)


# field -> accepted JSON types of a client message (null = absent); anything else
# is an invalid message (E_INVALID_MESSAGE), never an exception in the handlers
_CLIENT_FIELDS = {"session_id": (str,), "content": (str,), "metadata": (dict,),
                  "consent_grants": (list,), "parts": (list,), "tool_result": (dict,),
                  "tool_call_ack": (dict,), "tool_call_nack": (dict,),
                  "upload_request": (dict,)}
_PART_FIELDS = {"type": (str,), "text": (str,), "media": (dict,), "media_id": (str,),
                "mime_type": (str,), "url": (str,), "data": (str,)}


def parse_client(raw: str | bytes) -> dict:
    try:
        m = json.loads(raw)
    except RecursionError as e:  # pathologically nested JSON
        raise ValueError("message nested too deeply") from e
    if not isinstance(m, dict) or m.get("type") not in CLIENT_TYPES:
        raise ValueError("unknown or missing message type")
    for k, types in _CLIENT_FIELDS.items():
        v = m.get(k)
        if v is not None and not isinstance(v, types):
            raise ValueError(f"field {k!r} must be {types[0].__name__}")
    for p in m.get("parts") or ():
        if not isinstance(p, dict):
            raise ValueError("message parts must be objects")
        for k, types in _PART_FIELDS.items():
            v = p.get(k)
            if v is not None and not isinstance(v, types):
                raise ValueError(f"part field {k!r} must be {types[0].__name__}")
        for k in ("data", "url", "mime_type", "storage_ref"):
            v = (p.get("media") or {}).get(k)
            if v is not None and not isinstance(v, str):
                raise ValueError(f"media field {k!r} must be str")
    if not all(isinstance(g, str) for g in m.get("consent_grants") or ()):
        raise ValueError("consent_grants must be strings")
    return m


# ------------------------------------------------------------------ binary frames
MAGIC = b"OMNI"
HEADER_SIZE = 32
FLAG_COMPRESSED, FLAG_CHUNKED, FLAG_LAST = 0x01, 0x02, 0x04
TYPE_MEDIA_CHUNK, TYPE_UPLOAD = 1, 2
CHUNK_THRESHOLD = 1 << 20
CHUNK_SIZE = 64 << 10
_HDR = struct.Struct(">4sBBBBIII12s")


def encode_frame(ftype: int, payload: bytes, meta: dict | None = None, seq: int = 0,
                 media_id: bytes = b"", flags: int = 0) -> bytes:
    mb = json.dumps(meta or {}, separators=(",", ":")).encode() if meta else b""
    mid = (media_id or b"")[:12].ljust(12, b"\0")
    return _HDR.pack(MAGIC, PROTOCOL_VERSION, flags, ftype, 0, len(mb), len(payload), seq,
                     mid) + mb + payload


def decode_frame(buf: bytes) -> dict:
    if len(buf) < HEADER_SIZE:
        raise ValueError("frame shorter than header")
    magic, ver, flags, ftype, _, mlen, plen, seq, mid = _HDR.unpack_from(buf)
    if magic != MAGIC:
        raise ValueError("bad magic")
    if ver != PROTOCOL_VERSION:
        raise ValueError(f"unsupported frame version {ver}")
    if HEADER_SIZE + mlen + plen != len(buf):
        raise ValueError("length mismatch")
    meta = json.loads(buf[HEADER_SIZE:HEADER_SIZE + mlen]) if mlen else {}
    return {"version": ver, "flags": flags, "type": ftype, "seq": seq,
            "media_id": mid.rstrip(b"\0"), "meta": meta,
            "payload": buf[HEADER_SIZE + mlen:]}


def split_payload(ftype: int, payload: bytes, meta: dict | None, media_id: bytes) -> list[bytes]:
    if len(payload) <= CHUNK_THRESHOLD:
        return [encode_frame(ftype, payload, meta, 0, media_id, FLAG_LAST)]
    frames = []
    n = (len(payload) + CHUNK_SIZE - 1) // CHUNK_SIZE
    for i in range(n):
        part = payload[i * CHUNK_SIZE:(i + 1) * CHUNK_SIZE]
        fl = FLAG_CHUNKED | (FLAG_LAST if i == n - 1 else 0)
        frames.append(encode_frame(ftype, part, meta if i == 0 else None, i, media_id, fl))
    return frames
