"""Fuzz the facade's client-message parser (facade/protocol.py): any input
either parses into a message whose fields have the types the handlers read
(facade/server.py on_message, facade/handlers.py) or raises ValueError -- which
the server answers with E_INVALID_MESSAGE -- never another exception that would
end the connection's receive loop.  Binary media frames round-trip."""
import json

from hypothesis import given, settings
from hypothesis import strategies as st

from omnia_amd.facade import protocol as P

JSON = st.recursive(st.none() | st.booleans() | st.integers() | st.floats(allow_nan=False)
                    | st.text(max_size=8),
                    lambda c: st.lists(c, max_size=4) | st.dictionaries(st.text(max_size=6), c,
                                                                         max_size=4),
                    max_leaves=12)
FIELDS = ["session_id", "content", "metadata", "consent_grants", "parts", "tool_result",
          "tool_call_ack", "tool_call_nack", "upload_request"]


@given(st.sampled_from(sorted(P.CLIENT_TYPES) + ["bogus", None]),
       st.dictionaries(st.sampled_from(FIELDS), JSON, max_size=5))
@settings(max_examples=400, deadline=None)
def test_parse_client_accepts_well_typed_or_raises_value_error(typ, fields):
    raw = json.dumps({"type": typ, **fields})
    try:
        m = P.parse_client(raw)
    except ValueError:
        return
    # what the handlers do with a parsed message must not raise
    for k in ("tool_result", "tool_call_ack", "tool_call_nack", "upload_request"):
        (m.get(k) or {}).get("call_id", "")
    {str(k): str(v) for k, v in (m.get("metadata") or {}).items()}
    list(m.get("consent_grants") or [])
    for p in m.get("parts") or []:
        p.get("type", "text"), p.get("text", "")
        media = p.get("media") or {}
        for k in ("data", "url", "mime_type", "storage_ref"):
            assert isinstance(media.get(k, ""), str)


@given(st.binary(max_size=200))
@settings(max_examples=300, deadline=None)
def test_parse_client_on_garbage_bytes(raw):
    try:
        P.parse_client(raw)
    except ValueError:
        pass


def test_parse_client_deep_nesting_is_invalid_not_a_crash():
    raw = '{"type": "message", "content": "x", "metadata": {"a": ' + "[" * 100000 + \
        "]" * 100000 + "}}"
    try:
        P.parse_client(raw)
    except ValueError:
        pass


@given(st.binary(max_size=3000), st.dictionaries(st.text(max_size=5), st.integers(), max_size=3),
       st.integers(0, 2**31 - 1), st.binary(max_size=12))
@settings(max_examples=200, deadline=None)
def test_media_frames_round_trip(payload, meta, seq, mid):
    f = P.decode_frame(P.encode_frame(P.TYPE_UPLOAD, payload, meta, seq, mid, P.FLAG_LAST))
    assert f["payload"] == payload and f["meta"] == meta and f["seq"] == seq
    assert f["media_id"] == mid[:12].rstrip(b"\0")


@given(st.binary(max_size=100))
@settings(max_examples=300, deadline=None)
def test_decode_frame_garbage_raises_value_error(buf):
    try:
        P.decode_frame(P.MAGIC + buf)
    except ValueError:
        pass
