"""Property tests of the token-streaming path: the incremental UTF-8
detokenizer (engine/tokenizer.py) and the TP command ring (engine/tp.py).

* Streaming a token sequence piece by piece and flushing yields exactly the
  one-shot decode (invalid bytes as U+FFFD), and never holds back more than an
  incomplete multi-byte sequence (<= 3 bytes) -- the frames-per-token check of
  bench.py relies on that.
* The shared-memory ring delivers every command, header and payload intact
  and in order to every reader, whatever the interleaving of puts and gets
  (within its slot count)."""
import os

import numpy as np
from hypothesis import given, settings
from hypothesis import strategies as st

from omnia_amd.engine.tokenizer import Detokenizer, SyntheticTokenizer

TOK = SyntheticTokenizer(512, 300, (301,))
# byte tokens (incl. lead / continuation / invalid bytes), pseudo-words, specials
IDS = st.one_of(st.integers(0, 255), st.integers(256, 511),
                st.sampled_from([0xC3, 0xA9, 0xE2, 0x82, 0xAC, 0xF0, 0x9F, 0x98, 0x80]))


@given(st.lists(IDS, max_size=120))
@settings(max_examples=400, deadline=None)
def test_incremental_detokenizer_equals_one_shot_decode(ids):
    d = Detokenizer(TOK)
    parts = [d.push(t) for t in ids]
    parts.append(d.flush())
    assert "".join(parts) == TOK.decode(ids)


@given(st.lists(IDS, min_size=1, max_size=80))
@settings(max_examples=300, deadline=None)
def test_detokenizer_holds_back_at_most_one_partial_character(ids):
    d = Detokenizer(TOK)
    out = "".join(d.push(t) for t in ids)
    full = TOK.decode(ids)
    # what is still held is a suffix of the stream worth at most one character
    # (an incomplete code point: a lead byte + up to two continuation bytes)
    assert full.startswith(out)
    assert len(full) - len(out) <= 1


@given(st.lists(st.tuples(st.integers(0, 7), st.integers(0, 2000)), min_size=1, max_size=60),
       st.integers(1, 3), st.integers(2, 5))
@settings(max_examples=60, deadline=None)
def test_shm_ring_delivers_in_order_to_every_reader(cmds, readers, nslots):
    from omnia_amd.engine.tp import ShmRing

    path = f"/dev/shm/omnia-ring-prop-{os.getpid()}"
    w = ShmRing(path, True, nslots=nslots, payload=2048, readers=readers)
    rs = [ShmRing(path, False, reader=r) for r in range(readers)]
    got = [[] for _ in range(readers)]
    try:
        sent = []
        for i, (cmd, n) in enumerate(cmds):
            # drain readers whenever the ring is full (a put would wait)
            while int(w.ctrl[0]) - int(w.ctrl[8:8 + readers].min()) >= nslots:
                for r, ring in enumerate(rs):
                    if int(ring.ctrl[8 + r]) < int(ring.ctrl[0]):
                        h, body = ring.get(r)
                        got[r].append((h[0], h[1], bytes(body)))
                        ring.done(r)
            payload = np.full(n, i % 251, dtype=np.uint8)
            w.put([cmd, i], payload)
            sent.append((cmd, i, payload.tobytes()))
        for r, ring in enumerate(rs):
            while int(ring.ctrl[8 + r]) < int(ring.ctrl[0]):
                h, body = ring.get(r)
                got[r].append((h[0], h[1], bytes(body)))
                ring.done(r)
        for r in range(readers):
            assert got[r] == sent
    finally:
        for ring in rs:
            ring.close()
        w.close(unlink=True)
