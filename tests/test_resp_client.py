"""RESP client robustness: a command that times out or is cancelled while its
reply is outstanding must not leave that reply on the connection for the next
command to read (the client drops the connection instead), while an error
reply -- a complete reply -- keeps the connection."""
import asyncio

import pytest

from omnia_amd.utils.resp import RedisClient, RedisError, encode, read_reply


async def _slow_echo_server(delays: dict):
    """Replies to the i-th request the server receives (over all connections)
    with its second argument after delays.get(i, 0) s; ``ERR`` as the argument
    answers with an error reply."""
    conns = {"n": 0, "req": 0}

    async def handle(r, w):
        conns["n"] += 1
        try:
            while True:
                req = await read_reply(r)
                i = conns["req"]
                conns["req"] += 1
                await asyncio.sleep(delays.get(i, 0.0))
                arg = req[1]
                if arg == b"ERR":
                    w.write(b"-ERR boom\r\n")
                else:
                    w.write(b"$%d\r\n%s\r\n" % (len(arg), arg))
                await w.drain()
        except (ConnectionError, asyncio.IncompleteReadError):
            pass
        finally:
            w.close()

    srv = await asyncio.start_server(handle, "127.0.0.1", 0)
    return srv, srv.sockets[0].getsockname()[1], conns


def test_timeout_does_not_desynchronise_replies():
    async def run():
        srv, port, conns = await _slow_echo_server({0: 0.4})
        c = RedisClient(f"redis://127.0.0.1:{port}/0", timeout=0.1)
        with pytest.raises(asyncio.TimeoutError):
            await c.execute("ECHO", "first")
        # the late "first" reply must not answer this command
        assert await c.execute("ECHO", "second") == b"second"
        assert conns["n"] == 2  # the timed-out connection was dropped
        c.close()
        srv.close()

    asyncio.run(run())


def test_cancelled_command_does_not_desynchronise_replies():
    async def run():
        srv, port, _ = await _slow_echo_server({0: 0.3})
        c = RedisClient(f"redis://127.0.0.1:{port}/0", timeout=5.0)
        t = asyncio.ensure_future(c.execute("ECHO", "first"))
        await asyncio.sleep(0.05)
        t.cancel()
        with pytest.raises(asyncio.CancelledError):
            await t
        assert await c.execute("ECHO", "second") == b"second"
        c.close()
        srv.close()

    asyncio.run(run())


def test_error_reply_keeps_the_connection():
    async def run():
        srv, port, conns = await _slow_echo_server({})
        c = RedisClient(f"redis://127.0.0.1:{port}/0", timeout=1.0)
        with pytest.raises(RedisError):
            await c.execute("ECHO", "ERR")
        assert await c.execute("ECHO", "next") == b"next"
        assert conns["n"] == 1
        c.close()
        srv.close()

    asyncio.run(run())


def test_encode_roundtrip():
    async def run():
        r = asyncio.StreamReader()
        r.feed_data(encode("SET", b"k\r\n", 12, "v"))
        r.feed_eof()
        assert await read_reply(r) == [b"SET", b"k\r\n", b"12", b"v"]

    asyncio.run(run())
