"""Minimal Redis (RESP2) asyncio client + an in-process Redis-compatible server.

The reference uses go-redis for the runtime context store
(``pkg/runtime/promptkit/serveropts.go:93-130``), the session hot tier, the A2A
task store, the facade route table and Redis Streams (eval / memory events,
arena work queue).  The ``redis`` package is not installed here, so this
module speaks RESP directly.  ``MiniRedis`` (cf. miniredis in the reference's
tests) implements the command subset we use -- strings with TTL, hashes,
lists, sorted-set-free streams with consumer groups -- so every Redis-backed
path is testable without a server.
"""
from __future__ import annotations

import asyncio
import fnmatch
import itertools
import time


class RedisError(Exception):
    pass


# ------------------------------------------------------------------ protocol
def encode(*args) -> bytes:
    out = [b"*%d\r\n" % len(args)]
    for a in args:
        if isinstance(a, bytes):
            b = a
        elif isinstance(a, str):
            b = a.encode()
        else:
            b = str(a).encode()
        out.append(b"$%d\r\n%s\r\n" % (len(b), b))
    return b"".join(out)


async def read_reply(r: asyncio.StreamReader):
    line = await r.readline()
    if not line:
        raise ConnectionError("redis connection closed")
    t, body = line[:1], line[1:-2]
    if t == b"+":
        return body.decode()
    if t == b"-":
        raise RedisError(body.decode())
    if t == b":":
        return int(body)
    if t == b"$":
        n = int(body)
        if n < 0:
            return None
        data = await r.readexactly(n + 2)
        return data[:-2]
    if t == b"*":
        n = int(body)
        if n < 0:
            return None
        return [await read_reply(r) for _ in range(n)]
    raise RedisError(f"bad reply type {t!r}")


def _enc_reply(v) -> bytes:
    if v is None:
        return b"$-1\r\n"
    if isinstance(v, bool):
        return b":%d\r\n" % int(v)
    if isinstance(v, int):
        return b":%d\r\n" % v
    if isinstance(v, _Status):
        return b"+%s\r\n" % v.s.encode()
    if isinstance(v, _Err):
        return b"-%s\r\n" % v.s.encode()
    if isinstance(v, (bytes, str)):
        b = v if isinstance(v, bytes) else v.encode()
        return b"$%d\r\n%s\r\n" % (len(b), b)
    if isinstance(v, list):
        return b"*%d\r\n" % len(v) + b"".join(_enc_reply(x) for x in v)
    raise TypeError(type(v))


class _Status:
    def __init__(self, s):
        self.s = s


class _Err:
    def __init__(self, s):
        self.s = s


OK = _Status("OK")


# ------------------------------------------------------------------ client
class RedisClient:
    """Tiny pooled-by-lock asyncio client.  URL: redis://[:password@]host:port[/db]."""

    def __init__(self, url: str = "redis://127.0.0.1:6379/0", timeout: float = 5.0):
        self.url = url
        self.timeout = timeout
        rest = url.split("://", 1)[-1]
        self.password = None
        if "@" in rest:
            cred, rest = rest.rsplit("@", 1)
            self.password = cred.split(":", 1)[-1] or None
        hostport, _, db = rest.partition("/")
        host, _, port = hostport.partition(":")
        self.host, self.port = host or "127.0.0.1", int(port or 6379)
        self.db = int(db or 0)
        self._rw = None
        self._lock = asyncio.Lock()

    async def _conn(self):
        if self._rw is None:
            r, w = await asyncio.wait_for(asyncio.open_connection(self.host, self.port),
                                          self.timeout)
            self._rw = (r, w)
            if self.password:
                await self._raw("AUTH", self.password)
            if self.db:
                await self._raw("SELECT", self.db)
        return self._rw

    async def _raw(self, *args):
        r, w = self._rw
        w.write(encode(*args))
        await w.drain()
        return await asyncio.wait_for(read_reply(r), self.timeout)

    async def execute(self, *args):
        async with self._lock:
            try:
                await self._conn()
                return await self._raw(*args)
            except RedisError:
                raise  # a complete error reply: the connection stays in sync
            except BaseException:
                # connection lost, or a timeout / cancellation with the reply still
                # outstanding: that late reply would answer the NEXT command on this
                # connection, so drop it (the next command reconnects)
                self.close()
                raise

    def close(self):
        if self._rw is not None:
            try:
                self._rw[1].close()
            except Exception:
                pass
            self._rw = None

    # convenience
    async def ping(self):
        return await self.execute("PING")

    async def get(self, k):
        return await self.execute("GET", k)

    async def set(self, k, v, ex: int | None = None):
        if ex:
            return await self.execute("SET", k, v, "EX", int(ex))
        return await self.execute("SET", k, v)

    async def delete(self, *ks):
        return await self.execute("DEL", *ks)

    async def exists(self, k) -> bool:
        return bool(await self.execute("EXISTS", k))

    async def expire(self, k, s):
        return await self.execute("EXPIRE", k, int(s))

    async def xadd(self, stream, fields: dict, maxlen: int | None = None):
        args = ["XADD", stream]
        if maxlen:
            args += ["MAXLEN", "~", maxlen]
        args.append("*")
        for k, v in fields.items():
            args += [k, v]
        return await self.execute(*args)

    async def xgroup_create(self, stream, group, start="0"):
        try:
            return await self.execute("XGROUP", "CREATE", stream, group, start, "MKSTREAM")
        except RedisError as e:
            if "BUSYGROUP" not in str(e):
                raise

    async def xreadgroup(self, group, consumer, streams: dict, count=10, block_ms=None):
        args = ["XREADGROUP", "GROUP", group, consumer, "COUNT", count]
        if block_ms is not None:
            args += ["BLOCK", block_ms]
        args.append("STREAMS")
        args += list(streams.keys()) + list(streams.values())
        return await self.execute(*args)

    async def xack(self, stream, group, *ids):
        return await self.execute("XACK", stream, group, *ids)

    async def publish(self, channel, message) -> int:
        return await self.execute("PUBLISH", channel, message)

    async def subscribe(self, *channels) -> "Subscription":
        """A dedicated connection in subscribe mode.  Returns once the server
        confirmed every channel, so a PUBLISH issued after this cannot be lost."""
        sub = Subscription(self)
        await sub.open(*channels)
        return sub


class Subscription:
    """``async for channel, payload in sub`` over a SUBSCRIBE connection."""

    def __init__(self, client: RedisClient):
        self.c = client
        self._rw = None

    async def open(self, *channels):
        c = self.c
        r, w = await asyncio.wait_for(asyncio.open_connection(c.host, c.port), c.timeout)
        self._rw = (r, w)
        if c.password:
            w.write(encode("AUTH", c.password))
            await w.drain()
            await read_reply(r)
        w.write(encode("SUBSCRIBE", *channels))
        await w.drain()
        for _ in channels:
            await asyncio.wait_for(read_reply(r), c.timeout)  # ["subscribe", ch, n]

    async def get(self, timeout: float | None = None):
        """Next (channel, payload) message, or None on timeout / close."""
        r, _ = self._rw
        while True:
            try:
                m = await asyncio.wait_for(read_reply(r), timeout)
            except asyncio.TimeoutError:
                return None
            except (ConnectionError, asyncio.IncompleteReadError):
                return None
            if isinstance(m, list) and len(m) == 3 and m[0] in (b"message", "message"):
                ch, pl = m[1], m[2]
                return (ch.decode() if isinstance(ch, bytes) else ch,
                        pl.decode() if isinstance(pl, bytes) else pl)

    def __aiter__(self):
        return self

    async def __anext__(self):
        m = await self.get()
        if m is None:
            raise StopAsyncIteration
        return m

    def close(self):
        if self._rw is not None:
            try:
                self._rw[1].close()
            except Exception:
                pass
            self._rw = None


# ------------------------------------------------------------------ server
class MiniRedis:
    """In-process Redis-compatible server for tests and single-node mode."""

    def __init__(self):
        self.data: dict[bytes, object] = {}
        self.exp: dict[bytes, float] = {}
        self.streams: dict[bytes, list] = {}
        self.groups: dict[bytes, dict] = {}
        self._seq = itertools.count(1)
        self.server = None
        self.port = 0
        self.subs: dict[bytes, set] = {}  # channel -> subscribed connection writers

    async def start(self, host="127.0.0.1", port=0):
        self.server = await asyncio.start_server(self._handle, host, port, backlog=1024)
        self.port = self.server.sockets[0].getsockname()[1]
        return self

    @property
    def url(self) -> str:
        return f"redis://127.0.0.1:{self.port}/0"

    async def stop(self):
        if self.server:
            self.server.close()
            await self.server.wait_closed()

    def _alive(self, k):
        e = self.exp.get(k)
        if e is not None and e <= time.time():
            self.data.pop(k, None)
            self.exp.pop(k, None)
        return k in self.data

    async def _handle(self, r, w):
        mine: set = set()
        try:
            while True:
                req = await read_reply(r)
                if not isinstance(req, list) or not req:
                    break
                a = [x if isinstance(x, bytes) else str(x).encode() for x in req]
                if a[0].upper() in (b"SUBSCRIBE", b"UNSUBSCRIBE"):
                    sub = a[0].upper() == b"SUBSCRIBE"
                    for ch in a[1:]:
                        (self.subs.setdefault(ch, set()).add if sub else
                         self.subs.setdefault(ch, set()).discard)(w)
                        (mine.add if sub else mine.discard)(ch)
                        w.write(_enc_reply([a[0].lower(), ch, len(mine)]))
                    await w.drain()
                    continue
                try:
                    out = self.dispatch(a)
                except Exception as e:  # noqa: BLE001
                    out = _Err(f"ERR {e}")
                w.write(_enc_reply(out))
                await w.drain()
        except (ConnectionError, asyncio.IncompleteReadError):
            pass
        finally:
            for ch in mine:
                self.subs.get(ch, set()).discard(w)
            w.close()

    def c_publish(self, a):
        ch, msg = a[0], a[1]
        n = 0
        for w in list(self.subs.get(ch, ())):
            try:
                w.write(_enc_reply([b"message", ch, msg]))
                n += 1
            except Exception:  # noqa: BLE001 - a subscriber went away
                self.subs[ch].discard(w)
        return n

    def dispatch(self, a: list[bytes]):
        cmd = a[0].upper().decode()
        f = getattr(self, "c_" + cmd.lower(), None)
        if f is None:
            return _Err(f"ERR unknown command '{cmd}'")
        return f(a[1:])

    # --- strings / keys
    def c_ping(self, a):
        return _Status("PONG")

    def c_auth(self, a):
        return OK

    def c_select(self, a):
        return OK

    def c_set(self, a):
        k, v = a[0], a[1]
        self.data[k] = v
        self.exp.pop(k, None)
        i = 2
        while i < len(a):
            opt = a[i].upper()
            if opt == b"EX":
                self.exp[k] = time.time() + int(a[i + 1])
                i += 2
            elif opt == b"PX":
                self.exp[k] = time.time() + int(a[i + 1]) / 1000
                i += 2
            else:
                i += 1
        return OK

    def c_get(self, a):
        return self.data.get(a[0]) if self._alive(a[0]) else None

    def c_del(self, a):
        n = 0
        for k in a:
            if self._alive(k):
                n += 1
            self.data.pop(k, None)
            self.exp.pop(k, None)
            self.streams.pop(k, None)
        return n

    def c_exists(self, a):
        return sum(1 for k in a if self._alive(k) or k in self.streams)

    def c_expire(self, a):
        if not self._alive(a[0]):
            return 0
        self.exp[a[0]] = time.time() + int(a[1])
        return 1

    def c_ttl(self, a):
        if not self._alive(a[0]):
            return -2
        e = self.exp.get(a[0])
        return -1 if e is None else int(e - time.time())

    def c_keys(self, a):
        pat = a[0].decode()
        return [k for k in list(self.data) if self._alive(k) and fnmatch.fnmatch(k.decode(), pat)]

    def c_incr(self, a):
        v = int(self.data.get(a[0], b"0")) + 1 if self._alive(a[0]) else 1
        self.data[a[0]] = str(v).encode()
        return v

    # --- hashes
    def c_hset(self, a):
        h = self.data.setdefault(a[0], {})
        n = 0
        for i in range(1, len(a), 2):
            n += a[i] not in h
            h[a[i]] = a[i + 1]
        return n

    def c_hincrby(self, a):
        h = self.data.setdefault(a[0], {})
        v = int(h.get(a[1], b"0")) + int(a[2])
        h[a[1]] = str(v).encode()
        return v

    def c_hget(self, a):
        h = self.data.get(a[0]) if self._alive(a[0]) else None
        return None if not isinstance(h, dict) else h.get(a[1])

    def c_hgetall(self, a):
        h = self.data.get(a[0]) if self._alive(a[0]) else None
        if not isinstance(h, dict):
            return []
        return [x for kv in h.items() for x in kv]

    def c_hdel(self, a):
        h = self.data.get(a[0])
        if not isinstance(h, dict):
            return 0
        return sum(1 for f in a[1:] if h.pop(f, None) is not None)

    # --- lists
    def c_rpush(self, a):
        lst = self.data.setdefault(a[0], [])
        lst.extend(a[1:])
        return len(lst)

    def c_lrange(self, a):
        lst = self.data.get(a[0]) if self._alive(a[0]) else None
        if not isinstance(lst, list):
            return []
        s, e = int(a[1]), int(a[2])
        e = len(lst) if e == -1 else e + 1
        return lst[s:e]

    def c_llen(self, a):
        lst = self.data.get(a[0])
        return len(lst) if isinstance(lst, list) else 0

    # --- streams
    def c_xadd(self, a):
        k = a[0]
        i = 1
        maxlen = None
        if a[i].upper() == b"MAXLEN":
            i += 1
            if a[i] in (b"~", b"="):
                i += 1
            maxlen = int(a[i])
            i += 1
        i += 1  # '*'
        sid = f"{int(time.time() * 1000)}-{next(self._seq)}".encode()
        fields = a[i:]
        st = self.streams.setdefault(k, [])
        st.append((sid, fields))
        if maxlen and len(st) > maxlen:
            del st[: len(st) - maxlen]
        return sid

    def c_xlen(self, a):
        return len(self.streams.get(a[0], []))

    def c_xrange(self, a):
        return [[sid, list(f)] for sid, f in self.streams.get(a[0], [])]

    def c_xgroup(self, a):
        sub = a[0].upper()
        if sub == b"CREATE":
            k, g = a[1], a[2]
            gs = self.groups.setdefault(k, {})
            if g in gs:
                return _Err("BUSYGROUP Consumer Group name already exists")
            self.streams.setdefault(k, [])
            start = a[3]
            last = len(self.streams[k]) if start == b"$" else 0
            gs[g] = {"last": last, "pending": {}}
            return OK
        return _Err("ERR unsupported XGROUP subcommand")

    def c_xreadgroup(self, a):
        # GROUP g c [COUNT n] [BLOCK ms] STREAMS k... id...
        g, c = a[1], a[2]
        i = 3
        count = 10
        while a[i].upper() != b"STREAMS":
            if a[i].upper() == b"COUNT":
                count = int(a[i + 1])
            i += 2
        rest = a[i + 1:]
        keys, ids = rest[: len(rest) // 2], rest[len(rest) // 2:]
        out = []
        for k, sid in zip(keys, ids):
            grp = self.groups.get(k, {}).get(g)
            if grp is None:
                return _Err("NOGROUP No such key or consumer group")
            st = self.streams.get(k, [])
            if sid == b">":
                batch = st[grp["last"]: grp["last"] + count]
                grp["last"] += len(batch)
                for e in batch:
                    grp["pending"][e[0]] = (c, time.time(), e)
            else:
                batch = [p[2] for p in grp["pending"].values() if p[0] == c][:count]
            if batch:
                out.append([k, [[e[0], list(e[1])] for e in batch]])
        return out or None

    def c_xack(self, a):
        grp = self.groups.get(a[0], {}).get(a[1])
        if grp is None:
            return 0
        return sum(1 for i in a[2:] if grp["pending"].pop(i, None) is not None)

    def c_xpending(self, a):
        grp = self.groups.get(a[0], {}).get(a[1])
        return [len(grp["pending"]) if grp else 0, None, None, []]

    def c_xclaim(self, a):
        # XCLAIM k g consumer min-idle id...
        grp = self.groups.get(a[0], {}).get(a[1])
        if grp is None:
            return []
        c, min_idle = a[2], int(a[3]) / 1000
        out = []
        now = time.time()
        for i in a[4:]:
            p = grp["pending"].get(i)
            if p and now - p[1] >= min_idle:
                grp["pending"][i] = (c, now, p[2])
                out.append([p[2][0], list(p[2][1])])
        return out

    def c_xautoclaim(self, a):
        # XAUTOCLAIM k g consumer min-idle start [COUNT n]
        grp = self.groups.get(a[0], {}).get(a[1])
        if grp is None:
            return _Err("NOGROUP No such key or consumer group")
        c, min_idle = a[2], int(a[3]) / 1000
        count = 100
        if len(a) > 6 and a[5].upper() == b"COUNT":
            count = int(a[6])
        now = time.time()
        out = []
        for i, p in list(grp["pending"].items()):
            if len(out) >= count:
                break
            if now - p[1] >= min_idle:
                grp["pending"][i] = (c, now, p[2])
                out.append([p[2][0], list(p[2][1])])
        return [b"0-0", out, []]

    def c_flushall(self, a):
        self.data.clear()
        self.exp.clear()
        self.streams.clear()
        self.groups.clear()
        return OK
