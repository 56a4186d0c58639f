"""ConstDB op-stream ORACLE — test infrastructure only.

A CPU restatement of the reference's partial-replication apply path: the RESP messages a
Puller receives after the snapshot (``replica/pull.rs:160-235``) and the write-command
handlers they run (``cmd.rs``, ``type_counter.rs``, ``type_set.rs``, ``type_hash.rs``) on top
of the DB that the snapshot fold produced (``constdb_oracle.DB``). Like
``constdb_oracle``, only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s CPU
baseline may import it, and only as the checker.

Parity pinning: the reference has no test that applies a replicate stream (its only
integration test, ``bin/test.rs``, needs live servers), so this restatement is pinned by
hand-derived known-answer tests (``tests/test_ops_oracle.py``), "pinned by restatement +
KATs", like the merge fold. RESP framing follows ``conn/buf_read.rs:114-210`` and
``conn/buf_write.rs:127-160``; ``bytes2i64`` follows ``lib/utils.rs:3-28`` (wrapping).
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import List, Optional, Tuple

from constdb_oracle import (DB, Counter, Dict, Object, Set, OBJECT_ENC_BYTES, OBJECT_ENC_COUNTER,
                            OBJECT_ENC_DICT, OBJECT_ENC_SET, to_i64, to_u64)


class InvalidRequestMsg(Exception):
    """CstError::InvalidRequestMsg (lib.rs) raised by the RESP reader; offset = message start."""

    def __init__(self, offset: int, why: str):
        super().__init__(f"{why} at {offset}")
        self.offset = offset


# --------------------------------------------------------------------------------------
# RESP (conn/buf_read.rs, conn/buf_write.rs). Messages are tuples (kind, payload):
# ("str", b) "+", ("err", b) "-", ("int", i) ":", ("bulk", b) "$", ("nil", None) "$-1",
# ("arr", [..]) "*".
# --------------------------------------------------------------------------------------
def bytes2i64(b: bytes) -> Optional[int]:  # lib/utils.rs:3-28 (release build: wrapping)
    if len(b) == 0:
        return None
    result, invalid, negative = 0, True, False
    for i, c in enumerate(b):
        if i == 0 and c == 0x2D:
            negative = True
            continue
        if 0x30 <= c <= 0x39:
            invalid = False
            result = to_i64(result * 10 + (c - 0x30))
        else:
            break
    if invalid:
        return None
    return to_i64(-result) if negative else result


def get_int_bytes(n: int) -> bytes:  # resp.rs:20-26
    return str(n).encode()


def resp_encode(msg) -> bytes:  # buf_write.rs:127-150
    kind, v = msg
    if kind == "nil":
        return b"$-1\r\n"
    if kind == "bulk":
        return b"$" + str(len(v)).encode() + b"\r\n" + v + b"\r\n"
    if kind == "err":
        return b"-" + v + b"\r\n"
    if kind == "str":
        return b"+" + v + b"\r\n"
    if kind == "int":
        return b":" + str(v).encode() + b"\r\n"
    if kind == "arr":
        return b"*" + str(len(v)).encode() + b"\r\n" + b"".join(resp_encode(m) for m in v)
    raise ValueError(kind)


def _until_crlf(buf: bytes, cur: int) -> int:  # buf_read.rs:202-210: index of the '\n'
    i = buf.find(b"\r\n", cur)
    if i < 0:
        raise EOFError
    return i + 1


def _parse(buf: bytes, cur: int):  # buf_read.rs:114-171 -> (msg, size)
    if cur >= len(buf):
        raise EOFError
    t = buf[cur]
    if t == 0x2B or t == 0x2D:  # '+' '-'
        s = _until_crlf(buf, cur + 1)
        return ("str" if t == 0x2B else "err", buf[cur + 1:s - 1]), s - cur + 1
    if t == 0x3A:  # ':'
        s = _until_crlf(buf, cur + 1)
        i = bytes2i64(buf[cur + 1:s - 1])
        if i is None:
            raise ValueError("the ':' should be followed by an integer")
        return ("int", i), s - cur + 1
    if t == 0x24:  # '$'  read_bulk_string, buf_read.rs:173-200
        he = _until_crlf(buf, cur + 1)
        n = bytes2i64(buf[cur + 1:he - 1])
        if n is None:
            raise ValueError("the '$' should be followed by an integer")
        if n == -1:
            return ("nil", None), 5
        if n < 0:
            raise ValueError("invalid bulk string")
        se = _until_crlf(buf, he)
        if se - he != n + 2:
            raise ValueError("bulk string has wrong value of length")
        return ("bulk", buf[he + 1:se - 1]), se - cur + 1
    if t == 0x2A:  # '*'
        le = _until_crlf(buf, cur + 1)
        n = bytes2i64(buf[cur + 1:le - 1])
        if n is None:
            raise ValueError("the '*' should be followed by an integer")
        if n < 0:  # Vec::with_capacity(negative as usize) aborts the reference; an error here
            raise ValueError("negative array length")
        args, sub = [], le + 1
        for _ in range(n):
            m, sz = _parse(buf, sub)
            args.append(m)
            sub += sz
        return ("arr", args), sub - cur
    raise ValueError(f"unknown resp type {t}")


def resp_parse_stream(buf: bytes) -> List[tuple]:
    """Every complete message of `buf`, in order. A malformed message raises
    InvalidRequestMsg(offset); a truncated tail raises InvalidRequestMsg too (the reader
    would wait for more bytes, but a batch is complete by contract)."""
    out, cur = [], 0
    while cur < len(buf):
        try:
            m, sz = _parse(buf, cur)
        except EOFError:
            raise InvalidRequestMsg(cur, "truncated message")
        except ValueError as e:
            raise InvalidRequestMsg(cur, str(e))
        out.append(m)
        cur += sz
    return out


class _Args:
    """NextArg over an argument iterator (cmd.rs:348-397); every call consumes one arg."""

    def __init__(self, args):
        self.a = list(args)
        self.i = 0

    def next_arg(self):
        if self.i >= len(self.a):
            raise _CmdError("WrongArity")
        m = self.a[self.i]
        self.i += 1
        return m

    def next_bytes(self) -> bytes:  # cmd.rs:364-372
        k, v = self.next_arg()
        if k == "int":
            return get_int_bytes(v)
        if k in ("err", "str", "bulk"):
            return v
        raise _CmdError("should be non-array type")

    def next_i64(self) -> int:  # cmd.rs:374-381
        k, v = self.next_arg()
        if k == "int":
            return v
        if k in ("str", "bulk"):
            i = bytes2i64(v)
            if i is None:
                raise _CmdError("should be an integer")
            return i
        raise _CmdError("argument should be of type Integer or String or BulkString")

    def next_u64(self) -> int:  # cmd.rs:383-392
        i = self.next_i64()
        if i < 0:
            raise _CmdError("argument should be an unsigned integer")
        return i


class _CmdError(Exception):
    pass


# --------------------------------------------------------------------------------------
# Object / DB helpers the handlers use
# --------------------------------------------------------------------------------------
def updated_at(o: Object, uuid: int) -> None:  # object.rs:35-49
    if o.update_time < uuid:
        o.update_time = uuid
    if o.create_time < o.delete_time:
        if uuid < o.create_time:
            pass
        elif o.create_time <= uuid < o.delete_time:
            pass
        else:
            o.create_time = uuid  # created again


def query(db: DB, key: bytes, t: int) -> Optional[Object]:  # db.rs:52-66
    o = db.data.get(key)
    if o is None:
        return None
    e = db.expires.get(key)
    if e is not None:
        if o.create_time >= o.delete_time and o.create_time < e and e <= t:  # alive, created_before
            o.delete_time = e
            updated_at(o, e)
            db.deletes[key] = e
    return o


def counter_change(c: Counter, actor: int, value: int, uuid: int) -> None:  # type_counter.rs:37-51
    cur = c.data.get(actor)
    if cur is None:
        c.data[actor] = (value, uuid)
        c.sum = to_i64(c.sum + value)
    else:
        v, t = cur
        if t < uuid:
            c.data[actor] = (to_i64(v + value), t)
            c.sum = to_i64(c.sum + value)


def _query_or_create(db: DB, key: bytes, uuid: int, make) -> Object:
    o = query(db, key, uuid)
    if o is None:  # Object::new(enc, uuid, 0): ct = uuid, ut = 0, dt = 0 (object.rs:25-32)
        tag, enc = make()
        o = Object(uuid, 0, 0, tag, enc)
        db.data[key] = o
    return o


def _new_counter():
    return OBJECT_ENC_COUNTER, Counter()


def _new_set():
    return OBJECT_ENC_SET, Set()


def _new_dict():
    return OBJECT_ENC_DICT, Dict()


# --------------------------------------------------------------------------------------
# Write-command handlers (nodeid = the replicate message's node id, uuid = current_uuid)
# --------------------------------------------------------------------------------------
def set_command(db, nodeid, uuid, args):  # cmd.rs:188-210
    key = args.next_bytes()
    value = args.next_bytes()
    o = _query_or_create(db, key, uuid, lambda: (OBJECT_ENC_BYTES, value))
    if o.update_time > uuid:
        return
    if o.tag != OBJECT_ENC_BYTES:
        raise _CmdError("InvalidType")
    o.enc = value
    updated_at(o, uuid)


def delbytes_command(db, nodeid, uuid, args):  # cmd.rs:290-309
    key = args.next_bytes()
    o = _query_or_create(db, key, uuid, lambda: (OBJECT_ENC_BYTES, b""))
    if o.tag != OBJECT_ENC_BYTES:
        raise _CmdError("InvalidType")
    o.delete_time = max(o.delete_time, uuid)
    o.update_time = max(o.update_time, uuid)


def _incr_by(db, nodeid, uuid, args, d):  # type_counter.rs:169-204
    key = args.next_bytes()
    o = _query_or_create(db, key, uuid, _new_counter)
    if o.tag != OBJECT_ENC_COUNTER:
        raise _CmdError("InvalidType")
    counter_change(o.enc, nodeid, d, uuid)
    updated_at(o, uuid)


def incr_command(db, nodeid, uuid, args):
    _incr_by(db, nodeid, uuid, args, 1)


def decr_command(db, nodeid, uuid, args):
    _incr_by(db, nodeid, uuid, args, -1)


def delcnt_command(db, nodeid, uuid, args):  # type_counter.rs:142-167
    key = args.next_bytes()
    o = _query_or_create(db, key, uuid, _new_counter)
    if o.tag != OBJECT_ENC_COUNTER:
        raise _CmdError("InvalidType")
    o.update_time = max(o.update_time, uuid)
    o.delete_time = max(o.delete_time, uuid)
    while True:
        try:
            node = args.next_u64()
        except _CmdError:
            break
        v = args.next_i64()  # an error here returns after the earlier pairs were applied
        counter_change(o.enc, node, v, uuid)


def _members(args) -> List[bytes]:
    out = []
    while True:
        try:
            out.append(args.next_bytes())
        except _CmdError:
            return out


def sadd_command(db, nodeid, uuid, args):  # type_set.rs:13-40
    key = args.next_bytes()
    members = _members(args)
    o = _query_or_create(db, key, uuid, _new_set)
    if o.tag != OBJECT_ENC_SET:
        raise _CmdError("InvalidType")
    for m in members:
        o.enc.set(m, None, uuid)
    if uuid < o.delete_time:
        for m in members:
            o.enc.rem(m, o.delete_time)
    updated_at(o, uuid)


def srem_command(db, nodeid, uuid, args):  # type_set.rs:42-63
    key = args.next_bytes()
    members = _members(args)
    o = _query_or_create(db, key, uuid, _new_set)
    if o.tag != OBJECT_ENC_SET:
        raise _CmdError("InvalidType")
    for m in members:
        o.enc.rem(m, uuid)
    updated_at(o, uuid)


def _del_all(db, uuid, args, tag, make):  # type_set.rs:115-134, type_hash.rs:100-119
    key = args.next_bytes()
    o = _query_or_create(db, key, uuid, make)
    if o.tag != tag:
        raise _CmdError("InvalidType")
    for m in list(o.enc.add) + list(o.enc.dele):  # iter_all: the add map, then the del map
        o.enc.rem(m, uuid)
    o.delete_time = max(o.delete_time, uuid)
    o.update_time = max(o.update_time, uuid)


def delset_command(db, nodeid, uuid, args):
    _del_all(db, uuid, args, OBJECT_ENC_SET, _new_set)


def deldict_command(db, nodeid, uuid, args):
    _del_all(db, uuid, args, OBJECT_ENC_DICT, _new_dict)


def hset_command(db, nodeid, uuid, args):  # type_hash.rs:11-45
    key = args.next_bytes()
    kvs = []
    while True:
        try:
            f = args.next_bytes()
        except _CmdError:
            break
        kvs.append((f, args.next_bytes()))  # odd count: WrongArity before the DB is touched
    o = _query_or_create(db, key, uuid, _new_dict)
    if o.tag != OBJECT_ENC_DICT:
        raise _CmdError("InvalidType")
    for f, v in kvs:
        o.enc.set(f, v, uuid)
    if uuid < o.delete_time:
        for f, _ in kvs:
            o.enc.rem(f, o.delete_time)
    updated_at(o, uuid)


def hdel_command(db, nodeid, uuid, args):  # type_hash.rs:47-68
    key = args.next_bytes()
    fields = _members(args)
    o = _query_or_create(db, key, uuid, _new_dict)
    if o.tag != OBJECT_ENC_DICT:
        raise _CmdError("InvalidType")
    for f in fields:
        o.enc.rem(f, uuid)
    updated_at(o, uuid)


HANDLERS = {
    b"set": set_command, b"delbytes": delbytes_command, b"incr": incr_command, b"decr": decr_command,
    b"delcnt": delcnt_command, b"sadd": sadd_command, b"srem": srem_command, b"delset": delset_command,
    b"hset": hset_command, b"hdel": hdel_command, b"deldict": deldict_command,
}
# Commands in the reference's table (cmd.rs:97-133) that this path does not replay: spop picks
# a random member on the replica (type_set.rs:82-111, thread_rng_n, non-deterministic), `del`
# is never replicated (COMMAND_NO_REPLICATE), the rest are reads or server control.
UNSUPPORTED = {b"spop", b"del", b"node", b"replicas", b"sync", b"meet", b"client", b"repllog", b"info",
               b"get", b"desc", b"smembers", b"hget", b"hgetall"}


@dataclass
class ApplyStats:
    applied: int = 0        # replicate messages whose command ran (errors included)
    duplicates: int = 0     # uuid_he_sent > last_uuid (pull.rs:205-206)
    lost: int = 0           # uuid_he_sent < last_uuid (pull.rs:201-204) or a malformed replicate
    unknown: int = 0        # command not in the table (pull.rs:213-217)
    unsupported: int = 0    # in the table but not replayed here (UNSUPPORTED)
    cmd_errors: int = 0     # handler returned Err (pull.rs:219-221: logged, uuid advanced)
    replacks: int = 0
    uuid_he_sent: int = 0
    uuid_he_acked: int = 0


def apply_replicates(db: DB, stream: bytes, uuid_he_sent: int) -> ApplyStats:
    """Puller::apply_his_replicates over every message of `stream` in order
    (replica/pull.rs:160-235). A message that fails (lost commands, malformed) is dropped and
    the next one is tried: the reference pops it before it breaks, and the next main-loop visit
    continues with the following message."""
    st = ApplyStats(uuid_he_sent=uuid_he_sent)
    for kind, args in resp_parse_stream(stream):
        if kind != "arr":
            st.lost += 1
            continue
        a = _Args(args)
        try:
            name = a.next_bytes().lower()
        except _CmdError:
            st.lost += 1
            continue
        if name == b"replack":
            try:
                st.uuid_he_acked = a.next_u64()
                st.replacks += 1
            except _CmdError:
                st.lost += 1
            continue
        if name != b"replicate":
            st.lost += 1
            continue
        try:
            nodeid = a.next_u64()
            last_uuid = a.next_u64()
        except _CmdError:
            st.lost += 1
            continue
        if st.uuid_he_sent < last_uuid:
            st.lost += 1
            continue
        if st.uuid_he_sent > last_uuid:
            st.duplicates += 1
            continue
        try:
            current_uuid = a.next_u64()
            cmd = a.next_bytes().lower()
        except _CmdError:
            st.lost += 1
            continue
        rest = _Args(a.a[a.i:])
        h = HANDLERS.get(cmd)
        if h is None:
            if cmd in UNSUPPORTED:
                st.unsupported += 1
            else:
                st.unknown += 1
            st.uuid_he_sent = current_uuid
            continue
        try:
            h(db, nodeid, current_uuid, rest)
        except _CmdError:
            st.cmd_errors += 1
        st.applied += 1
        st.uuid_he_sent = current_uuid
    return st


# --------------------------------------------------------------------------------------
# Stream builders for tests and benches (what Server::repl_log_next sends, server.rs:290-314)
# --------------------------------------------------------------------------------------
def bulk(b) -> tuple:
    return ("bulk", b if isinstance(b, bytes) else str(b).encode())


def replicate_msg(nodeid: int, last_uuid: int, uuid: int, cmd: str, *args) -> bytes:
    items = [("bulk", b"replicate"), ("int", nodeid), ("int", last_uuid), ("int", uuid), ("bulk", cmd.encode())]
    for x in args:
        items.append(x if isinstance(x, tuple) else bulk(x))
    return resp_encode(("arr", items))


@dataclass
class StreamBuilder:
    """Builds a well-formed replicate stream: every message chains last_uuid -> uuid."""
    nodeid: int
    last_uuid: int
    parts: List[bytes] = field(default_factory=list)

    def cmd(self, uuid: int, name: str, *args) -> "StreamBuilder":
        self.parts.append(replicate_msg(self.nodeid, self.last_uuid, uuid, name, *args))
        self.last_uuid = uuid
        return self

    def raw(self, b: bytes) -> "StreamBuilder":
        self.parts.append(b)
        return self

    def bytes(self) -> bytes:
        return b"".join(self.parts)
