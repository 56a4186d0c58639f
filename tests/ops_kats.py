"""Hand-derived known answers for the op-stream apply, shared by the oracle test
(CPU) and the GPU parity test. Each case: a state DB, a replicate stream, the uuid_he_sent the
stream starts from, and the canonical dump the reference's handlers produce, derived by hand
from the cited lines (not by running the oracle)."""
import constdb_oracle as o
import constdb_ops_oracle as oo


def _db(objs=None, expires=None, deletes=None):
    d = o.DB()
    d.data.update(objs or {})
    d.expires.update(expires or {})
    d.deletes.update(deletes or {})
    return d


def _snap(db):
    return o.dump_all(db, o.NodeHeader())


def _counter(nodes, ct=1, ut=0, dt=0):
    c = o.Counter()
    c.data.update(nodes)
    c.cal_sum()
    return o.Object(ct, ut, dt, o.OBJECT_ENC_COUNTER, c)


def _set(adds=None, dels=None, ct=1, ut=0, dt=0):
    s = o.Set()
    for m, t in (adds or {}).items():
        s.set(m, None, t)
    for m, t in (dels or {}).items():
        s.rem(m, t)
    return o.Object(ct, ut, dt, o.OBJECT_ENC_SET, s)


def h(b: bytes) -> str:
    return b.hex()


def cases():
    """(name, state snapshot bytes, stream bytes, uuid_he_sent, expected dump text)."""
    out = []

    # set on an absent key: Object::new(Bytes(v), uuid, 0) then updated_at(uuid) (cmd.rs:188-210)
    sb = oo.StreamBuilder(2, 5).cmd(10, "set", b"k", b"v")
    out.append(("set_creates", _snap(_db()), sb.bytes(), 5,
                f"K {h(b'k')} 3 10 10 0\n V {h(b'v')}\n"))

    # set rejected when update_time > uuid (no type check reached); accepted otherwise
    st = _db({b"k": o.Object(3, 20, 0, o.OBJECT_ENC_BYTES, b"old"), b"j": o.Object(3, 4, 0, o.OBJECT_ENC_BYTES, b"o")})
    sb = oo.StreamBuilder(2, 5).cmd(10, "set", b"k", b"new").cmd(11, "set", b"j", b"nj")
    out.append(("set_update_time", _snap(st), sb.bytes(), 5,
                f"K {h(b'j')} 3 3 11 0\n V {h(b'nj')}\n"
                f"K {h(b'k')} 3 3 20 0\n V {h(b'old')}\n"))

    # set on a counter: InvalidType, nothing changes
    st = _db({b"c": _counter({1: (4, 2)}, ct=2)})
    sb = oo.StreamBuilder(2, 5).cmd(10, "set", b"c", b"x")
    out.append(("set_type_error", _snap(st), sb.bytes(), 5,
                f"K {h(b'c')} 0 2 0 0\n S 4\n N 1 4 2\n"))

    # incr: Counter::change inserts (1, uuid) for the message's node; later ops add only when the
    # node's time < uuid; the time never moves (type_counter.rs:37-51)
    sb = oo.StreamBuilder(7, 5).cmd(10, "incr", b"c").cmd(12, "incr", b"c").cmd(10, "incr", b"c").cmd(9, "decr", b"c")
    out.append(("incr_fold", _snap(_db()), sb.bytes(), 5,
                f"K {h(b'c')} 0 10 12 0\n S 2\n N 7 2 10\n"))

    # delcnt: update/delete times max, then the pairs; a bad value after a node id errors after
    # the earlier pairs ran (type_counter.rs:142-167)
    st = _db({b"c": _counter({1: (5, 3), 2: (9, 3)}, ct=2, ut=3)})
    sb = oo.StreamBuilder(2, 5).cmd(7, "delcnt", b"c", ("int", 1), ("int", -5), ("int", 3), ("int", 4),
                                    ("int", 2), oo.bulk(b"x"))
    out.append(("delcnt_partial", _snap(st), sb.bytes(), 5,
                f"K {h(b'c')} 0 2 7 7\n S 13\n N 1 0 3\n N 2 9 3\n N 3 4 7\n"))

    # delset reaches only members present when it runs; a later sadd below the delete time is
    # re-deleted at it (type_set.rs:34-37); srem never is. The sadd at 12 >= the delete time
    # recreates the object (updated_at: ct = 12)
    sb = (oo.StreamBuilder(2, 5).cmd(5, "sadd", b"s", b"a").cmd(10, "delset", b"s")
          .cmd(8, "sadd", b"s", b"b").cmd(12, "sadd", b"s", b"c").cmd(3, "srem", b"s", b"d"))
    out.append(("delset_scope", _snap(_db()), sb.bytes(), 5,
                f"K {h(b's')} 5 12 12 10\n"
                f" D {h(b'a')} 10\n D {h(b'b')} 10\n A {h(b'c')} 12\n D {h(b'd')} 3\n"))

    # member tags: ties go to the later op (lwwhash.rs:87-128); state tags compete too
    st = _db({b"s": _set(adds={b"x": 6}, dels={b"y": 9}, ct=1, ut=1)})
    sb = (oo.StreamBuilder(2, 5).cmd(6, "srem", b"s", b"x").cmd(9, "sadd", b"s", b"y")
          .cmd(4, "sadd", b"s", b"z").cmd(4, "srem", b"s", b"z"))
    out.append(("member_ties", _snap(st), sb.bytes(), 5,
                f"K {h(b's')} 5 1 9 0\n D {h(b'x')} 6\n A {h(b'y')} 9\n D {h(b'z')} 4\n"))

    # DB::query: an alive object created before its expire time, queried at or after it, is
    # deleted at the expire time, updated_at(expire) recreates it (ct = expire), deletes[k] set
    # (db.rs:52-66, object.rs:35-49); then the set applies
    st = _db({b"k": o.Object(5, 6, 0, o.OBJECT_ENC_BYTES, b"v1")}, expires={b"k": 8})
    sb = oo.StreamBuilder(2, 5).cmd(9, "set", b"k", b"v2")
    out.append(("query_expire", _snap(st), sb.bytes(), 5,
                f"K {h(b'k')} 3 8 9 8\n V {h(b'v2')}\nX {h(b'k')} 8\nR {h(b'k')} 8\n"))

    # hset: an odd argument count errors before the DB is touched (no object is created);
    # hset under a delete time re-deletes the field at it (type_hash.rs:37-42)
    st = _db({b"d": o.Object(1, 1, 30, o.OBJECT_ENC_DICT, o.Dict())})
    sb = (oo.StreamBuilder(2, 5).cmd(10, "hset", b"e", b"f", b"v", b"odd")
          .cmd(11, "hset", b"d", b"f", b"v").cmd(40, "hset", b"d", b"g", b"w"))
    out.append(("hset_rules", _snap(st), sb.bytes(), 5,
                f"K {h(b'd')} 4 40 40 30\n D {h(b'f')} 30\n A {h(b'g')} 40 {h(b'w')}\n"))

    # the uuid gate (pull.rs:199-209): a duplicate (last_uuid behind) is skipped, a message ahead
    # (lost commands) is dropped; unknown and unsupported commands advance uuid_he_sent
    parts = [oo.replicate_msg(2, 5, 10, "set", b"a", b"1"),
             oo.replicate_msg(2, 4, 11, "set", b"b", b"dup"),      # duplicate
             oo.replicate_msg(2, 12, 13, "set", b"c", b"lost"),    # lost
             oo.replicate_msg(2, 10, 14, "frobnicate", b"x"),      # unknown
             oo.replicate_msg(2, 14, 15, "spop", b"x"),            # unsupported
             oo.replicate_msg(2, 15, 16, "SET", b"d", b"2")]
    out.append(("uuid_gate", _snap(_db()), b"".join(parts), 5,
                f"K {h(b'a')} 3 10 10 0\n V {h(b'1')}\nK {h(b'd')} 3 16 16 0\n V {h(b'2')}\n"))

    # integer arguments: next_bytes gives the decimal form (resp.rs:20-26)
    sb = oo.StreamBuilder(2, 5).cmd(10, "sadd", ("int", 7), ("int", -3), b"m")
    out.append(("int_args", _snap(_db()), sb.bytes(), 5,
                f"K {h(b'7')} 5 10 10 0\n A {h(b'-3')} 10\n A {h(b'm')} 10\n"))
    return out
