"""Writes the reference-asserted op-stream fixtures under tests/golden/bintest_* (run from the repo
root: `python tests/golden/make_bintest.py`). Test infrastructure.

The reference's integration test (bin/test.rs:122-396) drives three replicas with random SET/DEL,
INCR/DECR/DEL, SADD/SREM/DEL and HSET/HDEL/DEL commands, each sent to a random replica a millisecond
or two after the previous one, and asserts that every replica then answers GET / SMEMBERS / HGETALL
exactly as a sequential model of the same commands (a HashMap / HashSet / i64 kept by the test). The
replicas see each other's commands as `replicate` messages (replica/pull.rs:184-235), so the state
every replica converges to is the replicate stream of all commands, in uuid order, applied to an
empty DB. Each fixture here is that stream:
  * the commands of one test function, drawn with a seeded generator (random.Random stands in for
    tokio's thread_rng_n: the same ranges and branch probabilities as the test), each tagged with the
    node id of the replica it was sent to and a uuid one or two milliseconds after the last
    (uuid = ms << 22, server.rs uuid layout);
  * client DEL turned into what del_command (cmd.rs:221-280) replicates from the originating replica's
    state: delbytes, delcnt with every node's negated value, delset, deldict -- or nothing for an absent
    or already-deleted key;
  * cut after the test's last asserting iteration, where the model's values are recorded
    (case.json pinning.model: the reference's own assertion);
  * applied.txt: the Python op-stream oracle's canonical dump of the stream applied to an empty DB
    (a regression reference; the model is what pins it to the reference).
"""
import json
import os
import random
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import constdb_oracle as o  # noqa: E402
import constdb_ops_oracle as oo  # noqa: E402

T0_MS = 1_700_000_000_000
NODES = (1, 2, 3)  # r1, r2, r3


class Run:
    """The three replicas as one converged DB, and the replicate stream of every command."""

    def __init__(self, seed):
        self.rng = random.Random(seed)
        self.db = o.DB()
        self.ms = T0_MS
        self.last_uuid = 5
        self.parts = []

    def n(self, k):  # thread_rng_n(k)
        return self.rng.randrange(k)

    def _next_uuid(self, gap_ms):
        self.ms += gap_ms
        return self.ms << 22

    def _emit(self, node, uuid, cmd, *args):
        msg = oo.replicate_msg(node, self.last_uuid, uuid, cmd, *args)
        st = oo.apply_replicates(self.db, msg, self.last_uuid)
        assert st.applied == 1 and st.cmd_errors == 0, (cmd, args)
        self.parts.append(msg)
        self.last_uuid = uuid

    def command(self, node, gap_ms, cmd, *args):
        """A client command sent to replica `node` (bin/test.rs exec!)."""
        uuid = self._next_uuid(gap_ms)
        if cmd != "del":
            self._emit(node, uuid, cmd, *args)
            return
        key = args[0]
        ob = oo.query(self.db, key, uuid)  # del_command (cmd.rs:221-280) on the originating replica
        if ob is None:
            return
        deleted = ob.create_time < ob.delete_time
        if ob.tag == o.OBJECT_ENC_COUNTER:
            if ob.update_time <= uuid and not deleted:
                pairs = []
                for nid, (v, _) in sorted(ob.enc.data.items()):
                    pairs += [("int", nid), ("int", -v)]
                self._emit(node, uuid, "delcnt", key, *pairs)
        elif ob.tag == o.OBJECT_ENC_BYTES:
            if ob.update_time <= uuid and not deleted:
                self._emit(node, uuid, "delbytes", key)
        elif ob.tag == o.OBJECT_ENC_SET:
            self._emit(node, uuid, "delset", key)
        else:
            self._emit(node, uuid, "deldict", key)

    def stream(self):
        return b"".join(self.parts)


def bytes_case(seed):
    """test_bytes (bin/test.rs:193-221): 1000 SET / DEL over key:0..4; GET of every key the model holds."""
    r = Run(seed)
    d = {}
    for _ in range(1000):
        rand = r.n(100)
        key = f"key:{rand % 5}".encode()
        c = NODES[r.n(100) % 3]
        if rand % 3 == 0:
            d.pop(key, None)
            r.command(c, 1, "del", key)
        else:
            value = f"value:{r.n(1000)}".encode()
            d[key] = value
            r.command(c, 1, "set", key, value)
    return r, {"GET": {k.decode(): v.decode() for k, v in d.items()}}, "bin/test.rs:193-221"


def counter_cases(seed):
    """test_counters (bin/test.rs:122-191): counter1 -- 1000 INCR / DECR, GET == v on every replica;
    counter2 -- INCR / DECR / DEL, asserted every 10th iteration (cut at the last, i = 90)."""
    r = Run(seed)
    v = 0
    for _ in range(1000):
        if r.n(10) % 2 == 0:
            v += 1
            cmd = "incr"
        else:
            v -= 1
            cmd = "decr"
        r.command(NODES[r.n(1000) % 3], 2, cmd, b"counter1")
    out = [("counter1", r, {"GET": {"counter1": v}}, "bin/test.rs:122-148")]
    r = Run(seed + 1)
    vv = None
    model = None
    for i in range(100):
        m = r.n(100) % 3
        if m == 0:
            vv = (vv or 0) + 1
            cmd = "incr"
        elif m == 1:
            vv = (vv or 0) - 1
            cmd = "decr"
        else:
            vv = None
            cmd = "del"
        r.command(NODES[r.n(100) % 3], 1, cmd, b"counter2")
        if i % 10 == 0:
            model = {"GET": {"counter2": vv}}
            if i == 90:
                break
    out.append(("counter2", r, model, "bin/test.rs:150-190"))
    return out


def set_cases(seed):
    """test_set (bin/test.rs:223-300): set1 -- 1000 SADD / SREM of member:0..99, SMEMBERS == the model;
    set2 -- SADD / SREM / DEL, asserted whenever the drawn client index is a multiple of 20 (cut there)."""
    r = Run(seed)
    s = set()
    for _ in range(1000):
        rand = r.n(100)
        member = f"member:{rand}".encode()
        if rand % 2 == 0:
            s.add(member)
            cmd = "sadd"
        else:
            s.discard(member)
            cmd = "srem"
        r.command(NODES[r.n(100) % 3], 1, cmd, b"set1", member)
    out = [("set1", r, {"SMEMBERS": {"set1": sorted(m.decode() for m in s)}}, "bin/test.rs:223-255")]
    r = Run(seed + 1)
    s = set()
    best = None
    for _ in range(1000):
        rand = r.n(20)
        member = f"member:{rand}".encode()
        k = rand % 9
        if k <= 3:
            s.add(member)
            cmd = "sadd"
        elif k <= 7:
            s.discard(member)
            cmd = "srem"
        else:
            s.clear()
            cmd = "del"
        i = r.n(100)
        if cmd == "del":
            r.command(NODES[i % 3], 1, cmd, b"set2")
        else:
            r.command(NODES[i % 3], 1, cmd, b"set2", member)
        if i % 20 == 0:
            best = (len(r.parts), {"SMEMBERS": {"set2": sorted(m.decode() for m in s)}}, r.ms, r.last_uuid)
    out.append(("set2", truncate(r, best), best[1], "bin/test.rs:257-300"))
    return out


def dict_cases(seed):
    """test_dict (bin/test.rs:302-396): dict1 -- 100 HSET / HDEL over field:0..9, HGETALL == the model;
    dict2 -- HSET / HDEL / DEL, asserted every 20th iteration (cut at the last, i = 980)."""
    r = Run(seed)
    d = {}
    for _ in range(100):
        rand = r.n(100)
        field = f"field:{r.n(10)}".encode()
        value = f"value:{r.n(50)}".encode()
        c = NODES[r.n(1000) % 3]
        if rand % 5 == 0:
            d.pop(field, None)
            r.command(c, 1, "hdel", b"dict1", field)
        else:
            d[field] = value
            r.command(c, 1, "hset", b"dict1", field, value)
    out = [("dict1", r, {"HGETALL": {"dict1": {k.decode(): v.decode() for k, v in d.items()}}},
            "bin/test.rs:302-334")]
    r = Run(seed + 1)
    m = {}
    model = None
    for i in range(1000):
        rand = r.n(100)
        field = f"field:{r.n(10)}".encode()
        value = f"value:{r.n(50)}".encode()
        c = NODES[r.n(1000) % 3]
        k = rand % 9
        if k <= 3:
            m[field] = value
            r.command(c, 1, "hset", b"dict2", field, value)
        elif k <= 7:
            m.pop(field, None)
            r.command(c, 1, "hdel", b"dict2", field)
        else:
            m.clear()
            r.command(c, 1, "del", b"dict2")
        if i % 20 == 0:
            model = {"HGETALL": {"dict2": {k2.decode(): v2.decode() for k2, v2 in m.items()}}}
            if i == 980:
                break
    out.append(("dict2", r, model, "bin/test.rs:336-396"))
    return out


def truncate(r, best):
    """The run cut after message count best[0] (a set2 assertion point): replayed from the stream."""
    n = best[0]
    t = Run(0)
    t.parts = r.parts[:n]
    t.db = o.DB()
    oo.apply_replicates(t.db, t.stream(), 5)
    return t


def main():
    cases = [("bytes",) + bytes_case(61)]
    cases += counter_cases(62)
    cases += set_cases(63)
    cases += dict_cases(64)
    empty = o.dump_all(o.DB(), o.NodeHeader(node_id=9, alias="n9"))
    for name, run, model, src in cases:
        d = os.path.join(HERE, "bintest_" + name)
        os.makedirs(d, exist_ok=True)
        stream = run.stream()
        db = o.DB()
        st = oo.apply_replicates(db, stream, 5)
        assert st.applied == len(run.parts) and st.lost == 0 and st.duplicates == 0 and st.cmd_errors == 0
        with open(os.path.join(d, "state.bin"), "wb") as f:
            f.write(empty)
        with open(os.path.join(d, "stream.bin"), "wb") as f:
            f.write(stream)
        with open(os.path.join(d, "applied.txt"), "wb") as f:
            f.write(o.canonical_dump(db))
        with open(os.path.join(d, "case.json"), "w") as f:
            json.dump({"source": src, "kind": "ops", "uuid_he_sent": 5, "messages": len(run.parts),
                       "pinning": {"kind": "reference-asserted", "model": model}}, f, indent=1, sort_keys=True)
            f.write("\n")
    print(f"{len(cases)} op-stream cases written under {HERE}")


if __name__ == "__main__":
    main()
