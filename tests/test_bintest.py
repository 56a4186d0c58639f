"""Reference-asserted op streams (tests/golden/bintest_*, written by tests/golden/make_bintest.py): the
commands of bin/test.rs:122-396 (SET/DEL, INCR/DECR/DEL, SADD/SREM/DEL, HSET/HDEL/DEL sent to three
replicas), replayed as the replicate stream every replica converges to. After it, the reference's test
asserts GET / SMEMBERS / HGETALL equal its sequential model on every replica (case.json pinning.model).

Checked here on the CPU: the op-stream oracle (oracle/constdb_ops_oracle.py, pull.rs:184-235 and the
handlers it cites) applied to the stream answers exactly the model -- through the reference's read
commands (get_command cmd.rs:167-184, smembers_command type_set.rs:69-81, hgetall_command
type_hash.rs:87-99) restated over the canonical dump -- and reproduces the frozen dump. The GPU op
apply and the snapshot merge of the converged replicas are checked against the same model in
tests/test_bintest_gpu.py."""
import json
import os

import pytest

import constdb_oracle as o
import constdb_ops_oracle as oo

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
CASES = sorted(d for d in os.listdir(GOLDEN) if d.startswith("bintest_"))


def load(name):
    d = os.path.join(GOLDEN, name)
    meta = json.load(open(os.path.join(d, "case.json")))
    state = open(os.path.join(d, "state.bin"), "rb").read()
    stream = open(os.path.join(d, "stream.bin"), "rb").read()
    want = open(os.path.join(d, "applied.txt"), "rb").read()
    return state, stream, want, meta


def views(dump: bytes):
    """The reference's read commands over a canonical dump: {key: (tag, ct, dt, value)} where value is
    the counter sum, the Bytes value, or the live members {member: value} (SetIter / DictIter,
    lwwhash.rs:229-248, 361-380: an add not shadowed by a strictly later del)."""
    keys = {}
    cur = None
    for line in dump.decode().split("\n"):
        if line.startswith("K "):
            _, kh, tag, ct, ut, dt = line.split()
            cur = bytes.fromhex(kh).decode()
            keys[cur] = {"tag": int(tag), "ct": int(ct), "dt": int(dt), "adds": {}, "dels": {}}
        elif line.startswith(" S "):
            keys[cur]["value"] = int(line.split()[1])
        elif line.startswith(" V "):
            keys[cur]["value"] = bytes.fromhex(line.split()[1] if len(line.split()) > 1 else "").decode()
        elif line.startswith(" A "):
            parts = line.split()
            m = bytes.fromhex(parts[1]).decode()
            keys[cur]["adds"][m] = (int(parts[2]), bytes.fromhex(parts[3]).decode() if len(parts) > 3 else None)
        elif line.startswith(" D "):
            parts = line.split()
            keys[cur]["dels"][bytes.fromhex(parts[1]).decode()] = int(parts[2])
        elif line[:1] in ("X", "R"):
            cur = None
    return keys


def get(keys, k):  # get_command (cmd.rs:167-184)
    o_ = keys.get(k)
    if o_ is None or o_["ct"] < o_["dt"]:
        return None
    return o_["value"]


def live(keys, k):  # smembers / hgetall: the set's live iterator (no object-deletion check)
    o_ = keys.get(k)
    if o_ is None:
        return None
    return {m: v for m, (t, v) in o_["adds"].items() if not (m in o_["dels"] and o_["dels"][m] > t)}


def check_model(dump: bytes, model: dict):
    keys = views(dump)
    for k, v in model.get("GET", {}).items():
        assert get(keys, k) == v, (k, get(keys, k), v)
    for k, members in model.get("SMEMBERS", {}).items():
        assert sorted(live(keys, k)) == members, k
    for k, kvs in model.get("HGETALL", {}).items():
        assert live(keys, k) == kvs, k


def test_fixture_set():
    assert [c[len("bintest_"):] for c in CASES] == ["bytes", "counter1", "counter2", "dict1", "dict2", "set1", "set2"]


@pytest.mark.parametrize("name", CASES)
def test_ops_oracle_answers_the_reference_model(name):
    state, stream, want, meta = load(name)
    assert meta["pinning"]["kind"] == "reference-asserted"
    db = o.fold_snapshots([state])
    st = oo.apply_replicates(db, stream, meta["uuid_he_sent"])
    assert st.applied == meta["messages"] and st.lost == 0 and st.duplicates == 0 and st.cmd_errors == 0
    got = o.canonical_dump(db)
    assert got == want
    check_model(got, meta["pinning"]["model"])
