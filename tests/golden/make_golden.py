"""Writes the frozen golden fixtures under tests/golden/ (run from the repo root:
`python tests/golden/make_golden.py`). Test infrastructure: the expected merge results come from the
Python oracle (oracle/constdb_oracle.py, a line-cited restatement of the reference's fold), so a
later change to either oracle -- or to the GPU path -- shows up against these files
(tests/test_golden.py) instead of moving the target silently.

Each case is a directory holding snap_<i>.bin (the snapshots in fold order, writer layout,
server.rs:183-215), merged.txt (the oracle's canonical dump of the fold, after DB::gc when the case
has a watermark) and case.json (watermark, the fold's type-conflict and Dict-merge counts, and where
the case comes from). Cases: every merge KAT of tests/test_oracle_kat.py (each cites
the reference lines it is derived from), the bin/test.rs:85-116 MEET scenarios (k1-k4, and k5 over
three replicas), and two 2000-key random replica sets from the seeded generator (one with DB::gc).
case.json's "pinning" says which cases the reference's own assertions pin (REFERENCE_ASSERTED), which
restate a cited rule, and which are oracle-only regression fixtures.
"""
import json
import os
import shutil
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, ROOT)

import constdb_oracle as o  # noqa: E402


def snap(objs=None, deletes=None, expires=None, node_id=1):
    db = o.DB()
    for k, v in (objs or {}).items():
        db.data[k] = v
    for k, t in (deletes or {}).items():
        db.deletes[k] = t
    for k, t in (expires or {}).items():
        db.expires[k] = t
    return o.dump_all(db, o.NodeHeader(node_id=node_id, alias=f"n{node_id}"))


def bytes_(ct, v, ut=0, dt=0):
    return o.Object(ct, ut, dt, o.OBJECT_ENC_BYTES, v)


def counter(nodes, ct=1, ut=0, dt=0):
    c = o.Counter()
    for n, (v, t) in nodes.items():
        c.data[n] = (v, t)
    c.cal_sum()
    return o.Object(ct, ut, dt, o.OBJECT_ENC_COUNTER, c)


def set_(adds, dels=None, ct=1, ut=0, dt=0):
    s = o.Set()
    for m, t in adds.items():
        s.set(m, None, t)
    for m, t in (dels or {}).items():
        s.rem(m, t)
    return o.Object(ct, ut, dt, o.OBJECT_ENC_SET, s)


def dict_(adds, dels=None, ct=1, ut=0, dt=0):
    d = o.Dict()
    for m, (t, v) in adds.items():
        d.set(m, v, t)
    for m, t in (dels or {}).items():
        d.rem(m, t)
    return o.Object(ct, ut, dt, o.OBJECT_ENC_DICT, d)


def kat_cases():
    t = 1 << 22
    return {
        "bytes_ct_tie": ("object.rs:71-73", [snap({b"k": bytes_(10, b"A", ut=3, dt=1)}),
                                              snap({b"k": bytes_(10, b"B", ut=9, dt=0)})], None),
        "bytes_max_ct": ("object.rs:71-76", [snap({b"k": bytes_(10, b"A", ut=50, dt=7)}),
                                              snap({b"k": bytes_(12, b"B", ut=11, dt=3)}),
                                              snap({b"k": bytes_(11, b"C", ut=12, dt=9)})], None),
        "counter_order_a": ("type_counter.rs:60-71", [snap({b"c": counter({1: (5, 10)})}),
                                                       snap({b"c": counter({1: (7, 11)})}),
                                                       snap({b"c": counter({1: (6, 12)})})], None),
        "counter_order_b": ("type_counter.rs:60-71", [snap({b"c": counter({1: (5, 10)})}),
                                                       snap({b"c": counter({1: (6, 12)})}),
                                                       snap({b"c": counter({1: (7, 11)})})], None),
        "counter_tie_insert": ("type_counter.rs:65-67,81-83",
                               [snap({b"c": counter({1: (5, 10), 2: (1, 3)})}),
                                snap({b"c": counter({1: (3, 10), 3: (4, 8)})}),
                                snap({b"c": counter({1: (9, 9), 3: (2, 9)})})], None),
        "counter_unmerged": ("type_counter.rs:111-126", [snap({b"c": counter({1: (5, 10), 2: (6, 1)})})], None),
        "non_bytes_head_times": ("object.rs:68,78-79", [snap({b"c": counter({1: (1, 1)}, ct=5, ut=6, dt=7)}),
                                                         snap({b"c": counter({1: (1, 2)}, ct=50, ut=60, dt=70)})],
                                 None),
        "type_conflict": ("db.rs:36-40, object.rs:80", [snap({b"k": counter({1: (1, 1)}, ct=5)}),
                                                         snap({b"k": bytes_(99, b"X")}),
                                                         snap({b"k": counter({1: (4, 2)}, ct=6)})], None),
        "set_ties_remote_dels": ("lwwhash.rs:87-107,319-323",
                                 [snap({b"s": set_({b"a": 5, b"b": 7}, {b"d": 10})}),
                                  snap({b"s": set_({b"d": 10, b"e": 1}, {b"a": 9})}),
                                  snap({b"s": set_({b"b": 6})})], None),
        "set_local_del": ("lwwhash.rs:87-128", [snap({b"s": set_({}, {b"m": 10})}), snap({b"s": set_({b"m": 9})})],
                          None),
        "dict_value_winner": ("lwwhash.rs:176-179", [snap({b"h": dict_({b"f": (5, b"x"), b"g": (9, b"y")})}),
                                                      snap({b"h": dict_({b"f": (5, b"z"), b"g": (8, b"w")})})],
                              None),
        "deletes_expires_last_pos": ("pull.rs:129-130, db.rs:68-76",
                                     [snap(deletes={b"a": 50, b"b": 1}, expires={b"x": 9}),
                                      snap(deletes={b"a": 20}, expires={b"x": 3})], None),
        "gc_lifo": ("db.rs:82-95", [snap(deletes={b"a": 5}), snap(deletes={b"b": 50}), snap(deletes={b"c": 6})], 10),
        "meet_bin_test": ("bin/test.rs:85-106",
                          [snap({}, node_id=3),
                           snap({b"k1": counter({1: (1, 1 * t)}), b"k2": counter({2: (2, 3 * t)}),
                                 b"k3": counter({1: (1, 8 * t), 2: (1, 9 * t)}), b"k4": counter({2: (4, 7 * t)})},
                                node_id=2)], None),
        # bin/test.rs:110-116: r3, r1 and r2 each INCR k5 once (after r3 MEETs r2, every node's
        # increment reaches the others); GET k5 == 3 on every replica. As snapshots: each replica
        # holds its own node's increment, and the merged counter sums to 3
        "meet_k5_three_replicas": ("bin/test.rs:110-116",
                                   [snap({b"k5": counter({3: (1, 20 * t)})}, node_id=3),
                                    snap({b"k5": counter({1: (1, 21 * t)})}, node_id=1),
                                    snap({b"k5": counter({2: (1, 22 * t)})}, node_id=2)], None),
        "canonical_sorted": ("canonical dump order", [snap({b"b": bytes_(1, b"\x00"),
                                                             b"a": set_({b"z": 1, b"y": 2}, {b"q": 3})},
                                                            deletes={b"d": 4}, expires={b"e": 5})], None),
    }


def random_cases():
    import constdb_amd as cdb
    from constdb_amd import configs
    cfg = cdb.gen_config(seed=2024, universe=2000, n_replicas=3, replica_hi=3, conflict_ppm=30000,
                         tie_permille=150, side_permille=250, mean_members=4, del_permille=300,
                         mix_set=25, mix_dict=25)
    snaps = [cdb.gen_snapshot(cfg, r) for r in range(3)]
    wm = (configs.T0_MS + (1 << 30)) << 22
    return {"random_2k": ("seeded generator, 2000 keys x 3 replicas", snaps, None),
            "random_2k_gc": ("the same with DB::gc after every time", snaps, wm)}


# What pins each case to the reference (case.json "pinning"): the values the reference's own test
# asserts (bin/test.rs GET results, checked in the frozen dump by tests/test_golden.py), a merge rule
# restated from the cited lines (the expected dump is the oracle's), or nothing but the oracle
# (a regression fixture: its parity with the reference is unpinned).
REFERENCE_ASSERTED = {
    "meet_bin_test": {"k1": 1, "k2": 2, "k3": 2, "k4": 4},  # bin/test.rs:97-98, 104, 108-109
    "meet_k5_three_replicas": {"k5": 3},                    # bin/test.rs:116
}


def pinning(name, src):
    if name in REFERENCE_ASSERTED:
        return {"kind": "reference-asserted", "counter_sums": REFERENCE_ASSERTED[name]}
    if name.startswith("random_"):
        return {"kind": "oracle-only regression fixture (parity unpinned)"}
    return {"kind": "rule restated from " + src}


def fold(snaps, wm):
    db = o.fold_snapshots(snaps)
    if wm is not None:
        db.gc(wm)
    return db


def main():
    cases = kat_cases()
    cases.update(random_cases())
    for name, (src, snaps, wm) in cases.items():
        d = os.path.join(HERE, name)
        shutil.rmtree(d, ignore_errors=True)
        os.makedirs(d)
        for i, s in enumerate(snaps):
            with open(os.path.join(d, f"snap_{i}.bin"), "wb") as f:
                f.write(s)
        db = fold(snaps, wm)
        with open(os.path.join(d, "merged.txt"), "wb") as f:
            f.write(o.canonical_dump(db))
        with open(os.path.join(d, "case.json"), "w") as f:
            json.dump({"source": src, "snapshots": len(snaps), "gc_watermark": wm,
                       "type_conflicts": db.type_conflicts, "dict_merges": db.dict_merges,
                       "pinning": pinning(name, src)}, f, indent=1)
            f.write("\n")
    print(f"{len(cases)} cases written under {HERE}")


if __name__ == "__main__":
    main()
