"""Small seeded random snapshot generator for parity tests (pure Python).

Builds R replica DBs over a shared key universe with deliberate hazards: time ties
(small time range), cross-replica type conflicts, members with add/del tags, dict
values, deletes/expires side maps, empty/long keys and values. Snapshots are written
with the reference writer layout via the oracle's dump_all (Bytes length-prefixed).
"""
import random

import constdb_oracle as o

T0 = 1_700_000_000_000 << 22


def _rand_bytes(rng, lo, hi):
    n = rng.randint(lo, hi)
    return bytes(rng.getrandbits(8) for _ in range(n))


def gen_replicas(seed, n_replicas=3, n_keys=40, p_key=0.6, type_mix=(0.4, 0.3, 0.15, 0.15),
                 p_conflict=0.05, t_range=8, n_members=6, n_nodes=4, p_side=0.1,
                 big_times=False):
    rng = random.Random(seed)
    keys = []
    for i in range(n_keys):
        r = rng.random()
        if r < 0.05:
            k = b""                                   # empty key (at most once)
            if k in keys:
                k = b"e%d" % i
        elif r < 0.1:
            k = _rand_bytes(rng, 60, 200)             # long keys
        else:
            k = b"k%d" % i + _rand_bytes(rng, 0, 3)
        if k not in keys:
            keys.append(k)
    tags = [o.OBJECT_ENC_BYTES, o.OBJECT_ENC_COUNTER, o.OBJECT_ENC_SET, o.OBJECT_ENC_DICT]
    key_type = {k: rng.choices(tags, weights=type_mix)[0] for k in keys}
    members = [b"m%d" % j for j in range(n_members)] + [b"", b"\xff\x00"]

    def t():
        base = T0 if big_times else 0
        return base + rng.randint(0, t_range)

    snaps = []
    for r in range(n_replicas):
        db = o.DB()
        for k in keys:
            if rng.random() >= p_key:
                continue
            tag = key_type[k]
            if rng.random() < p_conflict:
                tag = rng.choice(tags)
            ct, ut, dt = t(), t(), t()
            if tag == o.OBJECT_ENC_BYTES:
                enc = _rand_bytes(rng, 0, 40)
            elif tag == o.OBJECT_ENC_COUNTER:
                enc = o.Counter()
                for nd in rng.sample(range(1, n_nodes + 1), rng.randint(0, n_nodes)):
                    enc.data[nd] = (rng.randint(0, 1 << rng.choice([3, 20, 40])), t())
                enc.cal_sum()
            else:
                enc = o.Set() if tag == o.OBJECT_ENC_SET else o.Dict()
                for m in rng.sample(members, rng.randint(0, len(members))):
                    if rng.random() < 0.7:
                        enc.set(m, _rand_bytes(rng, 0, 12) if tag == o.OBJECT_ENC_DICT else None, t())
                    else:
                        enc.rem(m, t())
            db.data[k] = o.Object(ct, ut, dt, tag, enc)
        for k in keys:
            if rng.random() < p_side:
                db.deletes[k] = t()
            if rng.random() < p_side:
                db.expires[k] = t()
        hdr = o.NodeHeader(node_id=r + 1, alias=f"n{r + 1}", addr=f"127.0.0.1:{9001 + r}",
                           last_uuid=t())
        snaps.append(o.dump_all(db, hdr))
    return snaps
