"""Seeded random replicate streams for op-apply parity tests (pure Python).

Commands over a key universe shared with a snapgen state (so they hit existing keys of every
type, with type conflicts), small uuid ranges (ties with the state's times and each other),
expires in the state (DB::query's side effect), and stream-level hazards: duplicate and
out-of-order messages, unknown and unsupported commands, arity errors, integer arguments,
replack messages.
"""
import random

import constdb_ops_oracle as oo

CMDS = ["set", "delbytes", "incr", "decr", "delcnt", "sadd", "srem", "delset", "hset", "hdel", "deldict"]


def gen_stream(seed, keys, n_cmds=200, t_range=12, uuid_he_sent=5, members=None, hazards=True,
               weights=None, n_nodes=4):
    rng = random.Random(seed)
    members = members or [b"m%d" % j for j in range(6)] + [b"", b"\xff\x00"]
    keys = list(keys) + [b"new%d" % i for i in range(max(4, len(keys) // 4))]
    parts = []
    last = uuid_he_sent
    nodeid = rng.randint(1, n_nodes)

    def arg(b):
        if hazards and rng.random() < 0.05 and b.isdigit() and len(b) < 12:
            return ("int", int(b))            # an integer argument (next_bytes -> decimal)
        return oo.bulk(b)

    for _ in range(n_cmds):
        cmd = rng.choices(CMDS, weights=weights)[0] if weights else rng.choice(CMDS)
        k = rng.choice(keys)
        uuid = rng.randint(0, t_range)
        args = [arg(k)]
        if cmd == "set":
            args.append(oo.bulk(bytes(rng.getrandbits(8) for _ in range(rng.randint(0, 10))).replace(b"\r\n", b"..")))
        elif cmd == "delcnt":
            for _ in range(rng.randint(0, 3)):
                args += [("int", rng.randint(1, n_nodes)), ("int", rng.randint(-(1 << 20), 1 << 20))]
        elif cmd in ("sadd", "srem", "hdel"):
            for _ in range(rng.randint(0, 4)):
                args.append(arg(rng.choice(members)))
        elif cmd == "hset":
            for _ in range(rng.randint(0, 3)):
                args += [arg(rng.choice(members)), oo.bulk(bytes(rng.getrandbits(8) for _ in range(rng.randint(0, 6))).replace(b"\r\n", b".."))]
        name = cmd
        r = rng.random() if hazards else 1.0
        if r < 0.02:
            name = "frobnicate"                  # unknown: skipped, uuid advanced
        elif r < 0.04:
            name = "spop"                        # unsupported: skipped, uuid advanced
        elif r < 0.06:
            args = args[:0]                      # WrongArity: no key
        elif r < 0.07 and cmd == "hset":
            args = args + [oo.bulk(b"odd")]      # odd field count: error before the DB
        elif r < 0.08:
            name = name.upper()                  # command names are case-insensitive
        lu = last
        r2 = rng.random() if hazards else 1.0
        if r2 < 0.03:
            lu = last + 1 + rng.randint(0, 3)    # ahead: lost commands, dropped
        elif r2 < 0.06:
            lu = max(0, last - 1 - rng.randint(0, 3)) if last > 0 else last  # behind: duplicate
        parts.append(oo.replicate_msg(nodeid, lu, uuid, name, *args))
        if lu == last:
            last = uuid
        if hazards and rng.random() < 0.02:
            parts.append(oo.resp_encode(("arr", [oo.bulk(b"replack"), ("int", rng.randint(0, 99))])))
        if hazards and rng.random() < 0.01:
            parts.append(oo.resp_encode(("int", 5)))  # not an array: dropped
    return b"".join(parts)
