"""BASELINE.json's five configs as seeded generator presets.

Every config is a pure function of (seed, key index, replica): the host writer
(cdb_gen_snapshot, snapshot bytes for the decode path and the oracle) and the device
generator (cdb_gen_device, rows written straight into HBM) draw identical replica states.

  C1/C2  2-node MEET: 1M Bytes keys + 1M counters per node (counters carry the writing node's
         own id, one node each), 50 % key overlap per type; B merged into A (R = 2).
  C3     set/dict add-win merge: 4 replicas, each the state left by replaying 10M
         sadd/srem/hset/hdel commands (Zipf members) over 100K keys (one type per key on every
         replica) through the device op apply (R8, type_set.rs:13-67, type_hash.rs:11-71) on top
         of a synced state holding Expires and Deletes; merged with DB::gc at the median member
         time (db.rs:82-119).
  C4     8-replica anti-entropy: 60/30/5/5 Bytes/Counter/Set/Dict, 0.1 % type conflicts,
         p(key in replica) = 0.5; per GPU a 62.5M-key shard (N = 8 -> 500M keys).
  C5     Zipf hot keys: children per key ~ rank^-1.1 over 10M keys, 80M node/member rows over
         8 replicas; the hottest keys own ~10^6 members (lwwhash.rs:319-323,
         type_counter.rs:59-87 per-key loops).
"""
from __future__ import annotations

T0_MS = 1_700_000_000_000


def c4(cdb, universe=62_500_000, replicas=8, seed=4, lo=0, hi=None, shard=0, n_shards=1):
    return cdb.gen_config(seed=seed, universe=universe, n_replicas=replicas, key_permille=500,
                          mix_bytes=60, mix_counter=30, mix_set=5, mix_dict=5, conflict_ppm=1000,
                          tie_permille=20, max_nodes=8, mean_members=4, member_universe=16,
                          del_permille=200, side_permille=20, value_min=8, value_max=32,
                          shard=shard, n_shards=n_shards, replica_lo=lo,
                          replica_hi=replicas if hi is None else hi)


def c1(cdb, per_node=1_000_000, seed=1):
    """Universe 4 x per_node keys, half Bytes half Counter, p = 0.5: each node holds ~per_node
    keys of each type and half of a node's keys are also on the other node."""
    return cdb.gen_config(seed=seed, universe=4 * per_node, n_replicas=2, key_permille=500,
                          mix_bytes=50, mix_counter=50, mix_set=0, mix_dict=0, conflict_ppm=0,
                          tie_permille=20, max_nodes=1, mean_members=0, member_universe=1,
                          del_permille=0, side_permille=0, value_min=8, value_max=32,
                          flags=cdb.GEN_NODE_PER_REPLICA, replica_lo=0, replica_hi=2)


def c5(cdb, universe=10_000_000, events=80_000_000, replicas=8, seed=5):
    return cdb.gen_config(seed=seed, universe=universe, n_replicas=replicas, key_permille=500,
                          mix_bytes=0, mix_counter=40, mix_set=30, mix_dict=30, conflict_ppm=1000,
                          tie_permille=20, max_nodes=8, mean_members=4, member_universe=16,
                          del_permille=200, side_permille=20, value_min=8, value_max=32,
                          hot_zipf_milli=1100, hot_events=events, replica_lo=0, replica_hi=replicas)


def c3_ops_config(cdb, replica, keys=100_000, members=1000, seed=3):
    """Generator config of replica `replica`'s op stream: set/dict keys only, members drawn
    Zipf-skewed from `members` per key, only sadd/srem/hset/hdel. The seed is shared by every
    replica, so a key has ONE type everywhere (gen_type); `stream` salts the per-op draws, so each
    replica replays its own commands."""
    return cdb.gen_config(seed=seed, universe=keys, n_replicas=1, mix_bytes=0, mix_counter=0, mix_set=50,
                          mix_dict=50, member_universe=members, stream=replica + 1,
                          flags=cdb.GEN_OPS_ZIPF_MEMBERS | cdb.GEN_OPS_TAGS_ONLY)


def c3_base_config(cdb, replicas=4, keys=100_000, seed=3, side_permille=50):
    """The state every C3 replica syncs from first: no data entries, only Expires and Deletes for
    ~5 % of the keys each (pull.rs:129-130 -> DB::expire_at / DB::delete, db.rs:68-76). The
    reference creates a Deletes entry only through DB::delete (a snapshot's Deletes) or DB::query
    on an expired key (db.rs:53-66); delset / deldict only tag members (type_set.rs:117-135,
    type_hash.rs:102-120). So this is where the C3 states' Deletes -- the garbage DB::gc
    collects -- come from, besides the expiries the replayed commands trigger."""
    return cdb.gen_config(seed=seed * 1000 + 17, universe=keys, n_replicas=replicas, key_permille=0,
                          mix_bytes=0, mix_counter=0, mix_set=50, mix_dict=50, side_permille=side_permille,
                          replica_lo=0, replica_hi=replicas)


def c3_snapshots(cdb, ctx, ops_per_replica=10_000_000, replicas=4, keys=100_000, members=1000,
                 seed=3, zipf_milli=900, log=None):
    """The C3 replica states: replica r = its base state (c3_base_config: Expires + Deletes) with
    its own op stream applied by cdb_apply_ops (the device op apply of SURVEY §8f.2: DB::query's
    expiry included), written back as a snapshot by cdb_encode_snapshot. Returns the snapshot
    bytes of every replica."""
    db = cdb.DB(ctx)
    base = c3_base_config(cdb, replicas, keys, seed)
    snaps = []
    for r in range(replicas):
        ops_bytes = cdb.gen_ops(c3_ops_config(cdb, r, keys, members, seed), ops_per_replica, 0, zipf_milli)
        ops = cdb.decode_ops(ops_bytes, 0)
        del ops_bytes
        state = db.merge_snapshots([cdb.gen_snapshot(base, r)]).apply_ops(ops)
        data, _ = state.encode_snapshot(node_id=r + 1, alias=f"n{r + 1}", addr=f"127.0.0.1:{9001 + r}",
                                        replicas=None)
        snaps.append(data)
        if log:
            log(f"C3 replica {r}: {ops_per_replica} ops -> {len(data) / 1e6:.1f} MB snapshot")
    return snaps


def median_member_time(cdb, batches):
    """GC watermark of config C3: the median set/dict member tag time over every replica."""
    import numpy as np
    ts = [b.column_array(2, 4) for b in batches]
    ts = np.concatenate(ts) if ts else np.zeros(0, dtype=np.uint64)
    return int(np.sort(ts)[len(ts) // 2]) if len(ts) else 0


# Survey §8d member-row width is 34 B (set) / 42 B (dict): the share of dict members per config
DICT_MEMBER_SHARE = {"c1": 0.5, "c3": 0.5, "c4": 0.5, "c5": 0.5}
