"""ConstDB merge ORACLE — test infrastructure only.

This module is a CPU restatement of the reference's (fxsjy/ConstDB, Rust) snapshot
codec and CRDT merge fold, written from the cited file:line semantics. It exists to
check the product (``constdb_amd``'s HIP merge engine) and is NOT part of it:
only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg
may import it, and only as the checker.

Parity pinning:
  * codec: pinned by the reference's own golden vector ``snapshot.rs:372``
    (CRC-64 ``9519382692141102896`` of the varint test stream ``snapshot.rs:362-371``)
    and the varint round trips ``snapshot.rs:381-389``;
  * merge: the reference's own tests never assert a merge result, so the
    fold below is a literal restatement of ``db.rs:31-43``, ``object.rs:63-83``,
    ``type_counter.rs:59-91``, ``crdt/lwwhash.rs:87-128,176-181,319-323`` checked by
    hand-derived known-answer tests (tests/test_oracle_kat.py) and by the
    ``bin/test.rs:85-116`` MEET scenario. Merge parity is therefore
    "pinned by restatement + KATs", not by reference-run outputs (the Rust reference
    cannot be built here: no cargo/rustc, crates not vendored).

Pure Python: use it for small cases and fixtures. ``oracle/cdb_oracle.cpp`` is the
same restatement in C++ for medium sizes and the CPU baseline.
"""
from __future__ import annotations

import io
import struct
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Tuple

MASK64 = (1 << 64) - 1


def to_i64(x: int) -> int:
    x &= MASK64
    return x - (1 << 64) if x >> 63 else x


def to_u64(x: int) -> int:
    return x & MASK64


# --------------------------------------------------------------------------------------
# CRC-64/Jones as used through crc64 2.0.0 (Cargo.lock:197-200, snapshot.rs:3,40,62-64):
# reflected polynomial 0x95AC9329AC4BC9B5, init 0, no final xor. Pinned by
# snapshot.rs:372 (see tests/test_oracle_kat.py::test_reference_crc_golden).
# --------------------------------------------------------------------------------------
_CRC_POLY = 0x95AC9329AC4BC9B5
_CRC_TABLE = []
for _i in range(256):
    _c = _i
    for _ in range(8):
        _c = (_c >> 1) ^ _CRC_POLY if _c & 1 else _c >> 1
    _CRC_TABLE.append(_c)


def crc64_update(crc: int, data: bytes) -> int:
    t = _CRC_TABLE
    for b in data:
        crc = t[(crc ^ b) & 0xFF] ^ (crc >> 8)
    return crc


def crc64(data: bytes) -> int:
    return crc64_update(0, data)


# --------------------------------------------------------------------------------------
# Errors — CstError variants on the decode path (lib.rs:146-175)
# --------------------------------------------------------------------------------------
class CstError(Exception):
    pass


class InvalidSnapshot(CstError):  # lib.rs:157  InvalidSnapshot(usize)
    def __init__(self, offset: int):
        super().__init__(f"invalid data in snapshot at offset {offset}")
        self.offset = offset


class InvalidSnapshotChecksum(CstError):  # lib.rs:173
    pass


class InvalidType(CstError):  # lib.rs:151
    pass


class IoError(CstError):  # lib.rs:161 (UnexpectedEof from read_exact)
    pass


# --------------------------------------------------------------------------------------
# Snapshot writer (snapshot.rs:9-69)
# --------------------------------------------------------------------------------------
SNAPSHOT_FLAG_NODE = 2            # snapshot.rs:314
SNAPSHOT_FLAG_REPLICA_ADD = 3     # snapshot.rs:315
SNAPSHOT_FLAG_REPLICA_REM = 4     # snapshot.rs:316
SNAPSHOT_FLAG_DATAS = 5           # snapshot.rs:317
SNAPSHOT_FLAG_EXPIRES = 6         # snapshot.rs:318
SNAPSHOT_FLAG_DELETES = 7         # snapshot.rs:319
SNAPSHOT_FLAG_CHECKSUM = 8        # snapshot.rs:320

OBJECT_ENC_COUNTER = 0            # object.rs:19
OBJECT_ENC_BYTES = 3              # object.rs:20
OBJECT_ENC_DICT = 4               # object.rs:21
OBJECT_ENC_SET = 5                # object.rs:22


class SnapshotWriter:
    """snapshot.rs:9-69. Keeps a running CRC-64 over every byte written."""

    def __init__(self):
        self.buf = io.BytesIO()
        self.crc = 0

    def write_bytes(self, b: bytes) -> "SnapshotWriter":  # snapshot.rs:39-46
        b = bytes(b)
        self.crc = crc64_update(self.crc, b)
        self.buf.write(b)
        return self

    def write_byte(self, d: int) -> "SnapshotWriter":  # snapshot.rs:54-56
        return self.write_bytes(bytes([d & 0xFF]))

    def write_integer(self, i: int) -> "SnapshotWriter":  # snapshot.rs:25-37
        i = to_i64(i)
        if i < (1 << 6):
            # `[i as u8]`: negative values are truncated to one byte
            return self.write_bytes(bytes([i & 0xFF]))
        elif i < (1 << 14):
            v = (i & 0xFFFF) | (1 << 14)          # (i as i16) | 1 << 14
            return self.write_bytes(struct.pack(">H", v & 0xFFFF))
        elif i < (1 << 30):
            v = (i & 0xFFFFFFFF) | (1 << 31)      # (i as i32) | 1 << 31
            return self.write_bytes(struct.pack(">I", v & 0xFFFFFFFF))
        else:
            self.write_bytes(bytes([3 << 6]))
            return self.write_bytes(struct.pack(">q", i))

    def write_entry(self, key: bytes, obj: "Object") -> None:  # snapshot.rs:48-52
        self.write_integer(len(key))
        self.write_bytes(key)
        obj.save_snapshot(self)

    def checksum(self) -> int:  # snapshot.rs:62-64
        return self.crc

    def getvalue(self) -> bytes:
        return self.buf.getvalue()


# --------------------------------------------------------------------------------------
# CRDT types
# --------------------------------------------------------------------------------------
class LWWHash:
    """crdt/lwwhash.rs:11-128. add: member -> (t, value); dele: member -> t."""

    def __init__(self):
        self.size = 0                       # not serialized; excluded from parity
        self.add: Dict[bytes, Tuple[int, object]] = {}
        self.dele: Dict[bytes, int] = {}

    def set(self, k: bytes, v, t: int) -> bool:  # lwwhash.rs:87-107
        d = self.dele.get(k)
        if d is not None and d > t:
            return False
        a = self.add.get(k)
        if a is not None:
            if a[0] > t:
                return False
            self.add[k] = (t, v)
        else:
            self.dele.pop(k, None)
            self.add[k] = (t, v)
        self.size += 1
        return True

    def rem(self, k: bytes, t: int) -> bool:  # lwwhash.rs:109-128
        a = self.add.get(k)
        if a is not None and a[0] > t:
            return False
        d = self.dele.get(k)
        if d is not None:
            if d > t:
                return False
            self.dele[k] = t
        else:
            self.dele[k] = t
            self.add.pop(k, None)
        self.size -= 1
        return True

    def remove_time(self, k: bytes) -> Optional[int]:  # lwwhash.rs:54-66
        a, d = self.add.get(k), self.dele.get(k)
        if d is None:
            return None
        if a is None:
            return d
        return d if a[0] < d else None

    def remove_actually(self, k: bytes) -> None:  # lwwhash.rs:68-71
        self.add.pop(k, None)
        self.dele.pop(k, None)

    def live_iter(self):
        """SetIter / DictIter (lwwhash.rs:229-248, 361-380): adds not shadowed by a
        later-or-equal... strictly later del."""
        for k, (t, v) in list(self.add.items()):
            tt = self.dele.get(k)
            if tt is not None and tt > t:
                continue
            yield k, t, v

    def copy(self) -> "LWWHash":
        h = type(self)()
        h.size = self.size
        h.add = dict(self.add)
        h.dele = dict(self.dele)
        return h


class Set(LWWHash):  # lwwhash.rs:263-359
    def merge(self, other: "Set") -> None:  # lwwhash.rs:319-323
        for k, t, _ in other.live_iter():
            self.set(k, None, t)


class DictMergePanic(Exception):
    """lwwhash.rs:180 `unimplemented!()` — raised after the pre-panic loop ran."""


class Dict(LWWHash):  # lwwhash.rs:131-227
    def merge(self, other: "Dict", panic: bool = False) -> None:  # lwwhash.rs:176-181
        for k, t, v in other.live_iter():
            self.set(k, v, t)
        if panic:
            raise DictMergePanic()


class Counter:
    """type_counter.rs:18-126. data: node -> (v, t); sum is the load total or cal_sum."""

    def __init__(self):
        self.sum = 0
        self.data: Dict[int, Tuple[int, int]] = {}

    def merge(self, other: "Counter") -> None:  # type_counter.rs:59-87
        for nodeid in list(self.data.keys()):
            v, t = self.data[nodeid]
            o = other.data.get(nodeid)
            if o is not None:
                vv, tt = o
                if tt > t:
                    v = vv
                elif tt == t:
                    v = max(v, vv)
                self.data[nodeid] = (v, t)          # t is never updated
        for nodeid, (vv, tt) in other.data.items():
            cur = self.data.get(nodeid)
            if cur is not None:
                v, t = cur
                if tt > t:
                    v = vv
                elif tt == t:
                    v = max(v, vv)
                self.data[nodeid] = (v, t)
            else:
                self.data[nodeid] = (vv, tt)
        self.cal_sum()

    def cal_sum(self) -> None:  # type_counter.rs:89-91 (wrapping i64 in release)
        self.sum = to_i64(sum(v for v, _ in self.data.values()))

    def copy(self) -> "Counter":
        c = Counter()
        c.sum = self.sum
        c.data = dict(self.data)
        return c


TYPE_NAMES = {OBJECT_ENC_COUNTER: "counter", OBJECT_ENC_BYTES: "bytes",
              OBJECT_ENC_DICT: "dict", OBJECT_ENC_SET: "set"}


@dataclass
class Object:
    """object.rs:11-17. enc is one of Counter | bytes | Set | Dict; tag the wire tag."""
    create_time: int
    update_time: int
    delete_time: int
    tag: int
    enc: object

    def merge(self, other: "Object", dict_panic: bool = False) -> bool:  # object.rs:63-83
        my_ct, my_dt, my_ut = self.create_time, self.delete_time, self.update_time
        his_ct, his_dt, his_ut = other.create_time, other.delete_time, other.update_time
        if self.tag != other.tag:
            return False                                   # object.rs:80 Err(())
        if self.tag == OBJECT_ENC_COUNTER:
            self.enc.merge(other.enc)
        elif self.tag == OBJECT_ENC_BYTES:                 # object.rs:69-77
            if my_ct < his_ct:
                self.enc = other.enc
            self.create_time = max(my_ct, his_ct)
            self.delete_time = max(my_dt, his_dt)
            self.update_time = max(my_ut, his_ut)
        elif self.tag == OBJECT_ENC_DICT:
            self.enc.merge(other.enc, panic=dict_panic)
        elif self.tag == OBJECT_ENC_SET:
            self.enc.merge(other.enc)
        return True

    def save_snapshot(self, w: SnapshotWriter, bytes_len_prefix: bool = True) -> None:
        """object.rs:85-108. The reference writer emits Bytes values with NO length
        (object.rs:94-97) while its loader expects `len, bytes` (object.rs:114-117);
        fixtures use the loader's layout (bytes_len_prefix=True), see DESIGN.md."""
        w.write_integer(self.create_time)
        w.write_integer(self.update_time)
        w.write_integer(self.delete_time)
        w.write_byte(self.tag)
        if self.tag == OBJECT_ENC_COUNTER:                  # type_counter.rs:101-109
            w.write_integer(len(self.enc.data))
            for nodeid, (v, t) in self.enc.data.items():
                w.write_integer(nodeid)
                w.write_integer(v)
                w.write_integer(t)
        elif self.tag == OBJECT_ENC_BYTES:
            if bytes_len_prefix:
                w.write_integer(len(self.enc))
            w.write_bytes(self.enc)
        elif self.tag == OBJECT_ENC_SET:                    # lwwhash.rs:325-339
            w.write_integer(len(self.enc.add))
            for k, (t, _) in self.enc.add.items():
                w.write_integer(len(k)); w.write_bytes(k); w.write_integer(t)
            w.write_integer(len(self.enc.dele))
            for k, t in self.enc.dele.items():
                w.write_integer(len(k)); w.write_bytes(k); w.write_integer(t)
        elif self.tag == OBJECT_ENC_DICT:                   # lwwhash.rs:189-205
            w.write_integer(len(self.enc.add))
            for k, (t, v) in self.enc.add.items():
                w.write_integer(len(k)); w.write_bytes(k); w.write_integer(t)
                w.write_integer(len(v)); w.write_bytes(v)
            w.write_integer(len(self.enc.dele))
            for k, t in self.enc.dele.items():
                w.write_integer(len(k)); w.write_bytes(k); w.write_integer(t)
        else:
            raise InvalidType()

    def copy(self) -> "Object":
        enc = self.enc.copy() if hasattr(self.enc, "copy") else self.enc
        return Object(self.create_time, self.update_time, self.delete_time, self.tag, enc)


# --------------------------------------------------------------------------------------
# Snapshot loader (snapshot.rs:99-301)
# --------------------------------------------------------------------------------------
@dataclass
class Entry:
    kind: str          # Version | Node | ReplicaAdd | ReplicaDel | Data | Expires | Deletes
    args: tuple


class SnapshotLoader:
    """Literal restatement of snapshot.rs:107-301 over an in-memory buffer.

    checksum_mode:
      "reference" — snapshot.rs:207-213 exactly: the checksum is read with
                    read_integer and compared against a CRC that by then also covers
                    the checksum bytes (practically always InvalidSnapshotChecksum;
                    SURVEY §8a R2);
      "writer"    — the writer's layout (server.rs:205-207): 8 raw LE bytes of CRC over
                    everything up to and including flag 0x08. This is what the product
                    decoder verifies by default.
    """

    def __init__(self, data: bytes, checksum_mode: str = "writer"):
        self.data = bytes(data)
        self.off = 0
        self.crc = 0
        self.stat = ("Begin",)
        self.checksum_mode = checksum_mode

    # snapshot.rs:266-274
    def read_bytes(self, n: int) -> bytes:
        if n < 0 or self.off + n > len(self.data):
            raise IoError("unexpected eof")
        b = self.data[self.off:self.off + n]
        self.off += n
        self.crc = crc64_update(self.crc, b)
        return b

    def read_byte(self) -> int:  # snapshot.rs:276-278
        return self.read_bytes(1)[0]

    def read_integer(self) -> int:  # snapshot.rs:243-264
        flag = self.read_byte()
        k = (flag >> 6) & 3
        if k == 0:
            return flag & 0x3F
        if k == 1:
            return ((flag & 0x3F) << 8) | self.read_byte()
        if k == 2:
            b = self.read_bytes(3)
            return ((flag & 0x3F) << 24) | (b[0] << 16) | (b[1] << 8) | b[2]
        return struct.unpack(">q", self.read_bytes(8))[0]

    def _read_len(self) -> int:
        n = self.read_integer()
        if n < 0:  # `as usize` of a negative i64 -> an impossible read -> EOF
            raise IoError("unexpected eof")
        return n

    def _read_str(self) -> str:
        b = self.read_bytes(self._read_len())
        try:
            return b.decode("utf-8")
        except UnicodeDecodeError:  # snapshot.rs:143-145 unwraps -> panic; reported here
            raise InvalidSnapshot(self.off)

    def read_entry(self) -> Tuple[bytes, Object]:  # snapshot.rs:280-287
        key = self.read_bytes(self._read_len())
        return key, self.load_object()

    def read_key_int(self) -> Tuple[bytes, int]:  # snapshot.rs:289-295
        key = self.read_bytes(self._read_len())
        return key, to_u64(self.read_integer())

    def load_object(self) -> Object:  # object.rs:110-129
        ct = to_u64(self.read_integer())
        mt = to_u64(self.read_integer())
        dt = to_u64(self.read_integer())
        tag = self.read_byte()
        if tag == OBJECT_ENC_COUNTER:                      # type_counter.rs:111-126
            cnt = self._read_len()
            c = Counter()
            total = 0
            for _ in range(cnt):
                n = to_u64(self.read_integer())
                v = self.read_integer()
                t = to_u64(self.read_integer())
                c.data[n] = (v, t)
                total = to_i64(total + v)
            c.sum = total
            enc = c
        elif tag == OBJECT_ENC_BYTES:                      # object.rs:114-118
            s = self.read_integer()
            if s < 0:
                raise IoError("unexpected eof")
            enc = self.read_bytes(s)
        elif tag == OBJECT_ENC_SET:                        # lwwhash.rs:341-358
            s = Set()
            for _ in range(self._read_len()):
                k = self.read_bytes(self._read_len())
                t = to_u64(self.read_integer())
                s.set(k, None, t)
            for _ in range(self._read_len()):
                k = self.read_bytes(self._read_len())
                t = to_u64(self.read_integer())
                s.rem(k, t)
            enc = s
        elif tag == OBJECT_ENC_DICT:                       # lwwhash.rs:207-226
            d = Dict()
            for _ in range(self._read_len()):
                k = self.read_bytes(self._read_len())
                t = to_u64(self.read_integer())
                v = self.read_bytes(self._read_len())
                d.set(k, v, t)
            for _ in range(self._read_len()):
                k = self.read_bytes(self._read_len())
                t = to_u64(self.read_integer())
                d.rem(k, t)
            enc = d
        else:
            raise InvalidType()                            # object.rs:121
        return Object(ct, mt, dt, tag, enc)

    def convert_stat(self) -> None:  # snapshot.rs:222-241
        flag = self.read_byte()
        if flag == SNAPSHOT_FLAG_REPLICA_ADD:
            self.stat = ("Replicas", True)
        elif flag == SNAPSHOT_FLAG_REPLICA_REM:
            self.stat = ("Replicas", False)
        elif flag == SNAPSHOT_FLAG_DATAS:
            self.stat = ("Datas", self._read_len(), 0)
        elif flag == SNAPSHOT_FLAG_DELETES:
            self.stat = ("Deletes", self._read_len(), 0)
        elif flag == SNAPSHOT_FLAG_EXPIRES:
            self.stat = ("Expires", self._read_len(), 0)
        elif flag == SNAPSHOT_FLAG_CHECKSUM:
            self.stat = ("Checksum",)
        else:
            raise InvalidSnapshot(self.off)

    def next(self) -> Optional[Entry]:  # snapshot.rs:120-220
        while True:
            s = self.stat
            if s[0] == "Begin":
                self.read_bytes(7)                         # magic is not checked
                self.stat = ("Version",)
            elif s[0] == "Version":
                v = self.read_bytes(4)
                self.stat = ("Node",)
                return Entry("Version", (f"{v[0]}.{v[1]}.{v[2]}.{v[3]}",))
            elif s[0] == "Node":
                nodeid = to_u64(self.read_integer())
                alias = self._read_str()
                addr = self._read_str()
                uuid = to_u64(self.read_integer())
                self.convert_stat()
                return Entry("Node", (nodeid, alias, addr, uuid))
            elif s[0] == "Replicas" and s[1]:
                add_time = to_u64(self.read_integer())
                nodeid = to_u64(self.read_integer())
                alias = self._read_str()
                addr = self._read_str()
                uuid = to_u64(self.read_integer())
                self.convert_stat()
                return Entry("ReplicaAdd", (add_time, nodeid, alias, addr, uuid))
            elif s[0] == "Replicas":
                addr = self._read_str()
                t = to_u64(self.read_integer())
                self.convert_stat()
                return Entry("ReplicaDel", (addr, t))
            elif s[0] in ("Datas", "Deletes", "Expires"):
                size, cur = s[1], s[2]
                if cur < size:
                    self.stat = (s[0], size, cur + 1)
                    if s[0] == "Datas":
                        return Entry("Data", self.read_entry())
                    return Entry(s[0], self.read_key_int())
                self.convert_stat()
            elif s[0] == "Checksum":
                if self.checksum_mode == "reference":
                    got = self.read_integer()
                    if to_u64(got) != self.crc:
                        raise InvalidSnapshotChecksum()
                else:
                    expect = self.crc
                    got = struct.unpack("<Q", self.read_bytes(8))[0]
                    if got != expect:
                        raise InvalidSnapshotChecksum()
                self.stat = ("Finish",)
            else:
                return None


def load_snapshot(data: bytes, checksum_mode: str = "writer") -> List[Entry]:
    ld = SnapshotLoader(data, checksum_mode)
    out = []
    while True:
        e = ld.next()
        if e is None:
            return out
        out.append(e)


# --------------------------------------------------------------------------------------
# DB (db.rs:10-137)
# --------------------------------------------------------------------------------------
class DB:
    def __init__(self):
        self.data: Dict[bytes, Object] = {}
        self.expires: Dict[bytes, int] = {}
        self.deletes: Dict[bytes, int] = {}
        self.garbages: List[Tuple[bytes, Optional[bytes], int]] = []
        # build-side observability, not reference state
        self.type_conflicts = 0
        self.dict_merges = 0

    def merge_entry(self, key: bytes, value: Object, dict_panic: bool = False) -> None:
        """db.rs:31-43."""
        o = self.data.get(key)
        if o is None:
            self.data[key] = value
            return
        if o.tag == OBJECT_ENC_DICT and value.tag == OBJECT_ENC_DICT:
            self.dict_merges += 1
        if not o.merge(value, dict_panic=dict_panic):
            self.type_conflicts += 1                       # error! log; local kept

    def expire_at(self, key: bytes, t: int) -> None:  # db.rs:68-71
        self.expires[key] = t

    def delete(self, key: bytes, t: int) -> None:  # db.rs:73-76
        self.deletes[key] = t
        self.garbages.append((key, None, t))

    def gc(self, tombstone: int) -> None:  # db.rs:82-119 (LIFO, stops at first t > wm)
        while self.garbages:
            key, fld, t = self.garbages.pop()
            if t > tombstone:
                break
            if fld is None:
                v = self.deletes.get(key)
                if v is not None and v == t:
                    del self.deletes[key]
            else:  # dead path in the reference (delete_field is never called)
                o = self.data.get(key)
                if o is not None and o.tag in (OBJECT_ENC_DICT, OBJECT_ENC_SET):
                    rt = o.enc.remove_time(fld)
                    if rt is not None and rt < t:
                        o.enc.remove_actually(fld)

    def gc_member_tombstones(self, watermark: int) -> int:
        """BUILD EXTENSION (not reference behaviour, labelled as such in DESIGN.md):
        drop del-only members whose delete time is < watermark — what db.rs:96-115's
        field branch would do if delete_field (db.rs:78-80) were ever called."""
        n = 0
        for o in self.data.values():
            if o.tag in (OBJECT_ENC_DICT, OBJECT_ENC_SET):
                for k, t in list(o.enc.dele.items()):
                    if k not in o.enc.add and t < watermark:
                        del o.enc.dele[k]
                        n += 1
        return n

    def dump(self, w: SnapshotWriter) -> None:  # db.rs:122-136
        w.write_byte(SNAPSHOT_FLAG_DATAS).write_integer(len(self.data))
        for k, v in self.data.items():
            w.write_entry(k, v)
        w.write_byte(SNAPSHOT_FLAG_EXPIRES).write_integer(len(self.expires))
        for k, v in self.expires.items():
            w.write_integer(len(k)).write_bytes(k).write_integer(v)
        w.write_byte(SNAPSHOT_FLAG_DELETES).write_integer(len(self.deletes))
        for k, v in self.deletes.items():
            w.write_integer(len(k)).write_bytes(k).write_integer(v)


@dataclass
class NodeHeader:
    node_id: int = 1
    alias: str = "n1"
    addr: str = "127.0.0.1:9001"
    last_uuid: int = 0
    replicas_add: List[Tuple[int, int, str, str, int]] = field(default_factory=list)
    replicas_del: List[Tuple[str, int]] = field(default_factory=list)


def dump_all(db: DB, hdr: NodeHeader) -> bytes:
    """server.rs:183-215 + replica/replica.rs:100-119 (writer layout, Bytes len-prefixed)."""
    w = SnapshotWriter()
    w.write_bytes(b"CONSTDB")
    w.write_bytes(bytes([0, 1, 1, 1]))
    a, ad = hdr.alias.encode(), hdr.addr.encode()
    w.write_integer(hdr.node_id).write_integer(len(a)).write_bytes(a)
    w.write_integer(len(ad)).write_bytes(ad).write_integer(hdr.last_uuid)
    db.dump(w)
    for (t, nid, alias, addr, uuid) in hdr.replicas_add:
        al, adr = alias.encode(), addr.encode()
        w.write_byte(SNAPSHOT_FLAG_REPLICA_ADD).write_integer(t).write_integer(nid)
        w.write_integer(len(al)).write_bytes(al).write_integer(len(adr)).write_bytes(adr)
        w.write_integer(uuid)
    for (addr, t) in hdr.replicas_del:
        adr = addr.encode()
        w.write_byte(SNAPSHOT_FLAG_REPLICA_REM).write_integer(len(adr)).write_bytes(adr)
        w.write_integer(t)
    w.write_byte(SNAPSHOT_FLAG_CHECKSUM)
    w.write_bytes(struct.pack("<Q", w.checksum()))
    return w.getvalue()


# --------------------------------------------------------------------------------------
# The fold (replica/pull.rs:116-159): R snapshots applied in pos order into an empty DB.
# pos 0 plays the local DB (merging into an empty DB inserts verbatim, db.rs:33-35).
# --------------------------------------------------------------------------------------
def fold_snapshots(snapshots: List[bytes], dict_panic: bool = False,
                   checksum_mode: str = "writer") -> DB:
    db = DB()
    for snap in snapshots:
        for e in load_snapshot(snap, checksum_mode):
            if e.kind == "Data":
                k, v = e.args
                db.merge_entry(k, v, dict_panic=dict_panic)
            elif e.kind == "Deletes":
                db.delete(*e.args)
            elif e.kind == "Expires":
                db.expire_at(*e.args)
            # Version / Node / ReplicaAdd / ReplicaDel: replica metadata, host-side
    return db


def fold_replicas(snapshots: List[bytes], checksum_mode: str = "writer") -> List[dict]:
    """Replica-metadata merge (replica/pull.rs:131-156): ReplicaManager.replicas is an
    LWWHash<addr, ReplicaMeta> (replica/replica.rs:16-35). Snapshot 0 is the local node: its
    ReplicaAdd / ReplicaDel entries ARE its add / del maps (dump_snapshot, replica.rs:100-119).
    Every later snapshot is applied in stream order: ReplicaAdd -> add_replica -> set
    (skipped when it names the local node id, pull.rs:133-135), ReplicaDel -> remove_replica
    -> rem. Returns one dict per addr, sorted by addr (the shape of Merged.replicas())."""
    h = LWWHash()
    myself = None
    for i, snap in enumerate(snapshots):
        for e in load_snapshot(snap, checksum_mode):
            if e.kind == "Node" and i == 0:
                myself = e.args[0]
            elif e.kind == "ReplicaAdd":
                add_time, nid, alias, addr, uuid = e.args
                if i == 0:
                    h.add[addr.encode()] = (add_time, (nid, alias, uuid))
                elif nid != myself:
                    h.set(addr.encode(), (nid, alias, uuid), add_time)
            elif e.kind == "ReplicaDel":
                addr, t = e.args
                if i == 0:
                    h.dele[addr.encode()] = t
                else:
                    h.rem(addr.encode(), t)
    out = []
    for k in sorted(set(h.add) | set(h.dele)):
        d = {"addr": k.decode()}
        if k in h.add:
            t, (nid, alias, uuid) = h.add[k]
            d["add"] = (t, nid, alias, uuid)
        if k in h.dele:
            d["del"] = h.dele[k]
        out.append(d)
    return out


# --------------------------------------------------------------------------------------
# Canonical dump (the parity contract): keys sorted by bytes, members by
# bytes, counter nodes by id. Text, one record per line; identical format in
# oracle/cdb_oracle.cpp and the product's cdb_canonical_dump().
# --------------------------------------------------------------------------------------
def canonical_dump(db: DB) -> bytes:
    out = []
    for k in sorted(db.data):
        o = db.data[k]
        out.append(f"K {k.hex()} {o.tag} {o.create_time} {o.update_time} {o.delete_time}")
        if o.tag == OBJECT_ENC_BYTES:
            out.append(f" V {o.enc.hex()}")
        elif o.tag == OBJECT_ENC_COUNTER:
            out.append(f" S {o.enc.sum}")
            for n in sorted(o.enc.data):
                v, t = o.enc.data[n]
                out.append(f" N {n} {v} {t}")
        else:
            members = sorted(set(o.enc.add) | set(o.enc.dele))
            for m in members:
                if m in o.enc.add:
                    t, v = o.enc.add[m]
                    if o.tag == OBJECT_ENC_DICT:
                        out.append(f" A {m.hex()} {t} {v.hex()}")
                    else:
                        out.append(f" A {m.hex()} {t}")
                if m in o.enc.dele:
                    out.append(f" D {m.hex()} {o.enc.dele[m]}")
    for k in sorted(db.expires):
        out.append(f"X {k.hex()} {db.expires[k]}")
    for k in sorted(db.deletes):
        out.append(f"R {k.hex()} {db.deletes[k]}")
    return ("\n".join(out) + "\n").encode() if out else b""
