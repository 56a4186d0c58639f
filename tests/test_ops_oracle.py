"""Op-stream apply, CPU side: the oracle against hand-derived known answers, the
host decoder (cdb_decode_ops, no GPU needed) against the oracle's stream-level accounting, and
the RESP framing rules of conn/buf_read.rs."""
import pytest

import constdb_amd as cdb
import constdb_oracle as o
import constdb_ops_oracle as oo
from ops_kats import cases
from opsgen import gen_stream
from snapgen import gen_replicas


@pytest.mark.parametrize("case", cases(), ids=lambda c: c[0])
def test_oracle_kat(case):
    name, snap, stream, u0, want = case
    db = o.fold_snapshots([snap])
    oo.apply_replicates(db, stream, u0)
    assert o.canonical_dump(db).decode() == want


def test_resp_framing():
    assert oo.resp_parse_stream(b"*2\r\n$3\r\nabc\r\n:-12\r\n") == [("arr", [("bulk", b"abc"), ("int", -12)])]
    assert oo.resp_parse_stream(b"$-1\r\n+OK\r\n-ERR x\r\n") == [("nil", None), ("str", b"OK"), ("err", b"ERR x")]
    assert oo.bytes2i64(b"12ab") == 12 and oo.bytes2i64(b"-") is None and oo.bytes2i64(b"") is None
    for bad in (b"$3\r\na\r\nb\r\n", b"?x\r\n", b":x\r\n", b"*x\r\n"):  # CRLF inside a bulk payload, bad type, bad ints
        with pytest.raises(oo.InvalidRequestMsg):
            oo.resp_parse_stream(bad)


def _lib_ok():
    try:
        cdb.lib()
        return True
    except OSError:
        return False


needs_lib = pytest.mark.skipif(not _lib_ok(), reason="libcdbmerge.so not built")


@needs_lib
def test_decode_ops_errors():
    good = oo.replicate_msg(1, 5, 6, "set", b"k", b"v")
    with pytest.raises(cdb.InvalidRequestMsg) as e:
        cdb.decode_ops(good + b"$3\r\na\r\nb\r\n", 5)
    assert e.value.offset == len(good)
    with pytest.raises(cdb.NeedMoreMsg):
        cdb.decode_ops(good + good[:-3], 5)
    part = cdb.decode_ops(good + good[:-3], 5, allow_partial=True)
    assert not part.complete and part.consumed == len(good) and part.info().n_ops == 1


@needs_lib
@pytest.mark.parametrize("seed", range(40))
def test_decode_ops_matches_oracle_accounting(seed):
    snaps = gen_replicas(seed, n_replicas=2)
    db = o.fold_snapshots(snaps)
    stream = gen_stream(seed, list(db.data) + list(db.expires), n_cmds=150)
    st = oo.apply_replicates(db, stream, 5)
    info = cdb.decode_ops(stream, 5).info()
    for f in ("applied", "duplicates", "lost", "unknown", "unsupported", "replacks", "uuid_he_sent", "uuid_he_acked"):
        assert getattr(info, f) == getattr(st, f), f
    assert info.cmd_errors <= st.cmd_errors  # the rest are InvalidType, found on the device
