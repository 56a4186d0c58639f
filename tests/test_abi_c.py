"""The C ABI from C: tests/abi/abi_check.c is compiled with the system C compiler against
include/cdb_merge.h and linked to libcdbmerge.so. Compiling it pins sizeof/offsetof of every
public struct a binding mirrors by hand (INTEGRATION.md's Rust structs); running it walks the
boundary a host takes: gen -> decode -> ctx -> merge -> canonical dump."""
import os
import subprocess

import pytest

import constdb_amd as cdb

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _compile(tmp_path):
    from constdb_amd import build
    build.build()
    exe = str(tmp_path / "abi_check")
    subprocess.check_call(["gcc", "-std=c11", "-Wall", "-Wextra", "-Werror", "-I", os.path.join(ROOT, "include"),
                           "-o", exe, os.path.join(ROOT, "tests", "abi", "abi_check.c"),
                           "-L", os.path.join(ROOT, "constdb_amd"), "-lcdbmerge",
                           "-Wl,-rpath," + os.path.join(ROOT, "constdb_amd")])
    return exe


def test_abi_layout_and_decode_from_c(tmp_path):
    """Compiles (the layout pins) and runs the decode half; without a device cdb_ctx_create must
    answer CDB_NO_DEVICE (no CPU fallback)."""
    exe = _compile(tmp_path)
    out = subprocess.run([exe, str(tmp_path / "dump.txt")], capture_output=True, text=True)
    assert out.returncode == 0, out.stderr
    assert "no device" in out.stdout or "merged" in out.stdout


def _entries(dump: bytes):
    """A canonical dump as (section, key hex) -> entry lines: a data key's K line with its indented
    child lines, an X (expires) or R (deletes) line."""
    out = {}
    cur = None
    for line in dump.decode().splitlines():
        if line.startswith(" "):
            out[cur].append(line)
            continue
        tag, key = line.split(" ", 2)[:2]
        cur = ({"K": 0, "X": 1, "R": 2}[tag], key)
        assert cur not in out
        out[cur] = [line]
    return out


def _join(dumps):
    """The canonical dump of the union of several shards' dumps (shards own disjoint keys)."""
    merged = {}
    for d in dumps:
        e = _entries(d)
        assert not set(e) & set(merged)
        merged.update(e)
    lines = [ln for k in sorted(merged) for ln in merged[k]]
    return ("\n".join(lines) + "\n").encode() if lines else b""


@pytest.mark.gpu
def test_abi_merge_from_c(tmp_path):
    """From C: the host-batch merge, the HBM-resident pull (decode into HBM as records -> merge into
    the bucket layout -> cdb_dev_state_rows + cdb_dev_input_append -> second merge -> host view), and
    a two-slot multi-device context (cdb_ctx_create_multi -> cdb_merge_sharded, an aliased input
    refused): every dump equal to the oracle's fold of the same three replicas."""
    import cdb_oracle
    exe = _compile(tmp_path)
    out = subprocess.run([exe, str(tmp_path / "dump.txt"), str(tmp_path / "chain.txt"), str(tmp_path / "shard")],
                         capture_output=True, text=True)
    assert out.returncode == 0, (out.returncode, out.stdout, out.stderr)
    assert "merged" in out.stdout and "device chain" in out.stdout and "sharded" in out.stdout
    cfg = cdb.gen_config(seed=17, universe=3000, n_replicas=3, replica_hi=3)
    rc, want, _ = cdb_oracle.fold([cdb.gen_snapshot(cfg, r) for r in range(3)])
    assert rc == 0
    assert (tmp_path / "dump.txt").read_bytes() == want
    assert (tmp_path / "chain.txt").read_bytes() == want
    shards = [(tmp_path / f"shard.{d}").read_bytes() for d in range(2)]
    assert all(shards)
    assert _join(shards) == want
