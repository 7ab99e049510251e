"""Snapshot ingestion from the SYNC wire format: mkv_tree_build_wire parses the SCAN
response and the concatenated GET responses on the device. Checked against a restatement of the
reference client (src/sync.rs:150-214: read_line + trim_end, "KEYS <n>", "VALUE <v>" / "NOT_FOUND")
feeding the C oracle, including the reference's quirks (trailing whitespace trimmed, empty values are
a protocol error)."""
import pytest

pytestmark = pytest.mark.gpu

from merklekv_amd import MerkleError, MerkleTree  # noqa: E402
from oracle import coracle  # noqa: E402
from oracle.merkle_oracle import DEFAULT_SEED, pack, split_blob  # noqa: E402

WS = (" \t\n\x0b\x0c\r\u0085\u00a0\u1680" + "".join(chr(c) for c in range(0x2000, 0x200B))
      + "\u2028\u2029\u202f\u205f\u3000")  # Rust char::is_whitespace (Unicode White_Space)


def trim_end(b: bytes) -> bytes:
    """Rust str::trim_end (Unicode White_Space) on UTF-8 bytes (sync.rs:171, :203)."""
    return b.decode("utf-8", "surrogateescape").rstrip(WS).encode("utf-8", "surrogateescape")


def server_scan(keys) -> bytes:  # server.rs:580-587
    return b"KEYS %d\r\n" % len(keys) + b"".join(k + b"\r\n" for k in keys)


def server_get(v) -> bytes:  # server.rs:551-552
    return b"NOT_FOUND\r\n" if v is None else b"VALUE " + v + b"\r\n"


def client_snapshot(scan: bytes, gets: bytes):
    """sync.rs:122-143 + :150-214 restated: the records the reference would insert."""
    lines = scan.split(b"\n")
    head = trim_end(lines[0]).split()
    assert head[0] == b"KEYS"
    n = int(head[1])
    keys = [trim_end(l) for l in lines[1:1 + n]]
    glines = gets.split(b"\n")
    out = []
    for k, l in zip(keys, glines[:n]):
        l = trim_end(l)
        if l == b"NOT_FOUND":
            continue
        assert l.startswith(b"VALUE ")
        out.append((k, l[6:]))
    return out


def _oracle_root(records):
    if not records:
        return None
    return coracle.OracleTree.build(*pack([k for k, _ in records]), *pack([v for _, v in records])).root()


def test_wire_snapshot_synthetic_with_not_found():
    n = 20000
    kb, ko, vb, vo = coracle.gen_records(DEFAULT_SEED, 0, n)
    keys, vals = split_blob(kb, ko), split_blob(vb, vo)
    gets = [None if i % 97 == 5 else v for i, v in enumerate(vals)]  # keys deleted between SCAN and GET
    scan, get = server_scan(keys), b"".join(server_get(v) for v in gets)
    t = MerkleTree()
    t.build_wire(scan, get)
    rec = client_snapshot(scan, get)
    assert len(t) == len(rec) == n - len([g for g in gets if g is None])
    assert t.get_root_hash() == _oracle_root(rec)


def test_wire_trim_and_edge_records():
    keys = [b"a", b"b ", b"c\t", b"d\xc2\xa0", b"e\xe3\x80\x80", b"f\xe2\x80\x8b", b"g", b"dup", b"dup"]
    vals = [b"x  ", b"y", b"z\xe2\x80\xa8", b"w", b"v", b"u", b"with space inside", b"first", b"second"]
    scan, get = server_scan(keys), b"".join(server_get(v) for v in vals)
    t = MerkleTree()
    t.build_wire(scan, get)
    rec = client_snapshot(scan, get)
    assert [k for k, _ in rec][:3] == [b"a", b"b", b"c"]
    assert t.get_root_hash() == _oracle_root(rec)  # U+200B is not White_Space: kept; "dup": last wins


def test_wire_errors_match_reference():
    t = MerkleTree()
    with pytest.raises(MerkleError):
        t.build_wire(b"VALUES 1\r\nk v\r\n", b"VALUE v\r\n")       # not a KEYS header
    with pytest.raises(MerkleError):
        t.build_wire(b"KEYS 3\r\na\r\nb\r\n", b"VALUE 1\r\nVALUE 2\r\nVALUE 3\r\n")  # key list cut short
    with pytest.raises(MerkleError):
        t.build_wire(b"KEYS 2\r\na\r\nb\r\n", b"VALUE 1\r\n")      # a GET response missing
    with pytest.raises(MerkleError):
        t.build_wire(b"KEYS 1\r\na\r\n", b"VALUE \r\n")            # empty value: "VALUE" after trim_end
    with pytest.raises(MerkleError):
        t.build_wire(b"KEYS 1\r\na\r\n", b"ERROR boom\r\n")
    t.build_wire(b"KEYS 0\r\n", b"")
    assert t.get_root_hash() is None
    t.build_wire(b"KEYS 2\r\na\r\nb\r\n", b"NOT_FOUND\r\nNOT_FOUND\r\n")
    assert t.get_root_hash() is None and len(t) == 0
