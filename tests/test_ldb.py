"""LevelDB-format store (csrc/store/ldb.cpp).

Engine behaviour (random ops against a dict model across flushes, compactions, multi-level
trees and reopen; torn write-ahead-log tails; a held LOCK) plus the format cross-check both
ways against the reference's own LevelDB compiled from its source tree (tools/ref_leveldb.sh):
a store written here is dumped and point-read by the reference library with paranoid checks
and checksum verification (point reads go through the bloom filters, so a wrong filter loses
keys), and a multi-level store the reference library wrote is read here.
"""
import os
import random
import shutil
import subprocess

import pytest

from nodexa_chain_core_amd import core

_core = core()
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF_LEVELDB = "/root/reference/src/leveldb"


def _random_ops(rng, n, ref, db):
    for _ in range(n):
        if ref and rng.random() < 0.25:
            k = rng.choice(sorted(ref))
            db.delete(k)
            del ref[k]
        else:
            k = bytes(rng.randrange(256) for _ in range(rng.randrange(1, 14)))
            v = bytes(rng.randrange(256) for _ in range(rng.randrange(0, 120)))
            db.put(k, v)
            ref[k] = v


def test_random_ops_flush_compact_reopen(tmp_path):
    rng = random.Random(11)
    path = str(tmp_path / "db")
    kw = dict(write_buffer_size=32 << 10, max_file_size=16 << 10, level1_bytes=64 << 10)
    db = _core.LevelDB(path, **kw)
    ref = {}
    _random_ops(rng, 15000, ref, db)
    levels = db.files_per_level()
    assert sum(1 for n in levels[1:] if n) >= 2, levels  # data reached level 2 or deeper
    assert dict(db.items()) == ref
    keys = sorted(ref)
    for k in keys[::7]:
        assert db.get(k) == ref[k]
    assert db.get(b"\xff" * 20) is None
    # range scans
    lo, hi = keys[len(keys) // 4], keys[len(keys) // 2]
    assert [k for k, _ in db.items(lo, hi)] == [k for k in keys if lo <= k < hi]
    seq = db.last_sequence
    db.close()
    db = _core.LevelDB(path, **kw)
    assert db.last_sequence == seq
    assert dict(db.items()) == ref
    _random_ops(rng, 3000, ref, db)
    db.write([(b"batch-a", b"1"), (b"batch-b", b"2"), (b"batch-a", None)], sync=True)
    ref[b"batch-b"] = b"2"
    ref.pop(b"batch-a", None)
    db.compact()
    assert sum(db.files_per_level()[:-1]) == 0 or db.files_per_level()[0] == 0
    assert dict(db.items()) == ref
    db.close()


def test_unsynced_tail_and_torn_log(tmp_path):
    path = str(tmp_path / "db")
    db = _core.LevelDB(path)
    for i in range(200):
        db.put(b"k%04d" % i, b"v" * 50)
    db.close()
    logs = sorted(f for f in os.listdir(path) if f.endswith(".log"))
    # the records live in the log until the next open folds them into a table; cut the log
    # in the middle of its last record (a crash mid-append)
    log = os.path.join(path, logs[-1])
    size = os.path.getsize(log)
    assert size > 1000
    with open(log, "r+b") as f:
        f.truncate(size - 30)
    db = _core.LevelDB(path)
    got = dict(db.items())
    assert len(got) == 199 and all(got[b"k%04d" % i] == b"v" * 50 for i in range(199))
    db.close()


def test_lock_excludes_second_open(tmp_path):
    path = str(tmp_path / "db")
    db = _core.LevelDB(path)
    # fcntl locks are per process: a second process must fail to open the store
    r = subprocess.run(["python3", "-c", f"from nodexa_chain_core_amd import core; core().LevelDB({path!r})"],
                       cwd=ROOT, capture_output=True, text=True)
    assert r.returncode != 0 and "in use" in r.stderr
    # fcntl locks are per process, so this process keeps its own set of open stores
    with pytest.raises(Exception, match="already open in this process"):
        _core.LevelDB(path)
    (tmp_path / "x").mkdir()
    with pytest.raises(Exception, match="already open in this process"):
        _core.LevelDB(str(tmp_path / "x" / ".." / "db"))  # the same store under another spelling
    db.close()
    db2 = _core.LevelDB(path)  # closing released it
    db2.close()


def test_crc32c_bloom_hash_and_snappy():
    # CRC-32C check value and the RFC 3720 32-zero-byte vector
    assert _core.ldb_crc32c(b"123456789") == 0xE3069283
    assert _core.ldb_crc32c(bytes(32)) == 0x8A9136AA
    assert _core.ldb_bloom_hash(b"") == 0xBC9F1D34  # seed only, no tail mixing
    # snappy: literal "abcd" then copy-1 of length 8 at offset 4 -> "abcd" * 3
    raw = bytes([12, (4 - 1) << 2]) + b"abcd" + bytes([((8 - 4) << 2) | 1, 4])
    assert _core.snappy_uncompress(raw) == b"abcd" * 3
    assert _core.snappy_uncompress(bytes([12, 0x01, 0])) is None  # copy before any output


@pytest.fixture(scope="module")
def ref_tool():
    if not os.path.isdir(REF_LEVELDB):
        pytest.skip("reference LevelDB sources not present")
    try:
        out = subprocess.run(["bash", os.path.join(ROOT, "tools", "ref_leveldb.sh")], capture_output=True, text=True,
                             timeout=600, check=True)
    except (subprocess.CalledProcessError, OSError, subprocess.TimeoutExpired) as e:  # pragma: no cover
        pytest.skip(f"cannot build the reference LevelDB: {e}")
    return out.stdout.strip().splitlines()[-1]


def _ref(tool, *args, stdin=""):
    r = subprocess.run([tool, *args], input=stdin, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    return r.stdout


def test_reference_library_reads_our_store(tmp_path, ref_tool):
    rng = random.Random(3)
    path = str(tmp_path / "ours")
    db = _core.LevelDB(path, write_buffer_size=32 << 10, max_file_size=16 << 10, level1_bytes=64 << 10)
    ref = {}
    _random_ops(rng, 12000, ref, db)
    db.close()
    dump = _ref(ref_tool, "dump", path)
    got = {}
    for line in dump.splitlines():
        k, _, v = line.partition(" ")
        got[bytes.fromhex(k)] = bytes.fromhex(v)
    assert got == ref
    keys = sorted(ref)[::3] + [b"\xfe" * 9, b"absent"]
    out = _ref(ref_tool, "get", path, stdin="\n".join(k.hex() for k in keys) + "\n").split("\n")
    for k, line in zip(keys, out):
        assert (bytes.fromhex(line) if line != "-" else None) == ref.get(k), k
    # the reference can keep writing to (and compacting) it, and we read the result back
    _ref(ref_tool, "load", path, str(64 << 10), stdin="P 6e6577 76616c\nD " + sorted(ref)[0].hex() + "\n")
    ref[b"new"] = b"val"
    del ref[sorted(ref)[0]]
    _ref(ref_tool, "compact", path)
    db = _core.LevelDB(path)
    assert dict(db.items()) == ref
    db.close()


def test_we_read_reference_written_store(tmp_path, ref_tool):
    rng = random.Random(4)
    path = str(tmp_path / "theirs")
    ref, lines = {}, []
    for _ in range(30000):
        if ref and rng.random() < 0.2:
            k = rng.choice(list(ref))
            lines.append("D " + k.hex())
            del ref[k]
        else:
            k = bytes(rng.randrange(256) for _ in range(rng.randrange(1, 14)))
            v = bytes(rng.randrange(256) for _ in range(rng.randrange(0, 120)))
            lines.append(f"P {k.hex()} {v.hex() or '_'}")
            ref[k] = v
    _ref(ref_tool, "load", path, str(48 << 10), stdin="\n".join(lines) + "\n")
    assert any(f.endswith(".ldb") for f in os.listdir(path))
    db = _core.LevelDB(path)
    assert dict(db.items()) == ref
    for k in sorted(ref)[::11]:
        assert db.get(k) == ref[k]
    db.put(b"mine", b"1")
    db.close()
    assert bytes.fromhex(_ref(ref_tool, "get", path, stdin=b"mine".hex() + "\n").strip()) == b"1"
    shutil.rmtree(path)


def test_bounded_open_tables(tmp_path):
    """max_open_files: with far more table files than the bound, point reads and scans still see
    every key (least recently used tables are closed and reopened on demand)."""
    rng = random.Random(9)
    path = str(tmp_path / "db")
    kw = dict(write_buffer_size=8 << 10, max_file_size=4 << 10, level1_bytes=1 << 30, max_open_files=3)
    db = _core.LevelDB(path, **kw)
    ref = {}
    _random_ops(rng, 6000, ref, db)
    assert sum(db.files_per_level()) > 20
    for k in sorted(ref)[::5]:
        assert db.get(k) == ref[k]
    assert dict(db.items()) == ref
    db.close()
    db = _core.LevelDB(path, **kw)
    assert dict(db.items()) == ref
    db.close()
