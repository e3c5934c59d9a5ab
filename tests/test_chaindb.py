"""Chain databases in the reference's LevelDB layout (chain/blockindex.BlockTreeDB,
csrc/store/chaindb.cpp): blocks/index 'b'/'f'/'l' records and chainstate 'C'/'B'
records with value obfuscation, restart from them, recovery of blocks written after the last
index record, -reindex with the 'R' flag, an interrupted-flush 'H' marker, migration from the
journal layout, and the stores read by the reference's own LevelDB library.
"""
import os
import struct
import subprocess

import pytest

from nodexa_chain_core_amd import core

_core = core()
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _mine(st, n, spk=bytes([0x51])):
    from nodexa_chain_core_amd.miner.service import Miner

    m = Miner.local(st)
    try:
        m.generate(spk, n)
    finally:
        m.close()


def _utxo(st):
    s = st.coins.stats()
    return st.coins.best_block, s


def _state(path, **kw):
    from nodexa_chain_core_amd.chain.state import ChainState, make_params

    return ChainState(make_params("regtest"), str(path), **kw)


def test_varint_and_coin_codec():
    # serialize.h VARINT: 0 -> 00, 127 -> 7f, 128 -> 80 00, 255 -> 80 7f, 16383 -> fe 7f, 16384 -> ff 00
    txid = bytes(range(32))
    for n, enc in ((0, "00"), (127, "7f"), (128, "8000"), (255, "807f"), (16383, "fe7f"), (16384, "ff00")):
        assert _core.coin_db_key(txid, n) == b"C" + txid + bytes.fromhex(enc)
    p2pkh = bytes.fromhex("76a914") + bytes(range(20)) + bytes.fromhex("88ac")
    # height 120 coinbase: VARINT(241); 50 CLORE compresses to 0x32 (CompressAmount(5e9) = 50)
    v = _core.coin_db_serialize(5_000_000_000, p2pkh, 120, True)
    assert v == bytes.fromhex("8071") + bytes([50]) + b"\x00" + bytes(range(20))
    assert _core.coin_db_deserialize(v) == (5_000_000_000, p2pkh, 120, True)
    odd = bytes([0x6a, 3]) + b"abc"
    w = _core.coin_db_serialize(1234, odd, 7, False)
    assert _core.coin_db_deserialize(w) == (1234, odd, 7, False)
    assert _core.coin_db_deserialize(w[:-1]) is None


def test_store_restart_and_records(tmp_path):
    st = _state(tmp_path)
    assert st.db_format == "leveldb"
    _mine(st, 6)
    want = _utxo(st)
    tip = st.chain.tip().hash
    st.close()
    assert os.path.exists(tmp_path / "blocks" / "index" / "CURRENT")
    assert os.path.exists(tmp_path / "chainstate" / "CURRENT")
    assert not os.path.exists(tmp_path / "blocks" / "index.log")

    # the records, read back raw: obfuscated values, 'b' per block, 'f' file info, 'B' best block
    db = _core.LevelDB(str(tmp_path / "chainstate"))
    obf = _core.chaindb_obfuscation_key(db, False)
    assert len(obf) == 8 and obf != bytes(8)
    assert _core.chaindb_xor(db.get(b"B"), obf) == tip
    coins = db.items(b"C", b"D")
    assert len(coins) == want[1][0] >= 6
    db.close()
    db = _core.LevelDB(str(tmp_path / "blocks" / "index"))
    obf = _core.chaindb_obfuscation_key(db, False)
    recs = db.items(b"b", b"c")
    assert len(recs) == 7
    act = st.params.kawpow_activation_time
    for k, v in recs:
        height, status, ntx, fi, dpos, upos, hb = _core.decode_disk_index(_core.chaindb_xor(v, obf), act)
        assert status & 8 and fi == 0 and ntx == 1  # HAVE_DATA in blk00000
        if height > 0:
            assert status & 16 and status & 7 == 5  # HAVE_UNDO, VALID_SCRIPTS
        assert st.chain.block_hash(_core.BlockHeader.deserialize(hb, act)) == k[1:]
    blocks, size, undo_size, hf, hl, tf, tl = _core.decode_file_info(_core.chaindb_xor(db.get(b"f" + struct.pack("<i", 0)), obf))
    assert (blocks, hf, hl) == (7, 0, 6) and size == os.path.getsize(tmp_path / "blocks" / "blk00000.dat")
    assert undo_size == os.path.getsize(tmp_path / "blocks" / "rev00000.dat")
    db.close()

    st2 = _state(tmp_path)
    assert not st2.rebuilt  # coins and asset records loaded, nothing replayed
    assert st2.chain.tip().hash == tip and st2.height() == 6
    assert _utxo(st2)[0] == want[0] and _utxo(st2)[1] == want[1]
    _mine(st2, 1)
    st2.close()


def test_tail_recovery_reindex_and_head_marker(tmp_path):
    st = _state(tmp_path)
    _mine(st, 4)
    want = _utxo(st)[1]
    tip = st.chain.tip().hash
    st.close()
    # the last block's index record lost (written to the blk file, crash before its record)
    db = _core.LevelDB(str(tmp_path / "blocks" / "index"))
    db.delete(b"b" + tip, sync=True)
    db.close()
    st = _state(tmp_path)
    assert st.chain.tip().hash == tip and _utxo(st)[1] == want
    st.close()
    # -reindex: the index rebuilt from the blk files; the 'R' flag is cleared when it completes
    st = _state(tmp_path, reindex=True)
    assert st.chain.tip().hash == tip and not st.index_log.reindexing()
    st.close()
    # an interrupted reindex resumes on the next start
    db = _core.LevelDB(str(tmp_path / "blocks" / "index"))
    db.put(b"R", b"1", sync=True)
    db.close()
    st = _state(tmp_path)
    assert st.chain.tip().hash == tip and not st.index_log.reindexing()
    st.close()
    # 'H' (a reference flush that did not finish): the UTXO set is rebuilt, not trusted
    db = _core.LevelDB(str(tmp_path / "chainstate"))
    db.put(b"H", b"\x00", sync=True)
    db.close()
    st = _state(tmp_path)
    assert _utxo(st)[1] == want and st.coins_db.get(b"H") is None
    st.close()


def test_migration_from_journal_layout(tmp_path):
    st = _state(tmp_path, db_format="journal")
    _mine(st, 3)
    want = _utxo(st)[1]
    st.close()
    assert os.path.exists(tmp_path / "blocks" / "index.log")
    st = _state(tmp_path)
    assert st.db_format == "journal"
    st.close()
    st = _state(tmp_path, db_format="leveldb")  # reindexed from the blk files, UTXO set replayed
    assert st.height() == 3 and _utxo(st)[1] == want
    st.close()
    st = _state(tmp_path)
    assert st.db_format == "leveldb" and _utxo(st)[1] == want
    st.close()


@pytest.fixture(scope="module")
def ref_tool():
    if not os.path.isdir("/root/reference/src/leveldb"):
        pytest.skip("reference LevelDB sources not present")
    try:
        out = subprocess.run(["bash", os.path.join(ROOT, "tools", "ref_leveldb.sh")], capture_output=True, text=True,
                             timeout=600, check=True)
    except (subprocess.CalledProcessError, OSError, subprocess.TimeoutExpired) as e:  # pragma: no cover
        pytest.skip(f"cannot build the reference LevelDB: {e}")
    return out.stdout.strip().splitlines()[-1]


def test_reference_library_reads_chain_stores(tmp_path, ref_tool):
    st = _state(tmp_path)
    _mine(st, 5)
    coins = st.coins.stats()[0]
    st.close()
    for sub, prefix, n in (("blocks/index", "62", 6), ("chainstate", "43", None)):
        r = subprocess.run([ref_tool, "dump", str(tmp_path / sub)], capture_output=True, text=True, timeout=120)
        assert r.returncode == 0, r.stderr
        keys = [line.split(" ")[0] for line in r.stdout.splitlines()]
        assert sum(1 for k in keys if k.startswith(prefix)) == (n if n is not None else coins)
        assert "0e006f62667573636174655f6b6579" in keys  # "\x0e\x00obfuscate_key"


def test_indexes_persist_as_block_tree_records(tmp_path):
    flags = dict(txindex=True, addressindex=True, spentindex=True, timestampindex=True)
    h160 = bytes(range(20))
    spk = bytes.fromhex("76a914") + h160 + bytes.fromhex("88ac")
    st = _state(tmp_path, indexes=flags)
    _mine(st, 4, spk)
    tip = st.chain.tip()
    blk = st.get_block(tip.hash)
    cb = blk.vtx[0].txid()
    deltas = st.indexes.deltas(1, h160, "*")
    assert st.indexes.tx_block(cb) == tip.hash and len(deltas) >= 4
    st.close()

    # reference record layout: 't' txid -> VARINT(file) VARINT(pos) VARINT(offset after the header)
    db = _core.LevelDB(str(tmp_path / "blocks" / "index"))
    obf = _core.chaindb_obfuscation_key(db, False)
    v = _core.chaindb_xor(db.get(b"t" + cb), obf)
    assert v[0] == 0  # blk00000
    pos = st.block_pos[tip.hash]
    raw = open(tmp_path / "blocks" / "blk00000.dat", "rb").read()
    hdr_len = len(blk.header.serialize(st.params.kawpow_activation_time))
    off = v[-1]  # one-byte VARINTs here: file, pos (< 128 only for the first blocks) or more bytes
    assert raw[pos.offset + hdr_len + off: pos.offset + hdr_len + off + 4] == blk.vtx[0].serialize()[:4]
    # 'a' keys: type, hash160, asset name (CompactSize + "CLORE"), BE height, ...
    akeys = [k for k, _ in db.items(b"a", b"b")]
    mine = [k for k in akeys if k[2:22] == h160]  # (the community-fund outputs have their own address)
    assert len(mine) == len(deltas) and all(k[1] == 1 and k[22:28] == b"\x05CLORE" for k in mine)
    assert [k for k, _ in db.items(b"s", b"t")] and [k for k, _ in db.items(b"z", b"{")]
    db.close()

    st2 = _state(tmp_path, indexes=flags)
    assert st2.indexes.pending_changes == 0  # loaded from the records, not replayed
    assert st2.indexes.tx_block(cb) == tip.hash
    assert st2.indexes.deltas(1, h160, "*") == deltas
    st2.close()
    # turning an index off and on again rebuilds it (the stored 'F' flags differ)
    st3 = _state(tmp_path, indexes=dict(flags, txindex=False))
    st3.close()
    st4 = _state(tmp_path, indexes=flags)
    assert st4.indexes.tx_block(cb) == tip.hash and st4.indexes.deltas(1, h160, "*") == deltas
    st4.close()
