"""Incremental UTXO persistence (chainstate/coins.dat + coins.log): a flush writes only the outputs
changed since the previous one (CCoinsViewDB::BatchWrite's change set, src/txdb.cpp:91-), start-up
replays the journal onto the snapshot, a torn tail record from a crash is cut off, and compaction
folds the journal back into a snapshot."""
import os

import pytest


def _coin(core, view, i, value=None):
    txid = core.sha256d(b"coin-%d" % i)
    view.add(txid, i % 3, value if value is not None else 1000 + i, b"\x51" * (i % 40), i, i % 7 == 0)
    return txid, i % 3


def _stats(v):
    s = v.stats()
    return tuple(s) if isinstance(s, tuple) else (s.txouts, s.transactions, s.total, bytes(s.hash))


def test_journal_roundtrip_torn_tail_and_compaction(core, tmp_path):
    snap, log = str(tmp_path / "coins.dat"), str(tmp_path / "coins.log")
    v = core.CoinsView()
    outs = [_coin(core, v, i) for i in range(2000)]
    v.best_block = core.sha256d(b"b1")
    v.compact(snap, log)  # pending changes -> record 1, folded into a snapshot of 2000 coins
    assert v.journal_seq == 1 and os.path.getsize(log) == 0
    size0 = os.path.getsize(snap)
    # flush 1: 10 spends + 5 adds -> one small record, independent of the 2000-coin set
    for txid, n in outs[:10]:
        v.spend(txid, n)
    for i in range(5000, 5005):
        _coin(core, v, i)
    v.best_block = core.sha256d(b"b2")
    assert v.dirty == 15
    v.append_journal(log)
    assert v.dirty == 0 and v.journal_seq == 2
    rec1 = os.path.getsize(log)
    assert rec1 < size0 // 20
    # flush 2
    _coin(core, v, 6000)
    v.best_block = core.sha256d(b"b3")
    v.append_journal(log)
    want = _stats(v)
    w = core.CoinsView()
    assert w.load_with_journal(snap, log) and w.replayed == 2 and w.journal_seq == 3
    assert _stats(w) == want and w.best_block == core.sha256d(b"b3")
    # a crash in the middle of writing record 3: the torn tail is cut, records 1-2 stand
    full = os.path.getsize(log)
    _coin(core, v, 7000)
    v.best_block = core.sha256d(b"b4")
    v.append_journal(log)
    with open(log, "r+b") as f:
        f.truncate(os.path.getsize(log) - 7)
    w = core.CoinsView()
    assert w.load_with_journal(snap, log) and w.replayed == 2
    assert _stats(w) == want and os.path.getsize(log) == full
    # appends continue after the cut; compaction folds everything into the snapshot
    _coin(core, w, 8000)
    w.best_block = core.sha256d(b"b5")
    w.append_journal(log)
    want = _stats(w)
    w.compact(snap, log)
    assert os.path.getsize(log) == 0
    x = core.CoinsView()
    assert x.load_with_journal(snap, log) and x.replayed == 0 and _stats(x) == want and x.journal_seq == 4
    # records already folded into the snapshot are skipped if the journal truncate was lost
    x2 = core.CoinsView()
    _coin(core, x, 9000)
    x.best_block = core.sha256d(b"b6")
    x.append_journal(log)
    assert x2.load_with_journal(snap, log) and x2.replayed == 1 and _stats(x2) == _stats(x)


def test_chainstate_flushes_through_the_journal(core, tmp_path):
    from nodexa_chain_core_amd.chain.state import ChainState, make_params
    from nodexa_chain_core_amd.miner.service import Miner

    params = make_params("regtest")
    st = ChainState(params, str(tmp_path), db_format="journal")
    st.flush_interval = 3
    m = Miner.local(st)
    m.generate(bytes([0x51]), 7)
    m.close()
    st.flush()
    log = os.path.join(str(tmp_path), "chainstate", "coins.log")
    assert os.path.getsize(log) > 0 and st.coins.journal_seq >= 2  # first flush: snapshot, then records
    want = (st.coins.best_block, _stats(st.coins))
    st.close() if hasattr(st, "close") else None
    st2 = ChainState(params, str(tmp_path))  # the journal layout is detected
    assert st2.db_format == "journal"
    assert st2.height() == 7 and (st2.coins.best_block, _stats(st2.coins)) == want
    assert st2.coins.replayed >= 1
