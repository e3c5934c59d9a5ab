"""Signature cache (CSignatureCache, src/script/sigcache.cpp:76-86): signatures verified at mempool
acceptance are not verified again when the block that confirms the transaction is connected."""
from test_node_rpc import client, node_factory  # noqa: F401 — shared fixtures
from wallet_util import fund, mature_coin, spend


def test_mempool_signatures_are_reused_by_block_connect(core, node_factory):  # noqa: F811
    node, addr = node_factory()
    c = client(node)
    w = fund(c, 101)
    core.sigcache_clear()
    s0 = core.sigcache_stats()
    u = mature_coin(c)
    txid = c.sendrawtransaction(spend(c, u["txid"], u["vout"], u["amount"], w, 5.0))
    s1 = core.sigcache_stats()
    assert s1["inserts"] == s0["inserts"] + 1 and s1["entries"] == 1  # one P2PKH input verified
    c.generatetoaddress(1, addr)
    assert txid not in c.getrawmempool()
    s2 = core.sigcache_stats()
    # the block's connect found the signature in the cache (and dropped it: it will not be asked again)
    assert s2["hits"] == s1["hits"] + 1 and s2["entries"] == 0


def test_cache_modes_and_eviction(core, node_factory):  # noqa: F811
    node, addr = node_factory()
    c = client(node)
    w = fund(c, 101)
    u = mature_coin(c)
    raw = bytes.fromhex(spend(c, u["txid"], u["vout"], u["amount"], w, 5.0))
    tx = core.Transaction.deserialize(raw)
    vin = tx.vin[0]
    value, spk, _, _ = node.state._spent_coin(vin.prevout)
    args = (vin.script_sig, spk, list(vin.witness), core.STANDARD_SCRIPT_VERIFY_FLAGS, raw, 0, value)
    core.sigcache_clear()
    st = core.sigcache_stats
    assert core.verify_script(*args, 0)[0] and st()["entries"] == 0      # no cache
    assert core.verify_script(*args, 1)[0] and st()["entries"] == 1      # store
    h = st()["hits"]
    assert core.verify_script(*args, 2)[0] and st()["hits"] == h + 1     # use: hit, erased
    assert st()["entries"] == 0
    m = st()["misses"]
    assert core.verify_script(*args, 2)[0] and st()["misses"] == m + 1   # verified again on the host
    core.sigcache_set_max_bytes(0)
    assert core.verify_script(*args, 1)[0] and st()["entries"] == 0      # -maxsigcachesize=0: nothing kept
    core.sigcache_set_max_bytes(32 << 20)


def test_reinserted_entry_keeps_its_age(core, node_factory):  # noqa: F811
    """an entry erased by a block connect (use mode) and stored again later (mempool
    after a reorg) owns only its newest slot; eviction of its stale older slot must not drop it."""
    node, addr = node_factory()
    c = client(node)
    w = fund(c, 101)
    u = mature_coin(c)
    value, spk, _, _ = None, None, None, None
    checks = []
    for dest in (c.getnewaddress(), c.getnewaddress(), c.getnewaddress()):
        raw = bytes.fromhex(spend(c, u["txid"], u["vout"], u["amount"], dest, 5.0))
        tx = core.Transaction.deserialize(raw)
        vin = tx.vin[0]
        value, spk, _, _ = node.state._spent_coin(vin.prevout)
        checks.append(lambda mode, raw=raw, vin=vin, spk=spk, value=value: core.verify_script(
            vin.script_sig, spk, list(vin.witness), core.STANDARD_SCRIPT_VERIFY_FLAGS, raw, 0, value, mode)[0])
    a, b, cc = checks
    core.sigcache_clear()
    core.sigcache_set_max_bytes(2 * 32)  # two entries
    try:
        st = core.sigcache_stats
        assert a(1) and a(2) and st()["entries"] == 0  # A stored, then used (erased)
        assert b(1) and a(1) and st()["entries"] == 2   # B, then A again: slots [A(stale), B, A]
        assert cc(1) and st()["entries"] == 2           # C evicts the oldest live entry: B, not A
        h, m = st()["hits"], st()["misses"]
        assert a(2) and st()["hits"] == h + 1           # A survived
        assert b(2) and st()["misses"] == m + 1         # B was the one evicted
    finally:
        core.sigcache_set_max_bytes(32 << 20)
        core.sigcache_clear()
