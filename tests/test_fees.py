"""Fee estimation: the native CBlockPolicyEstimator (csrc/chain/fees.cpp).

`test_block_policy_estimates_reference_scenario` replays src/test/policyestimator_tests.cpp
(block_policy_estimates_test) step for step: 10 feerates x 4 txs per block, higher feerates mined
more often, then quiet blocks, a backlog and an all-mined phase, with the reference's bounds on
estimateFee. The node tests drive the estimator through AcceptToMemoryPool / ConnectTip and the
three RPCs (src/rpc/mining.cpp:1009-1212), and fee_estimates.dat across a restart."""
import struct

import pytest

from test_node_rpc import client, node_factory  # noqa: F401 — shared fixtures
from wallet_util import fund, spend

BASE_FEE, DELTA = 2000, 100
TX_VSIZE = 188  # the reference test's template: one 128-byte scriptSig input, one empty output


def _txid(block, j, k):
    return struct.pack("<III", block, j, k) + bytes(20)


def test_block_policy_estimates_reference_scenario(core):
    est = core.FeeEstimator()
    fees = [BASE_FEE * (j + 1) for j in range(10)]
    base_rate = BASE_FEE * 1000 // TX_VSIZE
    pending = [[] for _ in range(10)]
    blocknum = 0

    def add_all(b):
        for j in range(10):
            for k in range(4):
                t = _txid(b, j, k)
                est.process_tx(t, b, fees[j], TX_VSIZE, True)
                pending[j].append(t)

    while blocknum < 200:
        add_all(blocknum)
        block = []
        for h in range(blocknum % 10 + 1):  # 10/10 blocks take the top feerate, 1/10 the lowest
            block += pending[9 - h]
            pending[9 - h] = []
        blocknum += 1
        est.process_block(blocknum, block)
        if blocknum == 3:  # three buckets combined: ~9x base rate at target 2
            assert est.estimate_fee(1) == 0
            assert 9 * base_rate - DELTA < est.estimate_fee(2) < 9 * base_rate + DELTA

    orig = []
    for i in range(1, 10):
        orig.append(est.estimate_fee(i))
        if i > 2:
            assert orig[i - 1] <= orig[i - 2]  # monotonically decreasing
        if i % 2 == 0:  # scale 2: exact only for even targets
            mult = 11 - i
            assert mult * base_rate - DELTA < orig[i - 1] < mult * base_rate + DELTA
    for i in range(10, 49):
        orig.append(est.estimate_fee(i))

    while blocknum < 250:  # quiet blocks: estimates unchanged
        blocknum += 1
        est.process_block(blocknum, [])
    assert est.estimate_fee(1) == 0
    for i in range(2, 10):
        assert orig[i - 1] - DELTA < est.estimate_fee(i) < orig[i - 1] + DELTA

    while blocknum < 265:  # backlog that never confirms: estimates rise (or fail)
        add_all(blocknum)
        blocknum += 1
        est.process_block(blocknum, [])
    for i in range(1, 10):
        e = est.estimate_fee(i)
        assert e == 0 or e > orig[i - 1] - DELTA

    est.process_block(266, [t for j in range(10) for t in pending[j]])  # mine the whole backlog
    pending = [[] for _ in range(10)]
    assert est.estimate_fee(1) == 0
    for i in range(2, 10):
        e = est.estimate_fee(i)
        assert e == 0 or e > orig[i - 1] - DELTA

    blocknum = 266
    while blocknum < 665:  # everything mined every block: estimates fall below the original
        block = []
        for j in range(10):
            for k in range(4):
                t = _txid(blocknum, j, k)
                est.process_tx(t, blocknum, fees[j], TX_VSIZE, True)
                block.append(t)
        blocknum += 1
        est.process_block(blocknum, block)
    assert est.estimate_fee(1) == 0
    for i in range(2, 9):
        assert est.estimate_fee(i) < orig[i - 1] - DELTA

    # smart fee: clamped to half the recorded span, 85 % / 95 % thresholds
    rate, returned, reason, detail = est.estimate_smart_fee(6, True)
    assert rate > 0 and returned == 6 and reason
    assert detail["pass"]["endrange"] >= detail["pass"]["startrange"] >= 0
    eco, _, _, _ = est.estimate_smart_fee(6, False)
    assert 0 < eco <= rate
    assert est.estimate_smart_fee(1009, True)[0] == 0
    raw, info = est.estimate_raw_fee(6, 0.95, "short")
    assert raw > 0 and info["decay"] == pytest.approx(0.962) and info["scale"] == 1
    assert [est.highest_target_tracked(h) for h in ("short", "medium", "long")] == [12, 48, 1008]


def test_fee_estimates_file_roundtrip(core):
    est = core.FeeEstimator()
    for b in range(40):
        ids = []
        for j in range(8):
            t = _txid(b, j, 0)
            est.process_tx(t, b, 1000 * (j + 3), 250, True)
            ids.append(t)
        est.process_block(b + 1, ids[2:])  # the two cheapest wait (and then count as failures)
    blob = est.serialize()
    required, wrote, best = struct.unpack_from("<iiI", blob, 0)
    assert (required, wrote, best) == (149900, 4040402, 40)
    other = core.FeeEstimator()
    ok, err = other.deserialize(blob)
    assert ok, err
    for t in (2, 4, 8, 12):
        assert other.estimate_raw_fee(t, 0.85, "short")[0] == est.estimate_raw_fee(t, 0.85, "short")[0]
    assert other.estimate_smart_fee(4, True)[:2] == est.estimate_smart_fee(4, True)[:2]
    assert other.serialize() == est.serialize()
    nb = blob[20]  # bucket count (one-byte CompactSize), then the first horizon's decay
    assert nb < 253
    bad = bytearray(blob)
    off = 21 + 8 * nb
    assert struct.unpack_from("<d", bad, off)[0] == pytest.approx(0.9952)
    bad[off:off + 8] = struct.pack("<d", 1.5)
    ok, err = other.deserialize(bytes(bad))
    assert not ok and "Decay" in err
    ok, err = core.FeeEstimator().deserialize(blob[:100])
    assert not ok and err
    future = struct.pack("<i", 9_999_999) + blob[4:]
    assert not core.FeeEstimator().deserialize(future)[0]


def test_remove_counts_failures_and_reorgs_ignored(core):
    est = core.FeeEstimator()
    est.process_block(1, [])
    t = _txid(1, 0, 0)
    est.process_tx(t, 1, 5000, 200, True)
    assert est.tracked == 1
    est.process_tx(_txid(1, 1, 0), 0, 5000, 200, True)  # entry height != best seen: ignored
    est.process_tx(_txid(1, 2, 0), 1, 5000, 200, False)  # not current: ignored
    assert est.tracked == 1
    est.process_block(1, [t])  # a block at or below the best seen height changes nothing
    assert est.tracked == 1
    assert est.remove_tx(t, False) and est.tracked == 0
    assert not est.remove_tx(t, False)


def test_node_fee_estimation_rpcs_and_restart(core, node_factory):  # noqa: F811
    node, addr = node_factory(("-deprecatedrpc=estimatefee",))
    c = client(node)
    assert c.estimatesmartfee(6) == {"errors": ["Insufficient data or no feerate found"], "blocks": 0}
    assert c.estimatefee(6) == -1
    raw = c.estimaterawfee(6)
    assert set(raw) == {"short", "medium", "long"} and raw["short"]["errors"] and raw["long"]["scale"] == 24
    assert set(c.estimaterawfee(13)) == {"medium", "long"}
    for bad in (0, 1009):
        with pytest.raises(RuntimeError, match="Invalid conf_target"):
            c.estimatesmartfee(bad)
    with pytest.raises(RuntimeError, match="Invalid estimate_mode"):
        c.estimatesmartfee(6, "FAST")
    with pytest.raises(RuntimeError, match="Invalid threshold"):
        c.estimaterawfee(6, 1.5)

    fund(c, 160)
    coins = sorted((u for u in c.listunspent() if u["spendable"]), key=lambda u: u["txid"])
    for b in range(14):
        for k in range(4):
            u = coins.pop()
            fee = 0.01 * (1 + k % 2)
            c.sendrawtransaction(spend(c, u["txid"], u["vout"], u["amount"], addr, 1.0, fee=fee))
        c.generatetoaddress(1, addr)
    assert not c.getrawmempool()
    smart = c.estimatesmartfee(2)
    assert smart["feerate"] > 0 and smart["blocks"] == 2, smart
    assert c.estimatesmartfee(6, "ECONOMICAL")["blocks"] == 6
    assert c.estimatefee(2) > 0
    short = c.estimaterawfee(2, 0.85)["short"]
    assert short["feerate"] > 0 and short["pass"]["totalconfirmed"] > 0
    before = c.estimaterawfee(2, 0.85)["short"]["feerate"]

    node.stop()
    node2, _ = node_factory(("-deprecatedrpc=estimatefee",))
    c2 = client(node2)
    assert c2.estimaterawfee(2, 0.85)["short"]["feerate"] == before  # fee_estimates.dat reloaded
    assert c2.estimatesmartfee(2)["feerate"] == smart["feerate"]


def test_estimatefee_is_deprecated_by_default(core, node_factory):  # noqa: F811
    node, _ = node_factory()
    with pytest.raises(RuntimeError, match="deprecated"):
        client(node).estimatefee(6)
