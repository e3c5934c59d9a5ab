"""Fixtures that start past genesis: HeaderChain.add_anchor (a node's stored index below the first
header, as LoadBlockIndexDB leaves it) and the anchored synthetic chains of models/synthetic
(BASELINE config 5 at the headline epoch: tests/data/testnet_mixed_e384_10k.hdr)."""
import os

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
E384 = os.path.join(ROOT, "tests", "data", "testnet_mixed_e384_10k.hdr")


def test_anchor_links_heights_and_dgw(core):
    from nodexa_chain_core_amd.models import synthetic

    params = synthetic.synthetic_params("test")
    hs, base, work = synthetic.make_anchor(params, 2_880_000, 1_900_000_000)
    assert len(hs) == synthetic.ANCHOR_LEN and base == 2_880_000 - synthetic.ANCHOR_LEN
    c = core.HeaderChain(params)
    tip = c.add_anchor(hs, base, work)
    assert c.height() == 2_879_999 and tip.height == 2_879_999 and c.tip().hash == tip.hash
    assert c.at_height(base).height == base and c.at_height(base - 1) is None
    times, bits, a, bh = c.dgw_ancestors(tip.hash)
    assert a == 180 and bh == 2_879_999  # DarkGravityWave's whole window comes from the anchor
    nxt = core.BlockHeader()
    nxt.prev, nxt.time, nxt.height = tip.hash, tip.time + 60, 2_880_000
    assert c.next_bits(nxt) != 0
    with pytest.raises(ValueError):
        c.add_anchor(hs, base, work)  # already indexed
    broken = list(hs)
    broken[5], broken[6] = broken[6], broken[5]
    with pytest.raises(ValueError):
        core.HeaderChain(params).add_anchor(broken, base, work)  # does not link


@pytest.mark.skipif(not os.path.exists(E384), reason="headline fixture not generated")
def test_headline_fixture_shape(core):
    """The committed headline-epoch fixture: heights 2,880,000-2,889,999, KawPow epochs 384 and 385,
    an Equihash era at the end, and an anchor below it."""
    from nodexa_chain_core_amd.models import synthetic

    params, hs = synthetic.load(E384)
    anchor = synthetic.load_anchor(E384, params)
    assert anchor is not None and anchor[1] + len(anchor[0]) == hs[0].height == 2_880_000
    assert hs[-1].height == 2_889_999 and len(hs) == 10_000
    epochs = {h.height // core.EPOCH_LENGTH for h in hs if not h.is_equihash()}
    assert epochs == {384, 385}
    assert sum(h.is_equihash() for h in hs) > 0


@pytest.mark.skipif(not os.path.exists(E384), reason="headline fixture not generated")
def test_headline_fixture_prefix_verifies_on_cpu(core, tmp_path):
    """The first 48 headers of the headline fixture, on its anchor, pass the host golden model
    (KawPow light mode at epoch 384, DarkGravityWave from the anchor's window, contextual rules);
    without the anchor the first header has no parent; the anchor survives a save / load."""
    from nodexa_chain_core_amd.models import synthetic
    from nodexa_chain_core_amd.models.verify import process_headers

    params, hs = synthetic.load(E384)
    anchor = synthetic.load_anchor(E384, params)
    part = hs[:48]
    r = process_headers(synthetic.new_chain(params, anchor), part, part[-1].time + 3600)
    assert r["accepted"] == 48 and r["reject"] is None
    r = process_headers(synthetic.new_chain(params), part, part[-1].time + 3600)
    assert r["accepted"] == 0 and r["reject"]["reason"] == "prev-blk-not-found"
    path = str(tmp_path / "e384.hdr")
    synthetic.save(path, params, part, anchor)
    p2, h2 = synthetic.load(path)
    a2 = synthetic.load_anchor(path, p2)
    act = params.kawpow_activation_time
    assert a2[1:] == anchor[1:] and [h.serialize(act) for h in a2[0]] == [h.serialize(act) for h in anchor[0]]
    assert [h.serialize(act) for h in h2] == [h.serialize(act) for h in part]
