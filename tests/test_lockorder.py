"""DEBUG_LOCKORDER equivalent (utils/sync.py; reference src/sync.cpp:25-183)."""
import threading

import pytest

from nodexa_chain_core_amd.utils import sync


@pytest.fixture()
def lockorder():
    was = sync.enabled()
    sync.enable(True)
    sync.reset()
    yield
    sync.enable(was)
    sync.reset()


def test_inversion_detected(lockorder):
    a, b = sync.make_lock("A"), sync.make_lock("B")
    with a:
        with b:
            pass
    with b:
        with pytest.raises(sync.PotentialDeadlock, match="A -> B|B -> A"):
            a.acquire()
    with a:  # same order as first seen: fine, and re-entrant
        with a:
            with b:
                pass


def test_condition_on_ordered_lock(lockorder):
    lk = sync.make_lock("cs_main")
    cv = threading.Condition(lk)
    box = []

    def waiter():
        with cv:
            cv.wait_for(lambda: box, timeout=5)

    t = threading.Thread(target=waiter)
    t.start()
    with cv:
        box.append(1)
        cv.notify_all()
    t.join(5)
    assert not t.is_alive()


def test_node_runs_clean_under_lockorder(core, tmp_path, lockorder):
    """Mining, RPC and a two-node P2P sync with every Python-side lock order-checked."""
    from test_p2p import _node, _wait

    a = _node(core, tmp_path, "a", ["-listen", "-port=0", "-debuglockorder"])
    b = None
    try:
        a.miner.generate(a.mining_script, 5)
        b = _node(core, tmp_path, "b", [f"-connect=127.0.0.1:{a.connman.port}", "-debuglockorder"])
        assert _wait(lambda: b.state.height() == 5)
        b.miner.generate(b.mining_script, 1)
        assert _wait(lambda: a.state.height() == 6)
    finally:
        if b is not None:
            b.stop()
        a.stop()
