"""nodexad -gpus=0 on one MI355X: the node mines through its mining service (pipelined 2^25-nonce
windows, device-side stale-work abort, full share re-hash), getmininginfo reports the service's
hash rate, and every block it finds is accepted by ProcessNewBlock.

`-minertargetbits=28` makes the miner search for hashes below 2^228 although regtest accepts
almost any hash: a block then takes ~2^28 hashes (about a second at full rate), so the rate is
measured over whole windows rather than over the first few nonces of each template."""
import time

import pytest

pytestmark = pytest.mark.gpu


def test_node_setgenerate_hashrate_and_blocks(core, gpu, tmp_path):
    from nodexa_chain_core_amd.node import Node
    from nodexa_chain_core_amd.rpc.client import RPCClient
    from nodexa_chain_core_amd.utils.config import ArgsManager

    addr = core.base58check_encode(bytes([42]) + bytes(range(20)))
    args = ArgsManager()
    args.parse_parameters(["-regtest", f"-datadir={tmp_path}", "-rpcport=0", "-rpcuser=u", "-rpcpassword=p",
                           f"-miningaddress={addr}", "-printtoconsole=0", "-gpus=0", "-minertargetbits=28"])
    n = Node(args)
    n.start()
    try:
        c = RPCClient("127.0.0.1", n.rpc.port, "u", "p", timeout=300)
        assert c.generatetoaddress(1, addr, 1 << 40) and c.getblockcount() == 1  # DAG build + first block
        c.setgenerate(True)
        t0 = time.time()
        best = 0.0
        while time.time() - t0 < 90 and (c.getblockcount() < 4 or best == 0.0):
            time.sleep(1.0)
            best = max(best, c.getmininginfo()["hashespersec"])
        info = c.getmininginfo()
        c.setgenerate(False)
        assert c.getblockcount() >= 4
        assert best >= 200e6, info  # the service's windows run at the kernel's rate (epoch 0)
        assert info["gpus"] and info["gpus"][0]["epochs_resident"] == [0]
        assert n.miner.service.leader.stats["bad_shares"] == 0
        assert c.verifychain(4, 0) is True
        # every mined header carries a valid KawPow proof for its own nNonce64 / mix
        for h in range(1, c.getblockcount() + 1):
            blk = c.getblock(c.getblockhash(h))
            nonce = blk["nonce64"] if isinstance(blk["nonce64"], int) else int(blk["nonce64"], 16)
            res = c.getkawpowhash(blk["headerhash"], blk["mixhash"], "%016x" % nonce, h)
            assert res["result"] == "true", (h, res)
    finally:
        n.stop()
