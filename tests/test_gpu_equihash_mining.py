"""Equihash(200,9) mined by the node on one MI355X (the GPU twin of tests/test_equihash_mining.py):
nodexad -gpus=0 with the extension active mines Equihash blocks through setgenerate and
generatetoaddress (miner/equihash_search.EquihashGpuDevice inside the mining loop), the device-side
solution check (eq_verify_slots) agrees with the golden verifier and rejects a corrupted solution,
and a window's solution set equals the golden solver's."""
import time

import pytest

pytestmark = pytest.mark.gpu


def test_node_mines_equihash_on_gpu(core, gpu, tmp_path):
    from nodexa_chain_core_amd.node import Node
    from nodexa_chain_core_amd.rpc.client import RPCClient
    from nodexa_chain_core_amd.utils.config import ArgsManager

    addr = core.base58check_encode(bytes([42]) + bytes(range(20)))
    args = ArgsManager()
    args.parse_parameters(["-regtest", "-kawpowactivationtime=1524179367", f"-datadir={tmp_path}", "-rpcport=0", "-rpcuser=u", "-rpcpassword=p",
                           f"-miningaddress={addr}", "-printtoconsole=0", "-gpus=0",
                           "-equihash=%d" % (int(time.time()) - 100), "-minertargetbits=6"])
    n = Node(args)
    n.start()
    try:
        c = RPCClient("127.0.0.1", n.rpc.port, "u", "p", timeout=300)
        assert len(c.generatetoaddress(2, addr)) == 2
        c.setgenerate(True)
        deadline = time.time() + 90
        while c.getblockcount() < 5 and time.time() < deadline:
            time.sleep(0.2)
        info = c.getmininginfo()
        c.setgenerate(False)
        assert c.getblockcount() >= 5, info
        g = info["gpus"][0]
        assert g["algo"] == "equihash" and g["solutionspersec"] > 0 and g["last_device_ms"] > 0, g
        assert n.miner.service.leader.stats["bad_shares"] == 0
        act = n.params.kawpow_activation_time
        p = core.EquihashParams(200, 9)
        target = (1 << (256 - 6)) - 1
        for h in range(1, c.getblockcount() + 1):
            hdr = core.Block.deserialize(bytes.fromhex(c.getblock(c.getblockhash(h), 0)), act).header
            assert hdr.is_equihash()
            assert core.equihash_verify(p, hdr.equihash_input(), core.equihash_unpack(p, hdr.solution))[0]
            assert int.from_bytes(hdr.equihash_hash(act), "little") <= target  # -minertargetbits honoured
        assert c.verifychain(4, 0) is True
    finally:
        n.stop()


def test_device_window_matches_golden_solver(core, gpu):
    from nodexa_chain_core_amd.miner.equihash_search import EquihashGpuDevice
    from nodexa_chain_core_amd.miner.search import ALGO_EQUIHASH, Work, equihash_nonce256

    prefix = bytes(range(80))
    dev = EquihashGpuDevice(0, num_inst=4)
    w = Work(prefix, b"\xff" * 32, 1, 1, 0, 0, ALGO_EQUIHASH)  # every solution is a share
    dev.submit(0, w, 1000, 4)
    res = dev.wait(0)
    p = core.EquihashParams(200, 9)
    golden = set()
    for k in range(4):
        sols, _ = core.equihash_solve_cpu(p, prefix + equihash_nonce256(1000 + k), 16, 0)
        golden |= {(1000 + k, core.equihash_pack(p, s)) for s in sols}
    got = {(s.nonce, s.solution) for s in res.shares}
    assert res.hashes == len(golden) and res.algo == ALGO_EQUIHASH  # the exact solution count
    assert got <= golden and len(got) == min(4, len(golden))  # shares are golden solutions


def test_device_verdicts_catch_a_corrupted_solution(core, gpu):
    import torch

    from nodexa_chain_core_amd.ops import runtime
    from nodexa_chain_core_amd.ops.equihash import EquihashSolver

    s = EquihashSolver(num_inst=4)
    inputs = [bytes([7 + k]) * 112 for k in range(4)]
    s.launch(inputs)
    arrays = s.collect_arrays(verify="host")  # device verdicts and the golden verifier agree: all valid
    i = next(k for k, a in enumerate(arrays) if len(a))
    per = 1 + s.h.EQ_MAX_SOL * 512
    sols = s.sols.view(-1)
    a, b = int(sols[i * per + 1].item()), int(sols[i * per + 2].item())
    sols[i * per + 1], sols[i * per + 2] = b, a  # swap two leaves: ordering and collisions break
    s.h.launch_equihash_verify_slots(s.verify_kernel, s.h0, s.msgs.data_ptr(), 112, 4, s.sols.data_ptr(),
                                     s.verdicts.data_ptr(), runtime.current_stream_handle())
    v = s.verdicts.view(4, s.h.EQ_MAX_SOL).cpu().numpy()
    torch.cuda.synchronize()
    assert v[i, 0] not in (0, s.h.EQ_V_EMPTY)
    n = int(sols[i * per].item())
    assert (v[i, 1:n] == 0).all() and (v[i, n:] == s.h.EQ_V_EMPTY).all()
