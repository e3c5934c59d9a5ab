"""RPC method table: reference-compatible names, arguments and result shapes.

Parity tables: mining (src/rpc/mining.cpp:1283-1304), blockchain
(src/rpc/blockchain.cpp:1897), control/server (src/rpc/server.cpp:347,
src/rpc/misc.cpp:1469). Result keys follow the reference, including the
KawPow additions (getblock: headerhash / mixhash / nonce64; getblocktemplate:
pprpcheader / pprpcepoch, CommunityAutonomousAddress / Value; getkawpowhash:
result / digest / mix_hash / info / meets_target; pprpcsb: BIP22 results).
Engine additions are in the "gpu" category (getgpuinfo, equihash*, verifyheaders).
"""
from __future__ import annotations

import struct
import time

from .. import core
from ..chain.header import from_progpow, to_progpow
from ..utils import log
from .protocol import (RPC_DESERIALIZATION_ERROR, RPC_INVALID_ADDRESS_OR_KEY, RPC_INVALID_PARAMETER,
                       RPC_INVALID_PARAMS, RPC_MISC_ERROR, RPC_TRANSACTION_ERROR, RPC_TYPE_ERROR,
                       RPC_VERIFY_ALREADY_IN_CHAIN, RPC_VERIFY_ERROR, RPC_VERIFY_REJECTED, RPCError)

_core = core()


def _hex(b: bytes) -> str:
    return _core.u256_hex(b)


def _arg(params, i, default=None):
    return params[i] if len(params) > i and params[i] is not None else default


def _need(params, n, usage):
    if len(params) < n:
        raise RPCError(RPC_MISC_ERROR, usage)


def _parse_hash(s) -> bytes:
    if not isinstance(s, str) or len(s.strip().removeprefix("0x")) != 64:
        raise RPCError(RPC_INVALID_PARAMETER, "hash must be of length 64 (not %d)" % (len(s) if isinstance(s, str) else 0))
    try:
        return _core.u256_from_hex(s)
    except ValueError:
        raise RPCError(RPC_INVALID_PARAMETER, "hash must be hexadecimal string")


def _bip22(state) -> object:
    """BIP22ValidationResult (src/rpc/mining.cpp)."""
    if state.ok:
        return None
    return state.reject or "rejected"


def register(table, node) -> None:  # noqa: C901 — one table, like the reference's RegisterXRPCCommands
    class _StateProxy:  # the RPC table is registered (warm-up) before the chain is loaded
        def __getattr__(self, name):
            return getattr(node.state, name)

    st = _StateProxy()
    params = node.params

    # ------------------------------------------------------------------ control
    def rpc_help(p):
        """help ( "command" ) — list all commands, or get help for a specified command."""
        return table.help(_arg(p, 0))

    def rpc_stop(p):
        """stop — stop the node."""
        node.request_shutdown()
        return "Nodexa server stopping"

    def rpc_uptime(p):
        """uptime — seconds since the server started."""
        return int(time.time() - table.started)

    def rpc_getrpcinfo(p):
        """getrpcinfo — details of the RPC server (active commands)."""
        now = time.time()
        return {"active_commands": [{"method": m, "duration": int((now - t) * 1e6)} for m, t in table.active.values()]}

    def rpc_logging(p):
        """logging ( ["include",...] ["exclude",...] ) — get/set debug categories."""
        for c in _arg(p, 0, []) or []:
            log.enable(c)
        for c in _arg(p, 1, []) or []:
            log.disable(c)
        return log.active()

    def rpc_getmemoryinfo(p):
        """getmemoryinfo — host and device memory usage."""
        import resource

        out = {"locked": {"used": 0, "free": 0, "total": 0},
               "host_maxrss_kb": resource.getrusage(resource.RUSAGE_SELF).ru_maxrss}
        out["gpus"] = node.gpu_memory_info()
        return out

    for name, fn, args in [("help", rpc_help, ("command",)), ("stop", rpc_stop, ()), ("uptime", rpc_uptime, ()),
                           ("getrpcinfo", rpc_getrpcinfo, ()), ("logging", rpc_logging, ("include", "exclude")),
                           ("getmemoryinfo", rpc_getmemoryinfo, ("mode",))]:
        table.append("control", name, fn, args)

    # ------------------------------------------------------------------ blockchain
    def header_json(idx, hdr=None):
        hdr = hdr or idx.header
        tip = st.tip()
        nxt = st.chain.at_height(idx.height + 1) if st.chain.in_active_chain(idx) else None
        out = {
            "hash": _hex(idx.hash),
            "confirmations": (tip.height - idx.height + 1) if st.chain.in_active_chain(idx) else -1,
            "height": idx.height,
            "version": hdr.version,
            "versionHex": "%08x" % (hdr.version & 0xFFFFFFFF),
            "merkleroot": _hex(hdr.merkle_root),
            "time": hdr.time,
            "mediantime": idx.median_time_past(),
            "nonce": hdr.nonce,
            "bits": "%08x" % hdr.bits,
            "difficulty": _core.difficulty_from_bits(hdr.bits),
            "chainwork": "%064x" % idx.chain_work,
        }
        if hdr.time >= params.kawpow_activation_time:
            out["headerhash"] = _hex(hdr.kawpow_header_hash())
            out["mixhash"] = _hex(hdr.mix_hash)
            out["nonce64"] = hdr.nonce64
        if idx.height > 0:
            out["previousblockhash"] = _hex(idx.prev_hash)
        if nxt is not None:
            out["nextblockhash"] = _hex(nxt.hash)
        return out

    def lookup(hash_hex):
        h = _parse_hash(hash_hex)
        idx = st.chain.find(h)
        if idx is None:
            raise RPCError(RPC_INVALID_ADDRESS_OR_KEY, "Block not found")
        return idx

    def rpc_getblockcount(p):
        """getblockcount — height of the most-work fully-validated chain."""
        return st.height()

    def rpc_getbestblockhash(p):
        """getbestblockhash — hash of the tip."""
        return _hex(st.tip().hash)

    def rpc_getblockhash(p):
        """getblockhash height"""
        _need(p, 1, "getblockhash height")
        h = int(p[0])
        idx = st.chain.at_height(h)
        if idx is None:
            raise RPCError(RPC_INVALID_PARAMETER, "Block height out of range")
        return _hex(idx.hash)

    def rpc_getblockheader(p):
        """getblockheader "hash" ( verbose )"""
        _need(p, 1, 'getblockheader "hash" ( verbose )')
        idx = lookup(p[0])
        if not _arg(p, 1, True):
            return idx.header.serialize(params.kawpow_activation_time).hex()
        return header_json(idx)

    def rpc_getblock(p):
        """getblock "blockhash" ( verbosity ) — 0: hex, 1: json with txids, 2: json with decoded txs."""
        _need(p, 1, 'getblock "blockhash" ( verbosity )')
        idx = lookup(p[0])
        verbosity = _arg(p, 1, 1)
        if isinstance(verbosity, bool):
            verbosity = int(verbosity)
        raw = st.get_block_raw(idx.hash)
        if raw is None:
            raise RPCError(RPC_MISC_ERROR, "Block not available (pruned data)")
        if verbosity == 0:
            if not node.rpc_witness:  # -rpcserialversion=0: the block without witness data
                blk = _core.Block.deserialize(raw, params.kawpow_activation_time)
                return blk.serialize(params.kawpow_activation_time, False).hex()
            return raw.hex()
        blk = _core.Block.deserialize(raw, params.kawpow_activation_time)
        out = header_json(idx, blk.header)
        out["strippedsize"] = blk.stripped_size(params.kawpow_activation_time)
        out["size"] = blk.total_size(params.kawpow_activation_time)
        out["weight"] = blk.weight(params.kawpow_activation_time)
        if verbosity >= 2:
            out["tx"] = [tx_json(tx) for tx in blk.vtx]
        else:
            out["tx"] = [_hex(tx.txid()) for tx in blk.vtx]
        out["nTx"] = len(blk.vtx)
        return out

    def tx_json(tx):
        vin = []
        for i in tx.vin:
            if i.prevout.is_null():
                vin.append({"coinbase": i.script_sig.hex(), "sequence": i.sequence})
            else:
                vin.append({"txid": _hex(i.prevout.hash), "vout": i.prevout.n,
                            "scriptSig": {"hex": i.script_sig.hex()}, "sequence": i.sequence})
            if i.witness:
                vin[-1]["txinwitness"] = [w.hex() for w in i.witness]
        vout = []
        for n, o in enumerate(tx.vout):
            addr = _core.script_to_address(o.script_pubkey, params.pubkey_prefix, params.script_prefix)
            e = {"value": o.value / 1e8, "valueSat": o.value, "n": n, "scriptPubKey": {"hex": o.script_pubkey.hex()}}
            if addr:
                e["scriptPubKey"]["addresses"] = [addr]
            vout.append(e)
        return {"txid": _hex(tx.txid()), "hash": _hex(tx.wtxid()), "version": tx.version,
                "size": len(tx.serialize(True)), "vsize": (len(tx.serialize(False)) * 3 + len(tx.serialize(True)) + 3) // 4,
                "locktime": tx.lock_time, "vin": vin, "vout": vout, "hex": tx.serialize(node.rpc_witness).hex()}

    def rpc_getdifficulty(p):
        """getdifficulty — proof-of-work difficulty as a multiple of the minimum difficulty."""
        return _core.difficulty_from_bits(st.tip().bits)

    def rpc_getblockchaininfo(p):
        """getblockchaininfo — state of the chain."""
        tip = st.tip()
        out = {"chain": params.network_id, "blocks": tip.height, "headers": st.chain.height(),
               "bestblockhash": _hex(tip.hash), "difficulty": _core.difficulty_from_bits(tip.bits),
               "mediantime": tip.median_time_past(), "verificationprogress": 1.0,
               "initialblockdownload": st.is_initial_block_download(),
               "chainwork": "%064x" % tip.chain_work, "size_on_disk": node.blocks_size_on_disk(),
               "pruned": st.prune_mode, "warnings": node.get_warnings(),
               "bip9_softforks": st.versionbits.bip9_softforks(tip),
               "kawpow_activation_time": params.kawpow_activation_time,
               "equihash_activation_time": params.equihash_activation_time}
        if st.prune_mode:  # src/rpc/blockchain.cpp:1474-1490
            out["pruneheight"] = st.prune_height()
            out["automatic_pruning"] = st.prune_target != 1
            if st.prune_target != 1:
                out["prune_target_size"] = st.prune_target
        return out

    def rpc_getchaintips(p):
        """getchaintips — the active tip (side branches are tracked by the header chain)."""
        tip = st.tip()
        return [{"height": tip.height, "hash": _hex(tip.hash), "branchlen": 0, "status": "active"}]

    def rpc_invalidateblock(p):
        """invalidateblock "blockhash" """
        _need(p, 1, 'invalidateblock "blockhash"')
        idx = lookup(p[0])
        st.invalidate_block(idx.hash)
        return None

    def rpc_reconsiderblock(p):
        """reconsiderblock "blockhash" """
        _need(p, 1, 'reconsiderblock "blockhash"')
        idx = lookup(p[0])
        st.reconsider_block(idx.hash)
        return None

    def rpc_waitfornewblock(p):
        """waitfornewblock ( timeout_ms ) — wait for a new tip."""
        timeout = float(_arg(p, 0, 0)) / 1000.0
        old = st.tip().hash
        st.wait_for_tip_change(old, timeout if timeout > 0 else None)
        tip = st.tip()
        return {"hash": _hex(tip.hash), "height": tip.height}

    def rpc_verifychain(p):
        """verifychain ( checklevel nblocks ) — re-check stored blocks (structure + PoW, mix-only)."""
        nblocks = int(_arg(p, 1, 6))
        tip = st.tip()
        for h in range(max(1, tip.height - nblocks + 1), tip.height + 1):
            idx = st.chain.at_height(h)
            blk = st.get_block(idx.hash)
            if blk is None or not _core.check_block(blk, params, True)[0]:
                return False
            if not _core.check_proof_of_work(st.block_hash(blk.header), blk.header.bits, params):
                return False
        return True

    for name, fn, args in [
        ("getblockcount", rpc_getblockcount, ()), ("getbestblockhash", rpc_getbestblockhash, ()),
        ("getblockhash", rpc_getblockhash, ("height",)), ("getblockheader", rpc_getblockheader, ("blockhash", "verbose")),
        ("getblock", rpc_getblock, ("blockhash", "verbosity")), ("getdifficulty", rpc_getdifficulty, ()),
        ("getblockchaininfo", rpc_getblockchaininfo, ()), ("getchaintips", rpc_getchaintips, ()),
        ("invalidateblock", rpc_invalidateblock, ("blockhash",)),
        ("reconsiderblock", rpc_reconsiderblock, ("blockhash",)),
        ("waitfornewblock", rpc_waitfornewblock, ("timeout",)), ("verifychain", rpc_verifychain, ("checklevel", "nblocks")),
    ]:
        table.append("blockchain", name, fn, args)

    # ------------------------------------------------------------------ mining
    def rpc_getmininginfo(p):
        """getmininginfo — mining-related information (+ per-GPU rates)."""
        tip = st.tip()
        return {"blocks": tip.height, "currentblockweight": node.last_block_weight, "currentblocktx": node.last_block_tx,
                "difficulty": _core.difficulty_from_bits(tip.bits), "networkhashps": st.network_hashps(120, -1),
                "hashespersec": int(node.miner.hashrate), "pooledtx": len(st.mempool), "chain": params.network_id,
                "warnings": node.get_warnings(), "gpus": node.gpu_info(),
                "workers": node.miner.workers()}

    def rpc_getnetworkhashps(p):
        """getnetworkhashps ( nblocks height )"""
        return st.network_hashps(int(_arg(p, 0, 120)), int(_arg(p, 1, -1)))

    def rpc_getblocktemplate(p):
        """getblocktemplate ( TemplateRequest ) — BIP22/23 template + KawPow pprpcheader/pprpcepoch."""
        req = _arg(p, 0, {}) or {}
        mode = req.get("mode", "template")
        if mode == "proposal":
            data = req.get("data")
            if not isinstance(data, str):
                raise RPCError(RPC_TYPE_ERROR, "Missing data String key for proposal")
            blk = _core.Block.deserialize(bytes.fromhex(data), params.kawpow_activation_time)
            ok, reason, _ = _core.check_block(blk, params, True)
            return None if ok else reason
        if mode != "template":
            raise RPCError(RPC_INVALID_PARAMETER, "Invalid mode")
        if params.mining_requires_peers and not node.args.get_bool("bypassdownload", False) and node.peer_count() == 0:
            from .protocol import RPC_CLIENT_NOT_CONNECTED

            raise RPCError(RPC_CLIENT_NOT_CONNECTED, "Clore is not connected!")
        if params.mining_requires_peers and not node.args.get_bool("bypassdownload", False) \
                and st.is_initial_block_download():
            from .protocol import RPC_CLIENT_IN_INITIAL_DOWNLOAD

            raise RPCError(RPC_CLIENT_IN_INITIAL_DOWNLOAD, "Clore is downloading blocks...")
        lp = req.get("longpollid")
        if isinstance(lp, str) and len(lp) >= 64:
            want = _core.u256_from_hex(lp[:64])
            deadline = time.time() + 60
            while st.tip().hash == want and time.time() < deadline and not node.shutdown_requested():
                st.wait_for_tip_change(want, 1.0)
        tpl = node.template_for_gbt()
        blk = tpl.block
        hdr = blk.header
        # depends = 1-based template positions of in-template parents; sigops = GetTransactionSigOpCost
        # (segwit is active on every network, so never divided by 4): src/rpc/mining.cpp:585-617
        txs, pos = [], {blk.vtx[0].txid(): 0}
        for i, tx in enumerate(blk.vtx[1:], start=1):
            txid = tx.txid()
            pos[txid] = i
            e = st.mempool.get(txid)
            deps = sorted({pos[x.prevout.hash] for x in tx.vin if x.prevout.hash in pos})
            sigops = st.mempool_sigop_cost(txid) if e else _core.tx_legacy_sigops(tx.serialize(True)) * 4
            txs.append({"data": tx.serialize(True).hex(), "txid": _hex(txid), "hash": _hex(tx.wtxid()),
                        "depends": deps, "fee": e.fee if e else 0, "sigops": sigops,
                        "weight": len(tx.serialize(False)) * 3 + len(tx.serialize(True))})
        res = {
            "capabilities": ["proposal"],
            "version": hdr.version,
            **st.versionbits.gbt_fields(st.tip()),
            "previousblockhash": _hex(hdr.prev),
            "transactions": txs,
            "coinbaseaux": {"flags": ""},
            "coinbasevalue": blk.vtx[0].vout[0].value,
            "CommunityAutonomousAddress": params.community_autonomous_address,
            "CommunityAutonomousValue": blk.vtx[0].vout[1].value,
            "longpollid": _hex(hdr.prev) + str(st.transactions_updated),
            "target": "%064x" % tpl.target,
            "mintime": st.tip().median_time_past() + 1,
            "mutable": ["time", "transactions", "prevblock"],
            "noncerange": "00000000ffffffff",
            "sigoplimit": 80000,
            "sizelimit": 8000000,
            "weightlimit": 8000000,
            "curtime": hdr.time,
            "bits": "%08x" % hdr.bits,
            "height": tpl.height,
        }
        if tpl.witness_commitment:
            res["default_witness_commitment"] = tpl.witness_commitment.hex()
        if hdr.time >= params.equihash_activation_time:
            # Equihash(200,9) extension era (new; the reference has no Equihash): the 80-byte input
            # prefix of the cached template, for external solvers answering with equihashsubmit
            # (the analogue of pprpcheader / pprpcsb); a full block goes through submitblock as usual
            if node.mining_script is not None:
                res["equihash"] = node.register_equihash_template(tpl)
        elif hdr.time >= params.kawpow_activation_time and node.mining_script is not None:
            hh = node.register_pprpc_template(tpl)
            res["pprpcheader"] = hh
            res["pprpcepoch"] = tpl.height // _core.EPOCH_LENGTH
        return res

    def _submit(blk):
        h = st.block_hash(blk.header)
        idx = st.chain.find(h)
        if idx is not None and st.get_block_raw(h) is not None:
            return "duplicate"
        state = st.process_new_block(blk)
        if state.ok:
            node.last_block_tx = len(blk.vtx)
            node.last_block_weight = blk.weight(params.kawpow_activation_time)
        return _bip22(state)

    def rpc_submitblock(p):
        """submitblock "hexdata" ( "dummy" ) — BIP22 result (null on success)."""
        _need(p, 1, 'submitblock "hexdata"')
        try:
            blk = _core.Block.deserialize(bytes.fromhex(p[0]), params.kawpow_activation_time)
        except Exception:
            raise RPCError(RPC_DESERIALIZATION_ERROR, "Block decode failed")
        if not blk.vtx or not blk.vtx[0].is_coinbase():
            raise RPCError(RPC_DESERIALIZATION_ERROR, "Block does not start with a coinbase")
        return _submit(blk)

    def rpc_pprpcsb(p):
        """pprpcsb "header_hash" "mix_hash" "nonce" — submit a KawPow solution for a cached template."""
        if len(p) != 3:
            raise RPCError(RPC_MISC_ERROR, 'pprpcsb "header_hash" "mix_hash" "nonce"')
        header_hash, mix_hex, nonce_hex = p
        try:
            nonce = int(nonce_hex, 16)
        except (TypeError, ValueError):
            raise RPCError(RPC_INVALID_PARAMS, "Invalid hex nonce")
        tpl = node.pprpc_templates.get(header_hash)
        if tpl is None:
            raise RPCError(RPC_INVALID_PARAMS, "Block header hash not found in block data")
        blk = _core.Block.deserialize(tpl.block.serialize(params.kawpow_activation_time), params.kawpow_activation_time)
        hdr = blk.header
        hdr.nonce64 = nonce
        hdr.mix_hash = _core.u256_from_hex(mix_hex)
        blk.header = hdr
        pow_hash, _mix = st.chain.block_hash_full(hdr)
        if not _core.check_proof_of_work(pow_hash, hdr.bits, params):
            raise RPCError(RPC_DESERIALIZATION_ERROR, "Block does not solve the boundary")
        r = _submit(blk)
        return True if r is None else r

    def rpc_equihashsubmit(p):
        """equihashsubmit "input_hex" "nonce256_hex" "solution_hex" — submit an Equihash(200,9)
        solution for a template whose 80-byte input prefix getblocktemplate returned (the
        extension's pprpcsb). Returns true, or the BIP22 rejection reason."""
        if len(p) != 3:
            raise RPCError(RPC_MISC_ERROR, 'equihashsubmit "input_hex" "nonce256_hex" "solution_hex"')
        tpl = node.equihash_templates.get(str(p[0]).lower())
        if tpl is None:
            raise RPCError(RPC_INVALID_PARAMS, "Equihash input not found in block data")
        try:
            nonce256, solution = bytes.fromhex(p[1]), bytes.fromhex(p[2])
        except (TypeError, ValueError):
            raise RPCError(RPC_INVALID_PARAMS, "Invalid hex nonce or solution")
        if len(nonce256) != 32:
            raise RPCError(RPC_INVALID_PARAMS, "nonce256 must be 32 bytes")
        act = params.kawpow_activation_time
        blk = _core.Block.deserialize(tpl.block.serialize(act), act)
        hdr = blk.header
        hdr.nonce256 = nonce256
        hdr.solution = solution
        blk.header = hdr
        ep = _core.EquihashParams(params.equihash_n, params.equihash_k)
        if len(solution) != ep.solution_bytes or not _core.equihash_verify(ep, hdr.equihash_input(),
                                                                           _core.equihash_unpack(ep, solution))[0]:
            raise RPCError(RPC_DESERIALIZATION_ERROR, "Invalid Equihash solution")
        if not _core.check_proof_of_work(hdr.equihash_hash(act), hdr.bits, params):
            raise RPCError(RPC_DESERIALIZATION_ERROR, "Block does not solve the boundary")
        r = _submit(blk)
        return True if r is None else r

    def rpc_getkawpowhash(p):
        """getkawpowhash "header_hash" "mix_hash" "nonce" height ( "target" )"""
        if len(p) < 4:
            raise RPCError(RPC_MISC_ERROR, 'getkawpowhash "header_hash" "mix_hash" "nonce" height ( "target" )')
        header_hex, mix_hex, nonce_hex, height = p[0], p[1], p[2], int(p[3])
        try:
            nonce = int(nonce_hex, 16)
        except (TypeError, ValueError):
            raise RPCError(RPC_INVALID_PARAMS, "Invalid nonce hex string")
        if height > st.height() + 10:
            raise RPCError(RPC_DESERIALIZATION_ERROR, "Block height is to large")
        header_hash = bytes.fromhex(header_hex.removeprefix("0x").rjust(64, "0"))  # to_hash256: storage order
        ctx = _core.get_epoch_context(height // _core.EPOCH_LENGTH)
        fin, mix = _core.kawpow_hash(ctx, height, header_hash, nonce)
        mined_mix, mined_final = from_progpow(mix), from_progpow(fin)
        out = {"result": "true" if mined_mix == _core.u256_from_hex(mix_hex) else "false",
               "digest": _hex(mined_final), "mix_hash": _hex(mined_mix), "info": ""}
        if len(p) >= 5 and p[4] is not None:
            target = int.from_bytes(_core.u256_from_hex(p[4])[::-1], "big")
            out["meets_target"] = "true" if int.from_bytes(mined_final[::-1], "big") <= target else "false"
        return out

    def _script_for(address):
        spk = _core.address_to_script(address, params.pubkey_prefix, params.script_prefix)
        if spk is None:
            raise RPCError(RPC_INVALID_ADDRESS_OR_KEY, "Error: Invalid address")
        return spk

    def rpc_generatetoaddress(p):
        """generatetoaddress nblocks "address" ( maxtries )"""
        _need(p, 2, 'generatetoaddress nblocks "address" ( maxtries )')
        return node.miner.generate(_script_for(p[1]), int(p[0]), int(_arg(p, 2, 1_000_000)))

    def rpc_generate(p):
        """generate nblocks ( maxtries ) — mine to -miningaddress (wallet-less engine)."""
        _need(p, 1, "generate nblocks ( maxtries )")
        if node.mining_script is None:
            raise RPCError(RPC_MISC_ERROR, "Error: no -miningaddress configured (the engine has no wallet)")
        return node.miner.generate(node.mining_script, int(p[0]), int(_arg(p, 1, 1_000_000)))

    def rpc_getgenerate(p):
        """getgenerate — whether the internal GPU miner is running."""
        return node.miner.generating

    def rpc_setgenerate(p):
        """setgenerate generate ( genproclimit ) — start/stop the GPU miner."""
        _need(p, 1, "setgenerate generate ( genproclimit )")
        node.miner.set_generate(bool(p[0]), node.mining_script)
        return None

    def rpc_prioritisetransaction(p):
        """prioritisetransaction <txid> <dummy> <fee delta> — adjust a mempool entry's fee."""
        _need(p, 3, "prioritisetransaction <txid> <dummy value> <fee delta>")
        e = st.mempool.get(_parse_hash(p[0]))
        if e is not None:
            e.fee += int(p[2])
            e.fee_delta += int(p[2])
        return True

    for name, fn, args in [
        ("getmininginfo", rpc_getmininginfo, ()), ("getnetworkhashps", rpc_getnetworkhashps, ("nblocks", "height")),
        ("getblocktemplate", rpc_getblocktemplate, ("template_request",)),
        ("submitblock", rpc_submitblock, ("hexdata", "dummy")),
        ("pprpcsb", rpc_pprpcsb, ("header_hash", "mix_hash", "nonce")),
        ("equihashsubmit", rpc_equihashsubmit, ("input", "nonce256", "solution")),
        ("getkawpowhash", rpc_getkawpowhash, ("header_hash", "mix_hash", "nonce", "height", "target")),
        ("prioritisetransaction", rpc_prioritisetransaction, ("txid", "dummy", "fee_delta")),
        ("getgenerate", rpc_getgenerate, ()), ("setgenerate", rpc_setgenerate, ("generate", "genproclimit")),
    ]:
        table.append("mining", name, fn, args)
    table.append("generating", "generate", rpc_generate, ("nblocks", "maxtries"))
    table.append("generating", "generatetoaddress", rpc_generatetoaddress, ("nblocks", "address", "maxtries"))

    # ------------------------------------------------------------------ raw transactions / util
    def rpc_decoderawtransaction(p):
        """decoderawtransaction "hexstring" """
        _need(p, 1, 'decoderawtransaction "hexstring"')
        try:
            return tx_json(_core.Transaction.deserialize(bytes.fromhex(p[0])))
        except Exception:
            raise RPCError(RPC_DESERIALIZATION_ERROR, "TX decode failed")

    def rpc_sendrawtransaction(p):
        """sendrawtransaction "hexstring" ( allowhighfees ) — AcceptToMemoryPool, then relay
        (src/rpc/rawtransaction.cpp sendrawtransaction)."""
        _need(p, 1, 'sendrawtransaction "hexstring" ( allowhighfees )')
        try:
            tx = _core.Transaction.deserialize(bytes.fromhex(p[0]))
        except Exception:
            raise RPCError(RPC_DESERIALIZATION_ERROR, "TX decode failed")
        txid = tx.txid()
        if txid in st.mempool:
            return _hex(txid)
        if st.coins.get(txid, 0) is not None:
            raise RPCError(RPC_VERIFY_ALREADY_IN_CHAIN, "transaction already in block chain")
        max_fee = None if _arg(p, 1, False) else st.max_tx_fee  # nAbsurdFee = -maxtxfee unless allowhighfees
        ok, reason, _ = st.accept_to_mempool(tx, max_fee=max_fee)
        if not ok:
            code = RPC_TRANSACTION_ERROR if reason == "missing-inputs" else RPC_VERIFY_REJECTED
            raise RPCError(code, "Missing inputs" if reason == "missing-inputs" else f"16: {reason}")
        return _hex(txid)

    def rpc_gettxout(p):
        """gettxout "txid" n ( include_mempool ) — an unspent output (src/rpc/blockchain.cpp gettxout)."""
        _need(p, 2, 'gettxout "txid" n ( include_mempool )')
        txid, n = _parse_hash(p[0]), int(p[1])
        include_mempool = bool(_arg(p, 2, True))
        if include_mempool and any(i.prevout.hash == txid and i.prevout.n == n
                                   for e in st.mempool.values() for i in e.tx.vin):
            return None
        c = st.coins.get(txid, n)
        confirmations_tip = st.coins_tip()
        if c is None:
            if not include_mempool or txid not in st.mempool or n >= len(st.mempool[txid].tx.vout):
                return None
            o = st.mempool[txid].tx.vout[n]
            value, spk, height, coinbase, conf = o.value, o.script_pubkey, None, False, 0
        else:
            value, spk, height, coinbase = c
            conf = confirmations_tip.height - height + 1
        return {"bestblock": _hex(confirmations_tip.hash), "confirmations": conf, "value": value / 1e8,
                "scriptPubKey": _spk_json(spk), "coinbase": coinbase}

    def rpc_gettxoutsetinfo(p):
        """gettxoutsetinfo — statistics about the UTXO set."""
        with st.lock:
            st.flush()  # FlushStateToDisk first, as the reference does: the stats describe the stored set
            tip = st.coins_tip()
            txouts, ntx, total, h, bogo = st.coins.stats()
        return {"height": tip.height, "bestblock": _hex(tip.hash), "transactions": ntx, "txouts": txouts,
                "bogosize": bogo, "hash_serialized_2": _hex(h), "disk_size": st.chainstate_disk_size(),
                "total_amount": total / 1e8}

    def rpc_getrawmempool(p):
        """getrawmempool ( verbose )"""
        if _arg(p, 0, False):
            return {_hex(k): {"fee": e.fee / 1e8, "time": int(e.time)} for k, e in st.mempool.items()}
        return [_hex(k) for k in st.mempool]

    def rpc_getmempoolinfo(p):
        """getmempoolinfo — size / bytes of the template mempool."""
        sizes = [e.vsize() for e in st.mempool.values()]
        return {"size": len(sizes), "bytes": sum(sizes), "usage": st.mempool_usage(), "maxmempool": st.max_mempool_bytes,
                "mempoolminfee": max(st.mempool_min_fee(), st.min_relay_fee) / 1e8,
                "minrelaytxfee": st.min_relay_fee / 1e8}

    def rpc_getrawtransaction(p):
        """getrawtransaction "txid" ( verbose "blockhash" ) — mempool, the given block, -txindex, or a
        transaction with an unspent output (GetTransaction)."""
        _need(p, 1, 'getrawtransaction "txid" ( verbose "blockhash" )')
        txid = _parse_hash(p[0])
        tx, in_block = None, None
        e = st.mempool.get(txid)
        if e is not None:
            tx = e.tx
        elif _arg(p, 2) is not None:
            bh = _parse_hash(p[2])
            blk = st.get_block(bh)
            if blk is None:
                raise RPCError(RPC_INVALID_ADDRESS_OR_KEY, "Block hash not found")
            for t in blk.vtx:
                if t.txid() == txid:
                    tx, in_block = t, bh
                    break
        elif st.indexes.txindex and st.indexes.tx_block(txid) is not None:  # -txindex
            bh = st.indexes.tx_block(txid)
            blk = st.get_block(bh)
            for t in (blk.vtx if blk is not None else []):
                if t.txid() == txid:
                    tx, in_block = t, bh
                    break
        else:  # GetTransaction's fAllowSlow path: a transaction with an unspent output
            h = st.coins.height_of_txid(txid)
            idx = st.chain.at_height(h) if h is not None else None
            blk = st.get_block(idx.hash) if idx is not None else None
            for t in (blk.vtx if blk is not None else []):
                if t.txid() == txid:
                    tx, in_block = t, idx.hash
                    break
        if tx is None:
            raise RPCError(RPC_INVALID_ADDRESS_OR_KEY, "No such mempool transaction. Use -txindex or provide a block hash")
        if not _arg(p, 1, False):
            return tx.serialize(node.rpc_witness).hex()  # RPCSerializationFlags (-rpcserialversion)
        out = tx_json(tx)
        if in_block is not None:  # TxToJSON: confirmations / time of an active-chain block
            out["blockhash"] = _hex(in_block)
            idx = st.chain.find(in_block)
            if idx is not None and st.chain.in_active_chain(idx):
                out["confirmations"] = 1 + st.height() - idx.height
                out["time"] = out["blocktime"] = idx.time
            else:
                out["confirmations"] = 0
        return out

    def _spk_json(spk: bytes) -> dict:
        out = {"hex": spk.hex()}
        addr = _core.script_to_address(spk, params.pubkey_prefix, params.script_prefix)
        if addr:
            out["addresses"] = [addr]
            out["type"] = "scripthash" if spk[0] == 0xa9 else "pubkeyhash"
        return out

    def rpc_validateaddress(p):
        """validateaddress "address" """
        _need(p, 1, 'validateaddress "address"')
        spk = _core.address_to_script(p[0], params.pubkey_prefix, params.script_prefix)
        if spk is None:
            return {"isvalid": False}
        w = getattr(node, "wallet", None)
        out = {"isvalid": True, "address": p[0], "scriptPubKey": spk.hex(), "isscript": spk[0] == 0xa9,
               "ismine": bool(w is not None and w.is_mine(spk))}
        if out["ismine"] and len(spk) == 25:
            h = spk[3:23]
            out["pubkey"] = w.keys[h][1].hex()
            out["iscompressed"] = True
            out["account"] = w.labels.get(h, "")
            if h in w.hdpath:
                out["hdkeypath"] = w.hdpath[h]
                out["hdmasterkeyid"] = w.hd["master_id"][::-1].hex()
        return out

    for cat, name, fn, args in [
        ("rawtransactions", "decoderawtransaction", rpc_decoderawtransaction, ("hexstring",)),
        ("rawtransactions", "sendrawtransaction", rpc_sendrawtransaction, ("hexstring", "allowhighfees")),
        ("blockchain", "gettxout", rpc_gettxout, ("txid", "n", "include_mempool")),
        ("blockchain", "gettxoutsetinfo", rpc_gettxoutsetinfo, ()),
        ("blockchain", "getrawmempool", rpc_getrawmempool, ("verbose",)),
        ("blockchain", "getmempoolinfo", rpc_getmempoolinfo, ()),
        ("rawtransactions", "getrawtransaction", rpc_getrawtransaction, ("txid", "verbose", "blockhash")),
        ("util", "validateaddress", rpc_validateaddress, ("address",)),
    ]:
        table.append(cat, name, fn, args)

    # ------------------------------------------------------------------ engine (gpu)
    def rpc_getgpuinfo(p):
        """getgpuinfo — devices, resident DAG epochs, per-GPU hash rates."""
        return node.gpu_info()

    def rpc_verifyheaders(p):
        """verifyheaders ["hexheader",...] — batch full-PoW verification (GPU when available)."""
        _need(p, 1, 'verifyheaders ["hexheader",...]')
        hdrs = [_core.BlockHeader.deserialize(bytes.fromhex(x), params.kawpow_activation_time) for x in p[0]]
        return node.verify_headers(hdrs)

    def rpc_equihashsolve(p):
        """equihashsolve "input_hex" — solve Equihash(200,9) for a 112-byte input (GPU if available)."""
        _need(p, 1, 'equihashsolve "input_hex"')
        inp = bytes.fromhex(p[0])
        sols = node.equihash_solve(inp)
        return [_core.equihash_pack(_core.EquihashParams(200, 9), s).hex() for s in sols]

    def rpc_equihashverify(p):
        """equihashverify "input_hex" "solution_hex" """
        _need(p, 2, 'equihashverify "input_hex" "solution_hex"')
        ep = _core.EquihashParams(200, 9)
        ok, why = _core.equihash_verify(ep, bytes.fromhex(p[0]), _core.equihash_unpack(ep, bytes.fromhex(p[1])))
        return {"valid": ok, "reason": why}

    for name, fn, args in [("getgpuinfo", rpc_getgpuinfo, ()), ("verifyheaders", rpc_verifyheaders, ("headers",)),
                           ("equihashsolve", rpc_equihashsolve, ("input",)),
                           ("equihashverify", rpc_equihashverify, ("input", "solution"))]:
        table.append("gpu", name, fn, args)

    # ------------------------------------------------------------------ network (src/rpc/net.cpp subset)
    def _cm():
        return getattr(node, "connman", None)

    def rpc_getconnectioncount(p):
        """getconnectioncount — number of connected peers."""
        return node.peer_count()

    def rpc_getpeerinfo(p):
        """getpeerinfo — data about each connected peer."""
        cm = _cm()
        return [x.as_dict() for x in list(cm.peers)] if cm else []

    def rpc_getnetworkinfo(p):
        """getnetworkinfo — P2P state."""
        from ..net import protocol as P

        cm = _cm()
        return {"version": 40404, "subversion": P.USER_AGENT, "protocolversion": P.PROTOCOL_VERSION,
                "localservices": "%016x" % (cm.local_services if cm is not None else
                                            (0 if st.prune_mode else P.NODE_NETWORK) | P.NODE_WITNESS),
                "localrelay": True,
                "timeoffset": getattr(st, "time_offset", 0), "networkactive": cm is not None, "connections": node.peer_count(),
                "networks": cm.proxies.describe() if cm is not None else [],
                "relayfee": 0.00001, "incrementalfee": 0.00001,
                "localaddresses": ([{"address": cm.listen_addr[0], "port": cm.port, "score": 1}]
                                   if cm is not None and cm.port else [])
                + ([{"address": h, "port": pt, "score": sc} for (h, pt), sc in sorted(cm.local_addrs.items())]
                   if cm is not None else []), "warnings": node.get_warnings()}

    def rpc_addnode(p):
        """addnode "node" "add|remove|onetry" — only onetry/add connect immediately here."""
        _need(p, 2, 'addnode "node" "add|remove|onetry"')
        cm = _cm()
        if cm is None:
            raise RPCError(-9, "P2P networking is disabled (start with -listen, -port or -connect)")
        if p[1] not in ("add", "onetry", "remove"):
            raise RPCError(-8, "Error: Node could not be added")
        if p[1] == "remove":
            if p[0] not in cm.added_nodes:
                raise RPCError(-24, "Error: Node has not been added.")
            cm.added_nodes.remove(p[0])
            return None
        if p[1] == "add":
            if p[0] in cm.added_nodes:
                raise RPCError(-23, "Error: Node already added")
            cm.added_nodes.append(p[0])
        host, _, port = str(p[0]).rpartition(":")
        cm.connect(host or "127.0.0.1", int(port or params.default_port))
        return None

    def rpc_ping(p):
        """ping — request a pong from every peer."""
        cm = _cm()
        for x in list(cm.peers) if cm else []:
            x.send("ping", struct.pack("<Q", int(time.time() * 1e6)))
        return None

    for name, fn, args in [("getconnectioncount", rpc_getconnectioncount, ()), ("getpeerinfo", rpc_getpeerinfo, ()),
                           ("getnetworkinfo", rpc_getnetworkinfo, ()), ("addnode", rpc_addnode, ("node", "command")),
                           ("ping", rpc_ping, ())]:
        table.append("network", name, fn, args)
