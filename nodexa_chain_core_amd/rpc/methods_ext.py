"""Second half of the RPC table: the rest of the reference's control / blockchain / network /
raw-transaction / util commands that a wallet-less PoW engine can serve.

Parity tables: src/rpc/misc.cpp:1469 (getinfo, echo, echojson, setmocktime),
src/rpc/blockchain.cpp:1897 (clearmempool, getchaintxstats, decodeblock,
getmempoolentry / ancestors / descendants, savemempool, preciousblock, waitforblock,
waitforblockheight, pruneblockchain, getblockhashes), src/rpc/net.cpp:653
(disconnectnode, getaddednodeinfo, getnettotals, setban, listbanned, clearbanned,
setnetworkactive), src/rpc/rawtransaction.cpp:2203 (createrawtransaction,
decodescript, testmempoolaccept, gettxoutproof, verifytxoutproof) and
src/rpc/mining.cpp:1300 (estimatefee, estimatesmartfee, estimaterawfee).
Result keys and error codes follow the reference. What needs a UTXO set, the
address/spent indexes or a wallet (gettxout, getblockdeltas, signrawtransaction, ...)
stays DEFER, as SURVEY S4/S11/R7 mark it.
"""
from __future__ import annotations

import json
import os
import struct
import time

from .. import core
from ..utils import log
from ..chain.state import _compact_size, _read_compact_size
from .methods import _arg, _hex, _need, _parse_hash
from .protocol import (RPC_DESERIALIZATION_ERROR, RPC_INVALID_ADDRESS_OR_KEY, RPC_INVALID_PARAMETER,
                       RPC_METHOD_DEPRECATED, RPC_MISC_ERROR, RPC_TYPE_ERROR, RPCError)

_core = core()

RPC_CLIENT_NODE_ALREADY_ADDED = -23
RPC_CLIENT_NODE_NOT_ADDED = -24
RPC_CLIENT_NODE_NOT_CONNECTED = -29
RPC_CLIENT_INVALID_IP_OR_SUBNET = -30
RPC_CLIENT_P2P_DISABLED = -31
MAX_MONEY = 1_300_000_000 * 100_000_000  # MAX_MONEY (src/amount.h:29), 1.3B CLORE

# Opcode names for ScriptToAsmStr (src/script/script.cpp GetOpName).
_OPS = {0x00: "0", 0x4f: "-1", 0x50: "OP_RESERVED", 0x61: "OP_NOP", 0x62: "OP_VER", 0x63: "OP_IF",
        0x64: "OP_NOTIF", 0x65: "OP_VERIF", 0x66: "OP_VERNOTIF", 0x67: "OP_ELSE", 0x68: "OP_ENDIF",
        0x69: "OP_VERIFY", 0x6a: "OP_RETURN", 0x6b: "OP_TOALTSTACK", 0x6c: "OP_FROMALTSTACK",
        0x6d: "OP_2DROP", 0x6e: "OP_2DUP", 0x6f: "OP_3DUP", 0x70: "OP_2OVER", 0x71: "OP_2ROT",
        0x72: "OP_2SWAP", 0x73: "OP_IFDUP", 0x74: "OP_DEPTH", 0x75: "OP_DROP", 0x76: "OP_DUP", 0x77: "OP_NIP",
        0x78: "OP_OVER", 0x79: "OP_PICK", 0x7a: "OP_ROLL", 0x7b: "OP_ROT", 0x7c: "OP_SWAP", 0x7d: "OP_TUCK",
        0x7e: "OP_CAT", 0x7f: "OP_SUBSTR", 0x80: "OP_LEFT", 0x81: "OP_RIGHT", 0x82: "OP_SIZE",
        0x83: "OP_INVERT", 0x84: "OP_AND", 0x85: "OP_OR", 0x86: "OP_XOR", 0x87: "OP_EQUAL",
        0x88: "OP_EQUALVERIFY", 0x89: "OP_RESERVED1", 0x8a: "OP_RESERVED2", 0x8b: "OP_1ADD", 0x8c: "OP_1SUB",
        0x8d: "OP_2MUL", 0x8e: "OP_2DIV", 0x8f: "OP_NEGATE", 0x90: "OP_ABS", 0x91: "OP_NOT",
        0x92: "OP_0NOTEQUAL", 0x93: "OP_ADD", 0x94: "OP_SUB", 0x95: "OP_MUL", 0x96: "OP_DIV", 0x97: "OP_MOD",
        0x98: "OP_LSHIFT", 0x99: "OP_RSHIFT", 0x9a: "OP_BOOLAND", 0x9b: "OP_BOOLOR", 0x9c: "OP_NUMEQUAL",
        0x9d: "OP_NUMEQUALVERIFY", 0x9e: "OP_NUMNOTEQUAL", 0x9f: "OP_LESSTHAN", 0xa0: "OP_GREATERTHAN",
        0xa1: "OP_LESSTHANOREQUAL", 0xa2: "OP_GREATERTHANOREQUAL", 0xa3: "OP_MIN", 0xa4: "OP_MAX",
        0xa5: "OP_WITHIN", 0xa6: "OP_RIPEMD160", 0xa7: "OP_SHA1", 0xa8: "OP_SHA256", 0xa9: "OP_HASH160",
        0xaa: "OP_HASH256", 0xab: "OP_CODESEPARATOR", 0xac: "OP_CHECKSIG", 0xad: "OP_CHECKSIGVERIFY",
        0xae: "OP_CHECKMULTISIG", 0xaf: "OP_CHECKMULTISIGVERIFY", 0xb0: "OP_NOP1",
        0xb1: "OP_CHECKLOCKTIMEVERIFY", 0xb2: "OP_CHECKSEQUENCEVERIFY", 0xb3: "OP_NOP4", 0xb4: "OP_NOP5",
        0xb5: "OP_NOP6", 0xb6: "OP_NOP7", 0xb7: "OP_NOP8", 0xb8: "OP_NOP9", 0xb9: "OP_NOP10",
        0xc0: "OP_CLORE_ASSET"}
_OPS.update({0x50 + n: str(n) for n in range(1, 17)})


def script_asm(spk: bytes) -> str:
    """ScriptToAsmStr: pushes as hex (small ones as numbers), opcodes by name."""
    out, i = [], 0
    while i < len(spk):
        op = spk[i]
        i += 1
        if 0x01 <= op <= 0x4e:
            if op < 0x4c:
                n = op
            else:
                w = {0x4c: 1, 0x4d: 2, 0x4e: 4}[op]
                if i + w > len(spk):
                    out.append("[error]")
                    break
                n = int.from_bytes(spk[i:i + w], "little")
                i += w
            if i + n > len(spk):
                out.append("[error]")
                break
            data = spk[i:i + n]
            i += n
            out.append(str(_scriptnum_value(data)) if n <= 4 else data.hex())
        else:
            out.append(_OPS.get(op, "OP_UNKNOWN"))
    return " ".join(out)


def _scriptnum_value(data: bytes) -> int:
    """CScriptNum decoding: little-endian magnitude, sign in the top bit of the last byte."""
    if not data:
        return 0
    v = int.from_bytes(data, "little")
    if data[-1] & 0x80:
        return -(v & ~(0x80 << (8 * (len(data) - 1))))
    return v


def script_type(spk: bytes) -> str:
    """Solver() classes (src/script/standard.cpp) for the output templates the engine creates."""
    n = len(spk)
    if n == 25 and spk[:3] == b"\x76\xa9\x14" and spk[23:] == b"\x88\xac":
        return "pubkeyhash"
    if n == 23 and spk[:2] == b"\xa9\x14" and spk[22] == 0x87:
        return "scripthash"
    if n in (35, 67) and spk[0] == n - 2 and spk[-1] == 0xac:
        return "pubkey"
    if n >= 1 and spk[0] == 0x6a:
        return "nulldata"
    if n == 22 and spk[:2] == b"\x00\x14":
        return "witness_v0_keyhash"
    if n == 34 and spk[:2] == b"\x00\x20":
        return "witness_v0_scripthash"
    if n >= 3 and spk[-1] == 0xae and 0x51 <= spk[0] <= 0x60:
        return "multisig"
    return "nonstandard"


# ---------------------------------------------------------------- BIP37 partial merkle trees
def _tree_width(n: int, height: int) -> int:
    return (n + (1 << height) - 1) >> height


def _tree_hash(txids: list[bytes], height: int, pos: int) -> bytes:
    if height == 0:
        return txids[pos]
    left = _tree_hash(txids, height - 1, pos * 2)
    right = _tree_hash(txids, height - 1, pos * 2 + 1) if pos * 2 + 1 < _tree_width(len(txids), height - 1) else left
    return _core.sha256d(left + right)


def partial_merkle_tree(txids: list[bytes], match: list[bool]) -> bytes:
    """CPartialMerkleTree serialization (BIP37): nTransactions, vHash, vBits."""
    n = len(txids)
    height = 0
    while _tree_width(n, height) > 1:
        height += 1
    bits: list[bool] = []
    hashes: list[bytes] = []

    def build(h: int, pos: int) -> None:
        lo, hi = pos << h, min((pos + 1) << h, n)
        parent_of_match = any(match[lo:hi])
        bits.append(parent_of_match)
        if h == 0 or not parent_of_match:
            hashes.append(_tree_hash(txids, h, pos))
        else:
            build(h - 1, pos * 2)
            if pos * 2 + 1 < _tree_width(n, h - 1):
                build(h - 1, pos * 2 + 1)

    build(height, 0)
    vbits = bytearray((len(bits) + 7) // 8)
    for i, b in enumerate(bits):
        vbits[i // 8] |= int(b) << (i % 8)
    return struct.pack("<I", n) + _compact_size(len(hashes)) + b"".join(hashes) + _compact_size(len(vbits)) + bytes(vbits)


def parse_partial_merkle_tree(b: bytes, off: int = 0) -> tuple[bytes, list[bytes], int]:
    """ExtractMatches: (merkle root, matched txids, bytes consumed); ValueError when malformed."""
    (n,) = struct.unpack_from("<I", b, off)
    off += 4
    nh, off = _read_compact_size(b, off)
    hashes = [b[off + 32 * i: off + 32 * i + 32] for i in range(nh)]
    off += 32 * nh
    nb, off = _read_compact_size(b, off)
    vbits = b[off:off + nb]
    off += nb
    if n == 0 or nh > n or len(vbits) * 8 < nh or len(hashes[-1] if hashes else b"") != 32:
        raise ValueError("bad partial merkle tree")
    bits = [(vbits[i // 8] >> (i % 8)) & 1 for i in range(len(vbits) * 8)]
    height = 0
    while _tree_width(n, height) > 1:
        height += 1
    st = {"bit": 0, "hash": 0}
    matches: list[bytes] = []

    def walk(h: int, pos: int) -> bytes:
        if st["bit"] >= len(bits):
            raise ValueError("overflowed the bits array")
        parent_of_match = bits[st["bit"]]
        st["bit"] += 1
        if h == 0 or not parent_of_match:
            if st["hash"] >= len(hashes):
                raise ValueError("overflowed the hash array")
            x = hashes[st["hash"]]
            st["hash"] += 1
            if h == 0 and parent_of_match:
                matches.append(x)
            return x
        left = walk(h - 1, pos * 2)
        if pos * 2 + 1 < _tree_width(n, h - 1):
            right = walk(h - 1, pos * 2 + 1)
            if right == left:
                raise ValueError("duplicate hashes (CVE-2012-2459)")
        else:
            right = left
        return _core.sha256d(left + right)

    root = walk(height, 0)
    if (st["bit"] + 7) // 8 != len(vbits) or st["hash"] != len(hashes):
        raise ValueError("not all bits / hashes consumed")
    return root, matches, off


def register(table, node) -> None:  # noqa: C901 — one table, like the reference's RegisterXRPCCommands
    class _StateProxy:
        def __getattr__(self, name):
            return getattr(node.state, name)

    st = _StateProxy()
    params = node.params
    act = params.kawpow_activation_time

    def _cm(required: bool = True):
        cm = getattr(node, "connman", None)
        if cm is None and required:
            raise RPCError(RPC_CLIENT_P2P_DISABLED, "Error: Peer-to-peer functionality missing or disabled")
        return cm

    def _mempool_path():
        if node.datadir is None:
            raise RPCError(RPC_MISC_ERROR, "Unable to dump mempool to disk (no datadir)")
        return os.path.join(node.datadir, "mempool.dat")

    # ------------------------------------------------------------------ control / hidden
    def rpc_getinfo(p):
        """getinfo — DEPRECATED. Various state info (wallet fields omitted: no wallet)."""
        from ..net import protocol as P

        return {"deprecation-warning": "WARNING: getinfo is deprecated and will be fully removed in 0.16."
                                       " Projects should transition to using getblockchaininfo, getnetworkinfo,"
                                       " and getwalletinfo before upgrading to 0.16",
                "version": 40404, "protocolversion": P.PROTOCOL_VERSION, "blocks": st.height(), "timeoffset": 0,
                "connections": node.peer_count(), "proxy": "",
                "difficulty": _core.difficulty_from_bits(st.tip().bits),
                "testnet": params.network_id == "test", "relayfee": 0.00001, "errors": ""}

    def rpc_echo(p):
        """echo "message" ... — simply echo back the input arguments (testing)."""
        return list(p)

    def rpc_setmocktime(p):
        """setmocktime timestamp — set the local time (regtest only; 0 = wall clock)."""
        _need(p, 1, "setmocktime timestamp")
        if params.network_id != "regtest":
            raise RPCError(RPC_MISC_ERROR, "setmocktime for regression testing (-regtest mode) only")
        if not isinstance(p[0], int):
            raise RPCError(RPC_TYPE_ERROR, "Expected type number")
        node.state.mocktime = int(p[0])
        return None

    table.append("control", "getinfo", rpc_getinfo, ())
    table.append("hidden", "echo", rpc_echo, tuple(f"arg{i}" for i in range(10)))
    table.append("hidden", "echojson", rpc_echo, tuple(f"arg{i}" for i in range(10)))
    table.append("hidden", "setmocktime", rpc_setmocktime, ("timestamp",))

    # ------------------------------------------------------------------ blockchain
    def _entry_json(txid, e):
        anc, desc = st.mempool_ancestors(txid), st.mempool_descendants(txid)
        size = e.vsize()
        return {"size": size, "fee": e.fee / 1e8, "modifiedfee": e.fee / 1e8, "time": int(e.time),
                "height": e.height, "descendantcount": len(desc) + 1,
                "descendantsize": size + sum(st.mempool[t].vsize() for t in desc),
                "descendantfees": e.fee + sum(st.mempool[t].fee for t in desc),
                "ancestorcount": len(anc) + 1, "ancestorsize": size + sum(st.mempool[t].vsize() for t in anc),
                "ancestorfees": e.fee + sum(st.mempool[t].fee for t in anc), "wtxid": _hex(e.tx.wtxid()),
                "depends": sorted(_hex(t) for t in st.mempool_parents(txid))}

    def _pool_entry(txid_hex):
        txid = _parse_hash(txid_hex)
        e = st.mempool.get(txid)
        if e is None:
            raise RPCError(RPC_INVALID_ADDRESS_OR_KEY, "Transaction not in mempool")
        return txid, e

    def rpc_getmempoolentry(p):
        """getmempoolentry "txid" — mempool data for the given transaction."""
        _need(p, 1, 'getmempoolentry "txid"')
        txid, e = _pool_entry(p[0])
        return _entry_json(txid, e)

    def _relatives(p, fn, usage):
        _need(p, 1, usage)
        txid, _ = _pool_entry(p[0])
        rel = fn(txid)
        if not _arg(p, 1, False):
            return sorted(_hex(t) for t in rel)
        return {_hex(t): _entry_json(t, st.mempool[t]) for t in rel}

    def rpc_getmempoolancestors(p):
        """getmempoolancestors "txid" ( verbose ) — in-mempool ancestors."""
        return _relatives(p, st.mempool_ancestors, 'getmempoolancestors "txid" ( verbose )')

    def rpc_getmempooldescendants(p):
        """getmempooldescendants "txid" ( verbose ) — in-mempool descendants."""
        return _relatives(p, st.mempool_descendants, 'getmempooldescendants "txid" ( verbose )')

    def rpc_clearmempool(p):
        """clearmempool — remove every transaction from the mempool."""
        st.clear_mempool()
        return None

    def rpc_savemempool(p):
        """savemempool — dump the mempool to disk (mempool.dat)."""
        st.save_mempool(_mempool_path())
        return None

    def rpc_getchaintxstats(p):
        """getchaintxstats ( nblocks "blockhash" ) — transaction count / rate statistics."""
        if _arg(p, 1) is not None:
            idx = st.chain.find(_parse_hash(p[1]))
            if idx is None:
                raise RPCError(RPC_INVALID_ADDRESS_OR_KEY, "Block not found")
            if not st.chain.in_active_chain(idx):
                raise RPCError(RPC_INVALID_PARAMETER, "Block is not in main chain")
        else:
            idx = st.tip()
        spacing = 60
        if _arg(p, 0) is None:
            blockcount = max(0, min(30 * 24 * 60 * 60 // spacing, idx.height - 1))
        else:
            blockcount = int(p[0])
            if blockcount < 0 or (blockcount > 0 and blockcount >= idx.height):
                raise RPCError(RPC_INVALID_PARAMETER, "Invalid block count: should be between 0 and the block's height - 1")
        past = st.chain.at_height(idx.height - blockcount) if st.chain.in_active_chain(idx) else None
        txcount = st.chain_tx_count(idx)
        out = {"time": idx.time, "txcount": txcount, "window_block_count": blockcount}
        if blockcount > 0 and past is not None:
            dt = idx.median_time_past() - past.median_time_past()
            out["window_tx_count"] = txcount - st.chain_tx_count(past)
            out["window_interval"] = dt
            if dt > 0:
                out["txrate"] = out["window_tx_count"] / dt
        return out

    def rpc_decodeblock(p):
        """decodeblock "blockhex" — decode a serialized block (header fields + txids)."""
        _need(p, 1, 'decodeblock "blockhex"')
        try:
            blk = _core.Block.deserialize(bytes.fromhex(p[0]), act)
        except Exception:
            raise RPCError(RPC_DESERIALIZATION_ERROR, "Block decode failed")
        h = blk.header
        out = {"hash": _hex(st.block_hash(h)), "size": blk.total_size(act), "strippedsize": blk.stripped_size(act),
               "weight": blk.weight(act), "height": h.height, "version": h.version, "versionHex": "%08x" % (h.version & 0xFFFFFFFF),
               "merkleroot": _hex(h.merkle_root), "tx": [_hex(t.txid()) for t in blk.vtx], "time": h.time,
               "nonce": h.nonce, "bits": "%08x" % h.bits, "previousblockhash": _hex(h.prev)}
        if h.time >= act:
            out.update(headerhash=_hex(h.kawpow_header_hash()), mixhash=_hex(h.mix_hash), nonce64=h.nonce64)
        return out

    def rpc_preciousblock(p):
        """preciousblock "blockhash" — treat a block as if received before others with the same work."""
        _need(p, 1, 'preciousblock "blockhash"')
        if st.chain.find(_parse_hash(p[0])) is None:
            raise RPCError(RPC_INVALID_ADDRESS_OR_KEY, "Block not found")
        # the header chain already prefers the first-seen of equal-work tips; the active tip
        # only changes through invalidate/reconsider, so there is nothing to re-order here
        return None

    def _wait(pred, timeout_ms):
        deadline = time.time() + timeout_ms / 1000.0 if timeout_ms > 0 else None
        while not pred() and not node.shutdown_requested():
            left = None if deadline is None else deadline - time.time()
            if left is not None and left <= 0:
                break
            st.wait_for_tip_change(st.tip().hash, min(left, 1.0) if left is not None else 1.0)
        tip = st.tip()
        return {"hash": _hex(tip.hash), "height": tip.height}

    def rpc_waitforblock(p):
        """waitforblock "blockhash" ( timeout ) — wait until the block is the tip (or timeout ms)."""
        _need(p, 1, 'waitforblock "blockhash" ( timeout )')
        want = _parse_hash(p[0])
        return _wait(lambda: st.tip().hash == want, int(_arg(p, 1, 0)))

    def rpc_waitforblockheight(p):
        """waitforblockheight height ( timeout ) — wait until the tip is at least `height`."""
        _need(p, 1, "waitforblockheight height ( timeout )")
        h = int(p[0])
        return _wait(lambda: st.height() >= h, int(_arg(p, 1, 0)))

    def rpc_pruneblockchain(p):
        """pruneblockchain height — delete the blk / rev files whose blocks are all at or below
        `height` (or a unix time: blocks at least 2 hours older), keeping MIN_BLOCKS_TO_KEEP below
        the tip; returns the height pruned up to (src/rpc/blockchain.cpp:1133-1180)."""
        from ..chain.state import MIN_BLOCKS_TO_KEEP

        _need(p, 1, "pruneblockchain height")
        if not st.prune_mode:
            raise RPCError(RPC_MISC_ERROR, "Cannot prune blocks because node is not in prune mode.")
        height = int(p[0])
        if height < 0:
            raise RPCError(RPC_INVALID_PARAMETER, "Negative block height.")
        with st.lock:
            if height > 1_000_000_000:  # a block time, with TIMESTAMP_WINDOW of slack
                found = next((h for h in range(st.height() + 1) if st.chain.at_height(h).time >= height - 7200), None)
                if found is None:
                    raise RPCError(RPC_INVALID_PARAMETER, "Could not find block with at least the specified timestamp.")
                height = found
            tip = st.height()
            if tip < st.prune_after_height:
                raise RPCError(RPC_MISC_ERROR, "Blockchain is too short for pruning.")
            if height > tip:
                raise RPCError(RPC_INVALID_PARAMETER, "Blockchain is shorter than the attempted prune height.")
            if height > tip - MIN_BLOCKS_TO_KEEP:
                log.log_print("rpc", "Attempt to prune blocks close to the tip.  Retaining the minimum number of blocks.")
                height = tip - MIN_BLOCKS_TO_KEEP
            st.prune_block_files(st.files_to_prune(manual_height=height))
        return height

    def rpc_getblockhashes(p):
        """getblockhashes high low ( {"noOrphans", "logicalTimes"} ) — active-chain blocks with
        high > nTime >= low (the reference answers from -timestampindex; here a scan)."""
        _need(p, 2, "getblockhashes high low")
        high, low = int(p[0]), int(p[1])
        opts = _arg(p, 2, {}) or {}
        out = []
        if st.indexes.timestampindex:  # GetTimestampIndex: the index, active-chain blocks only with noOrphans
            for h in st.indexes.timestamps(low, high):
                idx = st.chain.find(h)
                if idx is None or (opts.get("noOrphans") and not st.chain.in_active_chain(idx)):
                    continue
                out.append({"blockhash": _hex(h), "logicalts": idx.time} if opts.get("logicalTimes") else _hex(h))
            return out
        for height in range(st.height() + 1):
            idx = st.chain.at_height(height)
            if low <= idx.time < high:
                out.append({"blockhash": _hex(idx.hash), "logicalts": idx.time} if opts.get("logicalTimes")
                           else _hex(idx.hash))
        return out

    for name, fn, args in [
        ("getmempoolentry", rpc_getmempoolentry, ("txid",)),
        ("getmempoolancestors", rpc_getmempoolancestors, ("txid", "verbose")),
        ("getmempooldescendants", rpc_getmempooldescendants, ("txid", "verbose")),
        ("clearmempool", rpc_clearmempool, ()), ("savemempool", rpc_savemempool, ()),
        ("getchaintxstats", rpc_getchaintxstats, ("nblocks", "blockhash")),
        ("decodeblock", rpc_decodeblock, ("blockhex",)), ("preciousblock", rpc_preciousblock, ("blockhash",)),
        ("pruneblockchain", rpc_pruneblockchain, ("height",)),
        ("getblockhashes", rpc_getblockhashes, ("high", "low", "options")),
    ]:
        table.append("blockchain", name, fn, args)
    table.append("hidden", "waitforblock", rpc_waitforblock, ("blockhash", "timeout"))
    table.append("hidden", "waitforblockheight", rpc_waitforblockheight, ("height", "timeout"))

    # ------------------------------------------------------------------ network
    def rpc_disconnectnode(p):
        """disconnectnode ( "address" nodeid ) — disconnect a peer by address or id."""
        cm = _cm()
        addr, nid = _arg(p, 0), _arg(p, 1)
        if (addr is None) == (nid is None) and not (addr == "" and nid is not None):
            raise RPCError(RPC_INVALID_PARAMETER, "Only one of address and nodeid should be provided.")
        if not cm.disconnect(address=addr or None, node_id=None if nid is None else int(nid)):
            raise RPCError(RPC_CLIENT_NODE_NOT_CONNECTED, "Node not found in connected nodes")
        return None

    def rpc_getaddednodeinfo(p):
        """getaddednodeinfo ( "node" ) — nodes added with addnode "add"."""
        cm = _cm()
        nodes = list(cm.added_nodes)
        if _arg(p, 0) is not None:
            if p[0] not in nodes:
                raise RPCError(RPC_CLIENT_NODE_NOT_ADDED, "Error: Node has not been added.")
            nodes = [p[0]]
        out = []
        for a in nodes:
            conns = [x for x in list(cm.peers) if f"{x.addr[0]}:{x.addr[1]}" == a or x.addr[0] == a]
            out.append({"addednode": a, "connected": bool(conns),
                        "addresses": [{"address": f"{x.addr[0]}:{x.addr[1]}",
                                       "connected": "inbound" if x.inbound else "outbound"} for x in conns]})
        return out

    def rpc_getnettotals(p):
        """getnettotals — network traffic totals."""
        cm = _cm()
        return {"totalbytesrecv": cm.total_recv, "totalbytessent": cm.total_sent, "timemillis": int(time.time() * 1000),
                "uploadtarget": cm.upload_target_info()}

    def rpc_setban(p):
        """setban "subnet" "add|remove" ( bantime absolute ) — manage the ban list."""
        _need(p, 2, 'setban "subnet" "add|remove" ( bantime absolute )')
        cm = _cm()
        addr = str(p[0]).split("/")[0]
        import ipaddress

        try:
            ipaddress.ip_address(addr)
        except ValueError:
            raise RPCError(RPC_CLIENT_INVALID_IP_OR_SUBNET, "Error: Invalid IP/Subnet")
        if p[1] == "add":
            if cm.is_banned(addr):
                raise RPCError(RPC_CLIENT_NODE_ALREADY_ADDED, "Error: IP/Subnet already banned")
            cm.ban(addr, int(_arg(p, 2, 0) or 0), bool(_arg(p, 3, False)), "manually added")
        elif p[1] == "remove":
            if not cm.unban(addr):
                raise RPCError(RPC_CLIENT_INVALID_IP_OR_SUBNET, "Error: Unban failed. Requested address/subnet was not previously banned.")
        else:
            raise RPCError(RPC_MISC_ERROR, 'setban "subnet" "add|remove" ( bantime absolute )')
        return None

    def rpc_listbanned(p):
        """listbanned — banned IPs/subnets."""
        return _cm().list_banned()

    def rpc_clearbanned(p):
        """clearbanned — clear all banned IPs."""
        _cm().banned.clear()
        return None

    def rpc_setnetworkactive(p):
        """setnetworkactive true|false — enable/disable all P2P network activity."""
        _need(p, 1, "setnetworkactive true|false")
        cm = _cm()
        cm.set_network_active(bool(p[0]))
        return cm.network_active

    for name, fn, args in [
        ("disconnectnode", rpc_disconnectnode, ("address", "nodeid")),
        ("getaddednodeinfo", rpc_getaddednodeinfo, ("node",)), ("getnettotals", rpc_getnettotals, ()),
        ("setban", rpc_setban, ("subnet", "command", "bantime", "absolute")), ("listbanned", rpc_listbanned, ()),
        ("clearbanned", rpc_clearbanned, ()), ("setnetworkactive", rpc_setnetworkactive, ("state",)),
    ]:
        table.append("network", name, fn, args)

    # ------------------------------------------------------------------ raw transactions
    def rpc_createrawtransaction(p):
        """createrawtransaction [{"txid":"id","vout":n,"sequence":n},...] {"address":amount,"data":"hex",...} ( locktime )"""
        _need(p, 2, "createrawtransaction [{\"txid\":\"id\",\"vout\":n},...] {\"address\":amount,...} ( locktime )")
        inputs, outputs = p[0], p[1]
        if isinstance(inputs, str):
            inputs = json.loads(inputs)
        if isinstance(outputs, str):
            outputs = json.loads(outputs)
        if not isinstance(inputs, list) or not isinstance(outputs, dict):
            raise RPCError(RPC_TYPE_ERROR, "Expected array of inputs and object of outputs")
        tx = _core.Transaction()
        tx.version = 2
        lock = int(_arg(p, 2, 0))
        if lock < 0 or lock > 0xFFFFFFFF:
            raise RPCError(RPC_INVALID_PARAMETER, "Invalid parameter, locktime out of range")
        tx.lock_time = lock
        vin = []
        for i in inputs:
            if "vout" not in i or not isinstance(i["vout"], int):
                raise RPCError(RPC_INVALID_PARAMETER, "Invalid parameter, missing vout key")
            if i["vout"] < 0:
                raise RPCError(RPC_INVALID_PARAMETER, "Invalid parameter, vout must be positive")
            ti, op = _core.TxIn(), _core.OutPoint()
            op.hash = _parse_hash(i.get("txid", ""))
            op.n = int(i["vout"])
            ti.prevout = op
            ti.sequence = int(i.get("sequence", 0xFFFFFFFE if lock else 0xFFFFFFFF))
            vin.append(ti)
        vout, seen = [], set()
        for k, v in outputs.items():
            o = _core.TxOut()
            if k == "data":
                data = bytes.fromhex(v)
                o.script_pubkey = b"\x6a" + _core.script_push_data(data)
                o.value = 0
            else:
                spk = _core.address_to_script(k, params.pubkey_prefix, params.script_prefix)
                if spk is None:
                    raise RPCError(RPC_INVALID_ADDRESS_OR_KEY, "Invalid Clore address: " + k)
                if k in seen:
                    raise RPCError(RPC_INVALID_PARAMETER, "Invalid parameter, duplicated address: " + k)
                seen.add(k)
                o.script_pubkey = spk
                o.value = round(float(v) * 1e8)
                if o.value < 0 or o.value > MAX_MONEY:
                    raise RPCError(RPC_TYPE_ERROR, "Amount out of range")
            vout.append(o)
        tx.vin, tx.vout = vin, vout
        return tx.serialize(True).hex()

    def rpc_decodescript(p):
        """decodescript "hexstring" — asm, type and P2SH address of a script."""
        _need(p, 1, 'decodescript "hexstring"')
        try:
            spk = bytes.fromhex(p[0])
        except ValueError:
            raise RPCError(RPC_INVALID_PARAMETER, "argument must be hexadecimal string")
        typ = script_type(spk)
        out = {"asm": script_asm(spk), "type": typ}
        addr = _core.script_to_address(spk, params.pubkey_prefix, params.script_prefix)
        if addr:
            out["reqSigs"] = 1
            out["addresses"] = [addr]
        if typ != "scripthash":
            p2sh = b"\xa9\x14" + _core.hash160(spk) + b"\x87"
            out["p2sh"] = _core.script_to_address(p2sh, params.pubkey_prefix, params.script_prefix)
        return out

    def rpc_testmempoolaccept(p):
        """testmempoolaccept ["rawtx"] ( allowhighfees ) — AcceptToMemoryPool without adding
        (src/rpc/rawtransaction.cpp testmempoolaccept)."""
        _need(p, 1, 'testmempoolaccept ["rawtx"] ( allowhighfees )')
        raws = p[0]
        if not isinstance(raws, list) or len(raws) != 1:
            raise RPCError(RPC_INVALID_PARAMETER, "Array must contain exactly one raw transaction for now")
        try:
            tx = _core.Transaction.deserialize(bytes.fromhex(raws[0]))
        except Exception:
            raise RPCError(RPC_DESERIALIZATION_ERROR, "TX decode failed")
        max_fee = None if _arg(p, 1, False) else st.max_tx_fee
        ok, why, _ = st.accept_to_mempool(tx, test_only=True, max_fee=max_fee)
        res = {"txid": _hex(tx.txid()), "allowed": ok}
        if not ok:
            res["reject-reason"] = ("18: " if why == "txn-already-in-mempool" else "16: ") + why
        return [res]

    def rpc_gettxoutproof(p):
        """gettxoutproof ["txid",...] ( "blockhash" ) — hex CMerkleBlock proving the txids are in a block."""
        _need(p, 1, 'gettxoutproof ["txid",...] ( "blockhash" )')
        want = [_parse_hash(t) for t in p[0]]
        if len(set(want)) != len(want):
            raise RPCError(RPC_INVALID_PARAMETER, "Invalid parameter, duplicated txid")
        blk = None
        if _arg(p, 1) is not None:
            blk = st.get_block(_parse_hash(p[1]))
            if blk is None:
                raise RPCError(RPC_INVALID_ADDRESS_OR_KEY, "Block not found")
        elif st.indexes.txindex:
            bh = st.indexes.tx_block(want[0])
            blk = st.get_block(bh) if bh is not None else None
            if blk is None:
                raise RPCError(RPC_INVALID_ADDRESS_OR_KEY, "Transaction not yet in block")
        else:  # no -txindex: scan the active chain from the tip
            for height in range(st.height(), -1, -1):
                b = st.get_block(st.chain.at_height(height).hash)
                if b is not None and want[0] in {t.txid() for t in b.vtx}:
                    blk = b
                    break
            if blk is None:
                raise RPCError(RPC_INVALID_ADDRESS_OR_KEY, "Transaction not yet in block")
        txids = [t.txid() for t in blk.vtx]
        if not set(want) <= set(txids):
            raise RPCError(RPC_INVALID_ADDRESS_OR_KEY, "Not all transactions found in specified or retrieved block")
        pmt = partial_merkle_tree(txids, [t in set(want) for t in txids])
        return (blk.header.serialize(act) + pmt).hex()

    def rpc_verifytxoutproof(p):
        """verifytxoutproof "proof" — txids the proof commits to ([] if the block is not in the active chain)."""
        _need(p, 1, 'verifytxoutproof "proof"')
        try:
            raw = bytes.fromhex(p[0])
            hdr, hlen = _header_prefix(raw)
            root, matches, _ = parse_partial_merkle_tree(raw, hlen)
        except (ValueError, IndexError, RuntimeError, struct.error):
            raise RPCError(RPC_DESERIALIZATION_ERROR, "Proof decode failed")
        if root != hdr.merkle_root:
            return []
        idx = st.chain.find(st.block_hash(hdr))
        if idx is None or not st.chain.in_active_chain(idx):
            raise RPCError(RPC_INVALID_ADDRESS_OR_KEY, "Block not found in chain")
        return [_hex(t) for t in matches]

    def _header_prefix(raw: bytes):
        """Parse the block header at the start of `raw` (80/120-byte or Equihash-extended)."""
        for n in (120, 80):  # KawPow / legacy sizes; extended headers are longer, tried below
            if len(raw) >= n:
                try:
                    h = _core.BlockHeader.deserialize(raw[:n], act)
                    if len(h.serialize(act)) == n:
                        return h, n
                except Exception:
                    pass
        # Equihash extension: 80 + 32 (nonce256) + compact-size solution
        sol_len, off = _read_compact_size(raw, 112)
        n = off + sol_len
        h = _core.BlockHeader.deserialize(raw[:n], act)
        return h, n

    for name, fn, args in [
        ("createrawtransaction", rpc_createrawtransaction, ("inputs", "outputs", "locktime")),
        ("decodescript", rpc_decodescript, ("hexstring",)),
        ("testmempoolaccept", rpc_testmempoolaccept, ("rawtxs", "allowhighfees")),
    ]:
        table.append("rawtransactions", name, fn, args)
    table.append("blockchain", "gettxoutproof", rpc_gettxoutproof, ("txids", "blockhash"))
    table.append("blockchain", "verifytxoutproof", rpc_verifytxoutproof, ("proof",))

    # ------------------------------------------------------------------ fee estimation
    # CBlockPolicyEstimator lives in csrc/chain/fees.cpp; these are src/rpc/mining.cpp:1009-1212.
    def _conf_target(v) -> int:
        """ParseConfirmTarget: 1 .. the long horizon's highest tracked target (1008)."""
        if isinstance(v, bool) or not isinstance(v, (int, float)):
            raise RPCError(RPC_TYPE_ERROR, "Expected type number")
        hi = st.fee_estimator.highest_target_tracked("long")
        t = int(v)
        if t < 1 or t > hi:
            raise RPCError(RPC_INVALID_PARAMETER, f"Invalid conf_target, must be between 1 - {hi}")
        return t

    def _amount(sat_per_kb: int) -> float:
        return round(sat_per_kb / 1e8, 8)

    def rpc_estimatefee(p):
        """estimatefee nblocks — DEPRECATED (needs -deprecatedrpc=estimatefee). Fee per kB for
        confirmation within nblocks from the medium horizon at 95 %, -1 without an estimate."""
        _need(p, 1, "estimatefee nblocks")
        if "estimatefee" not in node.args.get_list("deprecatedrpc"):
            raise RPCError(RPC_METHOD_DEPRECATED,
                           "estimatefee is deprecated and will be fully removed in v0.17. To use estimatefee in v0.16, "
                           "restart clore_blockchaind with -deprecatedrpc=estimatefee.\nProjects should transition to "
                           "using estimatesmartfee before upgrading to v0.17")
        if isinstance(p[0], bool) or not isinstance(p[0], (int, float)):
            raise RPCError(RPC_TYPE_ERROR, "Expected type number")
        r = st.fee_estimator.estimate_fee(max(1, int(p[0])))
        return -1.0 if r == 0 else _amount(r)

    def rpc_estimatesmartfee(p):
        """estimatesmartfee conf_target ( "estimate_mode" ) — {"feerate", "blocks"} or {"errors", "blocks"}."""
        _need(p, 1, 'estimatesmartfee conf_target ( "estimate_mode" )')
        target = _conf_target(p[0])
        conservative = True
        mode = _arg(p, 1)
        if mode is not None:
            if mode not in ("UNSET", "ECONOMICAL", "CONSERVATIVE"):
                raise RPCError(RPC_INVALID_PARAMETER, "Invalid estimate_mode parameter")
            conservative = mode != "ECONOMICAL"
        rate, returned, _reason, _est = st.fee_estimator.estimate_smart_fee(target, conservative)
        out = {"feerate": _amount(rate)} if rate else {"errors": ["Insufficient data or no feerate found"]}
        out["blocks"] = returned
        return out

    def rpc_estimaterawfee(p):
        """estimaterawfee conf_target ( threshold ) — per-horizon raw estimate with its pass / fail
        bucket ranges, for every horizon that tracks the target."""
        _need(p, 1, "estimaterawfee conf_target ( threshold )")
        target = _conf_target(p[0])
        threshold = 0.95 if _arg(p, 1) is None else float(p[1])
        if threshold < 0 or threshold > 1:
            raise RPCError(RPC_INVALID_PARAMETER, "Invalid threshold")

        def bucket(b):
            return {"startrange": round(b["startrange"]), "endrange": round(b["endrange"]),
                    **{k: round(b[k] * 100.0) / 100.0 for k in ("withintarget", "totalconfirmed", "inmempool",
                                                                 "leftmempool")}}
        out = {}
        for horizon in ("short", "medium", "long"):
            if target > st.fee_estimator.highest_target_tracked(horizon):
                continue
            rate, est = st.fee_estimator.estimate_raw_fee(target, threshold, horizon)
            h = {}
            if rate:
                h["feerate"] = _amount(rate)
                h["decay"] = est["decay"]
                h["scale"] = est["scale"]
                h["pass"] = bucket(est["pass"])
                if est["fail"]["startrange"] != -1:  # -1: every bucket passed, no fail range
                    h["fail"] = bucket(est["fail"])
            else:
                h["decay"] = est["decay"]
                h["scale"] = est["scale"]
                h["fail"] = bucket(est["fail"])
                h["errors"] = ["Insufficient data or no feerate found which meets threshold"]
            out[horizon] = h
        return out

    table.append("util", "estimatefee", rpc_estimatefee, ("nblocks",))
    table.append("util", "estimatesmartfee", rpc_estimatesmartfee, ("conf_target", "estimate_mode"))
    table.append("hidden", "estimaterawfee", rpc_estimaterawfee, ("conf_target", "threshold"))
