"""Address / spent / timestamp index RPCs (src/rpc/misc.cpp:880-1460, src/rpc/blockchain.cpp
getblockdeltas): getaddressbalance, getaddressdeltas, getaddressutxos, getaddresstxids,
getaddressmempool, getspentinfo, getblockdeltas. They read csrc/chain/indexes.* (enabled with
-addressindex / -spentindex / -timestampindex / -txindex); without the index they answer like the
reference does with its index disabled."""
from __future__ import annotations

from .. import core
from .protocol import RPC_INTERNAL_ERROR, RPC_INVALID_ADDRESS_OR_KEY, RPC_INVALID_PARAMETER, RPCError

_core = core()


def register(table, node) -> None:
    st = node.state
    params = node.params

    def _hex(h: bytes) -> str:
        return h[::-1].hex()

    def _address(type_: int, h160: bytes) -> str:
        prefix = params.pubkey_prefix if type_ == 1 else params.script_prefix
        return _core.base58check_encode(bytes([prefix]) + h160)

    def _addresses(p) -> list[tuple[bytes, int]]:
        """getAddressesFromParams: "address" or {"addresses": [...]}"""
        if not p:
            raise RPCError(RPC_INVALID_ADDRESS_OR_KEY, "Invalid address")
        arg = p[0]
        items = [arg] if isinstance(arg, str) else (arg.get("addresses") if isinstance(arg, dict) else None)
        if not isinstance(items, list) or not items:
            raise RPCError(RPC_INVALID_ADDRESS_OR_KEY, "Addresses is expected to be an array")
        out = []
        for a in items:
            spk = _core.address_to_script(str(a), params.pubkey_prefix, params.script_prefix)
            if spk is None:
                raise RPCError(RPC_INVALID_ADDRESS_OR_KEY, "Invalid address")
            out.append((spk[3:23], 1) if len(spk) == 25 else (spk[2:22], 2))
        return out

    def _need_address_index():
        if not st.indexes.addressindex:
            raise RPCError(RPC_INVALID_ADDRESS_OR_KEY, "No information available for address")

    def _obj(p) -> dict:
        return p[0] if p and isinstance(p[0], dict) else {}

    def rpc_getaddressbalance(p):
        """getaddressbalance {"addresses": [...]} ( includeAssets )"""
        addrs = _addresses(p)
        _need_address_index()
        include_assets = bool(p[1]) if len(p) > 1 else False
        per: dict[str, list[int]] = {}
        for h, t in addrs:
            for name, _, _, _, _, _, amount in st.indexes.deltas(t, h, "*" if include_assets else "CLORE"):
                b = per.setdefault(name, [0, 0])
                b[0] += amount
                if amount > 0:
                    b[1] += amount
        if include_assets:
            return [{"assetName": n, "balance": v[0], "received": v[1]} for n, v in sorted(per.items())]
        v = per.get("CLORE", [0, 0])
        return {"balance": v[0], "received": v[1]}

    def rpc_getaddressdeltas(p):
        """getaddressdeltas {"addresses": [...], "start": n, "end": n, "chainInfo": bool, "assetName": s}"""
        o = _obj(p)
        start, end = o.get("start"), o.get("end")
        if isinstance(start, int) and isinstance(end, int):
            if start <= 0 or end <= 0:
                raise RPCError(RPC_INVALID_ADDRESS_OR_KEY, "Start and end is expected to be greater than zero")
            if end < start:
                raise RPCError(RPC_INVALID_ADDRESS_OR_KEY, "End value is expected to be greater than start")
        else:
            start = end = 0
        asset = str(o.get("assetName", "CLORE"))
        addrs = _addresses(p)
        _need_address_index()
        deltas = []
        for h, t in addrs:
            for name, height, txi, txid, index, _, amount in st.indexes.deltas(t, h, asset, start, end):
                deltas.append({"assetName": name, "satoshis": amount, "txid": _hex(txid), "index": index,
                               "blockindex": txi, "height": height, "address": _address(t, h)})
        if o.get("chainInfo") and start and end:
            if start > st.height() or end > st.height():
                raise RPCError(RPC_INVALID_ADDRESS_OR_KEY, "Start or end is outside chain range")
            return {"deltas": deltas,
                    "start": {"hash": _hex(st.chain.at_height(start).hash), "height": start},
                    "end": {"hash": _hex(st.chain.at_height(end).hash), "height": end}}
        return deltas

    def rpc_getaddressutxos(p):
        """getaddressutxos {"addresses": [...], "chainInfo": bool, "assetName": s}"""
        o = _obj(p)
        asset = str(o.get("assetName", "CLORE"))
        addrs = _addresses(p)
        _need_address_index()
        rows = []
        for h, t in addrs:
            for name, txid, index, amount, script, height in st.indexes.unspent(t, h, asset):
                rows.append({"address": _address(t, h), "assetName": name, "txid": _hex(txid), "outputIndex": index,
                             "script": script.hex(), "satoshis": amount, "height": height})
        rows.sort(key=lambda r: r["height"])
        if o.get("chainInfo"):
            tip = st.tip()
            return {"utxos": rows, "hash": _hex(tip.hash), "height": tip.height}
        return rows

    def rpc_getaddresstxids(p):
        """getaddresstxids {"addresses": [...], "start": n, "end": n} ( includeAssets )"""
        o = _obj(p)
        start, end = o.get("start", 0), o.get("end", 0)
        if not (isinstance(start, int) and isinstance(end, int) and start > 0 and end > 0):
            start = end = 0
        include_assets = bool(p[1]) if len(p) > 1 else False
        addrs = _addresses(p)
        _need_address_index()
        seen: list[tuple[int, str]] = []
        keys = set()
        for h, t in addrs:
            for _, height, _, txid, _, _, _ in st.indexes.deltas(t, h, "*" if include_assets else "CLORE", start, end):
                k = (height, _hex(txid))
                if k not in keys:
                    keys.add(k)
                    seen.append(k)
        if len(addrs) > 1:
            seen.sort()
        return [txid for _, txid in seen]

    def rpc_getaddressmempool(p):
        """getaddressmempool {"addresses": [...]} ( includeAssets )"""
        addrs = _addresses(p)
        _need_address_index()
        include_assets = bool(p[1]) if len(p) > 1 else False
        want = {(h, t) for h, t in addrs}
        rows = []
        with st.lock:
            for txid, e in st.mempool.items():
                for i, vin in enumerate(e.tx.vin):
                    c = st.coins.get(vin.prevout.hash, vin.prevout.n)
                    if c is None:
                        pe = st.mempool.get(vin.prevout.hash)
                        if pe is None:
                            continue
                        o = pe.tx.vout[vin.prevout.n]
                        c = (o.value, o.script_pubkey, 0, False)
                    hit = _index_address(c[1], c[0])
                    if hit and (hit[0], hit[1]) in want and (include_assets or hit[2] == "CLORE"):
                        rows.append({"address": _address(hit[1], hit[0]), "assetName": hit[2], "txid": _hex(txid),
                                     "index": i, "satoshis": -hit[3], "timestamp": int(e.time),
                                     "prevtxid": _hex(vin.prevout.hash), "prevout": vin.prevout.n})
                for n, o in enumerate(e.tx.vout):
                    hit = _index_address(o.script_pubkey, o.value)
                    if hit and (hit[0], hit[1]) in want and (include_assets or hit[2] == "CLORE"):
                        rows.append({"address": _address(hit[1], hit[0]), "assetName": hit[2], "txid": _hex(txid),
                                     "index": n, "satoshis": hit[3], "timestamp": int(e.time)})
        rows.sort(key=lambda r: r["timestamp"])
        return rows

    def _index_address(spk: bytes, value: int):
        """(hash160, type, asset, amount) as the address index keys an output, or None."""
        if len(spk) == 25 and spk[:3] == b"\x76\xa9\x14" and spk[23:] == b"\x88\xac":
            return spk[3:23], 1, "CLORE", value
        if len(spk) == 23 and spk[:2] == b"\xa9\x14" and spk[22] == 0x87:
            return spk[2:22], 2, "CLORE", value
        if (len(spk) in (35, 67)) and spk[0] in (33, 65) and spk[-1] == 0xAC:
            return _core.hash160(spk[1:-1]), 1, "CLORE", value
        a = _core.parse_asset_script(spk)
        if a is not None:
            return a["hash160"], 1, a["name"], a["amount"]
        return None

    def rpc_getspentinfo(p):
        """getspentinfo {"txid": "...", "index": n}"""
        o = _obj(p)
        if not isinstance(o.get("txid"), str) or not isinstance(o.get("index"), int):
            raise RPCError(RPC_INVALID_ADDRESS_OR_KEY, "Invalid txid or index")
        try:
            txid = bytes.fromhex(o["txid"])[::-1]
        except ValueError:
            raise RPCError(RPC_INVALID_PARAMETER, "txid must be hexadecimal string")
        info = st.indexes.spent(txid, o["index"]) if st.indexes.spentindex and len(txid) == 32 else None
        if info is None:
            raise RPCError(RPC_INVALID_ADDRESS_OR_KEY, "Unable to get spent info")
        return {"txid": _hex(info[0]), "index": info[1], "height": info[2]}

    def rpc_getblockdeltas(p):
        """getblockdeltas "blockhash" """
        if not p:
            raise RPCError(RPC_INVALID_PARAMETER, 'getblockdeltas "blockhash"')
        try:
            h = bytes.fromhex(str(p[0]))[::-1]
        except ValueError:
            raise RPCError(RPC_INVALID_ADDRESS_OR_KEY, "Block not found")
        idx = st.chain.find(h) if len(h) == 32 else None
        if idx is None:
            raise RPCError(RPC_INVALID_ADDRESS_OR_KEY, "Block not found")
        blk = st.get_block(h)
        if blk is None:
            raise RPCError(RPC_INTERNAL_ERROR, "Can't read block from disk")
        active = st.chain.in_active_chain(idx)
        deltas = []
        for i, tx in enumerate(blk.vtx):
            txid = tx.txid()
            inputs = []
            if not tx.is_coinbase():
                for j, vin in enumerate(tx.vin):
                    info = st.indexes.spent(vin.prevout.hash, vin.prevout.n) if st.indexes.spentindex else None
                    if info is None:
                        raise RPCError(RPC_INTERNAL_ERROR, "Spent information not available")
                    d = {}
                    if info[4] in (1, 2):
                        d["address"] = _address(info[4], info[5])
                    d.update({"satoshis": -info[3], "index": j, "prevtxid": _hex(vin.prevout.hash),
                              "prevout": vin.prevout.n})
                    inputs.append(d)
            outputs = []
            for k, o in enumerate(tx.vout):
                d = {}
                spk = o.script_pubkey
                if len(spk) == 23 and spk[:2] == b"\xa9\x14":
                    d["address"] = _address(2, spk[2:22])
                elif len(spk) == 25 and spk[:3] == b"\x76\xa9\x14":
                    d["address"] = _address(1, spk[3:23])
                d.update({"satoshis": o.value, "index": k})
                outputs.append(d)
            deltas.append({"txid": _hex(txid), "index": i, "inputs": inputs, "outputs": outputs})
        hdr = blk.header
        out = {"hash": _hex(h), "confirmations": (st.height() - idx.height + 1) if active else -1,
               "size": len(blk.serialize(params.kawpow_activation_time)), "height": idx.height, "version": hdr.version,
               "merkleroot": _hex(hdr.merkle_root), "deltas": deltas, "time": hdr.time,
               "mediantime": idx.median_time_past(), "nonce": hdr.nonce, "bits": f"{hdr.bits:08x}",
               "chainwork": f"{idx.chain_work:064x}"}
        if idx.height > 0:
            out["previousblockhash"] = _hex(idx.prev_hash)
        if active and idx.height < st.height():
            out["nextblockhash"] = _hex(st.chain.at_height(idx.height + 1).hash)
        return out

    for cat, name, fn, args in [
        ("addressindex", "getaddressbalance", rpc_getaddressbalance, ("addresses", "includeAssets")),
        ("addressindex", "getaddressdeltas", rpc_getaddressdeltas, ("addresses",)),
        ("addressindex", "getaddressutxos", rpc_getaddressutxos, ("addresses",)),
        ("addressindex", "getaddresstxids", rpc_getaddresstxids, ("addresses", "includeAssets")),
        ("addressindex", "getaddressmempool", rpc_getaddressmempool, ("addresses", "includeAssets")),
        ("blockchain", "getspentinfo", rpc_getspentinfo, ("txid_index",)),
        ("blockchain", "getblockdeltas", rpc_getblockdeltas, ("blockhash",)),
    ]:
        table.append(cat, name, fn, args)
