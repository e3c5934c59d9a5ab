"""Asset JSON-RPC methods (src/rpc/assets.cpp:3035-3075): issue, issueunique, reissue, transfer,
transferfromaddress, listmyassets, listassets, getassetdata, listaddressesbyasset,
listassetbalancesbyaddress, getcacheinfo, and the restricted-asset family (issuequalifierasset,
issuerestrictedasset, reissuerestrictedasset, transferqualifier, addtagtoaddress,
removetagfromaddress, freezeaddress, unfreezeaddress, freezerestrictedasset,
unfreezerestrictedasset, listaddressesfortag, listtagsforaddress, listaddressrestrictions,
listglobalrestrictions, getverifierstring, checkaddresstag, checkaddressrestriction,
checkglobalrestriction, isvalidverifierstring). Quantities are asset units as floats on the wire."""
from __future__ import annotations

import fnmatch

from .. import core
from ..wallet import WalletError
from ..wallet.assets import AssetWallet
from .protocol import (RPC_INVALID_ADDRESS_OR_KEY, RPC_INVALID_PARAMETER, RPC_INVALID_REQUEST, RPC_WALLET_ERROR,
                       RPC_WALLET_INSUFFICIENT_FUNDS, RPCError)

_core = core()
COIN = 100_000_000


def _qty(v) -> int:
    try:
        q = round(float(v) * COIN)
    except (TypeError, ValueError):
        raise RPCError(RPC_INVALID_PARAMETER, "Invalid amount")
    if q <= 0:
        raise RPCError(RPC_INVALID_PARAMETER, "Invalid amount: must be greater than zero")
    return q


def register(table, node) -> None:
    st = node.state
    params = node.params

    def _arg(p, i, default=None):
        return p[i] if len(p) > i and p[i] is not None else default

    def aw() -> AssetWallet:
        return node.asset_wallet_instance()

    def call(fn, *a, **k):
        try:
            return fn(*a, **k)
        except WalletError as e:
            msg = str(e)
            if "Insufficient" in msg:
                raise RPCError(RPC_WALLET_INSUFFICIENT_FUNDS, msg)
            if "doesn't have asset" in msg:
                raise RPCError(RPC_INVALID_REQUEST, msg)
            if "Invalid" in msg or "aren't active" in msg:
                raise RPCError(RPC_INVALID_PARAMETER, msg)
            raise RPCError(RPC_WALLET_ERROR, msg)

    def _addr_of(h160: bytes) -> str:
        return _core.base58check_encode(bytes([params.pubkey_prefix]) + h160)

    def _h160(address: str) -> bytes:
        spk = _core.address_to_script(address, params.pubkey_prefix, params.script_prefix)
        if spk is None or len(spk) != 25:
            raise RPCError(RPC_INVALID_ADDRESS_OR_KEY, "Invalid Clore address: " + str(address))
        return spk[3:23]

    def _ipfs(v) -> bytes:
        if not v:
            return b""
        raw = _core.decode_asset_data(str(v))
        if not raw:
            raise RPCError(RPC_INVALID_PARAMETER, "Invalid IPFS/Txid hash")
        return raw

    def _txids(h: bytes) -> list:
        return [h[::-1].hex()]

    def _asset_json(meta: dict) -> dict:
        out = {"name": meta["name"], "amount": meta["amount"] / COIN, "units": meta["units"],
               "reissuable": meta["reissuable"], "has_ipfs": meta["has_ipfs"]}
        if meta["has_ipfs"]:
            key = "txid" if len(meta["ipfs"]) == 32 else "ipfs_hash"
            out[key] = _core.encode_asset_data(meta["ipfs"])
        v = st.assets.verifier(meta["name"])
        if v is not None:
            out["verifier_string"] = v
        return out

    # ------------------------------------------------------------------ wallet methods
    def rpc_issue(p):
        """issue "asset_name" qty "( to_address )" "( change_address )" ( units ) ( reissuable ) ( has_ipfs ) "( ipfs_hash )" """
        if not p:
            raise RPCError(RPC_INVALID_PARAMETER, 'issue "asset_name" qty ...')
        units = int(_arg(p, 4, 0))
        has_ipfs = bool(_arg(p, 6, False))
        ipfs = _ipfs(_arg(p, 7)) if has_ipfs else b""
        return _txids(call(aw().issue, p[0], _qty(_arg(p, 1, 1)), _arg(p, 2) or None, units,
                           bool(_arg(p, 5, True)), ipfs))

    def rpc_issueunique(p):
        """issueunique "root_name" [asset_tags] ( [ipfs_hashes] ) "( to_address )" "( change_address )" """
        if len(p) < 2 or not isinstance(p[1], list) or not p[1]:
            raise RPCError(RPC_INVALID_PARAMETER, 'issueunique "root_name" ["tag",...]')
        hashes = [_ipfs(h) for h in (_arg(p, 2, []) or [])]
        return _txids(call(aw().issue_unique, p[0], [str(t) for t in p[1]], hashes, _arg(p, 3) or None))

    def rpc_reissue(p):
        """reissue "asset_name" qty "to_address" "change_address" ( reissuable ) ( new_units ) "( new_ipfs )" """
        if len(p) < 3:
            raise RPCError(RPC_INVALID_PARAMETER, 'reissue "asset_name" qty "to_address"')
        return _txids(call(aw().reissue, p[0], _qty(p[1]), p[2], bool(_arg(p, 4, True)), int(_arg(p, 5, -1)),
                           _ipfs(_arg(p, 6))))

    def rpc_transfer(p):
        """transfer "asset_name" qty "to_address" "message" expire_time "change_address" "asset_change_address" """
        if len(p) < 3:
            raise RPCError(RPC_INVALID_PARAMETER, 'transfer "asset_name" qty "to_address"')
        _h160(p[2])
        return _txids(call(aw().transfer, p[0], _qty(p[1]), p[2], _ipfs(_arg(p, 3)), int(_arg(p, 4, 0)),
                           _arg(p, 6) or None))

    def _from_transfer(name, froms, qty, to, message, expire, clore_change, asset_change):
        for a in froms:
            _h160(a)
        if not aw().unspent(name):
            raise RPCError(RPC_INVALID_PARAMETER, "Wallet doesn't own the asset_name: " + name)
        _h160(to)
        return _txids(call(aw().transfer, name, _qty(qty), to, _ipfs(message), int(expire or 0),
                           asset_change or None, list(froms), clore_change or None))

    def rpc_transferfromaddress(p):
        """transferfromaddress "asset_name" "from_address" qty "to_address" "message" expire_time
        "clore_change_address" "asset_change_address" — only the asset coins held at from_address."""
        if len(p) < 4:
            raise RPCError(RPC_INVALID_PARAMETER, 'transferfromaddress "asset_name" "from_address" qty "to_address"')
        return _from_transfer(p[0], [p[1]], p[2], p[3], _arg(p, 4), _arg(p, 5, 0), _arg(p, 6), _arg(p, 7))

    def rpc_transferfromaddresses(p):
        """transferfromaddresses "asset_name" ["from_addresses"] qty "to_address" "message" expire_time
        "clore_change_address" "asset_change_address" (src/rpc/assets.cpp:1271)"""
        if len(p) < 4:
            raise RPCError(RPC_INVALID_PARAMETER, 'transferfromaddresses "asset_name" ["from_addresses"] qty '
                                                  '"to_address"')
        if not isinstance(p[1], list) or not p[1]:
            raise RPCError(RPC_INVALID_PARAMETER, "From addresses must be a non-empty array.")
        return _from_transfer(p[0], p[1], p[2], p[3], _arg(p, 4), _arg(p, 5, 0), _arg(p, 6), _arg(p, 7))

    def rpc_listmyassets(p):
        """listmyassets "( asset )" ( verbose ) ( count ) ( start ) ( confs )"""
        pattern = str(_arg(p, 0, "*"))
        verbose = bool(_arg(p, 1, False))
        bal = {k: v for k, v in aw().balances().items() if fnmatch.fnmatchcase(k, pattern)}
        names = sorted(bal)
        names = names[int(_arg(p, 3, 0)):][:int(_arg(p, 2, 2**31 - 1))]
        if not verbose:
            return {n: bal[n] / COIN for n in names}
        out = {}
        for n in names:
            outs = [{"txid": u["txid"][::-1].hex(), "vout": u["vout"], "amount": u["qty"] / COIN}
                    for u in aw().unspent(n)]
            out[n] = {"balance": bal[n] / COIN, "outpoints": outs}
        return out

    def rpc_issuequalifierasset(p):
        """issuequalifierasset "asset_name" qty "( to_address )" "( change_address )" ( has_ipfs ) "( ipfs_hash )" """
        if not p:
            raise RPCError(RPC_INVALID_PARAMETER, 'issuequalifierasset "asset_name" qty')
        name = p[0] if str(p[0]).startswith("#") else "#" + str(p[0])
        ipfs = _ipfs(_arg(p, 5)) if _arg(p, 4, False) else b""
        return _txids(call(aw().issue, name, _qty(_arg(p, 1, 1)), _arg(p, 2) or None, 0, False, ipfs))

    def rpc_issuerestrictedasset(p):
        """issuerestrictedasset "asset_name" qty "verifier" "to_address" "( change_address )" ( units ) ( reissuable ) ( has_ipfs ) "( ipfs_hash )" """
        if len(p) < 4:
            raise RPCError(RPC_INVALID_PARAMETER, 'issuerestrictedasset "asset_name" qty "verifier" "to_address"')
        name = p[0] if str(p[0]).startswith("$") else "$" + str(p[0])
        ipfs = _ipfs(_arg(p, 8)) if _arg(p, 7, False) else b""
        return _txids(call(aw().issue_restricted, name, _qty(p[1]), str(p[2]), p[3], int(_arg(p, 5, 0)),
                           bool(_arg(p, 6, True)), ipfs))

    def rpc_reissuerestrictedasset(p):
        """reissuerestrictedasset "asset_name" qty to_address ( change_verifier ) ( "new_verifier" ) ..."""
        if len(p) < 3:
            raise RPCError(RPC_INVALID_PARAMETER, 'reissuerestrictedasset "asset_name" qty "to_address"')
        name = p[0] if str(p[0]).startswith("$") else "$" + str(p[0])
        verifier = str(_arg(p, 4)) if _arg(p, 3, False) else None
        return _txids(call(aw().reissue, name, _qty(p[1]), p[2], bool(_arg(p, 7, True)), int(_arg(p, 6, -1)),
                           _ipfs(_arg(p, 8)), verifier))

    def rpc_transferqualifier(p):
        """transferqualifier "qualifier_name" qty "to_address" ..."""
        if len(p) < 3:
            raise RPCError(RPC_INVALID_PARAMETER, 'transferqualifier "qualifier_name" qty "to_address"')
        return _txids(call(aw().transfer, p[0], _qty(p[1]), p[2], _ipfs(_arg(p, 4)), int(_arg(p, 5, 0))))

    def _tag(add):
        def fn(p):
            if len(p) < 2:
                raise RPCError(RPC_INVALID_PARAMETER, '"tag_name" "to_address"')
            name = p[0] if str(p[0]).startswith("#") else "#" + str(p[0])
            _h160(p[1])
            return _txids(call(aw().tag_address, name, p[1], add))
        return fn

    def _freeze(freeze):
        def fn(p):
            if len(p) < 2:
                raise RPCError(RPC_INVALID_PARAMETER, '"asset_name" "address"')
            _h160(p[1])
            return _txids(call(aw().freeze_address, p[0], p[1], freeze))
        return fn

    def _global(freeze):
        def fn(p):
            if not p:
                raise RPCError(RPC_INVALID_PARAMETER, '"asset_name"')
            return _txids(call(aw().freeze_global, p[0], freeze))
        return fn

    # ------------------------------------------------------------------ chain-state methods
    def rpc_getassetdata(p):
        """getassetdata "asset_name" """
        if not p:
            raise RPCError(RPC_INVALID_PARAMETER, 'getassetdata "asset_name"')
        meta = st.assets.get(p[0])
        return None if meta is None else _asset_json(meta)

    def rpc_listassets(p):
        """listassets "( asset )" ( verbose ) ( count ) ( start )"""
        pattern = str(_arg(p, 0, "*"))
        verbose = bool(_arg(p, 1, False))
        names = sorted(n for n in st.assets.names() if fnmatch.fnmatchcase(n, pattern))
        start, count = int(_arg(p, 3, 0)), int(_arg(p, 2, 2**31 - 1))
        names = names[start:][:count] if start >= 0 else names[start:][:count]
        if not verbose:
            return names
        out = {}
        for n in names:
            meta = st.assets.get(n)
            d = _asset_json(meta)
            d["block_height"] = meta["height"]
            d["blockhash"] = meta["block"][::-1].hex()
            out[n] = d
        return out

    def rpc_listaddressesbyasset(p):
        """listaddressesbyasset "asset_name" ( onlytotal ) ( count ) ( start ) — needs -assetindex."""
        if not getattr(node, "asset_index", False):  # fAssetIndex (src/rpc/assets.cpp:1074)
            return "_This rpc call is not functional unless -assetindex is enabled. To enable, please run the wallet with -assetindex, this will require a reindex to occur"
        if not p:
            raise RPCError(RPC_INVALID_PARAMETER, 'listaddressesbyasset "asset_name"')
        rows = {_addr_of(h): amt / COIN for name, h, amt in st.assets.balances() if name == p[0]}
        if _arg(p, 1, False):
            return len(rows)
        return rows

    def rpc_listassetbalancesbyaddress(p):
        """listassetbalancesbyaddress "address" ( onlytotal ) ( count ) ( start ) — needs -assetindex."""
        if not getattr(node, "asset_index", False):  # fAssetIndex (src/rpc/assets.cpp:742)
            return "_This rpc call is not functional unless -assetindex is enabled. To enable, please run the wallet with -assetindex, this will require a reindex to occur"
        if not p:
            raise RPCError(RPC_INVALID_PARAMETER, 'listassetbalancesbyaddress "address"')
        h = _h160(p[0])
        rows = {name: amt / COIN for name, hh, amt in st.assets.balances() if hh == h}
        if _arg(p, 1, False):
            return len(rows)
        return rows

    def rpc_getcacheinfo(p):
        """getcacheinfo — sizes of the in-memory asset state (everything is resident)."""
        return {"assets": len(st.assets), "address balances": len(st.assets.balances()),
                "tags": len(st.assets.tags()), "restrictions": len(st.assets.restrictions()),
                "global restrictions": len(st.assets.global_restrictions())}

    def rpc_listaddressesfortag(p):
        """listaddressesfortag "tag_name" """
        if not p:
            raise RPCError(RPC_INVALID_PARAMETER, 'listaddressesfortag "tag_name"')
        return sorted(_addr_of(h) for q, h in st.assets.tags() if q == p[0])

    def rpc_listtagsforaddress(p):
        """listtagsforaddress "address" """
        h = _h160(p[0]) if p else None
        return sorted(q for q, hh in st.assets.tags() if hh == h)

    def rpc_listaddressrestrictions(p):
        """listaddressrestrictions "address" """
        h = _h160(p[0]) if p else None
        return sorted(r for r, hh in st.assets.restrictions() if hh == h)

    def rpc_listglobalrestrictions(p):
        """listglobalrestrictions"""
        return sorted(st.assets.global_restrictions())

    def rpc_getverifierstring(p):
        """getverifierstring "restricted_name" """
        if not p:
            raise RPCError(RPC_INVALID_PARAMETER, 'getverifierstring "restricted_name"')
        v = st.assets.verifier(p[0])
        if v is None:
            raise RPCError(RPC_INVALID_PARAMETER, "Verifier not found for asset: " + str(p[0]))
        return v

    def rpc_checkaddresstag(p):
        """checkaddresstag "address" "tag_name" """
        return st.assets.has_tag(p[1], _h160(p[0]))

    def rpc_checkaddressrestriction(p):
        """checkaddressrestriction "address" "restricted_name" """
        return st.assets.is_frozen(p[1], _h160(p[0]))

    def rpc_checkglobalrestriction(p):
        """checkglobalrestriction "restricted_name" """
        return st.assets.is_global_frozen(p[0])

    def rpc_isvalidverifierstring(p):
        """isvalidverifierstring "verifier_string" """
        if not p:
            raise RPCError(RPC_INVALID_PARAMETER, 'isvalidverifierstring "verifier_string"')
        ok, err, found = _core.check_verifier_string(_core.strip_verifier_string(str(p[0])))
        if not ok:
            raise RPCError(RPC_INVALID_PARAMETER, err)
        for q in found:
            if st.assets.get("#" + q) is None:
                raise RPCError(RPC_INVALID_PARAMETER, "Qualifier doesn't exist: #" + q)
        return "Valid Verifier"

    for cat, name, fn, args in [
        ("assets", "issue", rpc_issue, ("asset_name", "qty", "to_address", "change_address", "units", "reissuable",
                                         "has_ipfs", "ipfs_hash")),
        ("assets", "issueunique", rpc_issueunique, ("root_name", "asset_tags", "ipfs_hashes", "to_address",
                                                     "change_address")),
        ("assets", "listmyassets", rpc_listmyassets, ("asset", "verbose", "count", "start", "confs")),
        ("assets", "listassetbalancesbyaddress", rpc_listassetbalancesbyaddress, ("address", "onlytotal", "count",
                                                                                 "start")),
        ("assets", "getassetdata", rpc_getassetdata, ("asset_name",)),
        ("assets", "listaddressesbyasset", rpc_listaddressesbyasset, ("asset_name", "onlytotal", "count", "start")),
        ("assets", "transferfromaddress", rpc_transferfromaddress, ("asset_name", "from_address", "qty", "to_address",
                                                                     "message", "expire_time", "clore_change_address",
                                                                     "asset_change_address")),
        ("assets", "transferfromaddresses", rpc_transferfromaddresses, ("asset_name", "from_addresses", "qty",
                                                                         "to_address", "message", "expire_time",
                                                                         "clore_change_address",
                                                                         "asset_change_address")),
        ("assets", "transfer", rpc_transfer, ("asset_name", "qty", "to_address", "message", "expire_time",
                                               "change_address", "asset_change_address")),
        ("assets", "reissue", rpc_reissue, ("asset_name", "qty", "to_address", "change_address", "reissuable",
                                             "new_units", "new_ipfs")),
        ("assets", "listassets", rpc_listassets, ("asset", "verbose", "count", "start")),
        ("assets", "getcacheinfo", rpc_getcacheinfo, ()),
        ("restricted assets", "transferqualifier", rpc_transferqualifier, ("qualifier_name", "qty", "to_address",
                                                                           "change_address", "message", "expire_time")),
        ("restricted assets", "issuerestrictedasset", rpc_issuerestrictedasset, ("asset_name", "qty", "verifier",
                                                                                 "to_address", "change_address", "units",
                                                                                 "reissuable", "has_ipfs", "ipfs_hash")),
        ("restricted assets", "issuequalifierasset", rpc_issuequalifierasset, ("asset_name", "qty", "to_address",
                                                                               "change_address", "has_ipfs",
                                                                               "ipfs_hash")),
        ("restricted assets", "reissuerestrictedasset", rpc_reissuerestrictedasset, ("asset_name", "qty",
                                                                                     "to_address", "change_verifier",
                                                                                     "new_verifier",
                                                                                     "change_address", "new_units",
                                                                                     "reissuable", "new_ipfs")),
        ("restricted assets", "addtagtoaddress", _tag(True), ("tag_name", "to_address", "change_address", "asset_data")),
        ("restricted assets", "removetagfromaddress", _tag(False), ("tag_name", "to_address", "change_address",
                                                                    "asset_data")),
        ("restricted assets", "freezeaddress", _freeze(True), ("asset_name", "address", "change_address", "asset_data")),
        ("restricted assets", "unfreezeaddress", _freeze(False), ("asset_name", "address", "change_address",
                                                                  "asset_data")),
        ("restricted assets", "freezerestrictedasset", _global(True), ("asset_name", "change_address", "asset_data")),
        ("restricted assets", "unfreezerestrictedasset", _global(False), ("asset_name", "change_address",
                                                                          "asset_data")),
        ("restricted assets", "listaddressesfortag", rpc_listaddressesfortag, ("tag_name",)),
        ("restricted assets", "listtagsforaddress", rpc_listtagsforaddress, ("address",)),
        ("restricted assets", "listaddressrestrictions", rpc_listaddressrestrictions, ("address",)),
        ("restricted assets", "listglobalrestrictions", rpc_listglobalrestrictions, ()),
        ("restricted assets", "getverifierstring", rpc_getverifierstring, ("restricted_name",)),
        ("restricted assets", "checkaddresstag", rpc_checkaddresstag, ("address", "tag_name")),
        ("restricted assets", "checkaddressrestriction", rpc_checkaddressrestriction, ("address", "restricted_name")),
        ("restricted assets", "checkglobalrestriction", rpc_checkglobalrestriction, ("restricted_name",)),
        ("restricted assets", "isvalidverifierstring", rpc_isvalidverifierstring, ("verifier_string",)),
    ]:
        table.append(cat, name, fn, args)
