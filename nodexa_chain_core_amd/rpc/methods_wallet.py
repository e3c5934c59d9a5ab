"""Wallet JSON-RPC methods (src/wallet/rpcwallet.cpp, signrawtransaction from
src/rpc/rawtransaction.cpp): getnewaddress, getbalance, getunconfirmedbalance, listunspent,
sendtoaddress, sendmany, dumpprivkey, importprivkey, signrawtransaction, getwalletinfo.
Amounts are CLORE (floats) on the wire, as in the reference."""
from __future__ import annotations

from .. import core
from ..wallet import WalletError
from .protocol import (RPC_DESERIALIZATION_ERROR, RPC_INVALID_ADDRESS_OR_KEY, RPC_INVALID_PARAMETER,
                       RPC_METHOD_NOT_FOUND, RPC_TYPE_ERROR, RPC_WALLET_ERROR, RPC_WALLET_INSUFFICIENT_FUNDS,
                       RPCError)

_core = core()
COIN = 100_000_000


def _amount(v) -> int:
    try:
        a = round(float(v) * COIN)
    except (TypeError, ValueError):
        raise RPCError(RPC_TYPE_ERROR, "Amount is not a number or string")
    if a <= 0:
        raise RPCError(RPC_TYPE_ERROR, "Invalid amount for send")
    return a


def register(table, node) -> None:
    st = node.state
    params = node.params

    def wallet():
        if getattr(node, "wallet", None) is None:
            raise RPCError(RPC_METHOD_NOT_FOUND, "Method not found (wallet disabled)")
        return node.wallet

    def _arg(p, i, default=None):
        return p[i] if len(p) > i and p[i] is not None else default

    def _spk(address: str) -> bytes:
        spk = _core.address_to_script(address, params.pubkey_prefix, params.script_prefix)
        if spk is None:
            raise RPCError(RPC_INVALID_ADDRESS_OR_KEY, "Invalid Clore address")
        return spk

    def _wallet_call(fn, *a, **k):
        try:
            return fn(*a, **k)
        except WalletError as e:
            msg = str(e)
            code = RPC_WALLET_INSUFFICIENT_FUNDS if "Insufficient funds" in msg else RPC_WALLET_ERROR
            if "Invalid private key" in msg or "outside allowed range" in msg or "Invalid address" in msg:
                code = RPC_INVALID_ADDRESS_OR_KEY
            raise RPCError(code, msg)

    def rpc_getnewaddress(p):
        """getnewaddress ( "account" ) — a new P2PKH address from a fresh key."""
        return wallet().new_address(str(_arg(p, 0, "")))

    def rpc_getbalance(p):
        """getbalance ( "account" minconf ) — spendable (mature) wallet balance."""
        return wallet().balance(int(_arg(p, 1, 1))) / COIN

    def rpc_getunconfirmedbalance(p):
        """getunconfirmedbalance — wallet outputs in the mempool."""
        w = wallet()
        return (w.balance(0) - w.balance(1)) / COIN

    def rpc_listunspent(p):
        """listunspent ( minconf maxconf ["address",...] )"""
        w = wallet()
        want = set(_arg(p, 2, []) or [])
        out = []
        for u in w.unspent(int(_arg(p, 0, 1)), int(_arg(p, 1, 9_999_999))):
            addr = _core.script_to_address(u["scriptPubKey"], params.pubkey_prefix, params.script_prefix)
            if want and addr not in want:
                continue
            out.append({"txid": u["txid"][::-1].hex(), "vout": u["vout"], "address": addr,
                        "scriptPubKey": u["scriptPubKey"].hex(), "amount": u["amount"] / COIN,
                        "confirmations": u["confirmations"], "spendable": u["spendable"], "solvable": True,
                        "safe": u["confirmations"] > 0})
        return out

    def rpc_sendtoaddress(p):
        """sendtoaddress "address" amount ( "comment" "comment_to" subtractfeefromamount )"""
        if len(p) < 2:
            raise RPCError(RPC_INVALID_PARAMETER, 'sendtoaddress "address" amount')
        w = wallet()
        txid = _wallet_call(w.send, [(_spk(p[0]), _amount(p[1]))], subtract_fee=bool(_arg(p, 4, False)))
        return txid[::-1].hex()

    def rpc_sendmany(p):
        """sendmany "" {"address":amount,...} ( minconf "comment" ["address",...] )"""
        if len(p) < 2 or not isinstance(p[1], dict) or not p[1]:
            raise RPCError(RPC_INVALID_PARAMETER, 'sendmany "" {"address":amount,...}')
        outs = [(_spk(a), _amount(v)) for a, v in p[1].items()]
        txid = _wallet_call(wallet().send, outs)
        return txid[::-1].hex()

    def rpc_dumpprivkey(p):
        """dumpprivkey "address" """
        if not p:
            raise RPCError(RPC_INVALID_PARAMETER, 'dumpprivkey "address"')
        return _wallet_call(wallet().dump_privkey, p[0])

    def rpc_importprivkey(p):
        """importprivkey "privkey" ( "label" rescan ) — the UTXO set is always current: no rescan needed."""
        if not p:
            raise RPCError(RPC_INVALID_PARAMETER, 'importprivkey "privkey" ( "label" rescan )')
        _wallet_call(wallet().import_privkey, p[0], str(_arg(p, 1, "")))
        return None

    def rpc_getwalletinfo(p):
        """getwalletinfo"""
        w = wallet()
        return {"walletname": "wallet.json", "walletversion": 1, "balance": w.balance(1) / COIN,
                "unconfirmed_balance": (w.balance(0) - w.balance(1)) / COIN,
                "immature_balance": w.immature_balance() / COIN, "txcount": len(w.unspent(0)),
                "keypoolsize": len(w.keys), "paytxfee": 0.0}

    def rpc_signrawtransaction(p):
        """signrawtransaction "hexstring" ( [{"txid","vout","scriptPubKey","amount"},...] ["privkey",...]
        sighashtype ) — sign the inputs the wallet (or the given keys) can spend."""
        if not p:
            raise RPCError(RPC_INVALID_PARAMETER, 'signrawtransaction "hexstring" ( prevtxs privkeys sighashtype )')
        try:
            tx = _core.Transaction.deserialize(bytes.fromhex(p[0]))
        except Exception:
            raise RPCError(RPC_DESERIALIZATION_ERROR, "TX decode failed")
        hash_types = {"ALL": 1, "NONE": 2, "SINGLE": 3, "ALL|ANYONECANPAY": 0x81, "NONE|ANYONECANPAY": 0x82,
                      "SINGLE|ANYONECANPAY": 0x83}
        ht = hash_types.get(str(_arg(p, 3, "ALL")))
        if ht is None:
            raise RPCError(RPC_INVALID_PARAMETER, "Invalid sighash param")
        prevouts = {}
        for i in tx.vin:
            c = st._spent_coin(i.prevout)
            if c is not None:
                prevouts[(i.prevout.hash, i.prevout.n)] = (c[1], c[0])
        redeem = {}
        for d in _arg(p, 1, []) or []:
            try:
                h = bytes.fromhex(d["txid"])[::-1]
                prevouts[(h, int(d["vout"]))] = (bytes.fromhex(d["scriptPubKey"]),
                                                round(float(d.get("amount", 0)) * COIN))
                if d.get("redeemScript"):
                    rs = bytes.fromhex(d["redeemScript"])
                    redeem[_core.hash160(rs)] = rs
            except (KeyError, ValueError, TypeError):
                raise RPCError(RPC_DESERIALIZATION_ERROR, "expected object with {\"txid\",\"vout\",\"scriptPubKey\"}")
        w = wallet()
        keys = [_wallet_call(w.decode_wif, k) for k in (_arg(p, 2, []) or [])]
        tx, complete, errors = _wallet_call(w.sign, tx, prevouts, keys, ht, redeem)
        out = {"hex": tx.serialize(True).hex(), "complete": complete}
        if errors:
            out["errors"] = errors
        return out

    for cat, name, fn, args in [
        ("wallet", "getnewaddress", rpc_getnewaddress, ("account",)),
        ("wallet", "getbalance", rpc_getbalance, ("account", "minconf")),
        ("wallet", "getunconfirmedbalance", rpc_getunconfirmedbalance, ()),
        ("wallet", "listunspent", rpc_listunspent, ("minconf", "maxconf", "addresses")),
        ("wallet", "sendtoaddress", rpc_sendtoaddress,
         ("address", "amount", "comment", "comment_to", "subtractfeefromamount")),
        ("wallet", "sendmany", rpc_sendmany, ("fromaccount", "amounts", "minconf", "comment", "subtractfeefrom")),
        ("wallet", "dumpprivkey", rpc_dumpprivkey, ("address",)),
        ("wallet", "importprivkey", rpc_importprivkey, ("privkey", "label", "rescan")),
        ("wallet", "getwalletinfo", rpc_getwalletinfo, ()),
        ("rawtransactions", "signrawtransaction", rpc_signrawtransaction,
         ("hexstring", "prevtxs", "privkeys", "sighashtype")),
    ]:
        table.append(cat, name, fn, args)
