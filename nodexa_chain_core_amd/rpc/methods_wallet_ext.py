"""Remaining wallet JSON-RPC methods (src/wallet/rpcwallet.cpp:3525-3600, src/wallet/rpcdump.cpp):
watch-only imports (importaddress, importpubkey, importmulti), pruned-funds import / removal,
abortrescan, addwitnessaddress, bumpfee, getmasterkeyinfo, the account calls
(getreceivedbyaccount, listreceivedbyaccount, move, sendfrom), listwallets,
resendwallettransactions and sendfromaddress.

Two deliberate differences: bumpfee works here (the reference build throws "bumpfee has been
deprecated on the CLORE Wallet."; the replacement still needs -mempoolreplacement on the relaying
nodes, as BIP125 does), and account balances are computed from the resident wallet history rather
than a separate accounting database.
"""
from __future__ import annotations

import struct
import threading
import time

from .. import core
from ..wallet import WalletError
from ..wallet.wallet import EXT_COIN_TYPE, EXT_SECRET_PREFIX, _bip32_master, _ckd_priv, ext_key_b58, p2pkh
from .protocol import (RPC_DESERIALIZATION_ERROR, RPC_INVALID_ADDRESS_OR_KEY, RPC_INVALID_PARAMETER, RPC_MISC_ERROR,
                       RPC_TYPE_ERROR, RPC_WALLET_ERROR, RPC_WALLET_INSUFFICIENT_FUNDS, RPCError)

_core = core()
COIN = 100_000_000
EXT_PUBLIC_PREFIX = {"main": bytes.fromhex("0488B21E"), "test": bytes.fromhex("043587CF"),
                     "regtest": bytes.fromhex("043587CF")}
UNLOCK_NEEDED = "Error: Please enter the wallet passphrase with walletpassphrase first."


def ext_pub_b58(pub: bytes, c: bytes, network: str, depth: int = 0, fingerprint: bytes = b"\0" * 4,
                child: int = 0) -> str:
    """CExtPubKey::Encode under base58Prefixes[EXT_PUBLIC_KEY]."""
    return _core.base58check_encode(EXT_PUBLIC_PREFIX[network] + bytes([depth]) + fingerprint
                                    + struct.pack(">I", child) + c + pub)


def register(table, node) -> None:
    st = node.state
    params = node.params
    rescan_abort = threading.Event()
    node.rescan_abort = rescan_abort

    def wallet():
        return node.resolve_wallet()  # the request's /wallet/<name>, the only wallet, or an RPC error

    def _arg(p, i, default=None):
        return p[i] if len(p) > i and p[i] is not None else default

    def _unlocked(w):
        if w.locked:
            raise RPCError(-13, UNLOCK_NEEDED)

    def _amount(v) -> int:
        try:
            a = round(float(v) * COIN)
        except (TypeError, ValueError):
            raise RPCError(RPC_TYPE_ERROR, "Amount is not a number or string")
        if a <= 0:
            raise RPCError(RPC_TYPE_ERROR, "Invalid amount for send")
        return a

    def _spk(address: str) -> bytes:
        spk = _core.address_to_script(str(address), params.pubkey_prefix, params.script_prefix)
        if spk is None:
            raise RPCError(RPC_INVALID_ADDRESS_OR_KEY, "Invalid Clore address")
        return spk

    def _rescan():
        from .methods_wallet import rescan

        rescan(node)

    def _send_error(e: WalletError):
        msg = str(e)
        if "Insufficient funds" in msg:
            raise RPCError(RPC_WALLET_INSUFFICIENT_FUNDS, msg)
        if "walletpassphrase first" in msg:
            raise RPCError(-13, msg)
        raise RPCError(RPC_WALLET_ERROR, msg)

    # ------------------------------------------------------------------ watch-only imports
    def _import_script(w, spk: bytes, label: str, p2sh: bool, solvable: bool = False) -> None:
        try:
            if p2sh:
                w.add_redeem_script(spk)
                spk = b"\xa9\x14" + _core.hash160(spk) + b"\x87"
            w.add_watch(spk, label, solvable)
        except WalletError as e:
            raise RPCError(RPC_WALLET_ERROR, str(e))

    def rpc_importaddress(p):
        """importaddress "address" ( "label" rescan p2sh ) — watch an address or a hex script."""
        if not p:
            raise RPCError(RPC_INVALID_PARAMETER, 'importaddress "address" ( "label" rescan p2sh )')
        w = wallet()
        label, rescan, p2sh = str(_arg(p, 1, "")), bool(_arg(p, 2, True)), bool(_arg(p, 3, False))
        spk = _core.address_to_script(str(p[0]), params.pubkey_prefix, params.script_prefix)
        if spk is not None:
            if p2sh:
                raise RPCError(RPC_INVALID_ADDRESS_OR_KEY, "Cannot use the p2sh flag with an address - use a script "
                                                           "instead")
            _import_script(w, spk, label, False)
        else:
            try:
                script = bytes.fromhex(str(p[0]))
            except ValueError:
                raise RPCError(RPC_INVALID_ADDRESS_OR_KEY, "Invalid Clore address or script")
            _import_script(w, script, label, p2sh)
        if rescan:
            _rescan()
        return None

    def rpc_importpubkey(p):
        """importpubkey "pubkey" ( "label" rescan ) — watch the P2PKH and P2PK outputs of a key."""
        if not p:
            raise RPCError(RPC_INVALID_PARAMETER, 'importpubkey "pubkey" ( "label" rescan )')
        try:
            pub = bytes.fromhex(str(p[0]))
        except ValueError:
            raise RPCError(RPC_INVALID_ADDRESS_OR_KEY, "Pubkey must be a hex string")
        if len(pub) not in (33, 65) or _core.secp_pubkey_normalize(pub, len(pub) == 33) is None:
            raise RPCError(RPC_INVALID_ADDRESS_OR_KEY, "Pubkey is not a valid public key")
        w = wallet()
        label = str(_arg(p, 1, ""))
        _import_script(w, p2pkh(_core.hash160(pub)), label, False, True)
        _import_script(w, _core.script_push_data(pub) + b"\xac", label, False, True)
        if bool(_arg(p, 2, True)):
            _rescan()
        return None

    def rpc_importmulti(p):
        """importmulti [{"scriptPubKey": "<script>" | {"address": "<address>"}, "timestamp", "redeemscript",
        "pubkeys", "keys", "internal", "watchonly", "label"},...] ( {"rescan": bool} )"""
        if not p or not isinstance(p[0], list):
            raise RPCError(RPC_TYPE_ERROR, "Expected array of import requests")
        w = wallet()
        opts = _arg(p, 1, {}) or {}
        results, any_ok = [], False
        for req in p[0]:
            try:
                if not isinstance(req, dict) or "scriptPubKey" not in req or "timestamp" not in req:
                    raise RPCError(RPC_TYPE_ERROR, "Missing required fields")
                s = req["scriptPubKey"]
                if isinstance(s, dict):
                    spk = _spk(s.get("address", ""))
                else:
                    spk = bytes.fromhex(str(s))
                internal = bool(req.get("internal", False))
                label = "" if internal else str(req.get("label", ""))
                if internal and "label" in req:
                    raise RPCError(RPC_INVALID_PARAMETER, "Internal addresses should not have a label")
                keys = req.get("keys", []) or []
                pubs = req.get("pubkeys", []) or []
                rs = req.get("redeemscript")
                if rs:
                    w.add_redeem_script(bytes.fromhex(rs))
                if keys:
                    if w.locked:
                        raise RPCError(-13, UNLOCK_NEEDED)
                    for k in keys:
                        try:
                            w._add_secret(w.decode_wif(k), label)
                        except WalletError as e:
                            raise RPCError(RPC_INVALID_ADDRESS_OR_KEY, str(e))
                if not w.is_mine(spk):  # no key for it: the script is watched
                    w.add_watch(spk, label, bool(pubs or rs))
                for pub in pubs:
                    pb = bytes.fromhex(pub)
                    for s2 in (p2pkh(_core.hash160(pb)), _core.script_push_data(pb) + b"\xac"):
                        if not w.is_mine(s2):
                            w.add_watch(s2, label, True)
                results.append({"success": True})
                any_ok = True
            except RPCError as e:
                results.append({"success": False, "error": {"code": e.code, "message": e.message}})
            except (ValueError, WalletError) as e:
                results.append({"success": False, "error": {"code": RPC_MISC_ERROR, "message": str(e)}})
        if any_ok and opts.get("rescan", True):
            _rescan()
        return results

    def rpc_importprunedfunds(p):
        """importprunedfunds "rawtransaction" "txoutproof" — add a transaction confirmed in the
        active chain (proved by the merkle proof) to the wallet without a rescan."""
        if len(p) < 2:
            raise RPCError(RPC_INVALID_PARAMETER, 'importprunedfunds "rawtransaction" "txoutproof"')
        try:
            tx = _core.Transaction.deserialize(bytes.fromhex(p[0]))
        except Exception:  # noqa: BLE001
            raise RPCError(RPC_DESERIALIZATION_ERROR, "TX decode failed")
        txid = tx.txid()
        proved = table.commands["verifytxoutproof"].handler([p[1]])
        if txid[::-1].hex() not in proved:
            raise RPCError(RPC_INVALID_ADDRESS_OR_KEY, "Something wrong with merkleblock")
        hist = wallet().history
        if not hist.involves_me(tx):
            raise RPCError(RPC_INVALID_ADDRESS_OR_KEY, "No addresses in wallet correspond to included transaction")
        raw = bytes.fromhex(p[1])
        h = _core.BlockHeader.deserialize_prefix(raw, params.kawpow_activation_time, 0)[0]
        hist.add(tx, st.block_hash(h))
        return None

    def rpc_removeprunedfunds(p):
        """removeprunedfunds "txid" """
        if not p:
            raise RPCError(RPC_INVALID_PARAMETER, 'removeprunedfunds "txid"')
        try:
            txid = bytes.fromhex(p[0])[::-1]
        except ValueError:
            raise RPCError(RPC_INVALID_PARAMETER, "txid must be hexadecimal string")
        if not wallet().history.remove(txid):
            raise RPCError(RPC_INVALID_PARAMETER, "Transaction does not exist in wallet.")
        return None

    def rpc_abortrescan(p):
        """abortrescan — stop a rescan in progress (true if one was running)."""
        if getattr(node, "rescan_running", False):
            rescan_abort.set()
            return True
        return False

    # ------------------------------------------------------------------ keys
    def rpc_addwitnessaddress(p):
        """addwitnessaddress "address" — the P2SH-wrapped P2WPKH address of a wallet key."""
        if not p:
            raise RPCError(RPC_INVALID_PARAMETER, 'addwitnessaddress "address"')
        w = wallet()
        spk = _spk(p[0])
        if spk[:3] != b"\x76\xa9\x14" or spk[3:23] not in w.keys:
            raise RPCError(RPC_WALLET_ERROR, "Public key or redeemscript not known to wallet, or the key is "
                                             "uncompressed")
        sh = _core.hash160(b"\x00\x14" + spk[3:23])
        return _core.base58check_encode(bytes([params.script_prefix]) + sh)

    def rpc_getmasterkeyinfo(p):
        """getmasterkeyinfo — the BIP32 root and account extended keys of the HD wallet."""
        w = wallet()
        _unlocked(w)
        if w.hd is None:
            return {}
        net = params.network_id
        k, c = _bip32_master(w._hd_seed())
        out = {"bip32_root_private": ext_key_b58(k, c, net),
               "bip32_root_public": ext_pub_b58(_core.secp_pubkey_create(k, True), c, net)}
        path = [(44, True), (EXT_COIN_TYPE[net], True), (0, True)] if w.hd.get("bip44") else [(0, True)]
        parent = None
        for i, hard in path:
            parent = _core.secp_pubkey_create(k, True)
            k, c = _ckd_priv(k, c, i, hard)
        fp = _core.hash160(parent)[:4]
        depth, child = len(path), path[-1][0] | 0x80000000
        out["account_derivation_path"] = (f"m/44'/{EXT_COIN_TYPE[net]}'/0'" if w.hd.get("bip44") else "m/0'")
        out["account_extended_private_key"] = _core.base58check_encode(
            EXT_SECRET_PREFIX[net] + bytes([depth]) + fp + struct.pack(">I", child) + c + b"\x00" + k)
        out["account_extended_public_key"] = ext_pub_b58(_core.secp_pubkey_create(k, True), c, net, depth, fp, child)
        return out

    # ------------------------------------------------------------------ accounts
    def _label_of(w, spk: bytes) -> str | None:
        if spk in w.watch:
            return w.watch[spk].get("label", "")
        if len(spk) >= 25 and spk[:3] == b"\x76\xa9\x14":
            return w.labels.get(spk[3:23], "")
        return None

    def account_balance(w, acct: str, minconf: int) -> int:
        """GetAccountBalance: received to the account's addresses (minconf, mature), minus what the
        account sent (debit less change, fees included), plus move entries."""
        hist = w.history
        bal = 0
        for wtx in hist.ordered():
            conf = hist.confirmations(wtx)
            if conf < 0 or wtx.abandoned:
                continue
            if conf >= minconf and not (wtx.tx.is_coinbase() and conf <= _core.COINBASE_MATURITY):
                for o in wtx.tx.vout:
                    if w.is_mine(o.script_pubkey) and _label_of(w, o.script_pubkey) == acct:
                        bal += o.value
            debit = hist.debit(wtx)
            if debit and (wtx.from_account or "") == acct:
                # sent = debit less change (fee included); outputs to the wallet's own labelled
                # addresses are credited to their accounts above
                change = sum(o.value for o in wtx.tx.vout if w.is_mine(o.script_pubkey)
                             and _label_of(w, o.script_pubkey) == "change")
                bal -= debit - change
        for a, amount, *_ in hist.moves:
            if a == acct:
                bal += amount
        return bal

    def rpc_getreceivedbyaccount(p):
        """getreceivedbyaccount "account" ( minconf )"""
        if not p:
            raise RPCError(RPC_INVALID_PARAMETER, 'getreceivedbyaccount "account" ( minconf )')
        w = wallet()
        acct, minconf = str(p[0]), int(_arg(p, 1, 1))
        rec = w.history.received_by(minconf)
        return sum(v[0] for spk, v in rec.items() if _label_of(w, spk) == acct) / COIN

    def rpc_listreceivedbyaccount(p):
        """listreceivedbyaccount ( minconf include_empty include_watchonly )"""
        w = wallet()
        minconf, include_empty, watch = int(_arg(p, 0, 1)), bool(_arg(p, 1, False)), bool(_arg(p, 2, False))
        rec = w.history.received_by(minconf, watch)
        accts: dict[str, list] = {}
        for spk, (amount, conf, _) in rec.items():
            a = _label_of(w, spk)
            if a is None or a == "change":
                continue
            e = accts.setdefault(a, [0, 1 << 30, False])
            e[0] += amount
            e[1] = min(e[1], conf)
            e[2] |= w.is_watch(spk)
        if include_empty:
            for h in w.keys:
                lbl = w.labels.get(h, "")
                if lbl != "change":
                    accts.setdefault(lbl, [0, 0, False])
        out = []
        for a in sorted(accts):
            amount, conf, wo = accts[a]
            e = {"account": a, "amount": amount / COIN, "confirmations": conf if amount else 0, "label": a}
            if wo:
                e["involvesWatchonly"] = True
            out.append(e)
        return out

    def rpc_move(p):
        """move "fromaccount" "toaccount" amount ( minconf "comment" ) — an internal accounting entry."""
        if len(p) < 3:
            raise RPCError(RPC_INVALID_PARAMETER, 'move "fromaccount" "toaccount" amount ( minconf "comment" )')
        w = wallet()
        amount = _amount(p[2])
        now = int(time.time())
        comment = str(_arg(p, 4, ""))
        with w.history.lock:
            w.history.moves.append((str(p[0]), -amount, now, str(p[1]), comment))
            w.history.moves.append((str(p[1]), amount, now, str(p[0]), comment))
        w.history.save()
        return True

    def rpc_sendfrom(p):
        """sendfrom "fromaccount" "toaddress" amount ( minconf "comment" "comment_to" )"""
        if len(p) < 3:
            raise RPCError(RPC_INVALID_PARAMETER, 'sendfrom "fromaccount" "toaddress" amount ( minconf "comment" '
                                                  '"comment_to" )')
        w = wallet()
        _unlocked(w)
        acct, spk, amount, minconf = str(p[0]), _spk(p[1]), _amount(p[2]), int(_arg(p, 3, 1))
        if amount > account_balance(w, acct, minconf):
            raise RPCError(RPC_WALLET_INSUFFICIENT_FUNDS, "Account has insufficient funds")
        try:
            txid = w.send([(spk, amount)], comment=str(_arg(p, 4, "")), comment_to=str(_arg(p, 5, "")),
                          from_account=acct)
        except WalletError as e:
            _send_error(e)
        return txid[::-1].hex()

    def rpc_sendfromaddress(p):
        """sendfromaddress "from_address" "to_address" amount ( "comment" "comment_to" subtractfeefromamount
        conf_target "estimate_mode" ) — spend only that address's coins; the change returns to it."""
        if len(p) < 3:
            raise RPCError(RPC_INVALID_PARAMETER, 'sendfromaddress "from_address" "to_address" amount')
        w = wallet()
        from_spk = _core.address_to_script(str(p[0]), params.pubkey_prefix, params.script_prefix)
        if from_spk is None:
            raise RPCError(RPC_INVALID_ADDRESS_OR_KEY, "Invalid from address")
        to_spk = _core.address_to_script(str(p[1]), params.pubkey_prefix, params.script_prefix)
        if to_spk is None:
            raise RPCError(RPC_INVALID_ADDRESS_OR_KEY, "Invalid address")
        amount = _amount(p[2])
        have = sum(u["amount"] for u in w.unspent(1) if u["spendable"] and u["scriptPubKey"] == from_spk)
        if have < amount:
            raise RPCError(RPC_TYPE_ERROR, "From Address doesn't contain enough funds")
        _unlocked(w)
        try:
            txid = w.send([(to_spk, amount)], subtract_fee=bool(_arg(p, 5, False)), comment=str(_arg(p, 3, "")),
                          comment_to=str(_arg(p, 4, "")), from_scripts={from_spk}, change_spk=from_spk)
        except WalletError as e:
            _send_error(e)
        return txid[::-1].hex()

    # ------------------------------------------------------------------ misc
    def rpc_listwallets(p):
        """listwallets"""
        return list(getattr(node, "wallets", {}))

    def rpc_resendwallettransactions(p):
        """resendwallettransactions — re-announce the wallet's unconfirmed pool transactions."""
        w = wallet()
        out = []
        with st.lock:
            for wtx in w.history.ordered():
                txid = wtx.tx.txid()
                e = st.mempool.get(txid)
                if e is not None:
                    st._emit("transaction_added_to_mempool", e.tx)
                    out.append(txid[::-1].hex())
        return out

    def rpc_bumpfee(p):
        """bumpfee "txid" ( {"confTarget", "totalFee", "replaceable"} ) — replace an opted-in (BIP125)
        wallet transaction with one paying a higher fee out of its change."""
        if not p:
            raise RPCError(RPC_INVALID_PARAMETER, 'bumpfee "txid" ( options )')
        w = wallet()
        _unlocked(w)
        try:
            txid = bytes.fromhex(p[0])[::-1]
        except ValueError:
            raise RPCError(RPC_INVALID_PARAMETER, "txid must be hexadecimal string")
        opts = _arg(p, 1, {}) or {}
        if "confTarget" in opts and "totalFee" in opts:
            raise RPCError(RPC_INVALID_PARAMETER, "confTarget and totalFee options should not both be set. Please "
                                                  "provide either a confirmation target for fee estimation or an "
                                                  "explicit total fee for the transaction.")
        total = int(opts["totalFee"]) if "totalFee" in opts else None
        if total is not None and total <= 0:
            raise RPCError(RPC_INVALID_PARAMETER, f"Invalid totalFee {total} (must be greater than 0)")
        if txid not in w.history.txs:
            raise RPCError(RPC_INVALID_ADDRESS_OR_KEY, "Invalid or non-wallet transaction id")
        try:
            new, old_fee, new_fee = w.bump_fee(txid, total, bool(opts.get("replaceable", True)))
        except WalletError as e:
            msg = str(e)
            code = RPC_INVALID_PARAMETER if "Insufficient totalFee" in msg else RPC_WALLET_ERROR
            raise RPCError(code, msg)
        return {"txid": new[::-1].hex(), "origfee": old_fee / COIN, "fee": new_fee / COIN, "errors": []}

    for cat, name, fn, args in [
        ("wallet", "abortrescan", rpc_abortrescan, ()),
        ("wallet", "addwitnessaddress", rpc_addwitnessaddress, ("address",)),
        ("wallet", "bumpfee", rpc_bumpfee, ("txid", "options")),
        ("wallet", "getmasterkeyinfo", rpc_getmasterkeyinfo, ()),
        ("wallet", "getreceivedbyaccount", rpc_getreceivedbyaccount, ("account", "minconf")),
        ("wallet", "importaddress", rpc_importaddress, ("address", "label", "rescan", "p2sh")),
        ("wallet", "importmulti", rpc_importmulti, ("requests", "options")),
        ("wallet", "importprunedfunds", rpc_importprunedfunds, ("rawtransaction", "txoutproof")),
        ("wallet", "importpubkey", rpc_importpubkey, ("pubkey", "label", "rescan")),
        ("wallet", "listreceivedbyaccount", rpc_listreceivedbyaccount, ("minconf", "include_empty",
                                                                        "include_watchonly")),
        ("wallet", "listwallets", rpc_listwallets, ()),
        ("wallet", "move", rpc_move, ("fromaccount", "toaccount", "amount", "minconf", "comment")),
        ("wallet", "removeprunedfunds", rpc_removeprunedfunds, ("txid",)),
        ("wallet", "resendwallettransactions", rpc_resendwallettransactions, ()),
        ("wallet", "sendfrom", rpc_sendfrom, ("fromaccount", "toaddress", "amount", "minconf", "comment",
                                              "comment_to")),
        ("wallet", "sendfromaddress", rpc_sendfromaddress, ("from_address", "to_address", "amount", "comment",
                                                            "comment_to", "subtractfeefromamount", "conf_target",
                                                            "estimate_mode")),
    ]:
        table.append(cat, name, fn, args)
    node.account_balance = lambda acct, minconf=1: account_balance(wallet(), acct, minconf)
