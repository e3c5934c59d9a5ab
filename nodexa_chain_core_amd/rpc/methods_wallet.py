"""Wallet JSON-RPC methods (src/wallet/rpcwallet.cpp, signrawtransaction from
src/rpc/rawtransaction.cpp): getnewaddress, getbalance, getunconfirmedbalance, listunspent,
sendtoaddress, sendmany, dumpprivkey, importprivkey, signrawtransaction, getwalletinfo.
Amounts are CLORE (floats) on the wire, as in the reference."""
from __future__ import annotations

import os
import time

from .. import core
from ..wallet import WalletError
from .protocol import (RPC_DESERIALIZATION_ERROR, RPC_INVALID_ADDRESS_OR_KEY, RPC_INVALID_PARAMETER,
                       RPC_METHOD_NOT_FOUND, RPC_MISC_ERROR, RPC_TYPE_ERROR, RPC_WALLET_ERROR,
                       RPC_WALLET_INSUFFICIENT_FUNDS, RPCError)

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


def rescan(node, start_height: int = 0) -> int:
    """ScanForWalletTransactions: feed every active-chain block from start_height to the wallet
    history; returns the number of wallet transactions found."""
    st, hist = node.state, node.wallet.history
    if st.prune_mode and st.have_pruned and start_height < st.prune_height():
        raise RPCError(RPC_MISC_ERROR, "Can't rescan beyond pruned data. Use RPC call getblockchaininfo to "
                                       "determine your pruned height.")
    n = 0
    abort = getattr(node, "rescan_abort", None)
    if abort is not None:
        abort.clear()
    node.rescan_running = True
    try:
        n = _scan(node, st, hist, start_height, abort)
    finally:
        node.rescan_running = False
    return n


def _scan(node, st, hist, start_height: int, abort) -> int:
    n = 0
    for h in range(max(0, start_height), st.height() + 1):
        if abort is not None and abort.is_set():  # abortrescan
            break
        idx = st.chain.at_height(h)
        blk = st.get_block(idx.hash)
        if blk is None:
            continue
        for tx in blk.vtx:
            n += hist.add(tx, idx.hash, save=False)
    with st.lock:
        for e in list(st.mempool.values()):
            n += hist.add(e.tx, save=False)
    hist.save()
    return n


def register(table, node) -> None:
    st = node.state
    params = node.params

    def wallet():
        return node.resolve_wallet()  # the request's /wallet/<name>, the only wallet, or an RPC error

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
            if "walletpassphrase first" in msg:
                code = -13   # RPC_WALLET_UNLOCK_NEEDED
            elif "passphrase entered was incorrect" in msg:
                code = -14   # RPC_WALLET_PASSPHRASE_INCORRECT
            elif "unencrypted wallet" in msg or "encrypted wallet, but" in msg:
                code = -15   # RPC_WALLET_WRONG_ENC_STATE
            elif "Keypool ran out" in msg:
                code = -12   # RPC_WALLET_KEYPOOL_RAN_OUT
            raise RPCError(code, msg)

    def rpc_getnewaddress(p):
        """getnewaddress ( "account" ) — the next HD key (or a keypool key while locked)."""
        return _wallet_call(wallet().new_address, str(_arg(p, 0, "")))

    def rpc_getbalance(p):
        """getbalance ( "account" minconf include_watchonly ) — spendable (mature) wallet balance; a
        named account gives that account's balance (accounts = labels)."""
        w = wallet()
        minconf = int(_arg(p, 1, 1))
        acct = _arg(p, 0)
        if acct is not None and acct != "*":
            return node.account_balance(str(acct), minconf) / COIN
        total = w.balance(minconf)
        if bool(_arg(p, 2, False)):
            total += w.watch_balance(minconf)
        return total / COIN

    def rpc_getunconfirmedbalance(p):
        """getunconfirmedbalance — wallet outputs in the mempool."""
        w = wallet()
        return (w.balance(0) - w.balance(1)) / COIN

    def rpc_listunspent(p):
        """listunspent ( minconf maxconf ["address",...] )"""
        w = wallet()
        want = set(_arg(p, 2, []) or [])
        out = []
        for u in w.unspent(int(_arg(p, 0, 1)), int(_arg(p, 1, 9_999_999)), include_watch=True):
            addr = _core.script_to_address(u["scriptPubKey"], params.pubkey_prefix, params.script_prefix)
            if want and addr not in want:
                continue
            wo = u["watchonly"]
            solvable = w.watch[u["scriptPubKey"]]["solvable"] if wo else True
            e = {"txid": u["txid"][::-1].hex(), "vout": u["vout"], "address": addr,
                 "scriptPubKey": u["scriptPubKey"].hex(), "amount": u["amount"] / COIN,
                 "confirmations": u["confirmations"], "spendable": u["spendable"], "solvable": solvable,
                 "safe": u["confirmations"] > 0}
            lbl = w.watch[u["scriptPubKey"]]["label"] if wo else (w.labels.get(u["scriptPubKey"][3:23])
                                                                  if len(u["scriptPubKey"]) == 25 else None)
            if lbl is not None:
                e["account"] = lbl
            out.append(e)
        return out

    def rpc_sendtoaddress(p):
        """sendtoaddress "address" amount ( "comment" "comment_to" subtractfeefromamount )"""
        if len(p) < 2:
            raise RPCError(RPC_INVALID_PARAMETER, 'sendtoaddress "address" amount')
        w = wallet()
        txid = _wallet_call(w.send, [(_spk(p[0]), _amount(p[1]))], subtract_fee=bool(_arg(p, 4, False)),
                            comment=str(_arg(p, 2, "")))
        return txid[::-1].hex()

    def rpc_sendmany(p):
        """sendmany "" {"address":amount,...} ( minconf "comment" ["address",...] )"""
        if len(p) < 2 or not isinstance(p[1], dict) or not p[1]:
            raise RPCError(RPC_INVALID_PARAMETER, 'sendmany "" {"address":amount,...}')
        outs = [(_spk(a), _amount(v)) for a, v in p[1].items()]
        subtract = set(_arg(p, 4, []) or [])
        if subtract and list(p[1])[0] not in subtract:
            # the wallet subtracts the fee from the first output; move a subtract-from output first
            first = next(k for k, a in enumerate(p[1]) if a in subtract)
            outs.insert(0, outs.pop(first))
        acct = str(p[0]) if p[0] not in (None, "") else None
        txid = _wallet_call(wallet().send, outs, subtract_fee=bool(subtract), comment=str(_arg(p, 3, "")),
                            from_account=acct, minconf=int(_arg(p, 2, 1)))
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
        if bool(_arg(p, 2, True)):  # the balance is always current; the history needs the rescan
            rescan(node)
        return None

    def rpc_getwalletinfo(p):
        """getwalletinfo"""
        w = wallet()
        out = {"walletname": "wallet.json", "walletversion": 139900 if w.hd is not None else 60000,
               "balance": w.balance(1) / COIN, "unconfirmed_balance": (w.balance(0) - w.balance(1)) / COIN,
               "immature_balance": w.immature_balance() / COIN,
               "txcount": len(w.history.txs) if w.history is not None else len(w.unspent(0)),
               "keypoololdest": min(w.created.values(), default=0), "keypoolsize": len(w.pool),
               "paytxfee": w.pay_tx_fee / COIN}
        if w.encrypted:
            out["unlocked_until"] = w.unlocked_until
        if w.hd is not None:
            out["hdmasterkeyid"] = w.hd["master_id"][::-1].hex()
        return out

    def rpc_encryptwallet(p):
        """encryptwallet "passphrase" """
        if not p:
            raise RPCError(RPC_INVALID_PARAMETER, 'encryptwallet "passphrase"')
        _wallet_call(wallet().encrypt, str(p[0]))
        return "wallet encrypted; the keypool has been flushed and a new HD seed was generated (if you are using HD)."

    def rpc_walletpassphrase(p):
        """walletpassphrase "passphrase" timeout"""
        if len(p) < 2:
            raise RPCError(RPC_INVALID_PARAMETER, 'walletpassphrase "passphrase" timeout')
        _wallet_call(wallet().unlock, str(p[0]), int(p[1]))
        return None

    def rpc_walletlock(p):
        """walletlock"""
        w = wallet()
        if not w.encrypted:
            raise RPCError(-15, "Error: running with an unencrypted wallet, but walletlock was called.")
        w.lock_wallet()
        return None

    def rpc_walletpassphrasechange(p):
        """walletpassphrasechange "oldpassphrase" "newpassphrase" """
        if len(p) < 2:
            raise RPCError(RPC_INVALID_PARAMETER, 'walletpassphrasechange "oldpassphrase" "newpassphrase"')
        _wallet_call(wallet().change_passphrase, str(p[0]), str(p[1]))
        return None

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
        if w.locked and not keys:
            raise RPCError(-13, "Error: Please enter the wallet passphrase with walletpassphrase first.")
        tx, complete, errors = _wallet_call(w.sign, tx, prevouts, keys, ht, redeem)
        out = {"hex": tx.serialize(True).hex(), "complete": complete}
        if errors:
            out["errors"] = errors
        return out

    # ------------------------------------------------------------------ history and coin control
    def hist():
        return wallet().history

    def rpc_listtransactions(p):
        """listtransactions ( "account" count skip include_watchonly ) — the most recent entries."""
        count, skip = int(_arg(p, 1, 10)), int(_arg(p, 2, 0))
        if count < 0 or skip < 0:
            raise RPCError(RPC_INVALID_PARAMETER, "Negative count" if count < 0 else "Negative from")
        watch = bool(_arg(p, 3, False))
        acct = str(_arg(p, 0, "*"))
        entries = [e for w in hist().ordered() for e in hist().entries(w, watch)]
        if acct != "*":
            entries = [e for e in entries if e.get("account", "") == acct]
        for a, amount, t, other, comment in hist().moves:  # accounting entries ("move")
            if acct in ("*", a):
                entries.append({"account": a, "category": "move", "time": t, "amount": amount / COIN,
                                "otheraccount": other, "comment": comment})
        entries = entries[::-1][skip:skip + count][::-1]
        return entries

    def rpc_gettransaction(p):
        """gettransaction "txid" ( include_watchonly )"""
        if not p:
            raise RPCError(RPC_INVALID_PARAMETER, 'gettransaction "txid"')
        try:
            txid = bytes.fromhex(p[0])[::-1]
        except ValueError:
            raise RPCError(RPC_INVALID_PARAMETER, "txid must be hexadecimal string")
        w = hist().txs.get(txid)
        if w is None:
            raise RPCError(RPC_INVALID_ADDRESS_OR_KEY, "Invalid or non-wallet transaction id")
        credit, debit, fee = hist().credit(w), hist().debit(w), hist().fee(w)
        net = credit - debit
        out = {"amount": (net + (fee or 0) if debit else net) / COIN}
        if debit and fee is not None:
            out["fee"] = -fee / COIN
        ents = hist().entries(w)
        base = {k: v for k, v in (ents[0] if ents else {}).items()
                if k in ("confirmations", "blockhash", "blockindex", "blocktime", "txid", "time", "timereceived",
                         "bip125-replaceable", "walletconflicts", "comment", "to", "replaced_by_txid",
                         "replaces_txid")}
        if not ents:
            base = {"confirmations": hist().confirmations(w), "txid": p[0], "time": w.time, "timereceived": w.time}
        out.update(base)
        out["details"] = [{k: v for k, v in e.items() if k in ("account", "address", "category", "amount", "vout",
                                                                 "fee", "abandoned")} for e in ents]
        out["hex"] = w.tx.serialize(getattr(node, "rpc_witness", True)).hex()
        return out

    def rpc_listsinceblock(p):
        """listsinceblock ( "blockhash" target_confirmations include_watchonly include_removed )"""
        since = None
        if _arg(p, 0):
            try:
                since = st.chain.find(bytes.fromhex(p[0])[::-1])
            except ValueError:
                since = None
            if since is None:
                raise RPCError(RPC_INVALID_ADDRESS_OR_KEY, "Block not found")
        target = int(_arg(p, 1, 1))
        if target < 1:
            raise RPCError(RPC_INVALID_PARAMETER, "Invalid parameter")
        depth = st.height() + 1 - (since.height if since is not None and st.chain.in_active_chain(since) else -1)
        txs = []
        for w in hist().ordered():
            conf = hist().confirmations(w)
            if conf < depth:
                txs.extend(hist().entries(w))
        last = st.chain.at_height(max(0, st.height() + 1 - target))
        return {"transactions": txs, "removed": [], "lastblock": last.hash[::-1].hex()}

    def rpc_getreceivedbyaddress(p):
        """getreceivedbyaddress "address" ( minconf )"""
        if not p:
            raise RPCError(RPC_INVALID_PARAMETER, 'getreceivedbyaddress "address"')
        spk = _spk(p[0])
        if not wallet().is_mine(spk):
            return 0.0
        r = hist().received_by(int(_arg(p, 1, 1))).get(spk)
        return (r[0] if r else 0) / COIN

    def rpc_listreceivedbyaddress(p):
        """listreceivedbyaddress ( minconf include_empty include_watchonly )"""
        minconf, include_empty = int(_arg(p, 0, 1)), bool(_arg(p, 1, False))
        rec = hist().received_by(minconf)
        w = wallet()
        out = []
        for h in list(w.keys):
            spk = b"\x76\xa9\x14" + h + b"\x88\xac"
            r = rec.get(spk)
            if r is None and not include_empty:
                continue
            out.append({"address": w.address_of(h), "account": w.labels.get(h, ""), "amount": (r[0] if r else 0) / COIN,
                        "confirmations": r[1] if r else 0, "label": w.labels.get(h, ""), "txids": r[2] if r else []})
        return out

    def rpc_lockunspent(p):
        """lockunspent unlock ( [{"txid","vout"},...] )"""
        if not p:
            raise RPCError(RPC_INVALID_PARAMETER, "lockunspent unlock ( [{\"txid\",\"vout\"},...] )")
        unlock = bool(p[0])
        items = _arg(p, 1)
        if items is None:
            if unlock:
                hist().locked.clear()
            return True
        for d in items:
            try:
                key = (bytes.fromhex(d["txid"])[::-1], int(d["vout"]))
            except (KeyError, ValueError, TypeError):
                raise RPCError(RPC_INVALID_PARAMETER, "Invalid parameter, expected object with {\"txid\",\"vout\"}")
            if unlock:
                hist().locked.discard(key)
            else:
                hist().locked.add(key)
        return True

    def rpc_listlockunspent(p):
        """listlockunspent"""
        return [{"txid": h[::-1].hex(), "vout": n} for h, n in sorted(hist().locked)]

    def rpc_settxfee(p):
        """settxfee amount — fee rate in CLORE per kB for wallet sends."""
        if not p:
            raise RPCError(RPC_INVALID_PARAMETER, "settxfee amount")
        wallet().pay_tx_fee = round(float(p[0]) * COIN)  # payTxFee = CFeeRate(nAmount, 1000); 0 = estimate
        return True

    def rpc_getrawchangeaddress(p):
        """getrawchangeaddress"""
        return wallet().new_address("change")

    def rpc_fundrawtransaction(p):
        """fundrawtransaction "hexstring" ( options ) — add wallet inputs (and a change output) to
        cover the outputs and the fee; existing inputs stay. Returns {hex, fee, changepos}."""
        if not p:
            raise RPCError(RPC_INVALID_PARAMETER, 'fundrawtransaction "hexstring"')
        tx = None
        for witness in (False, True):  # DecodeHexTx(fTryNoWitness = true): output-only txs parse
            try:
                tx = _core.Transaction.deserialize(bytes.fromhex(p[0]), witness)
                break
            except Exception:  # noqa: BLE001
                continue
        if tx is None:
            raise RPCError(RPC_DESERIALIZATION_ERROR, "TX decode failed")
        opts = _arg(p, 1, {}) or {}
        w = wallet()
        fee_rate = round(float(opts["feeRate"]) * COIN) if "feeRate" in opts else w.fee_rate
        existing = []
        for i in tx.vin:
            c = st._spent_coin(i.prevout)
            if c is None:
                raise RPCError(RPC_INVALID_ADDRESS_OR_KEY, "Insufficient funds")
            existing.append({"txid": i.prevout.hash, "vout": i.prevout.n, "amount": c[0], "scriptPubKey": c[1]})
        need_out = list(tx.vout)
        change_spk = _spk(opts["changeAddress"]) if opts.get("changeAddress") else None
        try:  # the inputs already present count towards the outputs; wallet coins cover the rest + fee
            funded, fee = w.fund_and_sign(need_out, [], existing, fee_rate, change_spk, require_complete=False)
        except WalletError as e:
            raise RPCError(RPC_WALLET_INSUFFICIENT_FUNDS, str(e))
        # return it unsigned, as the reference does (signrawtransaction signs)
        vins = list(funded.vin)
        for v in vins:
            v.script_sig = b""
            v.witness = []
        funded.vin = vins
        changepos = -1
        for k, o in enumerate(funded.vout):
            if k >= len(need_out):
                changepos = k
        return {"hex": funded.serialize(True).hex(), "fee": fee / COIN, "changepos": changepos}

    def rpc_abandontransaction(p):
        """abandontransaction "txid" — forget an unconfirmed wallet transaction that is not in the pool."""
        if not p:
            raise RPCError(RPC_INVALID_PARAMETER, 'abandontransaction "txid"')
        txid = bytes.fromhex(p[0])[::-1]
        w = hist().txs.get(txid)
        if w is None:
            raise RPCError(RPC_INVALID_ADDRESS_OR_KEY, "Invalid or non-wallet transaction id")
        if hist().confirmations(w) > 0 or txid in st.mempool:
            raise RPCError(RPC_INVALID_ADDRESS_OR_KEY, "Transaction not eligible for abandonment")
        w.abandoned = True
        hist().save()
        return None

    def rpc_backupwallet(p):
        """backupwallet "destination" — a destination ending in ".dat" gets the reference's own
        format (a Berkeley DB wallet.dat that clore_blockchaind opens: wallet/walletdb.
        write_wallet_dat; an encrypted wallet whose BIP39 data is not held in that form must be
        unlocked), any other name a copy of this node's JSON wallet."""
        if not p:
            raise RPCError(RPC_INVALID_PARAMETER, 'backupwallet "destination"')
        w = wallet()
        with w.lock:
            w._save()
            try:
                if str(p[0]).endswith(".dat"):
                    from ..wallet.walletdb import write_wallet_dat

                    write_wallet_dat(w, p[0])
                else:
                    import shutil

                    shutil.copyfile(w.path, p[0])
            except WalletError as e:
                raise RPCError(-13, str(e))
            except (OSError, RuntimeError) as e:
                raise RPCError(RPC_WALLET_ERROR, f"Error: Wallet backup failed! {e}")
        return None

    def rpc_dumpwallet(p):
        """dumpwallet "filename" — every key as WIF with its label (the reference's dump format)."""
        if not p:
            raise RPCError(RPC_INVALID_PARAMETER, 'dumpwallet "filename"')
        w = wallet()
        if w.locked:
            raise RPCError(-13, "Error: Please enter the wallet passphrase with walletpassphrase first.")
        tip = st.tip()
        lines = ["# Wallet dump created by nodexa", f"# * Best block at time of backup was {tip.height} "
                 f"({tip.hash[::-1].hex()}),", ""]
        if w.hd is not None and w.hd.get("bip44"):  # the BIP39 words (src/wallet/rpcdump.cpp:710)
            words, pp = w.mnemonic()
            lines[2:2] = [f"# mnemonic: {words}", f"# mnemonic passphrase: {pp}"]
        for h, (sec, _) in w.keys.items():
            t = time.strftime("%Y-%m-%dT%H:%M:%SZ", time.gmtime(w.created.get(h, 0)))
            lbl = w.labels.get(h, "")
            tag = "change=1" if lbl == "change" else f"label={lbl}"
            lines.append(f"{w.encode_wif(sec)} {t} {tag} # addr={w.address_of(h)}")
        lines.append("\n# End of dump")
        try:
            with open(p[0], "w") as f:
                f.write("\n".join(lines) + "\n")
        except OSError as e:
            raise RPCError(RPC_WALLET_ERROR, f"Cannot open wallet dump file: {e}")
        return {"filename": os.path.abspath(p[0])}

    def rpc_getmywords(p):
        """getmywords — the BIP39 words (and passphrase, if one was used) this wallet derives from."""
        w = wallet()
        if w.locked:
            raise RPCError(-13, "Error: Please enter the wallet passphrase with walletpassphrase first.")
        try:
            words, pp = w.mnemonic()
        except WalletError as e:
            raise RPCError(RPC_WALLET_ERROR, str(e))
        out = {"word_list": words}
        if pp:
            out["passphrase"] = pp
        return out

    def rpc_importwallet(p):
        """importwallet "filename" — import the keys of a dumpwallet file, then rescan."""
        if not p:
            raise RPCError(RPC_INVALID_PARAMETER, 'importwallet "filename"')
        w = wallet()
        try:
            lines = open(p[0]).read().splitlines()
        except OSError:
            raise RPCError(RPC_INVALID_PARAMETER, "Cannot open wallet dump file")
        for line in lines:
            if not line.strip() or line.startswith("#"):
                continue
            fields = line.split()
            try:
                secret = w.decode_wif(fields[0])
            except WalletError:
                continue
            lbl = next((f[6:] for f in fields[2:] if f.startswith("label=")), "")
            w._add_secret(secret, "change" if "change=1" in fields else lbl)
        rescan(node)
        return None

    def rpc_keypoolrefill(p):
        """keypoolrefill ( newsize ) — derive keys into the pool (needs an unlocked wallet)."""
        _wallet_call(wallet().keypool_refill, int(_arg(p, 0, 100)))
        return None

    def rpc_listaddressgroupings(p):
        """listaddressgroupings — one group per address with its confirmed balance."""
        w = wallet()
        bal: dict[bytes, int] = {}
        for u in w.unspent(1):
            bal[u["scriptPubKey"]] = bal.get(u["scriptPubKey"], 0) + u["amount"]
        groups = []
        for spk, amount in bal.items():
            a = _core.script_to_address(spk, params.pubkey_prefix, params.script_prefix)
            if a:
                h = _core.base58check_decode(a)[1:]
                groups.append([[a, amount / COIN, w.labels.get(h, "")]])
        return groups

    def _h(address: str) -> bytes:
        raw = _core.base58check_decode(str(address))
        if raw is None or len(raw) != 21 or raw[0] != params.pubkey_prefix:
            raise RPCError(RPC_INVALID_ADDRESS_OR_KEY, "Invalid Clore address")
        return raw[1:]

    def rpc_getaccount(p):
        """getaccount "address" (deprecated accounts = labels)"""
        return wallet().labels.get(_h(p[0]), "") if p else ""

    def rpc_setaccount(p):
        """setaccount "address" "account" """
        if len(p) < 2:
            raise RPCError(RPC_INVALID_PARAMETER, 'setaccount "address" "account"')
        w = wallet()
        h = _h(p[0])
        if h not in w.keys:
            raise RPCError(RPC_MISC_ERROR, "setaccount can only be used with own address")
        with w.lock:
            w.labels[h] = str(p[1])
            w._save()
        return None

    def rpc_getaddressesbyaccount(p):
        """getaddressesbyaccount "account" """
        acct = str(_arg(p, 0, ""))
        w = wallet()
        return [w.address_of(h) for h in w.keys if w.labels.get(h, "") == acct]

    def rpc_getaccountaddress(p):
        """getaccountaddress "account" — an address of the account (a new one if it has none)."""
        acct = str(_arg(p, 0, ""))
        have = rpc_getaddressesbyaccount([acct])
        return have[0] if have else wallet().new_address(acct)

    def rpc_listaccounts(p):
        """listaccounts ( minconf ) — confirmed balance per label."""
        w = wallet()
        out: dict[str, float] = {w.labels.get(h, ""): 0.0 for h in w.keys if w.labels.get(h, "") != "change"}
        out.setdefault("", 0.0)
        for u in w.unspent(int(_arg(p, 0, 1))):
            if not u["spendable"]:
                continue
            a = _core.script_to_address(u["scriptPubKey"], params.pubkey_prefix, params.script_prefix)
            h = _core.base58check_decode(a)[1:] if a else None
            lbl = w.labels.get(h, "") if h else ""
            out[lbl if lbl != "change" else ""] = out.get(lbl if lbl != "change" else "", 0.0) + u["amount"] / COIN
        return out

    def rpc_rescanblockchain(p):
        """rescanblockchain ( start_height ) — rebuild the wallet history from the chain."""
        start = int(_arg(p, 0, 0))
        rescan(node, start)
        return {"start_height": start, "stop_height": st.height()}

    for cat, name, fn, args in [
        ("wallet", "listtransactions", rpc_listtransactions, ("account", "count", "skip", "include_watchonly")),
        ("wallet", "gettransaction", rpc_gettransaction, ("txid", "include_watchonly")),
        ("wallet", "listsinceblock", rpc_listsinceblock, ("blockhash", "target_confirmations", "include_watchonly",
                                                          "include_removed")),
        ("wallet", "getreceivedbyaddress", rpc_getreceivedbyaddress, ("address", "minconf")),
        ("wallet", "listreceivedbyaddress", rpc_listreceivedbyaddress, ("minconf", "include_empty",
                                                                        "include_watchonly")),
        ("wallet", "lockunspent", rpc_lockunspent, ("unlock", "transactions")),
        ("wallet", "listlockunspent", rpc_listlockunspent, ()),
        ("wallet", "settxfee", rpc_settxfee, ("amount",)),
        ("wallet", "getrawchangeaddress", rpc_getrawchangeaddress, ()),
        ("rawtransactions", "fundrawtransaction", rpc_fundrawtransaction, ("hexstring", "options")),
        ("wallet", "abandontransaction", rpc_abandontransaction, ("txid",)),
        ("wallet", "backupwallet", rpc_backupwallet, ("destination",)),
        ("wallet", "dumpwallet", rpc_dumpwallet, ("filename",)),
        ("wallet", "getmywords", rpc_getmywords, ()),
        ("wallet", "importwallet", rpc_importwallet, ("filename",)),
        ("wallet", "keypoolrefill", rpc_keypoolrefill, ("newsize",)),
        ("wallet", "listaddressgroupings", rpc_listaddressgroupings, ()),
        ("wallet", "getaccount", rpc_getaccount, ("address",)),
        ("wallet", "setaccount", rpc_setaccount, ("address", "account")),
        ("wallet", "getaddressesbyaccount", rpc_getaddressesbyaccount, ("account",)),
        ("wallet", "getaccountaddress", rpc_getaccountaddress, ("account",)),
        ("wallet", "listaccounts", rpc_listaccounts, ("minconf", "include_watchonly")),
        ("wallet", "rescanblockchain", rpc_rescanblockchain, ("start_height",)),
        ("wallet", "encryptwallet", rpc_encryptwallet, ("passphrase",)),
        ("wallet", "walletpassphrase", rpc_walletpassphrase, ("passphrase", "timeout")),
        ("wallet", "walletlock", rpc_walletlock, ()),
        ("wallet", "walletpassphrasechange", rpc_walletpassphrasechange, ("oldpassphrase", "newpassphrase")),
    ]:
        table.append(cat, name, fn, args)

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
