"""Wallet side of the asset layer: issuing, reissuing and transferring assets,
unique tokens, qualifiers and restricted assets, tagging / freezing addresses.

Parity (behaviour): CreateAssetTransaction / CreateReissueAssetTransaction /
CreateTransferAssetTransaction and the restricted-asset wallet paths (src/assets/assets.cpp:3855-4400,
src/rpc/assets.cpp). Every transaction is built with the consensus layout the node checks
(csrc/chain/assets.cpp check_tx_structure): burn output, CLORE change, owner / qualifier token
change, null-asset data, and the issue / reissue data output last. Consensus validity is then
decided by the node's own AcceptToMemoryPool, exactly as for a peer's transaction.
"""
from __future__ import annotations

from .. import core
from .wallet import WalletError

_core = core()
COIN = 100_000_000


def p2pkh_of(h160: bytes) -> bytes:
    return b"\x76\xa9\x14" + h160 + b"\x88\xac"
OWNER_AMOUNT = COIN


class AssetWallet:
    def __init__(self, wallet):
        self.w = wallet
        self.state = wallet.state
        self.params = wallet.params
        self.burn = _core.asset_burn_info(self.params)

    # ------------------------------------------------------------------ helpers
    def _h160(self, address: str) -> bytes:
        spk = _core.address_to_script(address, self.params.pubkey_prefix, self.params.script_prefix)
        if spk is None or len(spk) != 25 or spk[:3] != b"\x76\xa9\x14":
            raise WalletError(f"Invalid address: {address}")
        return spk[3:23]

    def _dest(self, address: str | None) -> bytes:
        return self._h160(address) if address else self._h160(self.w.new_address())

    def _burn_out(self, kind: str, n: int = 1):
        addr, amount = self.burn[kind]
        spk = _core.address_to_script(addr, self.params.pubkey_prefix, self.params.script_prefix)
        return _core.TxOut(amount * n, spk)

    def _flags(self):
        return self.state.asset_flags(self.state.coins_tip())

    def _require_active(self, restricted: bool = False) -> None:
        f = self._flags()
        if not f.assets:
            raise WalletError("Assets aren't active")
        if restricted and not f.msg_restricted:
            raise WalletError("Restricted assets aren't active")

    def unspent(self, name: str | None = None) -> list[dict]:
        """Asset outputs of wallet keys (confirmed, plus the wallet's unconfirmed pool outputs) not
        spent in the mempool."""
        st = self.state
        with st.lock:
            hashes = list(self.w.keys)
            pool_spent = {(i.prevout.hash, i.prevout.n) for e in st.mempool.values() for i in e.tx.vin}
            out = []
            for txid, n, value, spk, height, _ in st.coins.asset_outputs(hashes):
                if (txid, n) in pool_spent:
                    continue
                a = _core.parse_asset_script(spk)
                if a is None or (name is not None and a["name"] != name):
                    continue
                out.append({"txid": txid, "vout": n, "amount": value, "scriptPubKey": spk, "name": a["name"],
                            "qty": a["amount"], "hash160": a["hash160"], "height": height})
            # unconfirmed change of the wallet's own pool transactions (owner tokens spent and returned)
            mine = set(hashes)
            for txid, e in st.mempool.items():
                for n, o in enumerate(e.tx.vout):
                    a = _core.parse_asset_script(o.script_pubkey)
                    if a is None or a["hash160"] not in mine or (txid, n) in pool_spent:
                        continue
                    if name is not None and a["name"] != name:
                        continue
                    out.append({"txid": txid, "vout": n, "amount": o.value, "scriptPubKey": o.script_pubkey,
                                "name": a["name"], "qty": a["amount"], "hash160": a["hash160"], "height": -1})
            return out

    def balances(self) -> dict[str, int]:
        out: dict[str, int] = {}
        for u in self.unspent():
            out[u["name"]] = out.get(u["name"], 0) + u["qty"]
        return out

    def _take(self, name: str, qty: int, from_h160s: set | None = None) -> tuple[list[dict], int]:
        """Asset coins of `name` (held at `from_h160s` when given) covering `qty`, largest first, and
        the change."""
        coins = sorted((u for u in self.unspent(name) if from_h160s is None or u["hash160"] in from_h160s),
                       key=lambda u: -u["qty"])
        chosen, total = [], 0
        for u in coins:
            if total >= qty:
                break
            chosen.append(u)
            total += u["qty"]
        if total < qty:
            raise WalletError(f"Insufficient asset funds: {name}")
        return chosen, total - qty

    def _owner_inputs(self, token: str) -> tuple[list[dict], list]:
        """Spend the wallet's `token` (owner token or qualifier) and send it back to the wallet."""
        if not self.unspent(token):
            raise WalletError(f"Wallet doesn't have asset: {token}")
        ins, _ = self._take(token, 1)
        qty = sum(u["qty"] for u in ins)
        back = _core.TxOut(0, _core.asset_script_transfer(ins[0]["hash160"], token, qty))
        return ins, [back]

    def _send(self, pre, post, ins=()) -> bytes:
        tx, _ = self.w.fund_and_sign(pre, post, list(ins))
        ok, reason, _ = self.state.accept_to_mempool(tx)
        if not ok:
            raise WalletError(f"Transaction rejected: {reason}")
        return tx.txid()

    # ------------------------------------------------------------------ issue / reissue / transfer
    def issue(self, name: str, qty: int, to: str | None = None, units: int = 0, reissuable: bool = True,
              ipfs: bytes = b"") -> bytes:
        self._require_active()
        kind, err = _core.asset_name_type(name)
        h = self._dest(to)
        if kind == "ROOT" or kind == "SUB":
            ins, keep = ([], [])
            if kind == "SUB":
                ins, keep = self._owner_inputs(_core.asset_parent_name(name) + "!")
            pre = [self._burn_out("root" if kind == "ROOT" else "sub")] + keep
            post = [_core.TxOut(0, _core.asset_script_owner(h, name + "!")),
                    _core.TxOut(0, _core.asset_script_new(h, name, qty, units, 1 if reissuable else 0, ipfs))]
            return self._send(pre, post, ins)
        if kind == "QUALIFIER" or kind == "SUB_QUALIFIER":
            self._require_active(True)
            ins, keep = ([], [])
            if kind == "SUB_QUALIFIER":
                ins, keep = self._owner_inputs(_core.asset_parent_name(name))
            pre = [self._burn_out("qualifier" if kind == "QUALIFIER" else "subqualifier")] + keep
            post = [_core.TxOut(0, _core.asset_script_new(h, name, qty, 0, 0, ipfs))]
            return self._send(pre, post, ins)
        if kind == "MSGCHANNEL":
            self._require_active(True)
            ins, keep = self._owner_inputs(_core.asset_parent_name(name) + "!")
            pre = [self._burn_out("msgchannel")] + keep
            post = [_core.TxOut(0, _core.asset_script_new(h, name, COIN, 0, 0, ipfs))]
            return self._send(pre, post, ins)
        raise WalletError(f"Invalid asset name: {name} {err}".strip())

    def issue_unique(self, root: str, tags: list[str], ipfs: list[bytes] | None = None, to: str | None = None) -> bytes:
        self._require_active()
        h = self._dest(to)
        ins, keep = self._owner_inputs(root + "!")
        post = []
        for i, tag in enumerate(tags):
            name = f"{root}#{tag}"
            if _core.asset_name_type(name)[0] != "UNIQUE":
                raise WalletError(f"Invalid unique asset name: {name}")
            data = ipfs[i] if ipfs and i < len(ipfs) else b""
            post.append(_core.TxOut(0, _core.asset_script_new(h, name, COIN, 0, 0, data)))
        pre = [self._burn_out("unique", len(tags))] + keep
        return self._send(pre, post, ins)

    def issue_restricted(self, name: str, qty: int, verifier: str, to: str | None = None, units: int = 0,
                         reissuable: bool = True, ipfs: bytes = b"") -> bytes:
        self._require_active(True)
        if _core.asset_name_type(name)[0] != "RESTRICTED":
            raise WalletError(f"Invalid restricted asset name: {name}")
        h = self._dest(to)
        ins, keep = self._owner_inputs(name[1:] + "!")
        stripped = _core.strip_verifier_string(verifier)
        pre = [self._burn_out("restricted")] + keep + [_core.TxOut(0, _core.asset_script_null_verifier(stripped))]
        post = [_core.TxOut(0, _core.asset_script_new(h, name, qty, units, 1 if reissuable else 0, ipfs))]
        return self._send(pre, post, ins)

    def reissue(self, name: str, qty: int, to: str | None = None, reissuable: bool = True, new_units: int = -1,
                new_ipfs: bytes = b"", new_verifier: str | None = None) -> bytes:
        self._require_active()
        h = self._dest(to)
        root = name[1:] if name.startswith("$") else name
        ins, keep = self._owner_inputs(root + "!")
        pre = [self._burn_out("reissue")] + keep
        if new_verifier is not None:
            pre.append(_core.TxOut(0, _core.asset_script_null_verifier(_core.strip_verifier_string(new_verifier))))
        post = [_core.TxOut(0, _core.asset_script_reissue(h, name, qty, new_units, 1 if reissuable else 0, new_ipfs))]
        return self._send(pre, post, ins)

    def transfer(self, name: str, qty: int, to: str, message: bytes = b"", expire: int = 0,
                 change_to: str | None = None, from_addresses: list[str] | None = None,
                 clore_change_to: str | None = None) -> bytes:
        """CreateTransferAssetTransaction; `from_addresses` restricts the asset coins
        (transferfromaddress / transferfromaddresses), the change addresses are optional."""
        self._require_active()
        srcs = None if from_addresses is None else {self._h160(a) for a in from_addresses}
        ins, change = self._take(name, qty, srcs)
        outs = [_core.TxOut(0, _core.asset_script_transfer(self._h160(to), name, qty, message, expire))]
        if change:
            outs.append(_core.TxOut(0, _core.asset_script_transfer(self._dest(change_to), name, change)))
        change_spk = p2pkh_of(self._h160(clore_change_to)) if clore_change_to else None
        tx, _ = self.w.fund_and_sign(outs, [], list(ins), change_spk=change_spk)
        ok, reason, _ = self.state.accept_to_mempool(tx)
        if not ok:
            raise WalletError(f"Transaction rejected: {reason}")
        if self.w.history is not None:
            self.w.history.add(tx)
        return tx.txid()

    def build_transfer_many(self, name: str, dests: list[tuple[bytes, int]]):
        """CreateTransferAssetTransaction with one transfer output per (hash160, qty): the signed
        transaction, not yet submitted (reward distribution batches)."""
        self._require_active()
        ins, change = self._take(name, sum(q for _, q in dests))
        outs = [_core.TxOut(0, _core.asset_script_transfer(h, name, q)) for h, q in dests]
        if change:
            outs.append(_core.TxOut(0, _core.asset_script_transfer(self._dest(None), name, change)))
        tx, _ = self.w.fund_and_sign(outs, [], list(ins))
        return tx

    def send_message(self, channel: str, payload: bytes, expire: int = 0) -> bytes:
        """sendmessage (src/rpc/messages.cpp:310): the channel token goes back to the address it is
        held at, carrying the message (a message only counts when sent to the spending address)."""
        self._require_active(True)
        coins = self.unspent(channel)
        if not coins:
            raise WalletError(f"Wallet doesn't own the asset_name: {channel}")
        coin = coins[0]
        out = _core.TxOut(0, _core.asset_script_transfer(coin["hash160"], channel, coin["qty"], payload, expire))
        return self._send([out], [], [coin])

    # ------------------------------------------------------------------ tags and restrictions
    def tag_address(self, qualifier: str, address: str, add: bool) -> bytes:
        self._require_active(True)
        ins, keep = self._owner_inputs(qualifier)
        pre = keep + [_core.TxOut(0, _core.asset_script_null_tag(self._h160(address), qualifier, 1 if add else 0))]
        if add:
            pre = [self._burn_out("tag")] + pre
        return self._send(pre, [], ins)

    def freeze_address(self, restricted: str, address: str, freeze: bool) -> bytes:
        self._require_active(True)
        ins, keep = self._owner_inputs(restricted[1:] + "!")
        pre = keep + [_core.TxOut(0, _core.asset_script_null_tag(self._h160(address), restricted, 1 if freeze else 0))]
        return self._send(pre, [], ins)

    def freeze_global(self, restricted: str, freeze: bool) -> bytes:
        self._require_active(True)
        ins, keep = self._owner_inputs(restricted[1:] + "!")
        pre = keep + [_core.TxOut(0, _core.asset_script_null_global(restricted, 1 if freeze else 0))]
        return self._send(pre, [], ins)
