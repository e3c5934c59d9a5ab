"""Utility RPCs (src/rpc/misc.cpp:1475-1477, src/rpc/rawtransaction.cpp combinerawtransaction,
src/wallet/rpcwallet.cpp signmessage / addmultisigaddress): createmultisig, verifymessage,
signmessagewithprivkey, signmessage, addmultisigaddress, combinerawtransaction.

Signed messages hash ser_string("Clore Signed Message:\\n") || ser_string(message) with SHA256d
(strMessageMagic, src/validation.cpp:137) and carry a base64 compact recoverable signature."""
from __future__ import annotations

import base64
import hashlib

from .. import core
from ..wallet.wallet import _pushes, multisig_script, parse_multisig
from .protocol import (RPC_DESERIALIZATION_ERROR, RPC_INVALID_ADDRESS_OR_KEY, RPC_INVALID_PARAMETER,
                       RPC_METHOD_NOT_FOUND, RPC_TYPE_ERROR, RPCError)

_core = core()
MESSAGE_MAGIC = b"Clore Signed Message:\n"


def _ser_string(b: bytes) -> bytes:
    n = len(b)
    if n < 253:
        return bytes([n]) + b
    return b"\xfd" + n.to_bytes(2, "little") + b if n <= 0xFFFF else b"\xfe" + n.to_bytes(4, "little") + b


def message_hash(message: str) -> bytes:
    data = _ser_string(MESSAGE_MAGIC) + _ser_string(message.encode())
    return hashlib.sha256(hashlib.sha256(data).digest()).digest()


def register(table, node) -> None:
    st = node.state
    params = node.params

    def _need(p, n, usage):
        if len(p) < n:
            raise RPCError(RPC_INVALID_PARAMETER, usage)

    def _multisig(nrequired, keys) -> bytes:
        if not isinstance(keys, list):
            raise RPCError(RPC_TYPE_ERROR, "keys must be an array")
        m = int(nrequired)
        if m < 1:
            raise RPCError(RPC_INVALID_PARAMETER, "a multisignature address must require at least one key to redeem")
        if len(keys) < m:
            raise RPCError(RPC_INVALID_PARAMETER,
                           f"not enough keys supplied (got {len(keys)} keys, but need at least {m} to redeem)")
        if len(keys) > 16:
            raise RPCError(RPC_INVALID_PARAMETER,
                           "Number of addresses involved in the multisignature address creation > 16\nReduce the number")
        pubs = []
        for k in keys:
            k = str(k)
            pub = None
            try:
                raw = bytes.fromhex(k)
                pub = _core.secp_pubkey_normalize(raw, len(raw) == 33)
            except ValueError:
                w = getattr(node, "wallet", None)
                raw = _core.base58check_decode(k)
                if w is not None and raw is not None and len(raw) == 21 and raw[1:] in w.keys:
                    pub = w.keys[raw[1:]][1]
                elif raw is not None:
                    raise RPCError(RPC_INVALID_ADDRESS_OR_KEY, f"no full public key for address {k}")
            if pub is None:
                raise RPCError(RPC_INVALID_ADDRESS_OR_KEY, f" Invalid public key: {k}")
            pubs.append(pub)
        script = multisig_script(m, pubs)
        if len(script) > 520:
            raise RPCError(RPC_INVALID_PARAMETER, "redeemScript exceeds size limit: 520 > 520")
        return script

    def _p2sh_address(script: bytes) -> str:
        return _core.base58check_encode(bytes([params.script_prefix]) + _core.hash160(script))

    def rpc_createmultisig(p):
        """createmultisig nrequired ["key",...] -> {"address", "redeemScript"}"""
        _need(p, 2, "createmultisig nrequired [\"key\",...]")
        script = _multisig(p[0], p[1])
        return {"address": _p2sh_address(script), "redeemScript": script.hex()}

    def rpc_addmultisigaddress(p):
        """addmultisigaddress nrequired ["key",...] ( "account" ) — also remembered by the wallet."""
        _need(p, 2, "addmultisigaddress nrequired [\"key\",...]")
        if getattr(node, "wallet", None) is None:
            raise RPCError(RPC_METHOD_NOT_FOUND, "Method not found (wallet disabled)")
        return node.wallet.add_redeem_script(_multisig(p[0], p[1]))

    def rpc_verifymessage(p):
        """verifymessage "address" "signature" "message" """
        _need(p, 3, 'verifymessage "address" "signature" "message"')
        raw = _core.base58check_decode(str(p[0]))
        if raw is None or len(raw) != 21 or raw[0] not in (params.pubkey_prefix, params.script_prefix):
            raise RPCError(RPC_TYPE_ERROR, "Invalid address")
        if raw[0] != params.pubkey_prefix:
            raise RPCError(RPC_TYPE_ERROR, "Address does not refer to key")
        try:
            sig = base64.b64decode(str(p[1]), validate=True)
        except ValueError:
            raise RPCError(RPC_INVALID_ADDRESS_OR_KEY, "Malformed base64 encoding")
        pub = _core.secp_recover_compact(message_hash(str(p[2])), sig)
        return pub is not None and _core.hash160(pub) == raw[1:]

    def _sign_message(secret: bytes, compressed: bool, message: str) -> str:
        sig = _core.secp_sign_compact(message_hash(message), secret, compressed)
        if sig is None:
            raise RPCError(RPC_INVALID_ADDRESS_OR_KEY, "Sign failed")
        return base64.b64encode(sig).decode()

    def rpc_signmessagewithprivkey(p):
        """signmessagewithprivkey "privkey" "message" """
        _need(p, 2, 'signmessagewithprivkey "privkey" "message"')
        raw = _core.base58check_decode(str(p[0]))
        if raw is None or len(raw) not in (33, 34) or not _core.secp_seckey_valid(raw[1:33]):
            raise RPCError(RPC_INVALID_ADDRESS_OR_KEY, "Invalid private key")
        return _sign_message(raw[1:33], len(raw) == 34, str(p[1]))

    def rpc_signmessage(p):
        """signmessage "address" "message" (wallet key)"""
        _need(p, 2, 'signmessage "address" "message"')
        w = getattr(node, "wallet", None)
        if w is None:
            raise RPCError(RPC_METHOD_NOT_FOUND, "Method not found (wallet disabled)")
        raw = _core.base58check_decode(str(p[0]))
        if raw is None or len(raw) != 21 or raw[0] != params.pubkey_prefix:
            raise RPCError(RPC_TYPE_ERROR, "Invalid address")
        k = w.keys.get(raw[1:])
        if k is None:
            raise RPCError(RPC_INVALID_ADDRESS_OR_KEY, "Private key not available")
        return _sign_message(k[0], True, str(p[1]))

    def rpc_combinerawtransaction(p):
        """combinerawtransaction ["hexstring",...] — merge the signatures of partially signed copies."""
        _need(p, 1, 'combinerawtransaction ["hexstring",...]')
        if not isinstance(p[0], list) or not p[0]:
            raise RPCError(RPC_DESERIALIZATION_ERROR, "Missing transactions")
        try:
            txs = [_core.Transaction.deserialize(bytes.fromhex(h)) for h in p[0]]
        except Exception:  # noqa: BLE001
            raise RPCError(RPC_DESERIALIZATION_ERROR, "TX decode failed")
        merged = txs[0]
        vins = list(merged.vin)
        for i, vin in enumerate(vins):
            coin = st._spent_coin(vin.prevout)
            if coin is None:
                raise RPCError(RPC_INVALID_PARAMETER, "Input not found or already spent")
            value, spk = coin[0], coin[1]
            versions = [list(t.vin)[i] for t in txs if len(t.vin) > i]
            raw = merged.serialize(True)
            best = None
            for v in versions:  # a copy whose input already verifies wins
                ok, _ = _core.verify_script(v.script_sig, spk, list(v.witness), _core.STANDARD_SCRIPT_VERIFY_FLAGS,
                                            raw, i, value)
                if ok:
                    best = v
                    break
            if best is None:  # P2SH multisig: combine the partial signatures in key order
                redeem = next((_pushes(v.script_sig)[-1] for v in versions if _pushes(v.script_sig)), b"")
                ms = parse_multisig(redeem) if redeem else None
                if ms is not None:
                    m, pubs = ms
                    msg = _core.signature_hash(redeem, raw, i, 1, value, 0)
                    have = {}
                    for v in versions:
                        for push in _pushes(v.script_sig)[1:-1]:
                            for pub in pubs:
                                if pub not in have and push and _core.secp_verify(pub, push[:-1], msg):
                                    have[pub] = push
                    sigs = [have[pub] for pub in pubs if pub in have][:m]
                    best = vin
                    best.script_sig = b"\x00" + b"".join(_core.script_push_data(x) for x in sigs) + \
                        _core.script_push_data(redeem)
                else:
                    best = max(versions, key=lambda v: len(v.script_sig) + sum(len(x) for x in v.witness))
            vins[i] = best
        merged.vin = vins
        return merged.serialize(True).hex()

    for cat, name, fn, args in [
        ("util", "createmultisig", rpc_createmultisig, ("nrequired", "keys")),
        ("util", "verifymessage", rpc_verifymessage, ("address", "signature", "message")),
        ("util", "signmessagewithprivkey", rpc_signmessagewithprivkey, ("privkey", "message")),
        ("wallet", "signmessage", rpc_signmessage, ("address", "message")),
        ("wallet", "addmultisigaddress", rpc_addmultisigaddress, ("nrequired", "keys", "account")),
        ("rawtransactions", "combinerawtransaction", rpc_combinerawtransaction, ("txs",)),
    ]:
        table.append(cat, name, fn, args)
