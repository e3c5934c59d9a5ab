"""Relay policy: IsStandard / IsStandardTx output rules and BIP125 replacement helpers.

Parity (behaviour): src/policy/policy.cpp:19-160 — output templates (Solver classes, with the
asset templates: a P2PKH followed by OP_CLORE_ASSET payload, and the OP_CLORE_ASSET null-asset
data scripts), x-of-3 bare multisig, one OP_RETURN of at most 83 bytes, at most 100 null-asset
data outputs, dust = an output worth less than the fee to spend it at DUST_RELAY_TX_FEE
(asset outputs are never dust); src/policy/rbf.cpp SignalsOptInRBF.
"""
from __future__ import annotations

from .. import core

_core = core()

DUST_RELAY_TX_FEE = 3000      # sat per kB (src/policy/policy.h:50)
MAX_OP_RETURN_RELAY = 83      # nMaxDatacarrierBytes
MAX_NULL_ASSET_OUTPUTS = 100  # "tomany-op-clore-asset"
MAX_BIP125_RBF_SEQUENCE = 0xfffffffd
MAX_BIP125_REPLACEMENTS = 100  # MAX_BIP125_REPLACEMENT_CANDIDATES


def _push_only(script: bytes) -> bool:
    return _core.script_is_push_only(script)


def output_type(spk: bytes) -> str:
    """Solver() class of a scriptPubKey (src/script/standard.cpp), asset templates included."""
    n = len(spk)
    if n > 25 and spk[25] == 0xC0 and _core.parse_asset_script(spk) is not None:
        return "asset"
    if n >= 1 and spk[0] == 0xC0:
        return "null_asset" if _core.parse_null_asset_script(spk) is not None else "nonstandard"
    if n == 25 and spk[:3] == b"\x76\xa9\x14" and spk[23:] == b"\x88\xac":
        return "pubkeyhash"
    if n == 23 and spk[:2] == b"\xa9\x14" and spk[22] == 0x87:
        return "scripthash"
    if n in (35, 67) and spk[0] == n - 2 and spk[-1] == 0xAC:
        return "pubkey"
    if n == 22 and spk[:2] == b"\x00\x14":
        return "witness_v0_keyhash"
    if n == 34 and spk[:2] == b"\x00\x20":
        return "witness_v0_scripthash"
    if n >= 1 and spk[0] == 0x6A:
        return "nulldata" if _push_only(spk[1:]) else "nonstandard"
    if n >= 3 and spk[-1] == 0xAE and 0x51 <= spk[0] <= 0x60 and 0x51 <= spk[-2] <= 0x60:
        return "multisig"
    return "nonstandard"


def dust_threshold(value_spk: bytes, dust_fee: int = DUST_RELAY_TX_FEE) -> int:
    """GetDustThreshold: the fee, at dust_fee per kB, of the output plus an input spending it."""
    spk = value_spk
    if spk[:1] == b"\x6a" or _core.script_unspendable(spk):
        return 0
    size = 8 + (1 if len(spk) < 253 else 3) + len(spk)  # GetSerializeSize(txout)
    witness = len(spk) in (22, 34) and spk[0] == 0 and spk[1] == len(spk) - 2
    size += 32 + 4 + 1 + (107 // 4 if witness else 107) + 4
    return dust_fee * size // 1000


def is_dust(value: int, spk: bytes, dust_fee: int = DUST_RELAY_TX_FEE) -> bool:
    if output_type(spk) == "asset":
        return False
    return value < dust_threshold(spk, dust_fee)


def standard_outputs_reason(tx, witness_enabled: bool = True, permit_bare_multisig: bool = True,
                            datacarrier: bool = True, datacarrier_size: int = MAX_OP_RETURN_RELAY,
                            dust_fee: int = DUST_RELAY_TX_FEE) -> str:
    """The output half of IsStandardTx: '' when standard, else the reject reason. -datacarrier /
    -datacarriersize (fAcceptDatacarrier, nMaxDatacarrierBytes), -permitbaremultisig and
    -dustrelayfee select the policy knobs."""
    data_out = asset_data_out = 0
    for o in tx.vout:
        t = output_type(o.script_pubkey)
        if t == "nonstandard":
            return "scriptpubkey"
        if t == "multisig":
            m, n = o.script_pubkey[0] - 0x50, o.script_pubkey[-2] - 0x50
            if not (1 <= n <= 3 and 1 <= m <= n):
                return "scriptpubkey"
        if t == "nulldata" and (not datacarrier or len(o.script_pubkey) > datacarrier_size):
            return "scriptpubkey"
        if t == "null_asset" and len(o.script_pubkey) > MAX_OP_RETURN_RELAY:
            return "scriptpubkey"
        if not witness_enabled and t.startswith("witness"):
            return "scriptpubkey"
        if t == "nulldata":
            data_out += 1
        elif t == "null_asset":
            asset_data_out += 1
        elif t == "multisig" and not permit_bare_multisig:
            return "bare-multisig"
        elif is_dust(o.value, o.script_pubkey, dust_fee):
            return "dust"
    if data_out > 1:
        return "multi-op-return"
    if asset_data_out > MAX_NULL_ASSET_OUTPUTS:
        return "tomany-op-clore-asset"
    return ""


def signals_rbf(tx) -> bool:
    """SignalsOptInRBF: any input sequence at or below MAX_BIP125_RBF_SEQUENCE."""
    return any(i.sequence <= MAX_BIP125_RBF_SEQUENCE for i in tx.vin)
