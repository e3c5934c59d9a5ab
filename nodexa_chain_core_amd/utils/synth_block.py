"""Synthetic signed blocks for block-connection tests and benchmarks.

`make_signed_block(n_txs, ...)` returns a CoinsView holding one P2PKH (or P2WPKH) coin per
transaction and a block whose transactions each spend one of them with a real ECDSA signature
(RFC 6979, csrc/crypto/secp256k1.cpp) — the shape of an ordinary payments block. Keys are
derived deterministically from the seed so runs are reproducible.
"""
from __future__ import annotations

import hashlib

from .. import core

_core = core()


def _key(seed: int, i: int) -> bytes:
    while True:
        k = hashlib.sha256(f"nodexa-synth-{seed}-{i}".encode()).digest()
        if _core.secp_seckey_valid(k):
            return k
        i += 1 << 32


def make_signed_block(n_txs: int, seed: int = 0, witness_every: int = 0, height: int = 1000,
                      bad_at: int | None = None):
    """-> (block, view, height). Every `witness_every`-th spend is P2WPKH (0 = none); with
    `bad_at` the signature of that transaction is corrupted (a block ConnectBlock must reject)."""
    view = _core.CoinsView()
    cb = _core.Transaction()
    cb.version = 1
    cin = _core.TxIn()
    cin.script_sig = _core.script_push_int(height) + b"\x00"
    cb.vin = [cin]
    cb.vout = [_core.TxOut(0, b"\x51")]
    txs = [cb]
    for t in range(n_txs):
        sec = _key(seed, t)
        pub = _core.secp_pubkey_create(sec, True)
        h = _core.hash160(pub)
        witness = witness_every > 0 and t % witness_every == witness_every - 1
        spk = (b"\x00\x14" + h) if witness else (b"\x76\xa9\x14" + h + b"\x88\xac")
        prev = hashlib.sha256(f"prev-{seed}-{t}".encode()).digest()
        value = 50_000 + t
        view.add(prev, 0, value, spk, 1, False)
        tx = _core.Transaction()
        tx.version = 2
        vin = _core.TxIn()
        op = _core.OutPoint()
        op.hash, op.n = prev, 0
        vin.prevout = op
        vin.sequence = 0xffffffff
        tx.vin = [vin]
        tx.vout = [_core.TxOut(value - 1000, b"\x76\xa9\x14" + bytes(20) + b"\x88\xac")]
        raw = tx.serialize(True)
        if witness:
            msg = _core.signature_hash(b"\x76\xa9\x14" + h + b"\x88\xac", raw, 0, 1, value, 1)
        else:
            msg = _core.signature_hash(spk, raw, 0, 1, value, 0)
        sig = bytearray(_core.secp_sign(msg, sec))
        if bad_at == t:
            sig[-3] ^= 0x01  # inside S: still valid DER, wrong signature
        sig = bytes(sig) + b"\x01"
        if witness:
            vin.witness = [sig, pub]
            vin.script_sig = b""
        else:
            vin.script_sig = _core.script_push_data(sig) + _core.script_push_data(pub)
        tx.vin = [vin]
        txs.append(tx)
    blk = _core.Block()
    blk.vtx = txs
    return blk, view, height
