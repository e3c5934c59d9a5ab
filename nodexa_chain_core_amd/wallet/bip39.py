"""BIP39 mnemonics: entropy <-> word list, checksum validation and the PBKDF2 seed.

Parity (behaviour): CMnemonic::Generate / FromData / Check / ToSeed (src/wallet/bip39.cpp) — 11-bit
word indexes over entropy || SHA256(entropy)[: ENT/32 bits], seed = PBKDF2-HMAC-SHA512(mnemonic,
"mnemonic" || passphrase, 2048 rounds, 64 bytes). The word list is the standard BIP-0039 English
list (`bip39_words.txt`, checked against its published SHA-256 when loaded); the reference's
test/data/bip39_vectors.json pins all of it in tests/test_wallet.py.
"""
from __future__ import annotations

import hashlib
import os
import unicodedata

_WORDS: list[str] | None = None
_INDEX: dict[str, int] = {}
# sha256 of the canonical english.txt (one word per line, trailing newline)
WORDLIST_SHA256 = "2f5eed53a4727b4bf8880d8f3f199efc90e58503646d9ff8eff3a2ed3b24dbda"


def words() -> list[str]:
    global _WORDS
    if _WORDS is None:
        with open(os.path.join(os.path.dirname(__file__), "bip39_words.txt")) as f:
            w = f.read().split()
        if len(w) != 2048 or hashlib.sha256(("\n".join(w) + "\n").encode()).hexdigest() != WORDLIST_SHA256:
            raise RuntimeError("BIP39 word list is corrupt")
        _WORDS = w
        _INDEX.update({x: i for i, x in enumerate(w)})
    return _WORDS


def from_entropy(entropy: bytes) -> str:
    """CMnemonic::FromData: 16..32 bytes (a multiple of 4) -> 12..24 words."""
    if len(entropy) % 4 or not 16 <= len(entropy) <= 32:
        raise ValueError("entropy must be 16..32 bytes, a multiple of 4")
    wl = words()
    cs_bits = len(entropy) * 8 // 32
    bits = int.from_bytes(entropy, "big") << cs_bits | hashlib.sha256(entropy).digest()[0] >> (8 - cs_bits)
    n = (len(entropy) * 8 + cs_bits) // 11
    return " ".join(wl[(bits >> (11 * (n - 1 - i))) & 0x7FF] for i in range(n))


def generate(strength: int = 128) -> str:
    """CMnemonic::Generate (128 bits: 12 words, the -bip44 wallet default)."""
    return from_entropy(os.urandom(strength // 8))


def to_entropy(mnemonic: str) -> bytes | None:
    words()
    ws = mnemonic.split()
    if len(ws) % 3 or not 12 <= len(ws) <= 24:
        return None
    bits = 0
    for w in ws:
        i = _INDEX.get(w)
        if i is None:
            return None
        bits = bits << 11 | i
    cs_bits = len(ws) * 11 // 33
    ent_len = (len(ws) * 11 - cs_bits) // 8
    entropy = (bits >> cs_bits).to_bytes(ent_len, "big")
    if bits & ((1 << cs_bits) - 1) != hashlib.sha256(entropy).digest()[0] >> (8 - cs_bits):
        return None
    return entropy


def check(mnemonic: str) -> bool:
    """CMnemonic::Check: known words and a matching checksum."""
    return to_entropy(mnemonic) is not None


def to_seed(mnemonic: str, passphrase: str = "") -> bytes:
    """CMnemonic::ToSeed."""
    m = unicodedata.normalize("NFKD", mnemonic).encode()
    salt = ("mnemonic" + unicodedata.normalize("NFKD", passphrase)).encode()
    return hashlib.pbkdf2_hmac("sha512", m, salt, 2048, 64)
