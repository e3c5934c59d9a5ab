"""Native fuzzing (the reference's test_clore_fuzzy tier, src/test/test_clore_fuzzy.cpp, which
deserializes 17 wire / disk types from fuzzer input).

bin/fuzz_nodexa (csrc/fuzz/fuzz_main.cpp, libFuzzer + ASan + UBSan, host code only) runs a fixed
number of mutations from a seed corpus of real encodings: the regtest / main genesis blocks in
both header formats, KawPow testnet headers, a coinbase transaction, standard scripts, asset
verifier strings, the fee-estimator / asset / index snapshots, a DER signature and a two-page
Berkeley DB btree (the wallet.dat reader, store/bdb.cpp). A crash, a
sanitizer report or a broken round-trip invariant fails the run."""
import os
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))


def _seeds(core):
    main = core.make_chain_params("main")
    reg = core.make_chain_params("regtest")
    out = []
    for p in (main, reg):
        g = p.genesis
        out.append(b"\x00" + g.serialize(0))            # KawPow-format header
        out.append(b"\x01" + g.serialize(0xFFFFFFFF))   # legacy 80-byte header
        out.append(b"\x03" + g.header.serialize(0xFFFFFFFF))
        out.append(b"\x04" + g.vtx[0].serialize())
        out.append(b"\x05" + g.vtx[0].vout[0].script_pubkey)
    with open(os.path.join(HERE, "data", "testnet_kawpow_10k.hdr"), "rb") as f:
        raw = f.read(360)
    out += [b"\x02" + raw[i:i + 120] for i in range(0, 360, 120)]
    p2pkh = bytes.fromhex("76a914") + bytes(range(20)) + bytes.fromhex("88ac")
    out.append(b"\x05\x01" + p2pkh)
    out += [b"\x06" + s.encode() for s in ("#KYC & !#BANNED", "(#A | #B) & !#C", "true", "#KYC_1 & #AML")]
    est = core.FeeEstimator()
    for b in range(4):
        est.process_tx(bytes([b]) * 32, b, 5000 + b, 200, True)
        est.process_block(b + 1, [bytes([b]) * 32])
    out.append(b"\x07" + est.serialize())
    out.append(b"\x08" + core.AssetsState().serialize())
    out.append(b"\x0a" + bytes.fromhex("3044022057e8f2a6e4b4d3e8b8a7a9a9c1f2e1d0b0a090807060504030201000fedcba98"
                                       "022046e1f2a3b4c5d6e7f8091a2b3c4d5e6f708192a3b4c5d6e7f8091a2b3c4d5e6f"))
    out.append(b"\x0b" + bytes(80))
    out.append(b"\x0c" + bytes([2, 4, 1, 3, 1, 32, 17]) + bytes(range(40)))
    out.append(b"\x0d" + _bdb_seed())
    return out


def _bdb_seed() -> bytes:
    """A two-page Berkeley DB btree (512-byte pages): meta page, one leaf with one key/value."""
    import struct

    ps = 512
    meta = bytearray(ps)
    struct.pack_into("<III", meta, 12, 0x053162, 9, ps)
    meta[25] = 9
    struct.pack_into("<I", meta, 32, 1)   # last_pgno
    struct.pack_into("<I", meta, 88, 1)   # root
    leaf = bytearray(ps)
    struct.pack_into("<IIIHH", leaf, 8, 1, 0, 0, 2, ps - 16)
    leaf[24], leaf[25] = 1, 5
    for i, (off, item) in enumerate(((ps - 8, b"key"), (ps - 16, b"value"))):
        struct.pack_into("<H", leaf, 26 + 2 * i, off)
        struct.pack_into("<HB", leaf, off, len(item), 1)
        leaf[off + 3:off + 3 + len(item)] = item
    return bytes(meta + leaf)


def test_fuzz_native_core(core, tmp_path):
    from nodexa_chain_core_amd import _build

    try:
        exe = _build.build_fuzz()
    except subprocess.CalledProcessError as e:  # pragma: no cover - toolchain without libFuzzer
        pytest.skip(f"libFuzzer build unavailable: {e}")
    corpus = tmp_path / "corpus"
    corpus.mkdir()
    for i, s in enumerate(_seeds(core)):
        (corpus / f"seed{i:02d}").write_bytes(s)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:abort_on_error=1",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")
    r = subprocess.run([exe, str(corpus), "-runs=60000", "-seed=1", "-max_len=4096", "-timeout=20",
                        "-rss_limit_mb=4096", f"-artifact_prefix={tmp_path}/"],
                       capture_output=True, text=True, timeout=900, env=env)
    tail = (r.stdout + r.stderr)[-4000:]
    assert r.returncode == 0, tail
    assert "Done 60000 runs" in tail, tail
