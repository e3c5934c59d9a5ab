"""Derive the compact GOST R 34.11-2012 (Streebog) tables of csrc/pow/legacy_algos.cpp from a
dump of the reference's combined LPS table (src/algo/gost_streebog.c TG[8][256], C[12][64]).

TG[i][x] is linear in the S-box output pi(x): TG[i][x] = Lin_i(pi(x)) with Lin_i injective over
GF(2). So the 2048 words are 8 bases of 8 words (the images of 8 independent S-box outputs) plus
one 256-entry byte code (the coordinates of pi(x) in that basis, the same for every i). The
iteration constants are re-expressed as little-endian 64-bit words of the state layout.

    gcc -O2 -w -I/root/reference/src -o /tmp/gost/dump <harness including algo/gost_streebog.c>
    /tmp/gost/dump t > /tmp/gost/tables.json && python3 tools/gost_compact_tables.py /tmp/gost/tables.json
"""
import json
import sys


def main(path: str) -> None:
    d = json.load(open(path))
    tg = [[int(v, 16) for v in row] for row in d["TG"]]
    # greedy: 8 inputs whose TG[0] images are independent
    basis_x, rows = [], []  # rows: (reduced vector, combination mask over chosen basis)
    for x in range(256):
        v, m = tg[0][x], 0
        for rv, rm, piv in rows:
            if v >> piv & 1:
                v ^= rv
                m ^= rm
        if v:
            piv = v.bit_length() - 1
            rows.append((v, m ^ (1 << len(basis_x)), piv))
            basis_x.append(x)
        if len(basis_x) == 8:
            break
    assert len(basis_x) == 8

    def coords(v):
        m = 0
        for rv, rm, piv in rows:
            if v >> piv & 1:
                v ^= rv
                m ^= rm
        assert v == 0
        return m

    code = [coords(tg[0][x]) for x in range(256)]
    basis = [[tg[i][x] for x in basis_x] for i in range(8)]
    for i in range(8):  # the same code reproduces every row
        for x in range(256):
            acc = 0
            for b in range(8):
                if code[x] >> b & 1:
                    acc ^= basis[i][b]
            assert acc == tg[i][x], (i, x)
    c_words = [[int.from_bytes(bytes.fromhex(c)[8 * k:8 * k + 8], "little") for k in range(8)] for c in d["C"]]
    print("// basis[i][b]: LPS image of basis byte b at input byte position i")
    print("static const u64 kGostBasis[8][8] = {")
    for i in range(8):
        print("    {" + ", ".join(f"0x{v:016x}ULL" for v in basis[i]) + "},")
    print("};")
    print("// code[x]: the S-box output of x in that basis")
    print("static const u8 kGostCode[256] = {")
    for r in range(0, 256, 16):
        print("    " + ", ".join(f"{v:3d}" for v in code[r:r + 16]) + ",")
    print("};")
    print("// iteration constants C_1..C_12 as little-endian words of the state layout")
    print("static const u64 kGostC[12][8] = {")
    for w in c_words:
        print("    {" + ", ".join(f"0x{v:016x}ULL" for v in w) + "},")
    print("};")


if __name__ == "__main__":
    main(sys.argv[1])
