#include "uint256.hpp"

namespace nodexa {

std::string Uint256::hex() const {
    u8 rev[32];
    for (int i = 0; i < 32; ++i) rev[i] = data[31 - i];
    return hex_encode(rev, 32);
}

Uint256 Uint256::from_hex(const std::string& in) {
    // uint256S semantics: skip leading spaces and 0x, read up to 64 hex digits
    // right-aligned, ignore anything after the first non-hex character.
    size_t i = 0;
    while (i < in.size() && std::isspace((unsigned char)in[i])) ++i;
    if (i + 1 < in.size() && in[i] == '0' && (in[i + 1] == 'x' || in[i + 1] == 'X')) i += 2;
    size_t j = i;
    while (j < in.size() && std::isxdigit((unsigned char)in[j])) ++j;
    std::string digits = in.substr(i, j - i);
    if (digits.size() > 64) digits = digits.substr(digits.size() - 64);
    digits = std::string(64 - digits.size(), '0') + digits;
    Bytes b = hex_decode(digits);
    Uint256 r;
    for (int k = 0; k < 32; ++k) r.data[k] = b[31 - k];
    return r;
}

ArithU256& ArithU256::operator*=(u32 b) {
    u64 carry = 0;
    for (int i = 0; i < W; ++i) {
        u64 n = carry + u64(b) * pn[i];
        pn[i] = u32(n);
        carry = n >> 32;
    }
    return *this;
}

ArithU256& ArithU256::operator*=(const ArithU256& b) {
    ArithU256 a;
    for (int j = 0; j < W; ++j) {
        u64 carry = 0;
        for (int i = 0; i + j < W; ++i) {
            u64 n = carry + a.pn[i + j] + u64(pn[j]) * b.pn[i];
            a.pn[i + j] = u32(n);
            carry = n >> 32;
        }
    }
    *this = a;
    return *this;
}

unsigned ArithU256::bits() const {
    for (int pos = W - 1; pos >= 0; --pos)
        if (pn[pos]) return 32 * pos + (32 - __builtin_clz(pn[pos]));
    return 0;
}

ArithU256& ArithU256::operator<<=(unsigned shift) {
    ArithU256 a(*this);
    std::memset(pn, 0, sizeof(pn));
    const int k = int(shift / 32);
    shift %= 32;
    for (int i = 0; i < W; ++i) {
        if (i + k + 1 < W && shift != 0) pn[i + k + 1] |= (a.pn[i] >> (32 - shift));
        if (i + k < W) pn[i + k] |= (a.pn[i] << shift);
    }
    return *this;
}

ArithU256& ArithU256::operator>>=(unsigned shift) {
    ArithU256 a(*this);
    std::memset(pn, 0, sizeof(pn));
    const int k = int(shift / 32);
    shift %= 32;
    for (int i = 0; i < W; ++i) {
        if (i - k - 1 >= 0 && shift != 0) pn[i - k - 1] |= (a.pn[i] << (32 - shift));
        if (i - k >= 0) pn[i - k] |= (a.pn[i] >> shift);
    }
    return *this;
}

ArithU256& ArithU256::operator/=(const ArithU256& b) {
    bool small = true;  // divisor < 2^32 (DGW's n+1 and timespan): exact short division
    for (int i = 1; i < W; ++i) small = small && b.pn[i] == 0;
    if (small && b.pn[0] != 0) {
        const u64 d = b.pn[0];
        u64 rem = 0;
        for (int i = W - 1; i >= 0; --i) {
            const u64 cur = (rem << 32) | pn[i];
            pn[i] = u32(cur / d);
            rem = cur % d;
        }
        return *this;
    }
    const int num_bits = int(bits()), div_bits = int(b.bits());
    if (div_bits == 0) throw std::domain_error("division by zero");
    if (div_bits > num_bits) return *this = ArithU256();
    // binary long division on 64-bit limbs in registers: one compare / subtract / shift
    // per quotient bit (num_bits - div_bits + 1 of them; ~70 for a mainnet GetBlockProof)
    u64 n[4], d[4], q[4] = {0, 0, 0, 0};
    for (int i = 0; i < 4; ++i) {
        n[i] = u64(pn[2 * i]) | (u64(pn[2 * i + 1]) << 32);
        d[i] = u64(b.pn[2 * i]) | (u64(b.pn[2 * i + 1]) << 32);
    }
    int shift = num_bits - div_bits;
    {  // d <<= shift
        const int k = shift / 64, r = shift % 64;
        for (int i = 3; i >= 0; --i) {
            const u64 hi = i - k >= 0 ? d[i - k] : 0, lo = i - k - 1 >= 0 ? d[i - k - 1] : 0;
            d[i] = r ? (hi << r) | (lo >> (64 - r)) : hi;
        }
    }
    for (; shift >= 0; --shift) {
        bool ge = true;
        for (int i = 3; i >= 0; --i) {
            if (n[i] != d[i]) { ge = n[i] > d[i]; break; }
        }
        if (ge) {
            u64 borrow = 0;
            for (int i = 0; i < 4; ++i) {
                const unsigned __int128 t = (unsigned __int128)n[i] - d[i] - borrow;
                n[i] = u64(t);
                borrow = u64(t >> 64) & 1;
            }
            q[shift / 64] |= u64(1) << (shift % 64);
        }
        for (int i = 0; i < 3; ++i) d[i] = (d[i] >> 1) | (d[i + 1] << 63);
        d[3] >>= 1;
    }
    for (int i = 0; i < 4; ++i) {
        pn[2 * i] = u32(q[i]);
        pn[2 * i + 1] = u32(q[i] >> 32);
    }
    return *this;
}

double ArithU256::getdouble() const {
    double ret = 0.0, fact = 1.0;
    for (int i = 0; i < W; ++i) {
        ret += fact * pn[i];
        fact *= 4294967296.0;
    }
    return ret;
}

ArithU256& ArithU256::set_compact(u32 compact, bool* negative, bool* overflow) {
    const int size = int(compact >> 24);
    u32 word = compact & 0x007fffff;
    if (size <= 3) {
        word >>= 8 * (3 - size);
        *this = ArithU256(word);
    } else {
        *this = ArithU256(word);
        *this <<= unsigned(8 * (size - 3));
    }
    if (negative) *negative = word != 0 && (compact & 0x00800000) != 0;
    if (overflow)
        *overflow = word != 0 && ((size > 34) || (word > 0xff && size > 33) || (word > 0xffff && size > 32));
    return *this;
}

u32 ArithU256::get_compact(bool negative) const {
    int size = int((bits() + 7) / 8);
    u32 compact = 0;
    if (size <= 3) {
        compact = u32(low64() << (8 * (3 - size)));
    } else {
        ArithU256 bn = *this >> unsigned(8 * (size - 3));
        compact = u32(bn.low64());
    }
    if (compact & 0x00800000) {
        compact >>= 8;
        size++;
    }
    compact |= u32(size) << 24;
    compact |= (negative && (compact & 0x007fffff) ? 0x00800000 : 0);
    return compact;
}

}  // namespace nodexa
