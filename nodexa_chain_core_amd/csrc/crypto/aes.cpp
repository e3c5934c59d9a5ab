// AES-256-CBC: see aes.hpp.
#include "aes.hpp"

#include <cstring>

#include "../pow/x16r_prims.hpp"

namespace nodexa {

namespace {

u8 xtime(u8 x) { return u8((x << 1) ^ ((x & 0x80) ? 0x1b : 0)); }

u8 gmul(u8 a, u8 b) {
    u8 p = 0;
    while (b) {
        if (b & 1) p ^= a;
        a = xtime(a);
        b >>= 1;
    }
    return p;
}

struct Tables {
    u8 sbox[256], inv[256];
    Tables() {
        // S-box: multiplicative inverse in GF(2^8) followed by the affine map
        for (int i = 0; i < 256; ++i) {
            u8 inv_i = 0;
            for (int j = 1; j < 256 && i; ++j)
                if (gmul(u8(i), u8(j)) == 1) {
                    inv_i = u8(j);
                    break;
                }
            u8 s = inv_i;
            u8 r = s;
            for (int k = 0; k < 4; ++k) {
                s = u8((s << 1) | (s >> 7));
                r ^= s;
            }
            sbox[i] = u8(r ^ 0x63);
        }
        for (int i = 0; i < 256; ++i) inv[sbox[i]] = u8(i);
    }
};

const Tables& tables() {
    static const Tables t;
    return t;
}

void sub_bytes(u8 s[16], const u8* box) {
    for (int i = 0; i < 16; ++i) s[i] = box[s[i]];
}

void shift_rows(u8 s[16]) {
    u8 t[16];
    for (int c = 0; c < 4; ++c)
        for (int r = 0; r < 4; ++r) t[c * 4 + r] = s[((c + r) % 4) * 4 + r];
    std::memcpy(s, t, 16);
}

void inv_shift_rows(u8 s[16]) {
    u8 t[16];
    for (int c = 0; c < 4; ++c)
        for (int r = 0; r < 4; ++r) t[((c + r) % 4) * 4 + r] = s[c * 4 + r];
    std::memcpy(s, t, 16);
}

void mix_columns(u8 s[16]) {
    for (int c = 0; c < 4; ++c) {
        u8* a = s + 4 * c;
        const u8 a0 = a[0], a1 = a[1], a2 = a[2], a3 = a[3];
        a[0] = u8(xtime(a0) ^ (xtime(a1) ^ a1) ^ a2 ^ a3);
        a[1] = u8(a0 ^ xtime(a1) ^ (xtime(a2) ^ a2) ^ a3);
        a[2] = u8(a0 ^ a1 ^ xtime(a2) ^ (xtime(a3) ^ a3));
        a[3] = u8((xtime(a0) ^ a0) ^ a1 ^ a2 ^ xtime(a3));
    }
}

void inv_mix_columns(u8 s[16]) {
    for (int c = 0; c < 4; ++c) {
        u8* a = s + 4 * c;
        const u8 a0 = a[0], a1 = a[1], a2 = a[2], a3 = a[3];
        a[0] = u8(gmul(a0, 14) ^ gmul(a1, 11) ^ gmul(a2, 13) ^ gmul(a3, 9));
        a[1] = u8(gmul(a0, 9) ^ gmul(a1, 14) ^ gmul(a2, 11) ^ gmul(a3, 13));
        a[2] = u8(gmul(a0, 13) ^ gmul(a1, 9) ^ gmul(a2, 14) ^ gmul(a3, 11));
        a[3] = u8(gmul(a0, 11) ^ gmul(a1, 13) ^ gmul(a2, 9) ^ gmul(a3, 14));
    }
}

void add_round_key(u8 s[16], const u8* k) {
    for (int i = 0; i < 16; ++i) s[i] ^= k[i];
}

}  // namespace

Aes256::Aes256(const u8 key[32]) {
    const Tables& t = tables();
    std::memcpy(rk_, key, 32);
    u8 rcon = 1;
    for (int i = 8; i < 60; ++i) {  // 60 words of 4 bytes
        u8 w[4];
        std::memcpy(w, rk_ + 4 * (i - 1), 4);
        if (i % 8 == 0) {
            const u8 tmp = w[0];
            w[0] = u8(t.sbox[w[1]] ^ rcon);
            w[1] = t.sbox[w[2]];
            w[2] = t.sbox[w[3]];
            w[3] = t.sbox[tmp];
            rcon = xtime(rcon);
        } else if (i % 8 == 4) {
            for (auto& b : w) b = t.sbox[b];
        }
        for (int k = 0; k < 4; ++k) rk_[4 * i + k] = u8(rk_[4 * (i - 8) + k] ^ w[k]);
    }
}

void Aes256::encrypt_block(const u8 in[16], u8 out[16]) const {
    const Tables& t = tables();
    u8 s[16];
    std::memcpy(s, in, 16);
    add_round_key(s, rk_);
    for (int r = 1; r < 14; ++r) {
        sub_bytes(s, t.sbox);
        shift_rows(s);
        mix_columns(s);
        add_round_key(s, rk_ + 16 * r);
    }
    sub_bytes(s, t.sbox);
    shift_rows(s);
    add_round_key(s, rk_ + 16 * 14);
    std::memcpy(out, s, 16);
}

void Aes256::decrypt_block(const u8 in[16], u8 out[16]) const {
    const Tables& t = tables();
    u8 s[16];
    std::memcpy(s, in, 16);
    add_round_key(s, rk_ + 16 * 14);
    for (int r = 13; r > 0; --r) {
        inv_shift_rows(s);
        sub_bytes(s, t.inv);
        add_round_key(s, rk_ + 16 * r);
        inv_mix_columns(s);
    }
    inv_shift_rows(s);
    sub_bytes(s, t.inv);
    add_round_key(s, rk_);
    std::memcpy(out, s, 16);
}

Bytes aes256_cbc_encrypt(const u8 key[32], const u8 iv[16], const Bytes& plain) {
    const Aes256 aes(key);
    const size_t pad = 16 - plain.size() % 16;
    Bytes p = plain;
    p.insert(p.end(), pad, u8(pad));
    Bytes out(p.size());
    u8 prev[16];
    std::memcpy(prev, iv, 16);
    for (size_t off = 0; off < p.size(); off += 16) {
        u8 blk[16];
        for (int i = 0; i < 16; ++i) blk[i] = u8(p[off + size_t(i)] ^ prev[i]);
        aes.encrypt_block(blk, out.data() + off);
        std::memcpy(prev, out.data() + off, 16);
    }
    return out;
}

bool aes256_cbc_decrypt(const u8 key[32], const u8 iv[16], const Bytes& cipher, Bytes& plain) {
    plain.clear();
    if (cipher.empty() || cipher.size() % 16) return false;
    const Aes256 aes(key);
    Bytes out(cipher.size());
    const u8* prev = iv;
    for (size_t off = 0; off < cipher.size(); off += 16) {
        u8 blk[16];
        aes.decrypt_block(cipher.data() + off, blk);
        for (int i = 0; i < 16; ++i) out[off + size_t(i)] = u8(blk[i] ^ prev[i]);
        prev = cipher.data() + off;
    }
    const u8 pad = out.back();
    if (pad == 0 || pad > 16) return false;
    for (size_t i = out.size() - pad; i < out.size(); ++i)
        if (out[i] != pad) return false;
    out.resize(out.size() - pad);
    plain = std::move(out);
    return true;
}

void bytes_to_key_sha512(const std::string& passphrase, const Bytes& salt, int rounds, u8 key[32], u8 iv[16]) {
    Bytes buf(passphrase.begin(), passphrase.end());
    buf.insert(buf.end(), salt.begin(), salt.end());
    Hash512 h = sha512_hash(buf.data(), buf.size());
    for (int i = 1; i < rounds; ++i) h = sha512_hash(h.bytes, 64);
    std::memcpy(key, h.bytes, 32);
    std::memcpy(iv, h.bytes + 32, 16);
}

}  // namespace nodexa
