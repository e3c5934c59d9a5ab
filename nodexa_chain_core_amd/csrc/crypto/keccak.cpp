#include "keccak.hpp"

namespace nodexa {

const u64 kKeccakRoundConstants[24] = {
    0x0000000000000001ULL, 0x0000000000008082ULL, 0x800000000000808AULL, 0x8000000080008000ULL,
    0x000000000000808BULL, 0x0000000080000001ULL, 0x8000000080008081ULL, 0x8000000000008009ULL,
    0x000000000000008AULL, 0x0000000000000088ULL, 0x0000000080008009ULL, 0x000000008000000AULL,
    0x000000008000808BULL, 0x800000000000008BULL, 0x8000000000008089ULL, 0x8000000000008003ULL,
    0x8000000000008002ULL, 0x8000000000000080ULL, 0x000000000000800AULL, 0x800000008000000AULL,
    0x8000000080008081ULL, 0x8000000000008080ULL, 0x0000000080000001ULL, 0x8000000080008008ULL,
};

namespace {

// rho offsets indexed by lane position x + 5*y (Keccak reference, table 2).
constexpr unsigned kRho[25] = {0,  1,  62, 28, 27, 36, 44, 6,  55, 20, 3,  10, 43,
                               25, 39, 41, 45, 15, 21, 8,  18, 2,  61, 56, 14};

template <typename T, int ROUNDS>
inline void keccak_permute(T a[25]) {
    constexpr unsigned W = sizeof(T) * 8;
    for (int round = 0; round < ROUNDS; ++round) {
        // theta
        T c[5], d[5];
        for (int x = 0; x < 5; ++x) c[x] = a[x] ^ a[x + 5] ^ a[x + 10] ^ a[x + 15] ^ a[x + 20];
        for (int x = 0; x < 5; ++x) {
            T r = c[(x + 1) % 5];
            r = T((r << 1) | (r >> (W - 1)));
            d[x] = c[(x + 4) % 5] ^ r;
        }
        for (int i = 0; i < 25; ++i) a[i] ^= d[i % 5];
        // rho + pi: B[y, 2x+3y] = rot(A[x,y], r[x,y])
        T b[25];
        for (int x = 0; x < 5; ++x)
            for (int y = 0; y < 5; ++y) {
                const unsigned rot = kRho[x + 5 * y] % W;
                const T v = a[x + 5 * y];
                b[y + 5 * ((2 * x + 3 * y) % 5)] = rot ? T((v << rot) | (v >> (W - rot))) : v;
            }
        // chi
        for (int y = 0; y < 5; ++y)
            for (int x = 0; x < 5; ++x)
                a[x + 5 * y] = b[x + 5 * y] ^ (T(~b[(x + 1) % 5 + 5 * y]) & b[(x + 2) % 5 + 5 * y]);
        // iota
        a[0] ^= T(kKeccakRoundConstants[round]);
    }
}

template <size_t OUT_BYTES>
void keccak_sponge(const u8* data, size_t n, u8* out) {
    constexpr size_t rate = 200 - 2 * OUT_BYTES;
    u64 st[25] = {0};
    while (n >= rate) {
        for (size_t i = 0; i < rate / 8; ++i) st[i] ^= load_le64(data + 8 * i);
        keccakf1600(st);
        data += rate;
        n -= rate;
    }
    u8 last[rate];
    std::memset(last, 0, rate);
    std::memcpy(last, data, n);
    last[n] ^= 0x01;
    last[rate - 1] ^= 0x80;
    for (size_t i = 0; i < rate / 8; ++i) st[i] ^= load_le64(last + 8 * i);
    keccakf1600(st);
    std::memcpy(out, st, OUT_BYTES);
}

}  // namespace

void keccakf1600(u64 st[25]) { keccak_permute<u64, 24>(st); }
void keccakf800(u32 st[25]) { keccak_permute<u32, 22>(st); }

Hash256 keccak256(const u8* data, size_t n) {
    Hash256 h;
    keccak_sponge<32>(data, n, h.bytes);
    return h;
}

Hash512 keccak512(const u8* data, size_t n) {
    Hash512 h;
    keccak_sponge<64>(data, n, h.bytes);
    return h;
}

bool hash_le(const Hash256& a, const Hash256& b) {
    for (int i = 0; i < 4; ++i) {
        const u64 x = bswap64(a.w64[i]), y = bswap64(b.w64[i]);
        if (x != y) return x < y;
    }
    return true;
}

Hash256 hash256_from_hex(const std::string& hex) {
    Bytes b = hex_decode(hex);
    if (b.size() != 32) throw std::invalid_argument("expected 32-byte hex");
    Hash256 h;
    std::memcpy(h.bytes, b.data(), 32);
    return h;
}

std::string hash256_to_hex(const Hash256& h) { return hex_encode(h.bytes, 32); }

}  // namespace nodexa
