// Batch SHA-256d on gfx950 ("CPU + HIP device SHA256d for batch header hashing").
//
// sha256d_batch: one lane per fixed-length message (block headers: 80-byte KawPow inputs,
// 1459-byte Equihash-extended headers), digest = SHA256(SHA256(msg)) in the byte order of
// the reference's CHash256 / SerializeHash (src/hash.h:49,274).
// sha256d_merkle_level: one level of ComputeMerkleRoot (src/consensus/merkle.cpp): out[i] =
// SHA256d(in[2i] || in[2i+1]), the last node paired with itself on odd levels.
// Both are integer-ALU kernels (64 rounds of 32-bit rotates/adds per 64-byte block) with
// the message schedule in a 16-word register ring; SHA-256 has no MFMA shape.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "kernel_params.h"
#include "keccak_device.hpp"

__constant__ uint32_t SHA256_K[64] = {
    0x428a2f98u, 0x71374491u, 0xb5c0fbcfu, 0xe9b5dba5u, 0x3956c25bu, 0x59f111f1u, 0x923f82a4u, 0xab1c5ed5u,
    0xd807aa98u, 0x12835b01u, 0x243185beu, 0x550c7dc3u, 0x72be5d74u, 0x80deb1feu, 0x9bdc06a7u, 0xc19bf174u,
    0xe49b69c1u, 0xefbe4786u, 0x0fc19dc6u, 0x240ca1ccu, 0x2de92c6fu, 0x4a7484aau, 0x5cb0a9dcu, 0x76f988dau,
    0x983e5152u, 0xa831c66du, 0xb00327c8u, 0xbf597fc7u, 0xc6e00bf3u, 0xd5a79147u, 0x06ca6351u, 0x14292967u,
    0x27b70a85u, 0x2e1b2138u, 0x4d2c6dfcu, 0x53380d13u, 0x650a7354u, 0x766a0abbu, 0x81c2c92eu, 0x92722c85u,
    0xa2bfe8a1u, 0xa81a664bu, 0xc24b8b70u, 0xc76c51a3u, 0xd192e819u, 0xd6990624u, 0xf40e3585u, 0x106aa070u,
    0x19a4c116u, 0x1e376c08u, 0x2748774cu, 0x34b0bcb5u, 0x391c0cb3u, 0x4ed8aa4au, 0x5b9cca4fu, 0x682e6ff3u,
    0x748f82eeu, 0x78a5636fu, 0x84c87814u, 0x8cc70208u, 0x90befffau, 0xa4506cebu, 0xbef9a3f7u, 0xc67178f2u
};

__device__ __forceinline__ uint32_t rotr32(uint32_t x, int n) { return __builtin_amdgcn_alignbit(x, x, n); }

__device__ __forceinline__ void sha256_init(uint32_t s[8]) {
    const uint32_t h0[8] = {0x6a09e667u, 0xbb67ae85u, 0x3c6ef372u, 0xa54ff53au, 0x510e527fu, 0x9b05688cu, 0x1f83d9abu, 0x5be0cd19u};
#pragma unroll
    for (int i = 0; i < 8; ++i) s[i] = h0[i];
}

__device__ __forceinline__ void sha256_compress(uint32_t s[8], uint32_t w[16]) {
    uint32_t a = s[0], b = s[1], c = s[2], d = s[3], e = s[4], f = s[5], g = s[6], h = s[7];
#pragma unroll
    for (int i = 0; i < 64; ++i) {
        uint32_t wi;
        if (i < 16) {
            wi = w[i];
        } else {
            const uint32_t w15 = w[(i - 15) & 15], w2 = w[(i - 2) & 15];
            const uint32_t s0 = rotr32(w15, 7) ^ rotr32(w15, 18) ^ (w15 >> 3);
            const uint32_t s1 = rotr32(w2, 17) ^ rotr32(w2, 19) ^ (w2 >> 10);
            wi = w[i & 15] = w[i & 15] + s0 + w[(i - 7) & 15] + s1;
        }
        const uint32_t S1 = rotr32(e, 6) ^ rotr32(e, 11) ^ rotr32(e, 25);
        const uint32_t ch = (e & f) ^ (~e & g);
        const uint32_t t1 = h + S1 + ch + SHA256_K[i] + wi;
        const uint32_t S0 = rotr32(a, 2) ^ rotr32(a, 13) ^ rotr32(a, 22);
        const uint32_t mj = (a & b) ^ (a & c) ^ (b & c);
        h = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + S0 + mj;
    }
    s[0] += a; s[1] += b; s[2] += c; s[3] += d; s[4] += e; s[5] += f; s[6] += g; s[7] += h;
}

// SHA-256 of len bytes at m (any alignment), padding generated on the fly. A block that lies
// inside the message with a dword to spare is read as 17 aligned dwords and realigned in registers
// (v_alignbyte + byte swap): 17 loads instead of 64 byte loads per block, which matters for the
// 1487-byte Equihash headers (23 such blocks each) of the resident verify's side stream. The tail
// blocks (message end, padding, length) keep the byte path, so no load reaches past the message.
__device__ void sha256_bytes(const uint8_t* m, uint32_t len, uint32_t s[8]) {
    sha256_init(s);
    const uint32_t nblocks = (len + 9 + 63) / 64;
    const uint32_t mis = uint32_t(reinterpret_cast<uintptr_t>(m) & 3);
    const uint32_t* a = reinterpret_cast<const uint32_t*>(m - mis);
    // the next in-message block's dwords are loaded before this block is compressed, so the load
    // latency hides behind the 64 rounds (one lane hashes its message's blocks one after another)
    uint32_t nxt[17];
    if (64 + 4 <= len) {
#pragma unroll
        for (int k = 0; k < 17; ++k) nxt[k] = a[k];
    }
    for (uint32_t b = 0; b < nblocks; ++b) {
        uint32_t w[16];
        if ((b + 1) * 64 + 4 <= len) {
            uint32_t d[17];
#pragma unroll
            for (int k = 0; k < 17; ++k) d[k] = nxt[k];
            if ((b + 2) * 64 + 4 <= len) {
#pragma unroll
                for (int k = 0; k < 17; ++k) nxt[k] = a[(b + 1) * 16 + k];
            }
#pragma unroll
            for (int j = 0; j < 16; ++j) w[j] = __builtin_bswap32(__builtin_amdgcn_alignbyte(d[j + 1], d[j], mis));
        } else {
#pragma unroll
            for (int j = 0; j < 16; ++j) {
                uint32_t word = 0;
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    const uint32_t idx = b * 64 + uint32_t(j) * 4 + uint32_t(k);
                    const uint32_t byte = idx < len ? m[idx] : (idx == len ? 0x80u : 0u);
                    word = (word << 8) | byte;
                }
                w[j] = word;
            }
        }
        if (b == nblocks - 1) {
            w[14] = len >> 29;
            w[15] = len << 3;
        }
        sha256_compress(s, w);
    }
}

// Second pass of SHA256d: SHA-256 of the 32-byte digest held as 8 big-endian words.
__device__ __forceinline__ void sha256_of_digest(const uint32_t d[8], uint32_t s[8]) {
    uint32_t w[16];
#pragma unroll
    for (int i = 0; i < 8; ++i) w[i] = d[i];
    w[8] = 0x80000000u;
#pragma unroll
    for (int i = 9; i < 15; ++i) w[i] = 0;
    w[15] = 256;
    sha256_init(s);
    sha256_compress(s, w);
}

__device__ __forceinline__ void store_digest(uint8_t* o, const uint32_t s[8]) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        o[4 * i + 0] = uint8_t(s[i] >> 24);
        o[4 * i + 1] = uint8_t(s[i] >> 16);
        o[4 * i + 2] = uint8_t(s[i] >> 8);
        o[4 * i + 3] = uint8_t(s[i]);
    }
}

extern "C" __global__ __launch_bounds__(256) void sha256d_batch(Sha256dParams p) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= p.n) return;
    uint32_t s1[8], s2[8];
    sha256_bytes(p.in + size_t(i) * p.stride, p.len, s1);
    sha256_of_digest(s1, s2);
    store_digest(p.out + size_t(i) * 32, s2);
}

extern "C" __global__ __launch_bounds__(256) void sha256d_merkle_level(Sha256dParams p) {
    // p.n = output nodes, p.len = input nodes (32 bytes each)
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= p.n) return;
    const uint32_t l = 2 * i, r = (2 * i + 1 < p.len) ? 2 * i + 1 : 2 * i;
    uint32_t w[16];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const uint8_t* a = p.in + size_t(l) * 32 + 4 * j;
        const uint8_t* b = p.in + size_t(r) * 32 + 4 * j;
        w[j] = (uint32_t(a[0]) << 24) | (uint32_t(a[1]) << 16) | (uint32_t(a[2]) << 8) | a[3];
        w[8 + j] = (uint32_t(b[0]) << 24) | (uint32_t(b[1]) << 16) | (uint32_t(b[2]) << 8) | b[3];
    }
    uint32_t s1[8], s2[8];
    sha256_init(s1);
    sha256_compress(s1, w);
    uint32_t pad[16] = {0x80000000u, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 512};
    sha256_compress(s1, pad);
    sha256_of_digest(s1, s2);
    store_digest(p.out + size_t(i) * 32, s2);
}

// ---------------------------------------------------------------- K4: mix-only header check
// progpow::hash_no_verify (src/crypto/ethash/lib/ethash/progpow.cpp:498-550) for a batch of KawPow
// headers, fused with the SHA256d header hash it needs (K6): header hash = SHA256d of the 80-byte
// CKAWPOWInput (src/primitives/block.h:213-233), byte-reversed into ProgPoW order (GetHex ->
// to_hash256, src/hash.cpp:269-270); seed = keccak-f800(header hash, nonce64, "rAVENCOINKAWPOW");
// final = keccak-f800(seed[0..7], claimed mix, "RAVENCOIN"). The host then sends only the headers
// whose final meets their nBits boundary to the full (DAG) check — the reference's CheckBlockHeader
// does that cheap check first for the same reason (src/validation.cpp:11638-11665).
__device__ __forceinline__ uint32_t mo_le32(const uint8_t* p) {
    return uint32_t(p[0]) | (uint32_t(p[1]) << 8) | (uint32_t(p[2]) << 16) | (uint32_t(p[3]) << 24);
}

__device__ __forceinline__ void mo_store_le(uint8_t* o, uint32_t w) {
    o[0] = uint8_t(w); o[1] = uint8_t(w >> 8); o[2] = uint8_t(w >> 16); o[3] = uint8_t(w >> 24);
}

extern "C" __global__ __launch_bounds__(256) void kawpow_mixonly_batch(MixOnlyParams p) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= p.n) return;
    const uint8_t* h = p.headers + size_t(i) * p.stride;
    uint8_t* o = p.out + size_t(i) * 128;
    uint32_t s1[8], s2[8];
    sha256_bytes(h, 80, s1);
    sha256_of_digest(s1, s2);
    // ProgPoW word k of the byte-reversed digest is SHA state word 7-k (its big-endian bytes reversed)
    uint32_t st[25];
#pragma unroll
    for (int k = 0; k < 8; ++k) st[k] = s2[7 - k];
    st[8] = mo_le32(h + 80);   // nonce64 low
    st[9] = mo_le32(h + 84);   // nonce64 high
    const uint32_t pad1[15] = {0x72, 0x41, 0x56, 0x45, 0x4E, 0x43, 0x4F, 0x49, 0x4E, 0x4B, 0x41, 0x57, 0x50, 0x4F, 0x57};
#pragma unroll
    for (int k = 0; k < 15; ++k) st[10 + k] = pad1[k];
    uint32_t hh[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) hh[k] = st[k];
    keccak_f800(st);
    uint32_t mix[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) mix[k] = __builtin_bswap32(mo_le32(h + 88 + 28 - 4 * k));  // reversed mix_hash
#pragma unroll
    for (int k = 0; k < 8; ++k) st[8 + k] = mix[k];  // st[0..7] = seed state words
    const uint32_t pad2[9] = {0x72, 0x41, 0x56, 0x45, 0x4E, 0x43, 0x4F, 0x49, 0x4E};
#pragma unroll
    for (int k = 0; k < 9; ++k) st[16 + k] = pad2[k];
    keccak_f800(st);
    // nBits -> 256-bit target, big-endian bytes (arith_uint256::SetCompact; zero when negative or
    // overflowing, so nothing meets it)
    const uint32_t bits = mo_le32(h + 72);
    const uint32_t ex = bits >> 24;
    uint32_t mant = bits & 0x007fffffu;
    const bool neg = mant != 0 && (bits & 0x00800000u) != 0;
    const bool ovf = mant != 0 && (ex > 34 || (mant > 0xff && ex > 33) || (mant > 0xffff && ex > 32));
    uint8_t b[32];
#pragma unroll
    for (int k = 0; k < 32; ++k) b[k] = 0;
    if (!neg && !ovf) {
        if (ex <= 3) {
            mant >>= 8 * (3 - ex);
            b[31] = uint8_t(mant); b[30] = uint8_t(mant >> 8); b[29] = uint8_t(mant >> 16);
        } else {
            const uint32_t s = ex - 3;  // little-endian byte position of the mantissa's low byte
            for (uint32_t q = 0; q < 3; ++q)
                if (s + q < 32) b[31 - (s + q)] = uint8_t(mant >> (8 * q));
        }
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        mo_store_le(o + 4 * k, hh[k]);
        mo_store_le(o + 32 + 4 * k, st[k]);
        mo_store_le(o + 96 + 4 * k, mix[k]);
    }
#pragma unroll
    for (int k = 0; k < 32; ++k) o[64 + k] = b[k];
}
