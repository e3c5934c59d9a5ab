// Bitcoin-family wire/disk serialization primitives (little-endian ints,
// CompactSize, length-prefixed vectors). Parity: src/serialize.h
// (WriteCompactSize / ReadCompactSize, MAX_SIZE = 0x02000000).
#pragma once

#include "../util/common.hpp"
#include "uint256.hpp"

namespace nodexa {

constexpr u64 kMaxSerializeSize = 0x02000000;

class Writer {
public:
    Bytes buf;
    void u8_(u8 v) { buf.push_back(v); }
    void u16_(uint16_t v) { u8 b[2]; std::memcpy(b, &v, 2); raw(b, 2); }
    void u32_(u32 v) { u8 b[4]; store_le32(b, v); raw(b, 4); }
    void i32_(int32_t v) { u32_(u32(v)); }
    void u64_(u64 v) { u8 b[8]; store_le64(b, v); raw(b, 8); }
    void i64_(int64_t v) { u64_(u64(v)); }
    void raw(const u8* p, size_t n) { buf.insert(buf.end(), p, p + n); }
    void raw(const Bytes& b) { raw(b.data(), b.size()); }
    void u256(const Uint256& u) { raw(u.data, 32); }
    void compact_size(u64 n) {
        if (n < 253) u8_(u8(n));
        else if (n <= 0xffff) { u8_(253); u16_(uint16_t(n)); }
        else if (n <= 0xffffffffULL) { u8_(254); u32_(u32(n)); }
        else { u8_(255); u64_(n); }
    }
    void var_bytes(const Bytes& b) { compact_size(b.size()); raw(b); }
};

class Reader {
public:
    Reader(const u8* p, size_t n) : p_(p), n_(n) {}
    explicit Reader(const Bytes& b) : p_(b.data()), n_(b.size()) {}
    size_t pos() const { return pos_; }
    size_t remaining() const { return n_ - pos_; }
    bool empty() const { return pos_ == n_; }
    void need(size_t k) const { if (n_ - pos_ < k) throw std::out_of_range("Reader: unexpected end of data"); }
    const u8* take(size_t k) { need(k); const u8* r = p_ + pos_; pos_ += k; return r; }
    u8 u8_() { return *take(1); }
    uint16_t u16_() { uint16_t v; std::memcpy(&v, take(2), 2); return v; }
    u32 u32_() { return load_le32(take(4)); }
    int32_t i32_() { return int32_t(u32_()); }
    u64 u64_() { return load_le64(take(8)); }
    int64_t i64_() { return int64_t(u64_()); }
    Uint256 u256() { return Uint256::from_bytes(take(32)); }
    u64 compact_size() {
        const u8 c = u8_();
        u64 n;
        if (c < 253) n = c;
        else if (c == 253) { n = u16_(); if (n < 253) throw std::runtime_error("non-canonical ReadCompactSize()"); }
        else if (c == 254) { n = u32_(); if (n < 0x10000u) throw std::runtime_error("non-canonical ReadCompactSize()"); }
        else { n = u64_(); if (n < 0x100000000ULL) throw std::runtime_error("non-canonical ReadCompactSize()"); }
        if (n > kMaxSerializeSize) throw std::runtime_error("ReadCompactSize(): size too large");
        return n;
    }
    Bytes var_bytes() { const u64 n = compact_size(); const u8* q = take(size_t(n)); return Bytes(q, q + n); }

private:
    const u8* p_;
    size_t n_;
    size_t pos_ = 0;
};

}  // namespace nodexa
