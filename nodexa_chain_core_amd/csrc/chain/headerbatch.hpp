// A header batch laid out once for the device-resident verify pipeline (models/verify.py
// verify_batch_resident; BASELINE config 5).
//
// The reference verifies a `headers` message header by header under cs_main (ProcessNewBlock-
// Headers, src/validation.cpp:12017-12035; CheckBlockHeader :11638-11665). Here the batch is
// parsed straight from its wire bytes into one native object that owns the headers, so no
// per-header Python object is made or converted again, and packs, in one parallel pass, what the
// GPU pipeline uploads with ONE host-to-device copy:
//   rows   n x 128 B: bytes 0..119 the 120-byte KawPow header (the 80-byte legacy header, or the
//          80-byte CKAWPOWInput prefix of an Equihash header); nTime / nBits therefore sit at
//          bytes 68 / 72 of every row, where the DGW series reads them;
//   kinds  n B: 0 KawPow, 2 Equihash extension, 3 pre-KawPow (X16R / X16RV2);
//   eq_*   the Equihash headers: their batch index, 128-byte BLAKE2b message blocks (the 112-byte
//          input), packed 1344-byte solutions and the serialized headers (for SHA256d).
// HeaderChain::accept_headers then reads the batch's own headers (a contiguous range of them).
//
// from_bytes packs all of that straight from the wire bytes (a KawPow row IS its 120-byte wire
// form, a legacy or Equihash row the first 80 bytes of its, an Equihash input the first 112) and
// defers the BlockHeader objects: materialize() decodes them later, so the resident pipeline
// (ops/header_batch.py) decodes while the device verifies, and only the accept stays after it.
#pragma once

#include <memory>
#include <mutex>
#include <string>
#include <utility>
#include <vector>

#include "primitives.hpp"

namespace nodexa {

constexpr size_t kBatchRow = 128;

// Byte buffer whose resize leaves new bytes uninitialised: the batch's packing passes write every
// byte of the 1.3 MB row array themselves, in parallel, so a serial zero fill would be pure cost.
template <class T>
struct NoInitAlloc : std::allocator<T> {
    template <class U>
    struct rebind {
        using other = NoInitAlloc<U>;
    };
    NoInitAlloc() = default;
    template <class U>
    NoInitAlloc(const NoInitAlloc<U>&) {}
    template <class U>
    void construct(U* p) {
        ::new (static_cast<void*>(p)) U;
    }
    template <class U, class... A>
    void construct(U* p, A&&... a) {
        ::new (static_cast<void*>(p)) U(std::forward<A>(a)...);
    }
};
using RawBytes = std::vector<char, NoInitAlloc<char>>;

struct HeaderBatch {
    u32 act = 0;
    std::vector<BlockHeader> hs;  // complete once materialize() has run (from_headers: always)
    RawBytes kinds, rows;
    std::vector<u32> eq_index;
    std::string eq_msgs, eq_sols, eq_ser;
    size_t eq_ser_len = 0;   // bytes of one serialized Equihash header (all equal for (200, 9))
    bool eq_uniform = true;  // every Equihash header has a well-formed 1344-byte solution

    // `keep`: an owner of `data` that keeps it alive and unchanged for the batch's lifetime (an
    // immutable Python bytes object): the deferred decode then reads it in place, else the wire
    // records are copied
    static HeaderBatch from_bytes(const u8* data, size_t len, u32 kawpow_activation_time,
                                  std::shared_ptr<const void> keep = nullptr);
    static HeaderBatch from_headers(std::vector<BlockHeader> headers, u32 kawpow_activation_time);
    void pack();
    // decode the wire records into hs (parallel; no-op when done; concurrent callers wait for one)
    void materialize();
    const std::vector<BlockHeader>& headers() {
        materialize();
        return hs;
    }
    // header i, decoded on its own while the batch is not materialized yet
    BlockHeader header(size_t i);
    size_t size() const { return n_; }

private:
    std::string raw_;          // the wire records, back to back (from_bytes without an owner)
    std::shared_ptr<const void> keep_;
    const u8* src_ = nullptr;  // the owner's bytes (keep_ set)
    std::vector<size_t> off_;  // record offsets into raw_ (and raw_.size() at the end)
    size_t n_ = 0;
    bool materialized_ = true;
    std::shared_ptr<std::mutex> mu_ = std::make_shared<std::mutex>();  // shared_ptr: the batch stays movable
};

}  // namespace nodexa
