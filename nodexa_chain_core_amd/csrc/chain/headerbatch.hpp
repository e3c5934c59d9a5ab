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
#pragma once

#include <string>
#include <vector>

#include "primitives.hpp"

namespace nodexa {

constexpr size_t kBatchRow = 128;

struct HeaderBatch {
    u32 act = 0;
    std::vector<BlockHeader> hs;
    std::string kinds, rows;
    std::vector<u32> eq_index;
    std::string eq_msgs, eq_sols, eq_ser;
    size_t eq_ser_len = 0;   // bytes of one serialized Equihash header (all equal for (200, 9))
    bool eq_uniform = true;  // every Equihash header has a well-formed 1344-byte solution

    static HeaderBatch from_bytes(const u8* data, size_t len, u32 kawpow_activation_time);
    static HeaderBatch from_headers(std::vector<BlockHeader> headers, u32 kawpow_activation_time);
    void pack();
    size_t size() const { return hs.size(); }
};

}  // namespace nodexa
