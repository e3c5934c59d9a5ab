// Reader and writer of Berkeley DB btree files (the reference's wallet.dat).
//
// The reference keeps its wallet in a Berkeley DB 4.8 btree file with the records in a
// sub-database named "main" (src/wallet/db.cpp:235, 436, 536: Db::open(..., "main", DB_BTREE,
// ...)). This node keeps wallets as JSON (wallet/wallet.py); this reader is the one-way bridge
// that lets a reference wallet.dat be imported at start-up (wallet/walletdb.py). It needs no
// libdb: it walks the file's pages directly.
//
// Format (dbinc/db_page.h of Berkeley DB 4.x/5.x, btree version 8-10, host byte order, either
// endianness accepted):
//   page 0       btree meta page: magic 0x053162 @12, version @16, pagesize @20, encrypt_alg @24,
//                page type @25, metaflags @26 (bit 0: page checksums), last_pgno @32, root @88
//   page header  26 bytes: pgno @8, prev @12, next @16, entries u16 @20, hf_offset u16 @22,
//                level @24, type @25; the item index (u16 offsets) follows, after a 6-byte
//                checksum area when the file carries page checksums
//   internal     (type 3) BINTERNAL items: len u16, type u8, pad, child pgno u32 @4, nrecs, key
//   leaf         (type 5) alternating key / data items: BKEYDATA (len u16, type u8 = 1, bytes)
//                or BOVERFLOW (type 3, pgno @4, total length @8); type bit 0x80 = deleted
//   overflow     (type 7) pages chained by next_pgno, hf_offset bytes of payload each
//   sub-databases: the file's master btree maps each name to its own meta page number (stored in
//                network byte order by __db_master_update)
// Encrypted files (encrypt_alg != 0) and off-page duplicate trees are refused; neither occurs in
// a wallet.dat (the wallet encrypts secrets itself, CCryptoKeyStore).
#pragma once

#include <string>
#include <utility>
#include <vector>

namespace nodexa {
namespace bdb {

using Records = std::vector<std::pair<std::string, std::string>>;

// Every key/value pair of sub-database `subdb` of the btree file at `path`, in key order ("" reads
// the master database itself: the only one of a file without sub-databases). Throws
// std::runtime_error on a file that is not a readable btree or has no such sub-database.
Records read_btree(const std::string& path, const std::string& subdb);
// The same over the bytes of such a file (csrc/fuzz feeds it arbitrary input).
Records read_btree_bytes(std::string data, const std::string& subdb);

// Names of the sub-databases of the file (empty for a file without any).
std::vector<std::string> databases(const std::string& path);

// A btree file holding `records` (any order; duplicate keys refused) in sub-database `subdb`, in
// the layout Berkeley DB 4.8-5.3 writes without an environment (version 9, host byte order,
// LSNs "not logged", no checksums): master meta page, master leaf mapping the name to the
// sub-database's meta page (network byte order), that meta page, then the tree -- full leaf pages
// linked left to right, internal levels above them, items over the overflow size on overflow page
// chains. The file is written to `path`.tmp and renamed over `path`. The reference opens it as a
// wallet (src/wallet/db.cpp: Db::open(..., "main", DB_BTREE, ...)); libdb's own verifier accepts it
// (tests/test_walletdb.py).
void write_btree(const std::string& path, Records records, const std::string& subdb, uint32_t pagesize = 4096);
std::string write_btree_bytes(Records records, const std::string& subdb, uint32_t pagesize = 4096,
                              const std::string& uid = std::string());

}  // namespace bdb
}  // namespace nodexa
