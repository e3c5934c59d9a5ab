// AES-256 (FIPS-197) with CBC mode and PKCS#7 padding, for wallet key encryption.
//
// Parity (behaviour): CCrypter's AES-256-CBC (src/wallet/crypter.cpp, src/crypto/aes.cpp) and its
// key derivation BytesToKeySHA512AES — SHA512(passphrase || salt) iterated `rounds` times, key =
// first 32 bytes, IV = next 16. Table-driven software AES (the wallet encrypts a handful of keys;
// nothing here is hot).
#pragma once

#include <string>

#include "../util/common.hpp"

namespace nodexa {

class Aes256 {
public:
    explicit Aes256(const u8 key[32]);
    void encrypt_block(const u8 in[16], u8 out[16]) const;
    void decrypt_block(const u8 in[16], u8 out[16]) const;

private:
    u8 rk_[240];  // 15 round keys
};

// CBC with PKCS#7 padding; decrypt returns false on a bad padding.
Bytes aes256_cbc_encrypt(const u8 key[32], const u8 iv[16], const Bytes& plain);
bool aes256_cbc_decrypt(const u8 key[32], const u8 iv[16], const Bytes& cipher, Bytes& plain);
// BytesToKeySHA512AES: (key, iv) from passphrase, 8-byte salt and round count.
void bytes_to_key_sha512(const std::string& passphrase, const Bytes& salt, int rounds, u8 key[32], u8 iv[16]);

}  // namespace nodexa
