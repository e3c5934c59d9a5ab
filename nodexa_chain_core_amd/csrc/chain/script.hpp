// Minimal script building + Base58Check addresses (what block templates need).
//
// Parity: CScript push rules incl. CScriptNum encoding and the small-int
// opcodes (src/script/script.h: push_int64, operator<<(CScriptNum),
// operator<<(vector)), Base58Check (src/base58.cpp), P2PKH / P2SH destination
// scripts (GetScriptForDestination). Full script *evaluation* is out of scope
// for the PoW engine (DEFER).
#pragma once

#include "../util/common.hpp"

namespace nodexa {

enum Opcode : u8 {
    OP_0 = 0x00, OP_PUSHDATA1 = 0x4c, OP_PUSHDATA2 = 0x4d, OP_PUSHDATA4 = 0x4e, OP_1NEGATE = 0x4f,
    OP_1 = 0x51, OP_16 = 0x60, OP_RETURN = 0x6a, OP_DUP = 0x76, OP_EQUAL = 0x87, OP_EQUALVERIFY = 0x88,
    OP_HASH160 = 0xa9, OP_CHECKSIG = 0xac, OP_TRUE = 0x51,
};

class ScriptBuilder {
public:
    Bytes s;
    ScriptBuilder& op(u8 o) { s.push_back(o); return *this; }
    ScriptBuilder& push_data(const Bytes& d);
    ScriptBuilder& push_int(int64_t v);       // CScript << int64_t (small ints -> OP_n)
    ScriptBuilder& push_num(int64_t v);       // CScript << CScriptNum (always data push)
    static Bytes scriptnum(int64_t v);        // CScriptNum::serialize
};

std::string base58_encode(const Bytes& data);
bool base58_decode(const std::string& s, Bytes& out);
std::string base58check_encode(const Bytes& payload);
bool base58check_decode(const std::string& s, Bytes& payload);

// scriptPubKey for a Base58 address given the network's P2PKH / P2SH version
// bytes; returns false if the address is invalid for that network.
bool address_to_script(const std::string& addr, u8 pubkey_prefix, u8 script_prefix, Bytes& script);
std::string script_to_address(const Bytes& script, u8 pubkey_prefix, u8 script_prefix);  // "" if not P2PKH/P2SH

void hash160(const u8* data, size_t n, u8 out[20]);  // RIPEMD160(SHA256(x))
void ripemd160(const u8* data, size_t n, u8 out[20]);

}  // namespace nodexa
