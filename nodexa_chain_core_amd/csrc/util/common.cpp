#include "common.hpp"

namespace nodexa {

std::string hex_encode(const u8* data, size_t n) {
    static const char* digits = "0123456789abcdef";
    std::string out(n * 2, '0');
    for (size_t i = 0; i < n; ++i) {
        out[2 * i] = digits[data[i] >> 4];
        out[2 * i + 1] = digits[data[i] & 15];
    }
    return out;
}

static int hex_val(char c) {
    if (c >= '0' && c <= '9') return c - '0';
    if (c >= 'a' && c <= 'f') return c - 'a' + 10;
    if (c >= 'A' && c <= 'F') return c - 'A' + 10;
    return -1;
}

Bytes hex_decode(const std::string& hex_in) {
    std::string hex = hex_in;
    if (hex.size() >= 2 && hex[0] == '0' && (hex[1] == 'x' || hex[1] == 'X')) hex = hex.substr(2);
    if (hex.size() % 2) throw std::invalid_argument("hex string has odd length");
    Bytes out(hex.size() / 2);
    for (size_t i = 0; i < out.size(); ++i) {
        int h = hex_val(hex[2 * i]), l = hex_val(hex[2 * i + 1]);
        if (h < 0 || l < 0) throw std::invalid_argument("invalid hex digit");
        out[i] = u8((h << 4) | l);
    }
    return out;
}

}  // namespace nodexa
