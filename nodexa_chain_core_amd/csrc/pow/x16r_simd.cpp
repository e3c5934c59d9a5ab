#include "x16r_prims.hpp"
namespace nodexa {
Hash512 simd512(const u8*, size_t) { throw std::runtime_error("simd512: not implemented"); }
}
