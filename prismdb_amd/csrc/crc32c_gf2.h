// crc32c_gf2.h -- CRC-32C as linear algebra over GF(2).
//
// The CRC register of LevelDB's crc32c (util/crc32c.cc:276-377) is a 32-bit
// reflected LFSR over the Castagnoli polynomial.  With the pre/post
// conditioning (util/crc32c.cc:284,376) peeled off, feeding bytes is linear:
//
//   R(r, d)          register after feeding bytes d into register r
//   R(r, d)        = shift_|d|(r) ^ R(0, d)
//   R(r, w32)      = shift_4(r ^ w)            (w = LE 32-bit word)
//   shift_n        = register advanced over n zero bytes (a 32x32 bit matrix)
//
// Everything the engine needs -- the byte table, the LDS stride tables, the
// per-lane recombination matrices and CRC combination -- is derived here from
// the polynomial; no table is copied from the reference.
#pragma once

#include <cstddef>
#include <cstdint>

namespace prismdb {
namespace gf2 {

constexpr uint32_t kPolyReflected = 0x82F63B78u;  // Castagnoli, bit-reflected
constexpr uint32_t kConditioning = 0xFFFFFFFFu;   // kCRC32Xor, util/crc32c.cc:246

// A linear operator on the register: y = XOR of col[i] over set bits i of x.
struct Op {
  uint32_t col[32];
};

inline uint32_t Apply(const Op& m, uint32_t x) {
  uint32_t y = 0;
  for (int i = 0; i < 32; ++i)
    if ((x >> i) & 1u) y ^= m.col[i];
  return y;
}

// (a o b)(x) = a(b(x))
inline Op Compose(const Op& a, const Op& b) {
  Op r;
  for (int i = 0; i < 32; ++i) r.col[i] = Apply(a, b.col[i]);
  return r;
}

inline Op Identity() {
  Op r;
  for (int i = 0; i < 32; ++i) r.col[i] = 1u << i;
  return r;
}

// One zero bit through the reflected LFSR.
inline uint32_t StepBit(uint32_t r) { return (r >> 1) ^ (kPolyReflected & (0u - (r & 1u))); }

// Register advanced over one zero byte.
inline Op ShiftOneByte() {
  Op r;
  for (int i = 0; i < 32; ++i) {
    uint32_t v = 1u << i;
    for (int k = 0; k < 8; ++k) v = StepBit(v);
    r.col[i] = v;
  }
  return r;
}

// Register advanced over n zero bytes (square-and-multiply, O(log n) compositions).
inline Op ShiftBytes(uint64_t n) {
  Op result = Identity();
  Op power = ShiftOneByte();
  while (n != 0) {
    if (n & 1u) result = Compose(power, result);
    power = Compose(power, power);
    n >>= 1;
  }
  return result;
}

// Sarwate byte table: table[b] = shift_1(b), so that feeding byte x into r is
// r' = table[(r ^ x) & 0xff] ^ (r >> 8).
inline void ByteTable(uint32_t table[256]) {
  for (uint32_t b = 0; b < 256; ++b) {
    uint32_t v = b;
    for (int k = 0; k < 8; ++k) v = StepBit(v);
    table[b] = v;
  }
}

// Stride tables: t[k][b] = shift_S(b << 8k), so that shift_S(x) is
// t[0][x&0xff] ^ t[1][(x>>8)&0xff] ^ t[2][(x>>16)&0xff] ^ t[3][x>>24].
// (The reference's kStrideExtensionTable0..3 are this with S = 16 and the byte
// order reversed; util/crc32c.cc:65-243.)
inline void StrideTables(uint64_t stride_bytes, uint32_t t[4][256]) {
  const Op s = ShiftBytes(stride_bytes);
  for (int k = 0; k < 4; ++k)
    for (uint32_t b = 0; b < 256; ++b) t[k][b] = Apply(s, b << (8 * k));
}

// crc32c of A||B from crc32c(A), crc32c(B) and |B| (conditioned values, as
// returned by crc32c::Value/Extend).  Used to stitch split spans together.
inline uint32_t Combine(uint32_t crc_a, uint32_t crc_b, uint64_t len_b) {
  // Unconditioned: R(ra, B) = shift_|B|(ra) ^ R(0, B); R(0,B) = (crc_b ^ C) ^ shift_|B|(C).
  const Op s = ShiftBytes(len_b);
  uint32_t ra = crc_a ^ kConditioning;
  uint32_t rb = crc_b ^ kConditioning ^ Apply(s, kConditioning);
  return (Apply(s, ra) ^ rb) ^ kConditioning;
}

}  // namespace gf2
}  // namespace prismdb
