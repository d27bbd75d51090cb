// crc32c_host.cc -- the per-call CPU surface: leveldb::crc32c::Extend and the
// leveldb_crc32c_{extend,value,mask,unmask,combine,accelerated} C entry points.
//
// Per the drop-in contract, single-block Extend stays on the host (a GPU launch
// per 4 KiB call would lose).  Like the reference (util/crc32c.cc:265-280 +
// port::AcceleratedCRC32C, port/port_stdcxx.h:141-151) it picks a hardware
// path once, gated by the same known-answer self-test, and otherwise runs a
// portable table-driven loop (slicing-by-8 over tables derived in
// crc32c_gf2.h).  This is product code for the per-call surface; it is not the
// batch engine's fallback -- the batch entry points never run on the CPU.
#include <cstddef>
#include <cstdint>
#include <cstring>

#include "../../include/prismdb_crc32c.h"
#include "../../include/util/crc32c.h"
#include "crc32c_gf2.h"

namespace {

struct HostTables {
  uint32_t s8[8][256];  // s8[k][b] = shift_{k+1}(b): byte b followed by k zero bytes
  HostTables() {
    for (int k = 0; k < 8; ++k) {
      const prismdb::gf2::Op op = prismdb::gf2::ShiftBytes((uint64_t)k + 1);
      for (uint32_t b = 0; b < 256; ++b) s8[k][b] = prismdb::gf2::Apply(op, b);
    }
  }
};

const HostTables& Tables() {
  static const HostTables t;  // thread-safe init (C++11 magic statics)
  return t;
}

inline uint32_t LoadLE32(const uint8_t* p) {
  return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}

// Portable path: byte steps to 8-byte alignment, 8 bytes per step through the
// eight slice tables, byte steps for the tail.
uint32_t ExtendPortable(uint32_t crc, const uint8_t* p, size_t n) {
  const HostTables& t = Tables();
  uint32_t r = crc ^ prismdb::gf2::kConditioning;
  while (n != 0 && (reinterpret_cast<uintptr_t>(p) & 7u) != 0) {
    r = t.s8[0][(r ^ *p++) & 0xffu] ^ (r >> 8);
    --n;
  }
  while (n >= 8) {
    const uint32_t lo = LoadLE32(p) ^ r;
    const uint32_t hi = LoadLE32(p + 4);
    r = t.s8[7][lo & 0xff] ^ t.s8[6][(lo >> 8) & 0xff] ^ t.s8[5][(lo >> 16) & 0xff] ^
        t.s8[4][lo >> 24] ^ t.s8[3][hi & 0xff] ^ t.s8[2][(hi >> 8) & 0xff] ^
        t.s8[1][(hi >> 16) & 0xff] ^ t.s8[0][hi >> 24];
    p += 8;
    n -= 8;
  }
  while (n-- != 0) r = t.s8[0][(r ^ *p++) & 0xffu] ^ (r >> 8);
  return r ^ prismdb::gf2::kConditioning;
}

#if defined(__x86_64__)
// SSE4.2 CRC32 instruction computes exactly the reflected Castagnoli step.
__attribute__((target("sse4.2"))) uint32_t ExtendSse42(uint32_t crc, const uint8_t* p, size_t n) {
  uint64_t r = crc ^ prismdb::gf2::kConditioning;
  while (n != 0 && (reinterpret_cast<uintptr_t>(p) & 7u) != 0) {
    r = __builtin_ia32_crc32qi((uint32_t)r, *p++);
    --n;
  }
  while (n >= 8) {
    uint64_t w;
    std::memcpy(&w, p, 8);
    r = __builtin_ia32_crc32di(r, w);
    p += 8;
    n -= 8;
  }
  while (n-- != 0) r = __builtin_ia32_crc32qi((uint32_t)r, *p++);
  return (uint32_t)r ^ prismdb::gf2::kConditioning;
}
#endif

using ExtendFn = uint32_t (*)(uint32_t, const uint8_t*, size_t);

// Known-answer gate, as util/crc32c.cc:267-274: accept the hardware path only
// if it reproduces crc32c("TestCRCBuffer") == 0xdcbc59fa.
ExtendFn PickExtend() {
#if defined(__x86_64__)
  __builtin_cpu_init();
  if (__builtin_cpu_supports("sse4.2")) {
    static const char kTest[] = "TestCRCBuffer";
    if (ExtendSse42(0, reinterpret_cast<const uint8_t*>(kTest), sizeof(kTest) - 1) == 0xdcbc59fau)
      return &ExtendSse42;
  }
#endif
  return &ExtendPortable;
}

ExtendFn Impl() {
  static const ExtendFn fn = PickExtend();
  return fn;
}

}  // namespace

namespace leveldb {
namespace crc32c {

__attribute__((visibility("default"))) uint32_t Extend(uint32_t init_crc, const char* data,
                                                       size_t n) {
  return Impl()(init_crc, reinterpret_cast<const uint8_t*>(data), n);
}

}  // namespace crc32c
}  // namespace leveldb

extern "C" {

uint32_t leveldb_crc32c_extend(uint32_t init_crc, const char* data, size_t n) {
  return leveldb::crc32c::Extend(init_crc, data, n);
}

uint32_t leveldb_crc32c_value(const char* data, size_t n) { return leveldb::crc32c::Value(data, n); }

uint32_t leveldb_crc32c_mask(uint32_t crc) { return leveldb::crc32c::Mask(crc); }

uint32_t leveldb_crc32c_unmask(uint32_t masked_crc) { return leveldb::crc32c::Unmask(masked_crc); }

uint32_t leveldb_crc32c_combine(uint32_t crc_a, uint32_t crc_b, uint64_t len_b) {
  return prismdb::gf2::Combine(crc_a, crc_b, len_b);
}

int leveldb_crc32c_accelerated(void) { return Impl() != &ExtendPortable ? 1 : 0; }

// Portable path exposed for tests (so both host paths are parity-checked).
uint32_t prismdb_crc32c_extend_portable(uint32_t init_crc, const char* data, size_t n) {
  return ExtendPortable(init_crc, reinterpret_cast<const uint8_t*>(data), n);
}

}  // extern "C"
