// util/crc32c.h -- link-compatible replacement surface for LevelDB's crc32c.
//
// Same names, signatures and semantics as the reference header
// (util/crc32c.h:11-41), so table/format.cc:94-95, table/table_builder.cc:194-196,
// db/log_writer.cc:19,94-95, db/log_reader.cc:247-248 and
// benchmarks/db_bench.cc:2134 compile unchanged with `-I <this repo>/include`
// and link Extend from libprismdb_crc32c.so instead of util/crc32c.o.
// The batch (GPU) entry points live in prismdb_crc32c.h.
#ifndef PRISMDB_UTIL_CRC32C_H_
#define PRISMDB_UTIL_CRC32C_H_

#include <cstddef>
#include <cstdint>

namespace leveldb {
namespace crc32c {

// crc32c(A || data[0, n)) given init_crc == crc32c(A).  Out of line, exported
// as _ZN7leveldb6crc32c6ExtendEjPKcm by libprismdb_crc32c.so.
uint32_t Extend(uint32_t init_crc, const char* data, size_t n);

// crc32c(data[0, n))
inline uint32_t Value(const char* data, size_t n) { return Extend(0, data, n); }

// Stored checksums are masked so that a CRC over data that embeds CRCs stays
// well distributed: rotate right 15, add a constant.
static const uint32_t kMaskDelta = 0xa282ead8ul;

inline uint32_t Mask(uint32_t crc) { return ((crc << 17) | (crc >> 15)) + kMaskDelta; }

inline uint32_t Unmask(uint32_t masked_crc) {
  const uint32_t r = masked_crc - kMaskDelta;
  return (r << 15) | (r >> 17);
}

}  // namespace crc32c
}  // namespace leveldb

#endif  // PRISMDB_UTIL_CRC32C_H_
