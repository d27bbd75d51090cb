// ref_shim.cc -- TEST INFRASTRUCTURE ONLY (oracle/_ref build: not part of the
// product library; the built .so travels to the GPU box with the tree, where
// bench.py's cpu_baseline loads it as the reference CPU path).
//
// A thin extern "C" face over the reference's own crc32c::Extend, compiled
// together with /root/reference/util/crc32c.cc by oracle/Makefile into
// oracle/_ref/libref_crc32c.so.  Used (a) by oracle/gen_golden.py to produce
// golden vectors from the reference itself, and (b) by bench.py's cpu_baseline
// leg to time the reference crc32c::Value on the host cores.
#include <chrono>
#include <cstddef>
#include <cstdint>
#include <thread>
#include <vector>

#include "util/crc32c.h"  // resolved under /root/reference at build time

extern "C" {

uint32_t ref_crc32c_extend(uint32_t init, const char* data, size_t n) {
  return leveldb::crc32c::Extend(init, data, n);
}

uint32_t ref_crc32c_value(const char* data, size_t n) { return leveldb::crc32c::Value(data, n); }

uint32_t ref_crc32c_mask(uint32_t c) { return leveldb::crc32c::Mask(c); }

uint32_t ref_crc32c_unmask(uint32_t c) { return leveldb::crc32c::Unmask(c); }

// Which path the reference took: 1 = port::AcceleratedCRC32C (HAVE_CRC32C),
// 0 = portable slicing-by-4 (util/crc32c.cc:267-280).  This build never defines
// HAVE_CRC32C, so it reports 0.
int ref_crc32c_accelerated(void) {
#if defined(HAVE_CRC32C) && HAVE_CRC32C
  return 1;
#else
  return 0;
#endif
}

// Times crc32c::Value over nblocks blocks of block_len bytes at `stride`
// (db_bench's Crc32c loop, benchmarks/db_bench.cc:2126-2142, but over distinct
// buffers instead of one L1-hot buffer), `passes` times, on `threads` threads.
// Writes the per-block CRCs of the last pass into out (may be null).
// Returns wall seconds.
double ref_crc32c_time_blocks(const char* base, size_t stride, size_t block_len, size_t nblocks,
                              int threads, int passes, uint32_t* out) {
  if (threads < 1) threads = 1;
  auto t0 = std::chrono::steady_clock::now();
  std::vector<std::thread> pool;
  for (int t = 0; t < threads; ++t) {
    pool.emplace_back([=]() {
      size_t lo = nblocks * (size_t)t / (size_t)threads;
      size_t hi = nblocks * (size_t)(t + 1) / (size_t)threads;
      uint32_t sink = 0;
      for (int p = 0; p < passes; ++p) {
        for (size_t i = lo; i < hi; ++i) {
          uint32_t c = leveldb::crc32c::Value(base + i * stride, block_len);
          if (out != nullptr && p == passes - 1) out[i] = c;
          sink ^= c;
        }
      }
      volatile uint32_t keep = sink;
      (void)keep;
    });
  }
  for (auto& th : pool) th.join();
  auto t1 = std::chrono::steady_clock::now();
  return std::chrono::duration<double>(t1 - t0).count();
}

}  // extern "C"
