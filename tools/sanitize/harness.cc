// harness.cc -- host-side robustness driver for the sanitizer builds
// (tools/sanitize/Makefile, tests/test_sanitizers.py).  CPU only: no GPU is
// needed or touched beyond the runtime's "no device" answer.
//
//   harness sst   <file.ldb> <iters> <seed>   seeded mutations of an SST image
//                                             through leveldb_sst_block_spans
//   harness log   <file.bin> <iters> <seed>   seeded mutations of a log file
//                                             through leveldb_log_scan/replay
//   harness abi                               every C-ABI entry point with bad
//                                             arguments (EINVAL) and valid ones
//                                             (EDEVICE without a GPU)
//   harness threads <nthreads> <iters> <sst>  the C ABI, the host Extend and the
//                                             SST walker from many threads at once
//
// Every mutated image is copied into a heap block of exactly its size, so an
// out-of-bounds read by the walker or the scanner is an ASan report, not a
// silent read of the neighbouring bytes.  Exit status 0 = clean; a failed
// check prints what and aborts.
#include <atomic>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <thread>
#include <vector>

#include "../../include/prismdb_crc32c.h"
#include "../../include/prismdb_log.h"
#include "../../include/prismdb_sst.h"

// test hooks exported by the library (not in the public headers)
extern "C" {
uint32_t prismdb_crc32c_extend_portable(uint32_t init_crc, const char* data, size_t n);
void prismdb_crc32c_force_generic(int on);
uint64_t prismdb_crc32c_direct_max(uint64_t n);
int prismdb_test_hooks_enabled(void);
}

#define CHECK(c)                                                              \
  do {                                                                        \
    if (!(c)) {                                                               \
      std::fprintf(stderr, "CHECK failed at %s:%d: %s\n", __FILE__, __LINE__, #c); \
      std::abort();                                                           \
    }                                                                         \
  } while (0)

namespace {

std::vector<uint8_t> ReadFile(const char* path) {
  std::FILE* f = std::fopen(path, "rb");
  CHECK(f != nullptr);
  std::vector<uint8_t> v;
  uint8_t buf[65536];
  size_t n;
  while ((n = std::fread(buf, 1, sizeof buf, f)) > 0) v.insert(v.end(), buf, buf + n);
  std::fclose(f);
  return v;
}

uint32_t Le32(const uint8_t* p) { return p[0] | (p[1] << 8) | (p[2] << 16) | ((uint32_t)p[3] << 24); }

// One mutation of `img`: bit flips, a truncation, a run of varint
// continuation bytes (an overlong / overflowing varint) at a handle-heavy
// spot, or a random byte splat.
void Mutate(std::vector<uint8_t>& img, std::mt19937_64& rng, size_t hot_lo, size_t hot_hi) {
  if (img.empty()) return;
  switch (rng() % 5) {
    case 0: {  // 1-8 bit flips anywhere
      const int k = 1 + (int)(rng() % 8);
      for (int i = 0; i < k; ++i) img[rng() % img.size()] ^= (uint8_t)(1u << (rng() % 8));
      break;
    }
    case 1:  // truncation
      img.resize(rng() % img.size());
      break;
    case 2: {  // varint overflow in the handle area (footer / index block)
      if (hot_hi > img.size()) hot_hi = img.size();
      if (hot_lo >= hot_hi) hot_lo = 0;
      const size_t at = hot_lo + rng() % (hot_hi - hot_lo);
      const size_t len = 5 + rng() % 8;
      for (size_t i = at; i < img.size() && i < at + len; ++i) img[i] = 0x80 | (uint8_t)(rng() & 0x7F);
      if (rng() % 2 && at + len < img.size()) img[at + len] = 0x7F;
      break;
    }
    case 3: {  // random bytes in the handle area
      if (hot_hi > img.size()) hot_hi = img.size();
      if (hot_lo >= hot_hi) hot_lo = 0;
      for (int i = 0; i < 16; ++i) img[hot_lo + rng() % (hot_hi - hot_lo)] = (uint8_t)rng();
      break;
    }
    default: {  // a splat of 0xFF
      const size_t at = rng() % img.size();
      for (size_t i = at; i < img.size() && i < at + 1 + rng() % 64; ++i) img[i] = 0xFF;
      break;
    }
  }
}

int RunSst(const char* path, int iters, uint64_t seed) {
  const std::vector<uint8_t> base = ReadFile(path);
  std::mt19937_64 rng(seed);
  size_t ok = 0, corrupt = 0, unsupported = 0;
  for (int it = 0; it < iters; ++it) {
    std::vector<uint8_t> img = base;
    const int rounds = 1 + (int)(rng() % 3);
    for (int r = 0; r < rounds; ++r) Mutate(img, rng, img.size() > 4096 ? img.size() - 4096 : 0, img.size());
    // exactly-sized heap copy (ASan red zone right after the last byte)
    char* f = static_cast<char*>(std::malloc(img.size() ? img.size() : 1));
    if (!img.empty()) std::memcpy(f, img.data(), img.size());
    size_t n = 0;
    int rc = leveldb_sst_block_spans(f, img.size(), nullptr, nullptr, nullptr, 0, &n);
    if (rc == 0 || rc == PRISMDB_SST_ECAPACITY) {
      std::vector<uint64_t> off(n + 1);
      std::vector<uint32_t> len(n + 1);
      std::vector<uint8_t> kind(n + 1);
      size_t n2 = 0;
      rc = leveldb_sst_block_spans(f, img.size(), off.data(), len.data(), kind.data(), n, &n2);
      CHECK(rc == 0 && n2 == n);
      for (size_t i = 0; i < n; ++i) {
        // every listed span and its trailer lie inside the file
        CHECK(off[i] <= img.size() && len[i] <= img.size() - off[i] && img.size() - off[i] - len[i] >= 4);
        CHECK(kind[i] <= PRISMDB_SST_INDEX);
        const uint32_t c = leveldb_crc32c_value(f + off[i], len[i]);
        (void)(c == leveldb_crc32c_unmask(Le32(reinterpret_cast<const uint8_t*>(f) + off[i] + len[i])));
      }
      ++ok;
    } else {
      CHECK(rc == PRISMDB_SST_ECORRUPT || rc == PRISMDB_SST_EUNSUPPORTED);
      CHECK(std::strlen(leveldb_sst_last_error()) > 0);
      (rc == PRISMDB_SST_ECORRUPT ? corrupt : unsupported)++;
    }
    std::free(f);
  }
  std::printf("sst: %d mutants: %zu listed, %zu corrupt, %zu unsupported\n", iters, ok, corrupt, unsupported);
  return 0;
}

int RunLog(const char* path, int iters, uint64_t seed) {
  const std::vector<uint8_t> base = ReadFile(path);
  std::mt19937_64 rng(seed);
  size_t recs = 0, drops = 0;
  for (int it = 0; it < iters; ++it) {
    std::vector<uint8_t> img = base;
    if (it > 0) {
      const int rounds = 1 + (int)(rng() % 3);
      for (int r = 0; r < rounds; ++r) Mutate(img, rng, 0, img.size());
    }
    const size_t size = img.size();
    uint8_t* f = static_cast<uint8_t*>(std::malloc(size ? size : 1));
    if (size) std::memcpy(f, img.data(), size);
    const uint64_t initial = (rng() % 4 == 0 && size) ? rng() % (size + 100) : 0;
    const size_t cap = size / 7 + 1;
    std::vector<uint64_t> roff(cap);
    std::vector<uint32_t> rlen(cap);
    size_t n = 0;
    int rc = leveldb_log_scan(f, size, initial, roff.data(), rlen.data(), cap, &n);
    CHECK(rc == 0 && n <= cap);
    std::vector<uint8_t> bad(n ? n : 1);
    for (size_t i = 0; i < n; ++i) {
      CHECK(roff[i] + 7 + rlen[i] <= size);
      const uint32_t c = leveldb_crc32c_value(reinterpret_cast<const char*>(f) + roff[i] + 6, 1 + rlen[i]);
      bad[i] = c != leveldb_crc32c_unmask(Le32(f + roff[i])) ? 1 : 0;
    }
    const size_t dcap = 2 * (n + size / 32768 + 2);
    std::vector<uint64_t> rec_off(n + 1), drop_bytes(dcap);
    std::vector<uint32_t> rec_first(n + 1), rec_nfrag(n + 1), frag(n + 1);
    std::vector<int32_t> drop_reason(dcap);
    leveldb_log_replay_out o{};
    o.record_offset = rec_off.data();
    o.record_first = rec_first.data();
    o.record_nfrag = rec_nfrag.data();
    o.record_cap = n;
    o.fragment = frag.data();
    o.fragment_cap = n;
    o.drop_bytes = drop_bytes.data();
    o.drop_reason = drop_reason.data();
    o.drop_cap = dcap;
    const int checksum = (int)(rng() % 2);
    rc = leveldb_log_replay(f, size, initial, checksum, roff.data(), rlen.data(), checksum ? bad.data() : nullptr,
                            n, &o);
    CHECK(rc == 0);
    for (size_t r = 0; r < o.n_records; ++r) {
      CHECK(rec_first[r] + rec_nfrag[r] <= o.n_fragments);
      for (uint32_t k = 0; k < rec_nfrag[r]; ++k) CHECK(frag[rec_first[r] + k] < n);
    }
    char text[96];
    for (size_t d = 0; d < o.n_drops; ++d) CHECK(std::strlen(leveldb_log_reason(drop_reason[d], text, sizeof text)) > 0);
    recs += o.n_records;
    drops += o.n_drops;
    // a scan that disagrees with the file is refused, not trusted
    if (n > 0) {
      std::vector<uint32_t> wrong(rlen.begin(), rlen.begin() + n);
      wrong[n - 1] += 1u << 20;
      rc = leveldb_log_replay(f, size, initial, checksum, roff.data(), wrong.data(), checksum ? bad.data() : nullptr,
                              n, &o);
      CHECK(rc == LEVELDB_LOG_EINVAL || rc == 0);
    }
    std::free(f);
  }
  std::printf("log: %d mutants: %zu records, %zu drops\n", iters, recs, drops);
  return 0;
}

// Every batch entry point: bad arguments -> EINVAL with a message; valid
// arguments -> EDEVICE (no GPU here) with a message, never a crash.
int RunAbi(bool expect_no_device) {
  std::vector<uint8_t> data(1 << 16);
  std::vector<uint64_t> off = {0, 4096, 8192, 12288};
  std::vector<uint32_t> len = {4000, 4000, 4000, 4000};
  std::vector<uint32_t> out(4);
  std::vector<uint8_t> mm(4);
  const void* d = data.data();
  CHECK(leveldb_crc32c_batch(nullptr, nullptr, nullptr, nullptr, 0, nullptr, nullptr, 0, nullptr) == 0);
  CHECK(leveldb_crc32c_batch(d, nullptr, len.data(), nullptr, 4, out.data(), nullptr, 0, nullptr) ==
        PRISMDB_CRC32C_EINVAL);
  CHECK(leveldb_crc32c_batch(d, off.data(), len.data(), nullptr, 4, out.data(), nullptr, 0x80, nullptr) ==
        PRISMDB_CRC32C_EINVAL);
  CHECK(leveldb_crc32c_batch(d, off.data(), len.data(), nullptr, 4, out.data(), mm.data(),
                             PRISMDB_CRC32C_WRITE_TRAILER, nullptr) == PRISMDB_CRC32C_EINVAL);
  CHECK(leveldb_crc32c_batch_fixed(nullptr, 4096, 4096, 4, 0, out.data(), nullptr, 0, nullptr) ==
        PRISMDB_CRC32C_EINVAL);
  CHECK(leveldb_crc32c_batch_fixed(d, 1ull << 33, 1ull << 32, 1, 0, out.data(), nullptr, 0, nullptr) ==
        PRISMDB_CRC32C_EINVAL);
  std::vector<uint64_t> rev(off.rbegin(), off.rend());
  CHECK(leveldb_crc32c_batch_host(d, rev.data(), len.data(), nullptr, 4, out.data(), nullptr, 0) ==
        PRISMDB_CRC32C_EINVAL);
  int devs[2] = {0, 0};
  const void* bases[2] = {d, d};
  const uint64_t* offs[2] = {off.data(), off.data()};
  const uint32_t* lens[2] = {len.data(), len.data()};
  size_t ns[2] = {4, 4};
  CHECK(leveldb_crc32c_batch_multi(2, devs, bases, offs, lens, nullptr, ns, out.data(), nullptr, 0, nullptr) ==
        PRISMDB_CRC32C_EINVAL);
  CHECK(leveldb_crc32c_batch_multi(0, devs, bases, offs, lens, nullptr, ns, out.data(), nullptr, 0, nullptr) ==
        PRISMDB_CRC32C_EINVAL);
  CHECK(std::strlen(leveldb_crc32c_last_error()) > 0);
  if (expect_no_device) {
    CHECK(leveldb_crc32c_batch(d, off.data(), len.data(), nullptr, 4, out.data(), nullptr, 0, nullptr) ==
          PRISMDB_CRC32C_EDEVICE);
    CHECK(leveldb_crc32c_batch_fixed(d, 4096, 4000, 4, 0, out.data(), nullptr, 0, nullptr) == PRISMDB_CRC32C_EDEVICE);
    CHECK(leveldb_crc32c_batch_host(d, off.data(), len.data(), nullptr, 4, out.data(), nullptr, 0) ==
          PRISMDB_CRC32C_EDEVICE);
    CHECK(leveldb_crc32c_device_init(0) == PRISMDB_CRC32C_EDEVICE);
    CHECK(leveldb_crc32c_batch_multi(1, devs, bases, offs, lens, nullptr, ns, out.data(), nullptr, 0, nullptr) ==
          PRISMDB_CRC32C_EDEVICE);
    CHECK(std::strlen(leveldb_crc32c_last_error()) > 0);
  }
  // host surface
  CHECK(leveldb_crc32c_value("123456789", 9) == 0xE3069283u);
  CHECK(leveldb_crc32c_extend(leveldb_crc32c_value("1234", 4), "56789", 5) == 0xE3069283u);
  CHECK(leveldb_crc32c_unmask(leveldb_crc32c_mask(0xDEADBEEFu)) == 0xDEADBEEFu);
  CHECK(leveldb_crc32c_combine(leveldb_crc32c_value("1234", 4), leveldb_crc32c_value("56789", 5), 5) == 0xE3069283u);
  for (size_t n = 0; n < 300; ++n) {  // every alignment and tail of the host Extend on exact-size blocks
    char* b = static_cast<char*>(std::malloc(n ? n : 1));
    for (size_t i = 0; i < n; ++i) b[i] = (char)(i * 131 + 7);
    const uint32_t a = leveldb_crc32c_value(b, n);
    const uint32_t p = prismdb_crc32c_extend_portable(0, b, n);
    CHECK(a == p);
    std::free(b);
  }
  std::printf("abi: ok\n");
  return 0;
}

int RunThreads(int nthreads, int iters, const char* sst) {
  // the setters below store only with the test hooks on (read once, at the
  // first hook call): without this the run would race nothing
  setenv("PRISMDB_ENABLE_TEST_HOOKS", "1", 1);
  CHECK(prismdb_test_hooks_enabled() == 1);
  const std::vector<uint8_t> img = ReadFile(sst);
  std::atomic<int> failures{0};
  std::vector<std::thread> ts;
  for (int t = 0; t < nthreads; ++t) {
    ts.emplace_back([&, t] {
      std::vector<uint8_t> data(1 << 14, (uint8_t)t);
      std::vector<uint64_t> off = {0, 4096};
      std::vector<uint32_t> len = {4096, 4000};
      std::vector<uint32_t> out(2);
      std::vector<uint64_t> soff(4096);
      std::vector<uint32_t> slen(4096);
      std::vector<uint8_t> kind(4096);
      for (int i = 0; i < iters; ++i) {
        // argument errors and the no-device error, each with its thread-local message
        if (leveldb_crc32c_batch(data.data(), nullptr, len.data(), nullptr, 2, out.data(), nullptr, 0, nullptr) !=
            PRISMDB_CRC32C_EINVAL)
          failures++;
        if (std::strstr(leveldb_crc32c_last_error(), "non-NULL") == nullptr) failures++;
        const int rc = leveldb_crc32c_batch(data.data(), off.data(), len.data(), nullptr, 2, out.data(), nullptr, 0,
                                            nullptr);
        if (rc != PRISMDB_CRC32C_EDEVICE && rc != 0) failures++;
        if (leveldb_crc32c_batch_host(data.data(), off.data(), len.data(), nullptr, 2, out.data(), nullptr, 0) == 1)
          failures++;
        // the per-call host surface and the test hooks (atomics)
        if (leveldb_crc32c_value(reinterpret_cast<const char*>(data.data()), data.size()) !=
            prismdb_crc32c_extend_portable(0, reinterpret_cast<const char*>(data.data()), data.size()))
          failures++;
        prismdb_crc32c_force_generic(0);
        prismdb_crc32c_direct_max(prismdb_crc32c_direct_max(1u << 17));
        // the SST walker
        size_t n = 0;
        if (leveldb_sst_block_spans(reinterpret_cast<const char*>(img.data()), img.size(), soff.data(), slen.data(),
                                    kind.data(), soff.size(), &n) != 0)
          failures++;
      }
    });
  }
  for (auto& th : ts) th.join();
  std::printf("threads: %d x %d iterations, %d failures\n", nthreads, iters, failures.load());
  CHECK(failures.load() == 0);
  return 0;
}

}  // namespace

int main(int argc, char** argv) {
  if (argc < 2) {
    std::fprintf(stderr, "usage: harness sst|log|abi|threads ...\n");
    return 2;
  }
  const std::string mode = argv[1];
  if (mode == "sst" && argc == 5) return RunSst(argv[2], std::atoi(argv[3]), std::strtoull(argv[4], nullptr, 0));
  if (mode == "log" && argc == 5) return RunLog(argv[2], std::atoi(argv[3]), std::strtoull(argv[4], nullptr, 0));
  if (mode == "abi") return RunAbi(argc > 2 && std::string(argv[2]) == "nodevice");
  if (mode == "threads" && argc == 5) return RunThreads(std::atoi(argv[2]), std::atoi(argv[3]), argv[4]);
  std::fprintf(stderr, "bad arguments\n");
  return 2;
}
