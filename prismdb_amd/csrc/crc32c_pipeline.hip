// crc32c_pipeline.hip -- host-resident batches.
//
// PrismDB's blocks start and end in host memory: SST file pages read with
// pread during compaction (util/env_posix.cc:172-208) and blocks appended to a
// 32 MiB write buffer (:279-309).  leveldb_crc32c_batch_host streams such a
// batch through the device: spans are cut into chunks of <= kChunkBytes of
// consecutive file bytes; each chunk goes host -> (pinned staging, if the
// source is pageable) -> H2D -> batch kernel -> D2H of the 4-byte results, on
// kDepth streams so copies in both directions overlap the kernels.  The call
// is synchronous (like ReadBlock) and thread-safe: every calling thread gets
// its own staging ring per device.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <map>
#include <memory>
#include <string>
#include <vector>

#include "../../include/prismdb_crc32c.h"

namespace prismdb {
void SetLastError(const std::string& msg);  // crc32c_capi.hip: leveldb_crc32c_last_error()
}

namespace {

constexpr size_t kChunkBytes = 64ull << 20;  // one 64 MiB SST (include/leveldb/options.h:117)
constexpr size_t kChunkSpans = 1u << 16;     // descriptors per chunk
constexpr int kDepth = 3;

int PipeFail(int code, const std::string& msg) {
  prismdb::SetLastError(msg);
  return code;
}

struct Slot {
  hipStream_t stream = nullptr;
  hipEvent_t done = nullptr;
  uint8_t* h_stage = nullptr;  // pinned, kChunkBytes + 8
  uint8_t* d_data = nullptr;   // kChunkBytes + 8
  uint64_t* h_off = nullptr;   // pinned descriptors
  uint32_t* h_len = nullptr;
  uint32_t* h_init = nullptr;
  uint64_t* d_off = nullptr;
  uint32_t* d_len = nullptr;
  uint32_t* d_init = nullptr;
  uint32_t* d_out = nullptr;
  uint8_t* d_mm = nullptr;
  uint32_t* h_out = nullptr;   // pinned results
  uint8_t* h_mm = nullptr;
  // pending chunk
  bool busy = false;
  size_t first = 0, count = 0;
};

struct Ring {
  Slot slot[kDepth];
  bool ok = false;
  ~Ring() {
    for (Slot& s : slot) {
      if (s.stream) hipStreamSynchronize(s.stream);
      hipHostFree(s.h_stage);
      hipHostFree(s.h_off);
      hipHostFree(s.h_out);
      hipFree(s.d_data);
      hipFree(s.d_off);
      if (s.done) hipEventDestroy(s.done);
      if (s.stream) hipStreamDestroy(s.stream);
    }
  }
};

int MakeRing(Ring& r) {
  for (Slot& s : r.slot) {
    hipError_t e = hipStreamCreateWithFlags(&s.stream, hipStreamNonBlocking);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&s.done, hipEventDisableTiming);
    if (e == hipSuccess) e = hipHostMalloc(reinterpret_cast<void**>(&s.h_stage), kChunkBytes + 8);
    if (e == hipSuccess)
      e = hipHostMalloc(reinterpret_cast<void**>(&s.h_off), kChunkSpans * (8 + 4 + 4));
    if (e == hipSuccess) e = hipHostMalloc(reinterpret_cast<void**>(&s.h_out), kChunkSpans * (4 + 1));
    if (e == hipSuccess) e = hipMalloc(reinterpret_cast<void**>(&s.d_data), kChunkBytes + 8);
    if (e == hipSuccess) e = hipMalloc(reinterpret_cast<void**>(&s.d_off), kChunkSpans * (8 + 4 + 4 + 4 + 1));
    if (e != hipSuccess) return PipeFail(PRISMDB_CRC32C_EDEVICE, std::string("pipeline setup: ") + hipGetErrorString(e));
    s.h_len = reinterpret_cast<uint32_t*>(s.h_off + kChunkSpans);
    s.h_init = s.h_len + kChunkSpans;
    s.h_mm = reinterpret_cast<uint8_t*>(s.h_out + kChunkSpans);
    s.d_len = reinterpret_cast<uint32_t*>(s.d_off + kChunkSpans);
    s.d_init = s.d_len + kChunkSpans;
    s.d_out = s.d_init + kChunkSpans;
    s.d_mm = reinterpret_cast<uint8_t*>(s.d_out + kChunkSpans);
  }
  r.ok = true;
  return 0;
}

Ring* GetRing(int& rc) {
  thread_local std::map<int, std::unique_ptr<Ring>> rings;
  int dev = 0;
  hipGetDevice(&dev);
  std::unique_ptr<Ring>& r = rings[dev];
  if (!r) {
    r.reset(new Ring);
    rc = MakeRing(*r);
    if (rc != 0) {
      r.reset();
      return nullptr;
    }
  }
  rc = 0;
  return r.get();
}

bool IsPinned(const void* p) {
  hipPointerAttribute_t a;
  if (hipPointerGetAttributes(&a, p) != hipSuccess) {
    (void)hipGetLastError();  // clear the sticky "invalid value" for pageable memory
    return false;
  }
  return a.type == hipMemoryTypeHost;
}

}  // namespace

extern "C" {

int leveldb_crc32c_batch_host(const void* host_base, const uint64_t* off, const uint32_t* len,
                              const uint32_t* init, size_t n, uint32_t* out, uint8_t* mismatch,
                              uint32_t flags) {
  if (n == 0) return 0;
  if (host_base == nullptr || off == nullptr || len == nullptr)
    return PipeFail(PRISMDB_CRC32C_EINVAL, "host_base/off/len must be non-NULL");
  if (flags & ~(PRISMDB_CRC32C_MASK | PRISMDB_CRC32C_LOG_HEADER))
    return PipeFail(PRISMDB_CRC32C_EINVAL, "host batches take PRISMDB_CRC32C_MASK and _LOG_HEADER only");
  // Verify reads the stored checksum: the 4 bytes after the span, or with
  // LOG_HEADER the log record header 6 bytes before it.
  const bool hdr = (flags & PRISMDB_CRC32C_LOG_HEADER) != 0;
  const size_t lead = mismatch != nullptr && hdr ? 6 : 0;
  const size_t tail = mismatch != nullptr && !hdr ? 4 : 0;
  for (size_t i = 0; i < n; ++i) {
    if (lead + (size_t)len[i] + tail > kChunkBytes) return PipeFail(PRISMDB_CRC32C_EINVAL, "span larger than 64 MiB");
    if (i && off[i] < off[i - 1]) return PipeFail(PRISMDB_CRC32C_EINVAL, "spans must be sorted by offset");
    if (off[i] < lead) return PipeFail(PRISMDB_CRC32C_EINVAL, "log record header before the buffer start");
  }
  int rc = 0;
  Ring* ring = GetRing(rc);
  if (ring == nullptr) return rc;
  const uint8_t* src = static_cast<const uint8_t*>(host_base);
  const bool pinned = IsPinned(host_base);

  // Retire a slot: wait for its stream, hand its results to the caller.
  auto retire = [&](Slot& s) -> int {
    if (!s.busy) return 0;
    hipError_t e = hipEventSynchronize(s.done);
    if (e != hipSuccess) return PipeFail(PRISMDB_CRC32C_EDEVICE, std::string("pipeline: ") + hipGetErrorString(e));
    if (out) std::memcpy(out + s.first, s.h_out, s.count * 4);
    if (mismatch) std::memcpy(mismatch + s.first, s.h_mm, s.count);
    s.busy = false;
    return 0;
  };

  size_t i = 0;
  int k = 0;
  while (i < n) {
    Slot& s = ring->slot[k];
    if ((rc = retire(s)) != 0) return rc;
    // Chunk: consecutive spans whose bytes (plus trailers) fit kChunkBytes.
    const uint64_t lo = off[i] - lead;
    uint64_t hi = lo;
    size_t j = i;
    while (j < n && j - i < kChunkSpans) {
      const uint64_t end = std::max<uint64_t>(hi, off[j] + len[j] + tail);
      if (end - lo > kChunkBytes) break;
      hi = end;
      ++j;
    }
    const size_t cnt = j - i;
    for (size_t q = 0; q < cnt; ++q) {
      s.h_off[q] = off[i + q] - lo;
      s.h_len[q] = len[i + q];
      s.h_init[q] = init ? init[i + q] : 0u;
    }
    const size_t bytes = (size_t)(hi - lo);
    const uint8_t* from = src + lo;
    if (!pinned) {
      std::memcpy(s.h_stage, from, bytes);  // pageable source: stage through pinned memory
      from = s.h_stage;
    }
    hipError_t e = hipMemcpyAsync(s.d_data, from, bytes, hipMemcpyHostToDevice, s.stream);
    if (e == hipSuccess) e = hipMemcpyAsync(s.d_off, s.h_off, cnt * 8, hipMemcpyHostToDevice, s.stream);
    if (e == hipSuccess) e = hipMemcpyAsync(s.d_len, s.h_len, cnt * 4, hipMemcpyHostToDevice, s.stream);
    if (e == hipSuccess && init) e = hipMemcpyAsync(s.d_init, s.h_init, cnt * 4, hipMemcpyHostToDevice, s.stream);
    if (e != hipSuccess) return PipeFail(PRISMDB_CRC32C_EDEVICE, std::string("pipeline H2D: ") + hipGetErrorString(e));
    rc = leveldb_crc32c_batch(s.d_data, s.d_off, s.d_len, init ? s.d_init : nullptr, cnt, s.d_out,
                              mismatch ? s.d_mm : nullptr, flags, s.stream);
    if (rc != 0) return rc;  // message already set by leveldb_crc32c_batch
    e = hipMemcpyAsync(s.h_out, s.d_out, cnt * 4, hipMemcpyDeviceToHost, s.stream);
    if (e == hipSuccess && mismatch) e = hipMemcpyAsync(s.h_mm, s.d_mm, cnt, hipMemcpyDeviceToHost, s.stream);
    if (e == hipSuccess) e = hipEventRecord(s.done, s.stream);
    if (e != hipSuccess) return PipeFail(PRISMDB_CRC32C_EDEVICE, std::string("pipeline D2H: ") + hipGetErrorString(e));
    s.busy = true;
    s.first = i;
    s.count = cnt;
    i = j;
    k = (k + 1) % kDepth;
  }
  for (Slot& s : ring->slot)
    if ((rc = retire(s)) != 0) return rc;
  return 0;
}

}  // extern "C"
