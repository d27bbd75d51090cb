// crc32c_pipeline.hip -- host-resident batches.
//
// PrismDB's blocks start and end in host memory: SST file pages read with
// pread during compaction (util/env_posix.cc:172-208) and blocks appended to a
// 32 MiB write buffer (:279-309).  leveldb_crc32c_batch_host streams such a
// batch through the device.  Spans are cut into chunks of <= kChunkBytes of
// consecutive file bytes, and the work is split over two streams so the PCIe
// link never idles:
//   copy stream     chunk bytes host -> device, back to back (the bottleneck);
//   compute stream  per chunk: descriptors H2D (one packed copy), wait for the
//                   chunk's bytes, batch kernels, 4-byte results D2H.
// kDepth chunks are in flight; the host refills a slot once the compute
// stream has released it.  A pageable source is first staged into the slot's
// pinned buffer by several host threads (one memcpy thread reaches about half
// the link rate).  The call is synchronous (like ReadBlock) and thread-safe:
// a call leases a ring (its streams and slots) from a per-device pool for its
// duration, so memory follows the number of CONCURRENT calls, not the number
// of threads that ever called; at most kKeepIdle rings per device stay
// allocated between calls (each ~256 MiB pinned + ~256 MiB device).
#include <hip/hip_runtime.h>

#include <fcntl.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/prismdb_crc32c.h"

namespace prismdb {
void SetLastError(const std::string& msg);  // crc32c_capi.hip: leveldb_crc32c_last_error()
// crc32c_capi.hip: a ring's compute stream carries its own batch workspace
// (not one per thread that leases the ring), released with the ring
void RegisterEngineStream(hipStream_t s);
void ReleaseEngineStream(hipStream_t s);
bool TestHooksEnabled();  // crc32c_capi.hip: PRISMDB_ENABLE_TEST_HOOKS
}

namespace {

// per DMA (~1.2 ms of PCIe Gen5 x16), the slot size: 2 GiB of 4 KiB blocks
// stream at 51.7 GiB/s pinned / 50.7 pageable against 50.9 / 50.2 with
// 32 MiB chunks and 53.6 for the plain copy (profiles/r04/r04aa_pipe_chunks.json)
constexpr size_t kChunkBytes = 64ull << 20;
constexpr size_t kMaxSpan = 64ull << 20;     // one 64 MiB SST (include/leveldb/options.h:117)
constexpr size_t kSlotBytes = kMaxSpan + 8;  // a chunk holds one span of up to kMaxSpan
constexpr size_t kChunkSpans = 1u << 16;     // descriptors per chunk
constexpr int kDepth = 4;
constexpr size_t kKeepIdle = 2;  // idle rings kept per device
constexpr int kMaxDevices = 64;

// Test hook (not in the public header, like prismdb_crc32c_force_generic):
// the k-th chunk of every later call fails as a device error would, after the
// earlier chunks have been enqueued.  0 = off.
std::atomic<int> g_fail_after_chunks{0};
// Chunk size (tuning hook prismdb_pipeline_chunk_bytes; default kChunkBytes):
// spans are packed into chunks of at most this many bytes (a single span may
// be larger, up to kMaxSpan, the slot size).
std::atomic<size_t> g_chunk_bytes{kChunkBytes};

int PipeFail(int code, const std::string& msg) {
  prismdb::SetLastError(msg);
  return code;
}

struct Slot {
  hipEvent_t copied = nullptr;  // chunk bytes on the device (copy stream)
  hipEvent_t done = nullptr;    // results on the host, slot free (compute stream)
  uint8_t* h_stage = nullptr;   // pinned, kSlotBytes (pageable sources)
  uint8_t* d_data = nullptr;    // kSlotBytes
  uint8_t* h_desc = nullptr;    // pinned: off[cnt] | len[cnt] | init[cnt]
  uint8_t* d_desc = nullptr;
  uint32_t* d_out = nullptr;
  uint8_t* d_mm = nullptr;
  uint32_t* h_out = nullptr;  // pinned results
  uint8_t* h_mm = nullptr;
  bool busy = false;
  size_t first = 0, count = 0;
};

struct Ring {
  int device = 0;
  hipStream_t copy = nullptr, compute = nullptr;
  bool registered = false;  // compute's batch workspace (crc32c_capi.hip)
  Slot slot[kDepth];
  // Called with `device` current.  The ring's own streams are drained first;
  // its device blocks go back stream-ordered (no device-wide hipFree).
  ~Ring() {
    if (copy) (void)hipStreamSynchronize(copy);
    if (compute) (void)hipStreamSynchronize(compute);
    for (Slot& s : slot) {
      (void)hipHostFree(s.h_stage);
      (void)hipHostFree(s.h_desc);
      (void)hipHostFree(s.h_out);
      if (s.d_data) (void)hipFreeAsync(s.d_data, compute);
      if (s.d_desc) (void)hipFreeAsync(s.d_desc, compute);
      if (s.copied) (void)hipEventDestroy(s.copied);
      if (s.done) (void)hipEventDestroy(s.done);
    }
    if (compute) (void)hipStreamSynchronize(compute);
    // (after the slots: its pool trim then returns their blocks too)
    if (registered) prismdb::ReleaseEngineStream(compute);
    if (copy) (void)hipStreamDestroy(copy);
    if (compute) (void)hipStreamDestroy(compute);
  }
};

int MakeRing(Ring& r) {
  hipError_t e = hipStreamCreateWithFlags(&r.copy, hipStreamNonBlocking);
  if (e == hipSuccess) e = hipStreamCreateWithFlags(&r.compute, hipStreamNonBlocking);
  if (e == hipSuccess) {
    prismdb::RegisterEngineStream(r.compute);
    r.registered = true;
  }
  for (Slot& s : r.slot) {
    if (e == hipSuccess) e = hipEventCreateWithFlags(&s.copied, hipEventDisableTiming);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&s.done, hipEventDisableTiming);
    if (e == hipSuccess) e = hipHostMalloc(reinterpret_cast<void**>(&s.h_stage), kSlotBytes);
    if (e == hipSuccess) e = hipHostMalloc(reinterpret_cast<void**>(&s.h_desc), kChunkSpans * 16);
    if (e == hipSuccess) e = hipHostMalloc(reinterpret_cast<void**>(&s.h_out), kChunkSpans * (4 + 1));
    if (e == hipSuccess) e = hipMallocAsync(reinterpret_cast<void**>(&s.d_data), kSlotBytes, r.compute);
    if (e == hipSuccess) e = hipMallocAsync(reinterpret_cast<void**>(&s.d_desc), kChunkSpans * (16 + 4 + 1), r.compute);
    if (e != hipSuccess) break;
    s.h_mm = reinterpret_cast<uint8_t*>(s.h_out + kChunkSpans);
    s.d_out = reinterpret_cast<uint32_t*>(s.d_desc + kChunkSpans * 16);
    s.d_mm = reinterpret_cast<uint8_t*>(s.d_out + kChunkSpans);
  }
  if (e == hipSuccess) e = hipStreamSynchronize(r.compute);
  if (e != hipSuccess) return PipeFail(PRISMDB_CRC32C_EDEVICE, std::string("pipeline setup: ") + hipGetErrorString(e));
  return 0;
}

// Idle rings per device.  The pool itself is never destroyed: at exit() the
// HIP runtime (or a profiler wrapped around it) may already be tearing down,
// so the rings still in it are left to the OS.
struct RingPool {
  std::mutex mu;
  std::vector<Ring*> idle[kMaxDevices];
};
RingPool& Pool() {
  static RingPool* pool = new RingPool;
  return *pool;
}

// A ring for the duration of one call (current device).
struct RingLease {
  Ring* ring = nullptr;
  int Acquire() {
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return PipeFail(PRISMDB_CRC32C_EDEVICE, std::string("hipGetDevice: ") + hipGetErrorString(e));
    if (dev < 0 || dev >= kMaxDevices) return PipeFail(PRISMDB_CRC32C_EINVAL, "device ordinal out of range");
    {
      std::lock_guard<std::mutex> lk(Pool().mu);
      std::vector<Ring*>& idle = Pool().idle[dev];
      if (!idle.empty()) {
        ring = idle.back();
        idle.pop_back();
        return 0;
      }
    }
    std::unique_ptr<Ring> r(new Ring);
    r->device = dev;
    if (int rc = MakeRing(*r)) return rc;  // (the partial ring is freed by its destructor)
    ring = r.release();
    return 0;
  }
  // Back to the pool, or freed when kKeepIdle rings of this device are idle
  // already.  The ring is quiescent here (every call drains its slots).
  ~RingLease() {
    if (ring == nullptr) return;
    {
      std::lock_guard<std::mutex> lk(Pool().mu);
      std::vector<Ring*>& idle = Pool().idle[ring->device];
      if (idle.size() < kKeepIdle) {
        idle.push_back(ring);
        return;
      }
    }
    int cur = 0;
    const int dev = ring->device;
    (void)hipGetDevice(&cur);
    if (cur != dev) (void)hipSetDevice(dev);
    delete ring;
    if (cur != dev) (void)hipSetDevice(cur);
  }
};

bool IsPinned(const void* p) {
  hipPointerAttribute_t a;
  if (hipPointerGetAttributes(&a, p) != hipSuccess) {
    (void)hipGetLastError();  // clear the sticky "invalid value" for pageable memory
    return false;
  }
  return a.type == hipMemoryTypeHost;
}

// Staging threads for pageable sources: PRISMDB_STAGE_THREADS, else half the
// cores this process may use, capped at 8.
int StageThreads() {
  static const int n = [] {
    if (const char* e = std::getenv("PRISMDB_STAGE_THREADS")) {
      const int v = std::atoi(e);
      if (v >= 1) return std::min(v, 64);
    }
    const int hw = (int)std::thread::hardware_concurrency();
    return std::max(1, std::min(8, hw / 2));
  }();
  return n;
}

void ParallelCopy(uint8_t* dst, const uint8_t* src, size_t bytes) {
  const int t = bytes >= (4u << 20) ? StageThreads() : 1;
  if (t <= 1) {
    std::memcpy(dst, src, bytes);
    return;
  }
  const size_t piece = ((bytes + t - 1) / t + 4095) & ~size_t(4095);
  std::vector<std::thread> th;
  th.reserve(t - 1);
  for (int k = 1; k < t; ++k) {
    const size_t lo = k * piece;
    if (lo >= bytes) break;
    const size_t len = std::min(piece, bytes - lo);
    th.emplace_back([=] { std::memcpy(dst + lo, src + lo, len); });
  }
  std::memcpy(dst, src, std::min(piece, bytes));
  for (std::thread& x : th) x.join();
}

// True if the k bytes at p can be read and written by this process, checked
// without touching them from user code: the kernel copies them into a pipe
// and back (EFAULT instead of a fault on an unmapped or read-only page).  The
// bytes end up unchanged.  Sealing probes its first and last trailer slots
// with it, so that a read-only mapping (a file mmap'ed PROT_READ, an immutable
// Python bytes object) is refused with EINVAL rather than crashing in the
// trailer stores; the buffer TableBuilder seals is its writable heap append
// buffer (util/env_posix.cc:279-309).
bool HostWritable(uint8_t* p, size_t k) {
  int fd[2];
  if (pipe2(fd, O_CLOEXEC) != 0) return true;  // (cannot tell: leave it to the stores)
  bool ok = write(fd[1], p, k) == (ssize_t)k;
  if (ok) {
    ok = read(fd[0], p, k) == (ssize_t)k;
    if (!ok) {
      uint8_t sink[8];
      (void)!read(fd[0], sink, k);
    }
  }
  close(fd[0]);
  close(fd[1]);
  return ok;
}

}  // namespace

extern "C" {

int leveldb_crc32c_batch_host(const void* host_base, const uint64_t* off, const uint32_t* len,
                              const uint32_t* init, size_t n, uint32_t* out, uint8_t* mismatch,
                              uint32_t flags) {
  if (n == 0) return 0;
  if (host_base == nullptr || off == nullptr || len == nullptr)
    return PipeFail(PRISMDB_CRC32C_EINVAL, "host_base/off/len must be non-NULL");
  if (flags & ~(PRISMDB_CRC32C_MASK | PRISMDB_CRC32C_LOG_HEADER | PRISMDB_CRC32C_WRITE_TRAILER))
    return PipeFail(PRISMDB_CRC32C_EINVAL, "host batches take PRISMDB_CRC32C_MASK, _WRITE_TRAILER and _LOG_HEADER only");
  const bool seal = (flags & PRISMDB_CRC32C_WRITE_TRAILER) != 0;
  if (seal && mismatch != nullptr)
    return PipeFail(PRISMDB_CRC32C_EINVAL, "WRITE_TRAILER and verify are exclusive");
  // Verify reads the stored checksum: the 4 bytes after the span, or with
  // LOG_HEADER the log record header 6 bytes before it.  A seal writes it
  // there on the host (below): those bytes never travel to the device.
  const bool hdr = (flags & PRISMDB_CRC32C_LOG_HEADER) != 0;
  const size_t lead = mismatch != nullptr && hdr ? 6 : 0;
  const size_t tail = mismatch != nullptr && !hdr ? 4 : 0;
  for (size_t i = 0; i < n; ++i) {
    if (lead + (size_t)len[i] + tail > kMaxSpan) return PipeFail(PRISMDB_CRC32C_EINVAL, "span larger than 64 MiB");
    if (i && off[i] < off[i - 1]) return PipeFail(PRISMDB_CRC32C_EINVAL, "spans must be sorted by offset");
    if (off[i] < lead || (seal && hdr && off[i] < 6))
      return PipeFail(PRISMDB_CRC32C_EINVAL, "log record header before the buffer start");
  }
  if (seal) {  // the signature's const does not hold under WRITE_TRAILER
    uint8_t* const b = static_cast<uint8_t*>(const_cast<void*>(host_base));
    for (size_t i : {(size_t)0, n - 1}) {
      uint8_t* const t = hdr ? b + off[i] - 6 : b + off[i] + len[i];
      if (!HostWritable(t, 4))
        return PipeFail(PRISMDB_CRC32C_EINVAL, "WRITE_TRAILER: the host buffer is not writable at a trailer slot");
    }
  }
  RingLease lease;
  int rc = lease.Acquire();
  if (rc != 0) return rc;
  Ring* const ring = lease.ring;
  const uint8_t* src = static_cast<const uint8_t*>(host_base);
  const bool pinned = IsPinned(host_base);

  // Abandon the call: wait for everything this call enqueued (DMAs may still
  // read the caller's source, kernels and D2H copies still write the slots)
  // and release every slot without copying anything out, so that the next
  // call on this ring starts empty.  Returns the original failure.
  auto abort_call = [&](int code) -> int {
    const std::string msg = leveldb_crc32c_last_error();
    (void)hipStreamSynchronize(ring->copy);
    (void)hipStreamSynchronize(ring->compute);
    (void)hipGetLastError();
    for (Slot& q : ring->slot) q.busy = false;
    prismdb::SetLastError(msg);
    return code;
  };

  // Retire a slot: wait until the compute stream released it, hand its
  // results to the caller.  Sealing, the results are also stored into the
  // caller's buffer as each span's trailer -- 4 LE bytes right behind it, or
  // with LOG_HEADER the record header's crc 6 bytes before it -- where
  // TableBuilder::WriteRawBlock appends them to its 32 MiB write buffer
  // (table/table_builder.cc:192-197, util/env_posix.cc:279-309).  A chunk's
  // trailers go out while the next kDepth - 1 chunks are in flight.  (Left to
  // the caller after the call, 1.93 M scattered stores cost config 4's write
  // leg 12 % against its read leg: bench.py compaction_leg, round 4.)
  uint8_t* const dst = static_cast<uint8_t*>(const_cast<void*>(host_base));
  auto retire = [&](Slot& s) -> int {
    if (!s.busy) return 0;
    hipError_t e = hipEventSynchronize(s.done);
    if (e != hipSuccess) return PipeFail(PRISMDB_CRC32C_EDEVICE, std::string("pipeline: ") + hipGetErrorString(e));
    if (out) std::memcpy(out + s.first, s.h_out, s.count * 4);
    if (mismatch) std::memcpy(mismatch + s.first, s.h_mm, s.count);
    if (seal) {
      const uint64_t* o = off + s.first;
      const uint32_t* l = len + s.first;
      if (hdr) {
        for (size_t q = 0; q < s.count; ++q) std::memcpy(dst + o[q] - 6, s.h_out + q, 4);
      } else {
        for (size_t q = 0; q < s.count; ++q) std::memcpy(dst + o[q] + l[q], s.h_out + q, 4);
      }
    }
    s.busy = false;
    return 0;
  };

  size_t i = 0;
  int k = 0, chunks = 0;
  while (i < n) {
    Slot& s = ring->slot[k];
    if ((rc = retire(s)) != 0) return abort_call(rc);
    // Chunk: consecutive spans whose bytes (plus trailers) fit kChunkBytes;
    // a single span may be larger (up to kMaxSpan).
    const uint64_t lo = off[i] - lead;
    const uint64_t chunk_bytes = g_chunk_bytes.load(std::memory_order_relaxed);
    uint64_t hi = lo;
    size_t j = i;
    while (j < n && j - i < kChunkSpans) {
      const uint64_t end = std::max<uint64_t>(hi, off[j] + len[j] + tail);
      if (j > i && end - lo > chunk_bytes) break;
      hi = end;
      ++j;
    }
    const size_t cnt = j - i;
    uint64_t* h_off = reinterpret_cast<uint64_t*>(s.h_desc);
    uint32_t* h_len = reinterpret_cast<uint32_t*>(h_off + cnt);
    uint32_t* h_init = h_len + cnt;
    for (size_t q = 0; q < cnt; ++q) {
      h_off[q] = off[i + q] - lo;
      h_len[q] = len[i + q];
    }
    if (init) std::memcpy(h_init, init + i, cnt * 4);
    const size_t bytes = (size_t)(hi - lo);
    const uint8_t* from = src + lo;
    if (!pinned) {
      ParallelCopy(s.h_stage, from, bytes);  // pageable source: stage through pinned memory
      from = s.h_stage;
    }
    const uint64_t* d_off = reinterpret_cast<const uint64_t*>(s.d_desc);
    const uint32_t* d_len = reinterpret_cast<const uint32_t*>(d_off + cnt);
    const uint32_t* d_init = d_len + cnt;
    hipError_t e = hipMemcpyAsync(s.d_data, from, bytes, hipMemcpyHostToDevice, ring->copy);
    if (e == hipSuccess) e = hipEventRecord(s.copied, ring->copy);
    if (e == hipSuccess)
      e = hipMemcpyAsync(s.d_desc, s.h_desc, cnt * (init ? 16 : 12), hipMemcpyHostToDevice, ring->compute);
    if (e == hipSuccess) e = hipStreamWaitEvent(ring->compute, s.copied, 0);
    if (e != hipSuccess)
      return abort_call(PipeFail(PRISMDB_CRC32C_EDEVICE, std::string("pipeline H2D: ") + hipGetErrorString(e)));
    const int fail_after = g_fail_after_chunks.load(std::memory_order_relaxed);
    rc = fail_after > 0 && ++chunks >= fail_after
             ? PipeFail(PRISMDB_CRC32C_EDEVICE, "pipeline: injected failure (prismdb_pipeline_fail_after)")
             : leveldb_crc32c_batch(s.d_data, d_off, d_len, init ? d_init : nullptr, cnt, s.d_out,
                                    mismatch ? s.d_mm : nullptr, flags & ~PRISMDB_CRC32C_WRITE_TRAILER,
                                    ring->compute);
    if (rc != 0) return abort_call(rc);  // message already set by leveldb_crc32c_batch
    e = hipMemcpyAsync(s.h_out, s.d_out, cnt * 4, hipMemcpyDeviceToHost, ring->compute);
    if (e == hipSuccess && mismatch) e = hipMemcpyAsync(s.h_mm, s.d_mm, cnt, hipMemcpyDeviceToHost, ring->compute);
    if (e == hipSuccess) e = hipEventRecord(s.done, ring->compute);
    if (e != hipSuccess)
      return abort_call(PipeFail(PRISMDB_CRC32C_EDEVICE, std::string("pipeline D2H: ") + hipGetErrorString(e)));
    s.busy = true;
    s.first = i;
    s.count = cnt;
    i = j;
    k = (k + 1) % kDepth;
  }
  for (int q = 0; q < kDepth; ++q)
    if ((rc = retire(ring->slot[(k + q) % kDepth])) != 0) return abort_call(rc);
  return 0;
}

void prismdb_pipeline_fail_after(int chunks) {
  if (prismdb::TestHooksEnabled()) g_fail_after_chunks.store(chunks > 0 ? chunks : 0, std::memory_order_relaxed);
}

// Tuning hook: chunk size of later host batches (0: leave it; clamped to
// [1 MiB, kMaxSpan]); returns the previous value.
size_t prismdb_pipeline_chunk_bytes(size_t bytes) {
  if (bytes == 0 || !prismdb::TestHooksEnabled()) return g_chunk_bytes.load(std::memory_order_relaxed);
  const size_t b = bytes < (1u << 20) ? (1u << 20) : (bytes > kMaxSpan ? kMaxSpan : bytes);
  return g_chunk_bytes.exchange(b, std::memory_order_relaxed);
}

}  // extern "C"
