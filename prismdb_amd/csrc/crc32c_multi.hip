// crc32c_multi.hip -- several devices from one process (leveldb_crc32c_batch_multi).
//
// PrismDB runs its 8 partitions as threads of one process (db/db_impl.h:359,
// one background thread each, util/env_posix.cc:850-890).  Here partition p's
// block batch lives on device devices[p]: every device checksums its own
// batch (the one-launch or planner path, leveldb_crc32c_batch), and one RCCL
// gather -- grouped ncclSend / ncclRecv over xGMI, variable counts -- brings
// the 4-byte results (and the verify flags) to devices[0], partition after
// partition.  Blocks are independent, so the gather is the only exchange.
//
// A clique (the RCCL communicators of one device list, ncclCommInitAll) is
// created on the first call for that list and kept; its calls are serialized
// (RCCL communicators are not for concurrent use: calls with the same device
// list queue on the clique's mutex) on one internal stream per device, which
// waits for the caller's stream first and which the caller's stream waits for
// afterwards -- on every return, errors included.  Partition 0 writes its results straight into
// out0; the others go through per-device scratch, grown stream-ordered.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <atomic>
#include <chrono>
#include <cstring>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/prismdb_crc32c.h"

namespace prismdb {
void SetLastError(const std::string& msg);  // crc32c_capi.hip: leveldb_crc32c_last_error()
void RegisterEngineStream(hipStream_t s);   // crc32c_capi.hip: the stream's own batch workspace
bool TestHooksEnabled();                    // crc32c_capi.hip: PRISMDB_ENABLE_TEST_HOOKS
}

namespace {

int MultiFail(int code, const std::string& msg) {
  prismdb::SetLastError(msg);
  return code;
}

int HipFail(hipError_t e, const char* what) {
  return MultiFail(PRISMDB_CRC32C_EDEVICE, std::string("batch_multi: ") + what + ": " + hipGetErrorString(e));
}

int NcclFail(ncclResult_t r, const char* what) {
  return MultiFail(PRISMDB_CRC32C_EDEVICE, std::string("batch_multi: ") + what + ": " + ncclGetErrorString(r));
}

struct Clique {
  std::vector<int> devs;
  std::vector<ncclComm_t> comms;
  std::vector<hipStream_t> streams;  // one per device
  std::vector<hipEvent_t> events;    // one per device: stream handoffs with the caller
  std::vector<uint32_t*> out;        // per device (index 0 unused): its partition's results
  std::vector<uint8_t*> mm;
  std::vector<size_t> cap;
  // Per device, timing events of the last call on the clique stream: after
  // the hand-off from the caller (t0), after the device's own batch (t1),
  // after the gather (t2) -- read back by prismdb_crc32c_multi_timing.
  std::vector<hipEvent_t> t0, t1, t2;
  bool timed = false;  // the last call recorded all three
  double init_ms = 0;  // ncclCommInitAll's wall time
  std::mutex mu;
};

// Cliques live until the process exits (communicators and streams are not
// torn down inside exit(), where the runtime may be going away).
std::mutex g_mu;
std::vector<Clique*> g_cliques;
std::atomic<int> g_fail_after{-1};  // test hook: prismdb_crc32c_multi_fail_after

int GetClique(int ndev, const int* devices, Clique** out) {
  std::lock_guard<std::mutex> lk(g_mu);
  for (Clique* c : g_cliques) {
    if ((int)c->devs.size() == ndev && std::memcmp(c->devs.data(), devices, sizeof(int) * ndev) == 0) {
      *out = c;
      return 0;
    }
  }
  std::unique_ptr<Clique> c(new Clique);
  c->devs.assign(devices, devices + ndev);
  c->comms.resize(ndev);
  const auto w0 = std::chrono::steady_clock::now();
  ncclResult_t r = ncclCommInitAll(c->comms.data(), ndev, devices);
  if (r != ncclSuccess) return NcclFail(r, "ncclCommInitAll");
  c->init_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - w0).count();
  int cur = 0;
  (void)hipGetDevice(&cur);
  c->streams.resize(ndev);
  c->events.resize(ndev);
  c->out.assign(ndev, nullptr);
  c->mm.assign(ndev, nullptr);
  c->cap.assign(ndev, 0);
  c->t0.assign(ndev, nullptr);
  c->t1.assign(ndev, nullptr);
  c->t2.assign(ndev, nullptr);
  for (int p = 0; p < ndev; ++p) {
    hipError_t e = hipSetDevice(devices[p]);
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&c->streams[p], hipStreamNonBlocking);
    if (e == hipSuccess) prismdb::RegisterEngineStream(c->streams[p]);  // (used under the clique's mutex)
    if (e == hipSuccess) e = hipEventCreateWithFlags(&c->events[p], hipEventDisableTiming);
    if (e == hipSuccess) e = hipEventCreate(&c->t0[p]);
    if (e == hipSuccess) e = hipEventCreate(&c->t1[p]);
    if (e == hipSuccess) e = hipEventCreate(&c->t2[p]);
    if (e != hipSuccess) {
      (void)hipSetDevice(cur);
      return HipFail(e, "clique streams");
    }
  }
  (void)hipSetDevice(cur);
  *out = c.get();
  g_cliques.push_back(c.release());
  return 0;
}

}  // namespace

extern "C" {

int leveldb_crc32c_batch_multi(int ndev, const int* devices, const void* const* dev_base,
                               const uint64_t* const* dev_off, const uint32_t* const* dev_len,
                               const uint32_t* const* dev_init, const size_t* n, uint32_t* out0,
                               uint8_t* mismatch0, uint32_t flags, void* const* streams) {
  if (ndev < 1 || ndev > 64) return MultiFail(PRISMDB_CRC32C_EINVAL, "batch_multi: ndev must be 1..64");
  if (devices == nullptr || dev_base == nullptr || dev_off == nullptr || dev_len == nullptr || n == nullptr)
    return MultiFail(PRISMDB_CRC32C_EINVAL, "batch_multi: devices/dev_base/dev_off/dev_len/n must be non-NULL");
  if (out0 == nullptr && mismatch0 == nullptr)
    return MultiFail(PRISMDB_CRC32C_EINVAL, "batch_multi: out0 or mismatch0 is needed");
  if (flags & ~(PRISMDB_CRC32C_MASK | PRISMDB_CRC32C_WRITE_TRAILER | PRISMDB_CRC32C_LOG_HEADER |
                PRISMDB_CRC32C_UNORDERED))
    return MultiFail(PRISMDB_CRC32C_EINVAL, "batch_multi: unknown flag bits");
  flags &= ~PRISMDB_CRC32C_UNORDERED;  // (the clique's streams keep their calls in order)
  if ((flags & PRISMDB_CRC32C_WRITE_TRAILER) && mismatch0 != nullptr)
    return MultiFail(PRISMDB_CRC32C_EINVAL, "batch_multi: WRITE_TRAILER and verify are exclusive");
  for (int p = 0; p < ndev; ++p) {
    if (devices[p] < 0) return MultiFail(PRISMDB_CRC32C_EINVAL, "batch_multi: negative device ordinal");
    for (int q = 0; q < p; ++q)
      if (devices[q] == devices[p]) return MultiFail(PRISMDB_CRC32C_EINVAL, "batch_multi: a device is listed twice");
    if (n[p] != 0 && (dev_base[p] == nullptr || dev_off[p] == nullptr || dev_len[p] == nullptr))
      return MultiFail(PRISMDB_CRC32C_EINVAL, "batch_multi: a partition's base/off/len is NULL");
  }
  int cur = 0;
  hipError_t e = hipGetDevice(&cur);
  if (e != hipSuccess) return HipFail(e, "hipGetDevice");
  for (int p = 0; p < ndev; ++p) {  // tables and self-test on every device first
    const int rc = leveldb_crc32c_device_init(devices[p]);
    if (rc != 0) return rc;
  }
  Clique* c = nullptr;
  int rc = GetClique(ndev, devices, &c);
  if (rc != 0) return rc;
  std::lock_guard<std::mutex> lk(c->mu);
  c->timed = false;
  // Once the first command is on a clique stream, every return goes through
  // here: the caller's streams wait for everything the call enqueued (its
  // batches, scratch growth, the gather), so a caller that frees or reuses
  // its buffers after an error never races the clique's work.  If a hand-off
  // itself fails, the clique's streams are drained instead.
  int enqueued = 0;  // clique streams [0, enqueued) may hold work of this call
  auto finish = [&](int code) {
    for (int p = 0; p < enqueued; ++p) {
      hipError_t h = hipSetDevice(devices[p]);
      hipStream_t user = streams != nullptr ? static_cast<hipStream_t>(streams[p]) : nullptr;
      if (h == hipSuccess) h = hipEventRecord(c->events[p], c->streams[p]);
      if (h == hipSuccess) h = hipStreamWaitEvent(user, c->events[p], 0);
      if (h != hipSuccess) {
        (void)hipStreamSynchronize(c->streams[p]);
        if (code == 0) code = HipFail(h, "hand-off to the caller's stream");
      }
    }
    (void)hipSetDevice(cur);
    return code;
  };
  // the clique's streams start after the caller's, and partitions > 0 get
  // scratch for their results
  for (int p = 0; p < ndev; ++p) {
    if ((e = hipSetDevice(devices[p])) != hipSuccess) return finish(HipFail(e, "hipSetDevice"));
    hipStream_t user = streams != nullptr ? static_cast<hipStream_t>(streams[p]) : nullptr;
    if ((e = hipEventRecord(c->events[p], user)) != hipSuccess) return finish(HipFail(e, "hipEventRecord"));
    if ((e = hipStreamWaitEvent(c->streams[p], c->events[p], 0)) != hipSuccess)
      return finish(HipFail(e, "hipStreamWaitEvent"));
    enqueued = p + 1;
    if ((e = hipEventRecord(c->t0[p], c->streams[p])) != hipSuccess) return finish(HipFail(e, "hipEventRecord"));
    if (p > 0 && c->cap[p] < n[p]) {
      if (c->out[p] != nullptr) (void)hipFreeAsync(c->out[p], c->streams[p]);  // out and mm: one block
      c->out[p] = nullptr;
      c->mm[p] = nullptr;
      c->cap[p] = 0;
      const size_t cap = n[p] + n[p] / 4 + 1024;
      void* blk = nullptr;
      if ((e = hipMallocAsync(&blk, cap * 5, c->streams[p])) != hipSuccess) return finish(HipFail(e, "scratch"));
      c->out[p] = static_cast<uint32_t*>(blk);
      c->mm[p] = reinterpret_cast<uint8_t*>(c->out[p] + cap);
      c->cap[p] = cap;
    }
  }
  // every partition's batch on its own device
  const int fail_after = g_fail_after.load(std::memory_order_relaxed);
  for (int p = 0; p < ndev; ++p) {
    if (n[p] != 0) {
      if ((e = hipSetDevice(devices[p])) != hipSuccess) return finish(HipFail(e, "hipSetDevice"));
      uint32_t* o = out0 == nullptr ? nullptr : (p == 0 ? out0 : c->out[p]);
      uint8_t* m = mismatch0 == nullptr ? nullptr : (p == 0 ? mismatch0 : c->mm[p]);
      rc = leveldb_crc32c_batch(dev_base[p], dev_off[p], dev_len[p], dev_init != nullptr ? dev_init[p] : nullptr,
                                n[p], o, m, flags, c->streams[p]);
      if (rc != 0) return finish(rc);
    }
    if ((e = hipSetDevice(devices[p])) != hipSuccess) return finish(HipFail(e, "hipSetDevice"));
    if ((e = hipEventRecord(c->t1[p], c->streams[p])) != hipSuccess) return finish(HipFail(e, "hipEventRecord"));
    if (p == fail_after)
      return finish(MultiFail(PRISMDB_CRC32C_EDEVICE, "batch_multi: injected failure (test hook)"));
  }
  // the gather to devices[0]: partition p's results at offset n[0] + ... + n[p-1]
  if (ndev > 1) {
    ncclResult_t r = ncclGroupStart();
    if (r != ncclSuccess) return finish(NcclFail(r, "ncclGroupStart"));
    size_t at = n[0];
    for (int p = 1; p < ndev && r == ncclSuccess; ++p) {
      if (n[p] == 0) continue;
      if (out0 != nullptr) {
        r = ncclSend(c->out[p], n[p], ncclUint32, 0, c->comms[p], c->streams[p]);
        if (r == ncclSuccess) r = ncclRecv(out0 + at, n[p], ncclUint32, p, c->comms[0], c->streams[0]);
      }
      if (r == ncclSuccess && mismatch0 != nullptr) {
        r = ncclSend(c->mm[p], n[p], ncclUint8, 0, c->comms[p], c->streams[p]);
        if (r == ncclSuccess) r = ncclRecv(mismatch0 + at, n[p], ncclUint8, p, c->comms[0], c->streams[0]);
      }
      at += n[p];
    }
    const ncclResult_t r2 = ncclGroupEnd();
    if (r != ncclSuccess) return finish(NcclFail(r, "ncclSend/ncclRecv"));
    if (r2 != ncclSuccess) return finish(NcclFail(r2, "ncclGroupEnd"));
  }
  for (int p = 0; p < ndev; ++p) {
    if ((e = hipSetDevice(devices[p])) != hipSuccess) return finish(HipFail(e, "hipSetDevice"));
    if ((e = hipEventRecord(c->t2[p], c->streams[p])) != hipSuccess) return finish(HipFail(e, "hipEventRecord"));
  }
  c->timed = true;
  // the caller's streams resume after the clique's work
  return finish(0);
}

// Diagnostics (not in the public header): the phases of the last successful
// call on the clique of this device list, per device p, after waiting for it:
// batch_ms[p] = its own batch (hand-off to batch end on its clique stream),
// gather_ms[p] = batch end to the end of its part of the gather (on devices[0]:
// until every partition has arrived); *init_ms = ncclCommInitAll's wall time
// when the clique was created.  Read-only.  0; -1 if no such clique or call.
int prismdb_crc32c_multi_timing(int ndev, const int* devices, float* batch_ms, float* gather_ms, double* init_ms) {
  if (ndev < 1 || devices == nullptr) return -1;
  Clique* c = nullptr;
  {
    std::lock_guard<std::mutex> lk(g_mu);
    for (Clique* x : g_cliques)
      if ((int)x->devs.size() == ndev && std::memcmp(x->devs.data(), devices, sizeof(int) * ndev) == 0) c = x;
  }
  if (c == nullptr) return -1;
  std::lock_guard<std::mutex> lk(c->mu);
  if (init_ms != nullptr) *init_ms = c->init_ms;
  if (!c->timed) return -1;
  int cur = 0;
  (void)hipGetDevice(&cur);
  int rc = 0;
  for (int p = 0; p < ndev && rc == 0; ++p) {
    float b = 0, g = 0;
    hipError_t e = hipSetDevice(devices[p]);
    if (e == hipSuccess) e = hipEventSynchronize(c->t2[p]);
    if (e == hipSuccess) e = hipEventElapsedTime(&b, c->t0[p], c->t1[p]);
    if (e == hipSuccess) e = hipEventElapsedTime(&g, c->t1[p], c->t2[p]);
    if (e != hipSuccess) rc = HipFail(e, "multi timing");
    if (batch_ms != nullptr) batch_ms[p] = b;
    if (gather_ms != nullptr) gather_ms[p] = g;
  }
  (void)hipSetDevice(cur);
  return rc;
}

// Test hook (not in the public header): fail every call right after
// partition p's batch is enqueued (-1: off); returns the previous value.
int prismdb_crc32c_multi_fail_after(int p) {
  if (!prismdb::TestHooksEnabled()) return g_fail_after.load();  // (crc32c_capi.hip)
  return g_fail_after.exchange(p < 0 ? -1 : p);
}

}  // extern "C"
