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
//
// Enqueue.  A partition's planner-path batch is ~10 launches and event
// operations of host work; issued device after device from one thread, the
// last device of 8 would start its batch 7 enqueues after the first, and the
// gather waits for the last.  So partitions 1..ndev-1 are enqueued by one
// persistent worker thread per device of the clique (its hand-off from the
// caller's stream, scratch growth, batch and timing event), while the calling
// thread enqueues partition 0; the gather and the hand-back follow once all
// have enqueued.  Workers spin briefly for the next call (back-to-back
// calls), then sleep on a condition variable.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstring>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/prismdb_crc32c.h"

namespace prismdb {
void SetLastError(const std::string& msg);  // crc32c_capi.hip: leveldb_crc32c_last_error()
void RegisterEngineStream(hipStream_t s);   // crc32c_capi.hip: the stream's own batch workspace
bool TestHooksEnabled();                    // crc32c_capi.hip: PRISMDB_ENABLE_TEST_HOOKS
}

namespace {

using Clock = std::chrono::steady_clock;

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

// One call's arguments, shared with the workers for the call's duration.
struct CallArgs {
  const void* const* dev_base;
  const uint64_t* const* dev_off;
  const uint32_t* const* dev_len;
  const uint32_t* const* dev_init;
  const size_t* n;
  uint32_t* out0;
  uint8_t* mismatch0;
  uint32_t flags;
  void* const* streams;
  bool scratch0;  // partition 0's results go through scratch too (self-gather hook)
  int last;       // partitions > last skip their batch (fail_after hook; ndev otherwise)
  Clock::time_point t_call;
};

struct Clique;

// A persistent enqueue thread for one device of a clique.
struct Worker {
  std::thread th;
  std::mutex mu;
  std::condition_variable cv;
  std::atomic<uint32_t> go{0};   // call generation posted by the caller
  std::atomic<uint32_t> fin{0};  // call generation this worker has finished
  const CallArgs* args = nullptr;
  int rc = 0;
  std::string err;
};

struct Clique {
  std::vector<int> devs;
  std::vector<ncclComm_t> comms;
  std::vector<hipStream_t> streams;  // one per device
  std::vector<hipEvent_t> events;    // one per device: stream handoffs with the caller
  std::vector<uint32_t*> out;        // per device (index 0: self-gather hook only): its partition's results
  std::vector<uint8_t*> mm;
  std::vector<size_t> cap;
  // Per device, timing events of the last call on the clique stream: after
  // the hand-off from the caller (t0), after the device's own batch (t1),
  // after the gather (t2) -- read back by prismdb_crc32c_multi_timing.
  std::vector<hipEvent_t> t0, t1, t2;
  // Per device, host wall times of the last call: from the call's entry to
  // the start of the partition's enqueue, and the enqueue itself (hand-off,
  // scratch, batch, event), in us; and the whole call's.
  std::vector<double> h_start_us, h_enq_us;
  std::vector<uint8_t> handed;  // the call's work reached this device's clique stream
  double h_call_us = 0;
  bool timed = false;  // the last call recorded all three
  double init_ms = 0;  // ncclCommInitAll's wall time
  std::vector<std::unique_ptr<Worker>> workers;  // per device, created on first use
  uint32_t gen = 0;
  std::mutex mu;
};

// Cliques live until the process exits (communicators, streams and worker
// threads are not torn down inside exit(), where the runtime may be going
// away; the workers sleep on their condition variables).
std::mutex g_mu;
std::vector<Clique*> g_cliques;
std::atomic<int> g_fail_after{-1};    // test hook: prismdb_crc32c_multi_fail_after
std::atomic<int> g_self_gather{0};    // test hook: prismdb_crc32c_multi_self_gather

// Partition p's share of a call, on whichever thread: hand-off from the
// caller's stream, scratch, the batch, its timing event.  Returns 0 or the
// error (message set on this thread).
int EnqueuePartition(Clique* c, int p, const CallArgs& a) {
  const auto h0 = Clock::now();
  c->h_start_us[p] = std::chrono::duration<double, std::micro>(h0 - a.t_call).count();
  hipError_t e = hipSetDevice(c->devs[p]);
  if (e != hipSuccess) return HipFail(e, "hipSetDevice");
  hipStream_t user = a.streams != nullptr ? static_cast<hipStream_t>(a.streams[p]) : nullptr;
  if ((e = hipEventRecord(c->events[p], user)) != hipSuccess) return HipFail(e, "hipEventRecord");
  if ((e = hipStreamWaitEvent(c->streams[p], c->events[p], 0)) != hipSuccess) return HipFail(e, "hipStreamWaitEvent");
  c->handed[p] = 1;
  if ((e = hipEventRecord(c->t0[p], c->streams[p])) != hipSuccess) return HipFail(e, "hipEventRecord");
  const bool scratch = p > 0 || a.scratch0;
  if (scratch && c->cap[p] < a.n[p]) {
    if (c->out[p] != nullptr) (void)hipFreeAsync(c->out[p], c->streams[p]);  // out and mm: one block
    c->out[p] = nullptr;
    c->mm[p] = nullptr;
    c->cap[p] = 0;
    const size_t cap = a.n[p] + a.n[p] / 4 + 1024;
    void* blk = nullptr;
    if ((e = hipMallocAsync(&blk, cap * 5, c->streams[p])) != hipSuccess) return HipFail(e, "scratch");
    c->out[p] = static_cast<uint32_t*>(blk);
    c->mm[p] = reinterpret_cast<uint8_t*>(c->out[p] + cap);
    c->cap[p] = cap;
  }
  if (a.n[p] != 0 && p <= a.last) {
    uint32_t* o = a.out0 == nullptr ? nullptr : (scratch ? c->out[p] : a.out0);
    uint8_t* m = a.mismatch0 == nullptr ? nullptr : (scratch ? c->mm[p] : a.mismatch0);
    const int rc = leveldb_crc32c_batch(a.dev_base[p], a.dev_off[p], a.dev_len[p],
                                        a.dev_init != nullptr ? a.dev_init[p] : nullptr, a.n[p], o, m, a.flags,
                                        c->streams[p]);
    if (rc != 0) return rc;
  }
  if ((e = hipEventRecord(c->t1[p], c->streams[p])) != hipSuccess) return HipFail(e, "hipEventRecord");
  c->h_enq_us[p] = std::chrono::duration<double, std::micro>(Clock::now() - h0).count();
  return 0;
}

void WorkerLoop(Clique* c, int p) {
  Worker& w = *c->workers[p];
  (void)hipSetDevice(c->devs[p]);
  uint32_t seen = 0;
  for (;;) {
    // the next call: spin ~50 us first (calls issued back to back), then sleep
    uint32_t g = w.go.load(std::memory_order_acquire);
    const auto s0 = Clock::now();
    while (g == seen && Clock::now() - s0 < std::chrono::microseconds(50)) g = w.go.load(std::memory_order_acquire);
    if (g == seen) {
      std::unique_lock<std::mutex> lk(w.mu);
      w.cv.wait(lk, [&] { return w.go.load(std::memory_order_acquire) != seen; });
      g = w.go.load(std::memory_order_acquire);
    }
    seen = g;
    w.rc = EnqueuePartition(c, p, *w.args);
    w.err = w.rc != 0 ? std::string(leveldb_crc32c_last_error()) : std::string();
    w.fin.store(g, std::memory_order_release);
  }
}

int StartWorker(Clique* c, int p) {
  if (c->workers[p] != nullptr) return 0;
  std::unique_ptr<Worker> w(new Worker);
  c->workers[p] = std::move(w);
  try {
    c->workers[p]->th = std::thread(WorkerLoop, c, p);
    c->workers[p]->th.detach();
  } catch (const std::exception& ex) {
    c->workers[p].reset();
    return MultiFail(PRISMDB_CRC32C_EDEVICE, std::string("batch_multi: worker thread: ") + ex.what());
  }
  return 0;
}

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
  const auto w0 = Clock::now();
  ncclResult_t r = ncclCommInitAll(c->comms.data(), ndev, devices);
  if (r != ncclSuccess) return NcclFail(r, "ncclCommInitAll");
  c->init_ms = std::chrono::duration<double, std::milli>(Clock::now() - w0).count();
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
  c->h_start_us.assign(ndev, 0.0);
  c->h_enq_us.assign(ndev, 0.0);
  c->handed.assign(ndev, 0);
  c->workers.resize(ndev);
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

Clique* FindClique(int ndev, const int* devices) {
  std::lock_guard<std::mutex> lk(g_mu);
  for (Clique* x : g_cliques)
    if ((int)x->devs.size() == ndev && std::memcmp(x->devs.data(), devices, sizeof(int) * ndev) == 0) return x;
  return nullptr;
}

}  // namespace

extern "C" {

int leveldb_crc32c_batch_multi(int ndev, const int* devices, const void* const* dev_base,
                               const uint64_t* const* dev_off, const uint32_t* const* dev_len,
                               const uint32_t* const* dev_init, const size_t* n, uint32_t* out0,
                               uint8_t* mismatch0, uint32_t flags, void* const* streams) {
  const auto t_call = Clock::now();
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
  const int fail_after = g_fail_after.load(std::memory_order_relaxed);
  const bool self = g_self_gather.load(std::memory_order_relaxed) != 0;
  CallArgs args{dev_base, dev_off,   dev_len, dev_init, n,
                out0,     mismatch0, flags,   streams,  self,
                fail_after >= 0 && fail_after < ndev ? fail_after : ndev, t_call};
  std::fill(c->handed.begin(), c->handed.end(), 0);
  // Once the first command is on a clique stream, every return goes through
  // here: the caller's streams wait for everything the call enqueued (its
  // batches, scratch growth, the gather), so a caller that frees or reuses
  // its buffers after an error never races the clique's work.  If a hand-off
  // itself fails, the clique's streams are drained instead.
  auto finish = [&](int code) {
    for (int p = 0; p < ndev; ++p) {
      if (!c->handed[p]) continue;
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
    c->h_call_us = std::chrono::duration<double, std::micro>(Clock::now() - t_call).count();
    return code;
  };
  // every partition's batch on its own device: partitions >= 1 (and 0 under
  // the self-gather hook) by their devices' workers, partition 0 here
  const int first_worker = self ? 0 : 1;
  for (int p = first_worker; p < ndev; ++p)
    if ((rc = StartWorker(c, p)) != 0) return finish(rc);
  const uint32_t g = ++c->gen;
  for (int p = first_worker; p < ndev; ++p) {
    Worker& w = *c->workers[p];
    w.args = &args;
    {
      std::lock_guard<std::mutex> wl(w.mu);
      w.go.store(g, std::memory_order_release);
    }
    w.cv.notify_one();
  }
  int first_err = 0;
  std::string first_msg;
  if (!self) {
    first_err = EnqueuePartition(c, 0, args);
    if (first_err != 0) first_msg = leveldb_crc32c_last_error();
  }
  for (int p = first_worker; p < ndev; ++p) {  // join, in partition order for the error reported
    Worker& w = *c->workers[p];
    for (uint32_t spins = 0; w.fin.load(std::memory_order_acquire) != g; ++spins)
      if (spins >= 4096) std::this_thread::yield();
    if (w.rc != 0 && first_err == 0) {
      first_err = w.rc;
      first_msg = w.err;
    }
  }
  if (first_err != 0) {
    prismdb::SetLastError(first_msg);
    return finish(first_err);
  }
  if (args.last < ndev)
    return finish(MultiFail(PRISMDB_CRC32C_EDEVICE, "batch_multi: injected failure (test hook)"));
  // The gather to devices[0]: partition p's results at offset n[0] + ... +
  // n[p-1].  Under the self-gather hook partition 0's results also travel,
  // from its scratch to out0 by a send / receive to itself on devices[0]'s
  // communicator: the same grouped call sequence on a one-device clique.
  if (ndev > 1 || self) {
    ncclResult_t r = ncclGroupStart();
    if (r != ncclSuccess) return finish(NcclFail(r, "ncclGroupStart"));
    size_t at = 0;
    for (int p = 0; p < ndev && r == ncclSuccess; ++p) {
      const size_t np = n[p];
      if (np == 0 || (p == 0 && !self)) {
        at += np;
        continue;
      }
      if (out0 != nullptr) {
        r = ncclSend(c->out[p], np, ncclUint32, 0, c->comms[p], c->streams[p]);
        if (r == ncclSuccess) r = ncclRecv(out0 + at, np, ncclUint32, p, c->comms[0], c->streams[0]);
      }
      if (r == ncclSuccess && mismatch0 != nullptr) {
        r = ncclSend(c->mm[p], np, ncclUint8, 0, c->comms[p], c->streams[p]);
        if (r == ncclSuccess) r = ncclRecv(mismatch0 + at, np, ncclUint8, p, c->comms[0], c->streams[0]);
      }
      at += np;
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
  Clique* c = FindClique(ndev, devices);
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

// Diagnostics (not in the public header): host wall times of the last
// successful call on this device list, in us: start_us[p] = from the call's
// entry to the start of partition p's enqueue (its skew against the others),
// enqueue_us[p] = that enqueue (hand-off, scratch, batch launches, event),
// *call_us = the whole call.  0; -1 if no such clique or call.
int prismdb_crc32c_multi_host_timing(int ndev, const int* devices, double* start_us, double* enqueue_us,
                                     double* call_us) {
  if (ndev < 1 || devices == nullptr) return -1;
  Clique* c = FindClique(ndev, devices);
  if (c == nullptr) return -1;
  std::lock_guard<std::mutex> lk(c->mu);
  if (!c->timed) return -1;
  for (int p = 0; p < ndev; ++p) {
    if (start_us != nullptr) start_us[p] = c->h_start_us[p];
    if (enqueue_us != nullptr) enqueue_us[p] = c->h_enq_us[p];
  }
  if (call_us != nullptr) *call_us = c->h_call_us;
  return 0;
}

// Test hook (not in the public header): fail every call right after
// partition p's batch is enqueued -- partitions after p enqueue no batch --
// (-1: off); returns the previous value.
int prismdb_crc32c_multi_fail_after(int p) {
  if (!prismdb::TestHooksEnabled()) return g_fail_after.load();  // (crc32c_capi.hip)
  return g_fail_after.exchange(p < 0 ? -1 : p);
}

// Test hook (not in the public header): with on != 0, partition 0 is also
// enqueued by a worker thread and its results reach out0 through the grouped
// ncclSend / ncclRecv, to itself -- the gather's call sequence on a
// one-device clique.  Returns the previous setting.
int prismdb_crc32c_multi_self_gather(int on) {
  if (!prismdb::TestHooksEnabled()) return g_self_gather.load();
  return g_self_gather.exchange(on != 0 ? 1 : 0);
}

}  // extern "C"
