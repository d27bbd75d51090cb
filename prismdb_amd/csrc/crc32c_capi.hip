// crc32c_capi.hip -- C ABI of the batch engine (include/prismdb_crc32c.h).
//
// Per-device context (tables in HBM, CU count, self-test) is created once with
// std::call_once; after that every call is lock-free.  The descriptor paths
// need a workspace (ticket map, span records, split-path scratch); it is
// cached per (thread, device, stream) so concurrent callers on distinct
// streams never share one, grown stream-ordered (hipMallocAsync /
// hipFreeAsync: no device-wide synchronisation), and released when the
// thread exits or when the thread has used more than kMaxWorkspaces streams.
#include <hip/hip_runtime.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <list>
#include <mutex>
#include <string>
#include <utility>

#include "../../include/prismdb_crc32c.h"
#include "crc32c_device.h"
#include "crc32c_gf2.h"

namespace prismdb {
// Streams the engine creates for itself (pipeline rings, batch_multi
// cliques) carry their own workspace: defined below.
void RegisterEngineStream(hipStream_t s);
void ReleaseEngineStream(hipStream_t s);
}  // namespace prismdb

namespace {

using prismdb::dev::DeviceTables;
using prismdb::dev::SpanBatch;
using prismdb::dev::SplitCounters;
using prismdb::dev::SplitWs;

thread_local std::string t_last_error;
// The calling thread's last descriptor batch: its split counters and stream
// (read back only by the test hook prismdb_crc32c_last_split).
thread_local const prismdb::dev::SplitCounters* t_last_counters = nullptr;
thread_local hipStream_t t_last_stream = nullptr;
thread_local bool t_last_direct = false;
thread_local bool t_last_pair = false;  // the planner batch launched the pair-run kernel
thread_local const uint32_t* t_last_stats = nullptr;
// Whether that batch ran on an engine-owned stream (a pipeline ring, a clique
// stream), whose workspace any thread may release (ReleaseEngineStream), and
// the release epoch then: the hooks above refuse to read it after a release.
thread_local bool t_last_owned = false;
thread_local uint64_t t_last_epoch = 0;
std::atomic<uint64_t> g_release_epoch{0};

// The calling thread's last batch ran on an engine stream whose workspace
// has been released since (by any thread): its pointers are gone.
bool LastBatchStale() {
  return t_last_owned && t_last_epoch != g_release_epoch.load(std::memory_order_acquire);
}

int Fail(int code, const std::string& msg) {
  t_last_error = msg;
  return code;
}

int FailHip(hipError_t e, const char* what) {
  return Fail(PRISMDB_CRC32C_EDEVICE, std::string(what) + ": " + hipGetErrorString(e));
}

constexpr int kMaxDevices = 64;

struct DeviceCtx {
  std::once_flag once;
  int status = 0;
  std::string error;
  DeviceTables* tabs = nullptr;
  int cus = 0;
  hipStream_t release = nullptr;  // frees of released workspaces (non-blocking: waits for nothing else)
};

DeviceCtx g_ctx[kMaxDevices];

// Test hooks (read on every call: atomics, relaxed).
// Route fixed-stride batches through the generic span kernel.
std::atomic<bool> g_force_generic{false};
// Which planner-path descriptor batches go through the lane kernel first
// (spans of kLaneMinLen..kLaneMaxLen bytes; the rest follow on the generic
// path): 0 = log-record batches (PRISMDB_CRC32C_LOG_HEADER), 1 = all, -1 = none.
std::atomic<int> g_lane_mode{0};
// Descriptor batches of at most this many spans take the one-launch kernel.
std::atomic<uint64_t> g_direct_max{prismdb::dev::kDirectPlainSpans};
// The one-launch path's ticket capacity (tests shrink it to reach the
// whole-span fallback) and its debug flags (DirectWs::dbg).
std::atomic<uint32_t> g_direct_cap{prismdb::dev::kDirectTickets};
std::atomic<uint32_t> g_direct_dbg{0};
// Descriptor batches of more than g_direct_max spans (without LOG_HEADER):
// windows of the one-launch kernel (1), the planner path (0), or (2, the
// default) windows up to two of them for batches that seal or verify block
// trailers (RunBatch), the planner path otherwise and beyond.  Two
// windows of SST files (twelve files, 201 744 spans) take 13.4 us per file,
// against 21.6 on the planner path, whose 5-7 launches and segment pass cost
// ~120 us per call; from there on the planner's balance wins, and on mixed
// span sizes it wins at any size (profiles/r04/r04h_bench.json,
// r04h_configs.json).  The one-launch kernel deals each wave a static run
// of consecutive spans, and a group leaves its CU only when its slowest wave
// is done: on spans of mixed sizes the windows lose to the planner's
// task-balanced slices (config-3 mix 65.7 against 74.8 % of the roofline,
// random spans 70.3 against 77.1 %), on uniform SST spans they win (72.8
// against 70.8 %; profiles/r04/r04e_configs.json).
std::atomic<int> g_windows{2};

void BuildTables(DeviceTables* t) {
  namespace g = prismdb::gf2;
  g::StrideTables(prismdb::dev::kStrideBytes, t->stride);
  g::StrideTables(4u, t->slice4);
  for (int l = 0; l < 64; ++l) {
    const g::Op m = g::ShiftBytes(prismdb::dev::kStrideBytes - 4u * (uint32_t)l);
    for (int n = 0; n < 8; ++n)
      for (uint32_t v = 0; v < 16; ++v) t->lane_nib[n][v][l] = g::Apply(m, v << (4 * n));
  }
  const g::Op s = g::ShiftBytes(prismdb::dev::kSegment);
  for (int i = 0; i < 32; ++i) t->shift_seg[i] = s.col[i];
  const g::Op s64 = g::ShiftBytes(64ull * prismdb::dev::kSegment);
  for (int i = 0; i < 32; ++i) t->shift_seg64[i] = s64.col[i];
  for (int l = 0; l < 64; ++l) {
    const g::Op m = g::ShiftBytes((63ull - (uint64_t)l) * prismdb::dev::kSegment);
    for (int i = 0; i < 32; ++i) t->lane_seg[i][l] = m.col[i];
  }
  // one-launch path: tickets of 2^lg chunks of 4 KiB
  const g::Op c = g::ShiftBytes(4096u);
  for (int i = 0; i < 32; ++i) t->shift_chunk[i] = c.col[i];
  for (int lg = 0; lg <= prismdb::dev::kTicketLgMax; ++lg) {
    const g::Op m = g::ShiftBytes(4096ull << lg);
    g::Op p = g::Identity();  // M^(63 - l), l = 63 down to 0; then M^64
    for (int l = 63; l >= 0; --l) {
      for (int i = 0; i < 32; ++i) t->tick_lane[lg][i][l] = p.col[i];
      p = g::Compose(m, p);
    }
    for (int i = 0; i < 32; ++i) t->tick64[lg][i] = p.col[i];
  }
}

int RunBatch(DeviceCtx& ctx, const SpanBatch& base_args, bool desc, bool verify, hipStream_t s, int route);

// Device known-answer self-test (util/crc32c.cc:269-273 vector, plus a 4 KiB
// block and a > kLongSpan span checked against the host Extend), through both
// descriptor paths: the one-launch kernel (route 1) and the planner (route 2).
int SelfTest(DeviceCtx& ctx) {
  const size_t kBig = prismdb::dev::kLongSpan + 3 * prismdb::dev::kSegment + 77;
  const size_t bytes = 64 + 4096 + kBig;
  unsigned char* h = new unsigned char[bytes];
  std::memset(h, 0, 64);
  std::memcpy(h + 1, "TestCRCBuffer", 13);
  uint64_t z = 0x5EED0001ull;
  for (size_t i = 64; i < bytes; ++i) {
    z = z * 6364136223846793005ull + 1442695040888963407ull;
    h[i] = (unsigned char)(z >> 56);
  }
  const uint64_t off[3] = {1, 64, 64 + 4096};
  const uint32_t len[3] = {13, 4096, (uint32_t)kBig};
  const uint32_t want[3] = {0xdcbc59fau,
                            leveldb_crc32c_value(reinterpret_cast<const char*>(h) + 64, 4096),
                            leveldb_crc32c_value(reinterpret_cast<const char*>(h) + 64 + 4096, kBig)};
  unsigned char* d = nullptr;
  const size_t desc_at = (bytes + 15) & ~size_t(15);
  hipError_t e = hipMalloc(&d, desc_at + 64);
  if (e != hipSuccess) {
    delete[] h;
    return FailHip(e, "self-test hipMalloc");
  }
  uint64_t* d_off = reinterpret_cast<uint64_t*>(d + desc_at);  // 24 B
  uint32_t* d_len = reinterpret_cast<uint32_t*>(d_off + 3);     // 12 B
  uint32_t* d_out = d_len + 3;                                  // 12 B
  e = hipMemcpy(d, h, bytes, hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMemcpy(d_off, off, sizeof(off), hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMemcpy(d_len, len, sizeof(len), hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMemset(d_out, 0, sizeof(uint32_t) * 3);
  if (e != hipSuccess) {
    (void)hipFree(d);
    delete[] h;
    return FailHip(e, "self-test upload");
  }
  SpanBatch a{};
  a.base = d;
  a.off = d_off;
  a.len = d_len;
  a.n = 3;
  a.out = d_out;
  int rc = 0;
  for (int route = 1; route <= 2 && rc == 0; ++route) {
    uint32_t got[3] = {0, 0, 0};
    e = hipMemset(d_out, 0, sizeof(got));
    if (e != hipSuccess) rc = FailHip(e, "self-test memset");
    if (rc == 0) rc = RunBatch(ctx, a, true, false, nullptr, route);
    if (rc == 0) {
      e = hipStreamSynchronize(nullptr);
      if (e != hipSuccess) rc = FailHip(e, "self-test sync");
    }
    if (rc == 0) {
      e = hipMemcpy(got, d_out, sizeof(got), hipMemcpyDeviceToHost);
      if (e != hipSuccess) rc = FailHip(e, "self-test download");
    }
    if (rc == 0 && (got[0] != want[0] || got[1] != want[1] || got[2] != want[2])) {
      char buf[200];
      std::snprintf(buf, sizeof(buf), "device self-test (%s path): got %08x %08x %08x want %08x %08x %08x",
                    route == 1 ? "one-launch" : "planner", got[0], got[1], got[2], want[0], want[1], want[2]);
      rc = Fail(PRISMDB_CRC32C_ESELFTEST, buf);
    }
  }
  (void)hipFree(d);
  delete[] h;
  return rc;
}

void InitDevice(DeviceCtx& ctx, int device) {
  hipError_t e = hipDeviceGetAttribute(&ctx.cus, hipDeviceAttributeMultiprocessorCount, device);
  if (e != hipSuccess || ctx.cus <= 0) {
    ctx.status = FailHip(e, "hipDeviceGetAttribute(multiprocessor count)");
    ctx.error = t_last_error;
    return;
  }
  e = hipStreamCreateWithFlags(&ctx.release, hipStreamNonBlocking);
  if (e != hipSuccess) {
    ctx.status = FailHip(e, "release stream");
    ctx.error = t_last_error;
    return;
  }
  DeviceTables* host = new DeviceTables;
  std::memset(host, 0, sizeof(DeviceTables));
  BuildTables(host);
  e = hipMalloc(&ctx.tabs, sizeof(DeviceTables));
  if (e == hipSuccess) e = hipMemcpy(ctx.tabs, host, sizeof(DeviceTables), hipMemcpyHostToDevice);
  delete host;
  if (e != hipSuccess) {
    ctx.status = FailHip(e, "table upload");
    ctx.error = t_last_error;
    return;
  }
  ctx.status = SelfTest(ctx);
  if (ctx.status != 0) ctx.error = t_last_error;
}

int GetCtx(DeviceCtx** out) {
  int device = 0;
  hipError_t e = hipGetDevice(&device);
  if (e != hipSuccess) return FailHip(e, "hipGetDevice");
  if (device < 0 || device >= kMaxDevices) return Fail(PRISMDB_CRC32C_EINVAL, "device ordinal out of range");
  DeviceCtx& ctx = g_ctx[device];
  std::call_once(ctx.once, [&]() { InitDevice(ctx, device); });
  if (ctx.status != 0) return Fail(ctx.status, ctx.error);
  *out = &ctx;
  return 0;
}

// ---- workspaces, per (thread, device, stream) ----
// Fixed part, allocated once: split-path counters, segment records and
// results, the long-span table, the planner's block sums.  Growing parts,
// sized for the largest batch seen: the span records (16 B + a 4-byte task
// count per span, plus the slice starts), the lane path's list (9 B per span)
// and the one-launch path's ticket workspace (allocated on its first use).
// Growth frees the old block on the stream, behind the work still reading
// it (hipFreeAsync), so one thread's growth never stalls other streams.
struct Workspace {
  int device = -1;
  hipStream_t stream = nullptr;
  // Completion of the last batch of each slot parity (the one-launch path's
  // calls alternate between two slots; the planner path marks done[gen & 1]):
  // waiting for both covers everything that used the workspace.
  hipEvent_t done[2] = {nullptr, nullptr};
  // The planner path's side stream (created on first use): the segment pass
  // runs there, concurrently with the span kernel, between a fork and a join
  // event on the batch's stream.
  hipStream_t side = nullptr;
  hipEvent_t fork = nullptr, join = nullptr;
  void* mem = nullptr;
  char* grow = nullptr;
  size_t cap_rec = 0;
  uint32_t cap_streams = 0;  // the span-kernel streams the slice starts of `grow` were sized for
  char* qgrow = nullptr;
  size_t cap_q = 0;
  char* sgrow = nullptr;  // sealing planner batches without `out`: their results for the trailer pass
  size_t cap_s = 0;
  char* direct = nullptr;  // word, done | ticket map | partials | per-span counters
  uint32_t gen = 0;
  // Planner calls alternate between two counter blocks (pcall parity); each
  // call's plan kernel zeroes the block of the next.  dirty: a call used its
  // block and failed before its plan kernel was enqueued, so the next call
  // fills its block first.
  uint32_t pcall = 0;
  bool dirty = false;
  bool owned = false;  // an engine stream's (g_owned), not a thread's
  SplitWs ws{};
};

// A thread that has used more streams than this evicts its least recently
// used workspace.
constexpr size_t kMaxWorkspaces = 8;

// Give w's device memory back: wait for the last batch that used it (its
// event -- valid even when the caller has destroyed the stream; nothing
// device-wide), free every block on the device's release stream, and trim
// the default pool so the memory leaves the process's pool too.
void SyncAndRelease(Workspace& w) {
  {
    const char* t = reinterpret_cast<const char*>(t_last_counters);
    const char* c = reinterpret_cast<const char*>(w.ws.counters);
    if (c != nullptr && t >= c && t < c + 2 * prismdb::dev::kCounterBlock) t_last_counters = nullptr;
  }
  if (w.direct != nullptr && t_last_stats == reinterpret_cast<const uint32_t*>(w.direct + 32)) t_last_stats = nullptr;
  int cur = 0;
  (void)hipGetDevice(&cur);
  if (w.device != cur) (void)hipSetDevice(w.device);
  for (hipEvent_t ev : w.done)
    if (ev != nullptr) (void)hipEventSynchronize(ev);
  const hipStream_t rs = g_ctx[w.device].release;
  for (void* blk : {static_cast<void*>(w.mem), static_cast<void*>(w.grow), static_cast<void*>(w.qgrow),
                    static_cast<void*>(w.sgrow), static_cast<void*>(w.direct)})
    if (blk != nullptr) (void)hipFreeAsync(blk, rs);
  (void)hipStreamSynchronize(rs);
  hipMemPool_t pool = nullptr;
  if (hipDeviceGetDefaultMemPool(&pool, w.device) == hipSuccess) (void)hipMemPoolTrimTo(pool, 0);
  for (hipEvent_t ev : w.done)
    if (ev != nullptr) (void)hipEventDestroy(ev);
  if (w.side != nullptr) {  // (idle: its last work is behind a join the done events cover)
    (void)hipStreamSynchronize(w.side);
    (void)hipStreamDestroy(w.side);
  }
  for (hipEvent_t ev : {w.fork, w.join})
    if (ev != nullptr) (void)hipEventDestroy(ev);
  if (w.device != cur) (void)hipSetDevice(cur);
  w = Workspace{};
}

struct WorkspaceCache {
  std::list<Workspace> lru;  // most recently used first
  ~WorkspaceCache() {
    // A worker thread gives its device memory back when it exits.  The main
    // thread's thread-local destructors run inside exit(), where the HIP
    // runtime (or a profiler wrapped around it) may be tearing down already:
    // its workspaces are left to the OS (as the host pipeline's rings are).
    if (syscall(SYS_gettid) == getpid()) return;
    for (Workspace& w : lru) SyncAndRelease(w);
  }
};

// Slice starts needed for n spans: nslices + 1 <= n/2 + 32 * streams + 2
// (crc32c_slice_scan_kernel: K = m S slices with m <= kSlicesPerStream or
// enough slices to keep <= 63 tasks each).
size_t SliceCap(size_t n, uint32_t streams) {
  return n / 2 + 2 * (size_t)prismdb::dev::kSlicesPerStream * streams + 4;
}

constexpr uint64_t kCapSeg = 1u << 20;   // 1 Mi segments = 32 GiB of long spans per call
constexpr uint32_t kCapLong = 1u << 18;

WorkspaceCache& ThreadWorkspaces() {
  thread_local WorkspaceCache cache;
  return cache;
}

// Streams the engine itself owns and lends to one caller at a time (the host
// pipeline's ring streams, leased from a per-device pool across threads;
// batch_multi's clique streams):
// their workspace belongs to the stream, not to the calling thread, and is
// released with it (prismdb::ReleaseEngineStream) -- as thread-local entries
// they piled up (up to kMaxWorkspaces per thread that ever leased a ring) or
// cycled through the LRU.
std::mutex g_owned_mu;
std::list<Workspace> g_owned;  // (list: entries never move)
// Lock-free snapshot of the owned streams' handles, so a batch on any other
// stream -- every PrismDB partition thread's own -- never takes g_owned_mu:
// slots are written under the mutex, read with relaxed loads.  More engine
// streams than slots at once (not reached: kKeepIdle rings per device plus
// the live leases and clique streams) send every lookup through the mutex.
constexpr int kOwnedSlots = 256;
std::atomic<hipStream_t> g_owned_keys[kOwnedSlots];
std::atomic<int> g_owned_spill{0};  // registered streams that found no free slot

// Allocates w's fixed part on stream s (device current).
int InitWorkspace(Workspace& w, int device, hipStream_t s) {
  w.device = device;
  w.stream = s;
  hipError_t e = hipSuccess;
  const size_t bytes = 2 * prismdb::dev::kCounterBlock + kCapSeg * (16 + 4) + (size_t)kCapLong * (8 + 8 + 4) +
                       (size_t)prismdb::dev::kMaxPlanBlocks * 8;
  e = hipEventCreateWithFlags(&w.done[0], hipEventDisableTiming);
  if (e == hipSuccess) e = hipEventCreateWithFlags(&w.done[1], hipEventDisableTiming);
  if (e == hipSuccess) e = hipMallocAsync(&w.mem, bytes, s);
  // both planner counter blocks start zeroed (then each call zeroes the next's)
  if (e == hipSuccess) e = hipMemsetAsync(w.mem, 0, 2 * prismdb::dev::kCounterBlock, s);
  if (e != hipSuccess) {
    for (hipEvent_t ev : w.done)
      if (ev != nullptr) (void)hipEventDestroy(ev);
    w = Workspace{};
    return FailHip(e, "workspace allocation");
  }
  char* p = static_cast<char*>(w.mem);
  w.ws.counters = reinterpret_cast<SplitCounters*>(p);  // two counter blocks, one per call parity
  p += 2 * prismdb::dev::kCounterBlock;
  w.ws.seg_rec = reinterpret_cast<prismdb::dev::SpanRec*>(p);
  p += kCapSeg * 16;
  w.ws.long_span = reinterpret_cast<uint64_t*>(p);
  p += (size_t)kCapLong * 8;
  w.ws.long_first = reinterpret_cast<uint64_t*>(p);
  p += (size_t)kCapLong * 8;
  w.ws.seg_out = reinterpret_cast<uint32_t*>(p);
  p += kCapSeg * 4;
  w.ws.long_nseg = reinterpret_cast<uint32_t*>(p);
  p += (size_t)kCapLong * 4;
  w.ws.bsum = reinterpret_cast<uint64_t*>(p);
  w.ws.cap_seg = kCapSeg;
  w.ws.cap_long = kCapLong;
  return 0;
}


Workspace* FindWorkspace(hipStream_t s, int& rc) {
  int device = 0;
  hipError_t e = hipGetDevice(&device);
  if (e != hipSuccess) {
    rc = FailHip(e, "hipGetDevice");
    return nullptr;
  }
  bool maybe_owned = s != nullptr && g_owned_spill.load(std::memory_order_acquire) > 0;
  for (int k = 0; k < kOwnedSlots && !maybe_owned && s != nullptr; ++k)
    maybe_owned = g_owned_keys[k].load(std::memory_order_acquire) == s;
  if (maybe_owned) {
    std::lock_guard<std::mutex> lk(g_owned_mu);
    for (Workspace& w : g_owned) {
      if (w.stream != s) continue;
      if (w.mem == nullptr && (rc = InitWorkspace(w, device, s)) != 0) {
        w.stream = s;  // (stays registered: the next call retries)
        return nullptr;
      }
      w.owned = true;
      rc = 0;
      return &w;
    }
  }
  WorkspaceCache& cache = ThreadWorkspaces();
  auto& lru = cache.lru;
  for (auto it = lru.begin(); it != lru.end(); ++it) {
    if (it->device == device && it->stream == s) {
      if (it != lru.begin()) lru.splice(lru.begin(), lru, it);
      rc = 0;
      return &lru.front();
    }
  }
  if (lru.size() >= kMaxWorkspaces) {
    SyncAndRelease(lru.back());
    lru.pop_back();
  }
  lru.emplace_front();
  if ((rc = InitWorkspace(lru.front(), device, s)) != 0) {
    lru.pop_front();
    return nullptr;
  }
  return &lru.front();
}

// Replace *blk (size irrelevant) by a fresh block of `bytes` on stream s; the
// old one is freed behind the work already enqueued on s.
int GrowBlock(char** blk, size_t bytes, hipStream_t s, const char* what) {
  if (*blk != nullptr) {
    hipError_t e = hipFreeAsync(*blk, s);
    *blk = nullptr;
    if (e != hipSuccess) return FailHip(e, what);
  }
  hipError_t e = hipMallocAsync(reinterpret_cast<void**>(blk), bytes, s);
  if (e != hipSuccess) {
    *blk = nullptr;
    return FailHip(e, what);
  }
  return 0;
}

int PlannerWorkspace(Workspace& w, hipStream_t s, size_t nspans, uint32_t streams, bool lane, SplitWs* out) {
  // The slice starts' room depends on the stream count too: a block sized
  // for fewer streams is grown, and the layout below follows the block's own
  // sizing, never the call's (round 4's one-sequence span kernel, planned
  // for half the streams, overran it).
  if (w.cap_rec < nspans || w.cap_streams < streams) {
    const size_t cap = nspans < 4096 ? 4096 : nspans + nspans / 4;
    const uint32_t cs = streams > w.cap_streams ? streams : w.cap_streams;
    const size_t bytes = cap * (16 + 4) + SliceCap(cap, cs) * 8 + 16;
    w.cap_rec = 0;
    w.cap_streams = cs;
    if (int rc = GrowBlock(&w.grow, bytes, s, "span record workspace")) return rc;
    w.cap_rec = cap;
  }
  if (lane && w.cap_q < nspans) {
    const size_t cap = nspans < 4096 ? 4096 : nspans + nspans / 4;
    w.cap_q = 0;
    if (int rc = GrowBlock(&w.qgrow, cap * 9 + 1024, s, "lane list workspace")) return rc;
    w.cap_q = cap;
  }
  w.ws.list = lane ? reinterpret_cast<uint32_t*>(w.qgrow) : nullptr;
  w.ws.qout = lane ? reinterpret_cast<uint32_t*>(w.qgrow + w.cap_q * 4) : nullptr;
  w.ws.qmm = lane ? reinterpret_cast<uint8_t*>(w.qgrow + w.cap_q * 8) : nullptr;
  w.ws.rec = reinterpret_cast<prismdb::dev::SpanRec*>(w.grow);
  w.ws.slice_start = reinterpret_cast<uint64_t*>(w.grow + w.cap_rec * 16);
  w.ws.cnt = reinterpret_cast<uint32_t*>(w.grow + w.cap_rec * 16 + SliceCap(w.cap_rec, w.cap_streams) * 8);
  // Planner tiles: whole multiples of its block size, at most kMaxPlanBlocks.
  namespace d = prismdb::dev;
  const uint64_t per = (nspans + d::kMaxPlanBlocks - 1) / d::kMaxPlanBlocks;
  w.ws.tile = (per + d::kPlanThreads - 1) / d::kPlanThreads * d::kPlanThreads;
  w.ws.nblocks = (uint32_t)((nspans + w.ws.tile - 1) / w.ws.tile);
  w.ws.nstreams = streams;
  *out = w.ws;
  return 0;
}

// The one-launch path's workspace: four claim words (call g uses word g % 4
// and zeroes word (g + 2) % 4 for the call after next; calls of a stream run
// in stream order, so the word a call zeroes is idle), the usage counters, and
// two slots (call parity) of: the ticket map (32-B entries of four words
// tagged with the call's gen), the tagged partial registers and the per-span
// ticket counters (zero between calls: a span's combiner resets its own).
int DirectWorkspace(Workspace& w, hipStream_t s, prismdb::dev::DirectWs* out) {
  namespace d = prismdb::dev;
  const size_t cap = d::kDirectTickets;
  const size_t slot_bytes = cap * (32 + 8 + 4);
  const size_t bytes = 256 + 4096 + 2 * slot_bytes;
  if (w.direct == nullptr) {
    if (int rc = GrowBlock(&w.direct, bytes, s, "ticket workspace")) return rc;
    hipError_t e = hipMemsetAsync(w.direct, 0, bytes, s);
    if (e != hipSuccess) return FailHip(e, "ticket workspace memset");
  }
  // Generations: the words a call writes carry gen's low 16 bits (its tag),
  // so words of earlier calls never match.  At the wrap (2^16 calls) the
  // workspace is zeroed again (a fill kernel in stream order: behind both
  // slots' last calls, ahead of the next one -- every one-launch call is an
  // ordered launch) and the count restarts.
  if ((++w.gen & d::kTagMask) == 0) {
    hipError_t e = hipMemsetAsync(w.direct, 0, bytes, s);
    if (e != hipSuccess) return FailHip(e, "ticket workspace memset");
    w.gen = 1;
  }
  char* p = w.direct;
  out->word = reinterpret_cast<unsigned long long*>(p + 8 * (w.gen & 3u));
  out->next = reinterpret_cast<unsigned long long*>(p + 8 * ((w.gen + 2u) & 3u));
  out->stats = reinterpret_cast<uint32_t*>(p + 32);
  out->help = reinterpret_cast<uint32_t*>(p + 256);
  char* sl = p + 256 + 4096 + (size_t)(w.gen & 1u) * slot_bytes;
  out->tmap = reinterpret_cast<uint64_t*>(sl);
  out->part = reinterpret_cast<uint64_t*>(sl + cap * 32);
  out->cdone = reinterpret_cast<uint32_t*>(sl + cap * 40);
  out->cap = g_direct_cap.load(std::memory_order_relaxed);
  out->dbg = g_direct_dbg.load(std::memory_order_relaxed);
  out->tag = w.gen & d::kTagMask;  // 0 is the zeroed workspace's
  return 0;
}

enum Route { kRouteAuto = 0, kRouteDirect = 1, kRoutePlanner = 2 };

// A descriptor batch of more spans than one launch of the one-launch kernel
// takes, as ceil(n / wmax) equal windows of consecutive spans, one launch of
// that kernel each, back to back on the caller's stream.  (Round 4 first ran
// the windows on two side streams so a window's start-up would overlap its
// predecessor's tail; but the kernel's grid is one group per CU with static
// runs dealt for every wave at once, and two such kernels in flight shared
// the CUs: twelve SST files per call took 18.0 us per file that way against
// 12.8 us in calls of seven files, profiles/r04/r04g_bench.json.)
int RunWindows(DeviceCtx& ctx, const SpanBatch& a, bool verify, hipStream_t s, uint64_t wmax) {
  const uint64_t cap = 64ull * (uint64_t)ctx.cus * (prismdb::dev::kDirectThreads / 64);  // one span run per wave
  if (wmax > cap) wmax = cap;
  const uint64_t nwin = (a.n + wmax - 1) / wmax;
  uint64_t at = 0;
  for (uint64_t k = 0; k < nwin; ++k) {
    const uint64_t m = (a.n - at) / (nwin - k);  // equal windows, the remainder spread over the last ones
    SpanBatch p = a;
    p.off += at;
    p.len += at;
    if (p.init != nullptr) p.init += at;
    if (p.out != nullptr) p.out += at;
    if (p.mismatch != nullptr) p.mismatch += at;
    p.n = m;
    if (int rc = RunBatch(ctx, p, true, verify, s, kRouteDirect)) return rc;
    at += m;
  }
  return 0;
}

// Launch sequence.  Fixed stride, aligned, <= 4 KiB: one kernel.  Descriptor
// batches of <= g_direct_max spans: one kernel (crc32c_direct.hip).  The
// rest: plan (span records, long spans cut into segments) -> span pass (long
// spans skipped) -> segment pass -> combine, with the lane kernel and its
// list in front for log-record batches.
// The workspace's side stream and its fork / join events, created on first use.
int SideStream(Workspace* w) {
  if (w->side != nullptr) return 0;
  hipError_t e = hipStreamCreateWithFlags(&w->side, hipStreamNonBlocking);
  if (e == hipSuccess) e = hipEventCreateWithFlags(&w->fork, hipEventDisableTiming);
  if (e == hipSuccess) e = hipEventCreateWithFlags(&w->join, hipEventDisableTiming);
  return e == hipSuccess ? 0 : FailHip(e, "side stream");
}

int RunBatch(DeviceCtx& ctx, const SpanBatch& base_args, bool desc, bool verify, hipStream_t s, int route) {
  SpanBatch a = base_args;
  // PRISMDB_CRC32C_UNORDERED is accepted and has no effect: every launch is
  // in stream order (an any-order launch is not supported on gfx9, and it
  // measured slower where it ran: 25.9 against 24.9 us per SST file)
  a.flags &= ~PRISMDB_CRC32C_UNORDERED;
  a.tabs = ctx.tabs;
  a.role = prismdb::dev::kRoleSpans;
  // Fast path: fixed stride, 4-byte aligned, 4..4096-byte multiple-of-4 spans
  // (verify: up to 4092 bytes and not a multiple of 256, so that the stored
  // trailer word fits round 0's padding lanes).
  const uint32_t max_len = 4u * prismdb::dev::kChunkWords - (verify ? 4u : 0u);
  if (!desc && (verify || a.out != nullptr) && (!verify || (a.len_c & 255u) != 0) &&
      (a.flags & (prismdb::dev::kFlagWriteTrailer | prismdb::dev::kFlagLogHeader)) == 0 &&
      a.len_c >= 4 && a.len_c <= max_len && (a.len_c & 3u) == 0 &&
      (a.stride & 3u) == 0 && (reinterpret_cast<uintptr_t>(a.base) & 3u) == 0 &&
      !g_force_generic.load(std::memory_order_relaxed)) {
    hipError_t e = prismdb::dev::launch_fixed(a, verify, ctx.cus, s);
    return e == hipSuccess ? 0 : FailHip(e, "fixed kernel launch");
  }
  int rc = 0;
  Workspace* w = FindWorkspace(s, rc);
  if (w == nullptr) return rc;
  // Whatever follows, the workspace's events mark the end of this call's
  // work: the one-launch kernel's own completion (hipExtLaunchKernel's stop
  // event), or a marker after the planner path's last launch (ordered: it
  // covers everything before it).
  struct MarkDone {
    Workspace* w;
    hipStream_t s;
    bool by_launch = false;
    ~MarkDone() {
      if (!by_launch) (void)hipEventRecord(w->done[w->gen & 1u], s);
    }
  } mark{w, s};
  // Between a fork onto the workspace's side stream and its join, an error
  // return still joins the side stream back into s (before `mark` records
  // the done event, which must cover the side stream's kernels: the next
  // call's growth or reuse of the lists and segment records waits on it).
  struct SideJoin {
    Workspace* w;
    hipStream_t s;
    bool armed = false;
    ~SideJoin() {
      if (armed && (hipEventRecord(w->join, w->side) != hipSuccess || hipStreamWaitEvent(s, w->join, 0) != hipSuccess))
        (void)hipStreamSynchronize(w->side);
    }
  } side_join{w, s};
  // One launch: <= direct_max spans (2^17), or, by default (wmode 2), a
  // batch that seals or verifies block trailers (not log records) up to the
  // kernel's capacity -- the SST-file batches the windows below would
  // otherwise cut in two.
  const int wmode = g_windows.load(std::memory_order_relaxed);
  const bool block_trailers = verify || (a.flags & prismdb::dev::kFlagWriteTrailer) != 0;
  const bool sst_batch = wmode == 2 && block_trailers && !(a.flags & prismdb::dev::kFlagLogHeader);
  const bool direct = desc && (route == kRouteDirect ||
                               (route == kRouteAuto && (a.n <= g_direct_max.load(std::memory_order_relaxed) || sst_batch)));
  if (direct && a.n <= prismdb::dev::kDirectMaxSpans &&
      a.n <= 64ull * (uint64_t)ctx.cus * (prismdb::dev::kDirectThreads / 64)) {
    prismdb::dev::DirectWs d{};
    if ((rc = DirectWorkspace(*w, s, &d)) != 0) return rc;
    t_last_direct = true;
    t_last_stats = d.stats;
    t_last_stream = s;
    t_last_owned = w->owned;
    t_last_epoch = g_release_epoch.load(std::memory_order_acquire);
    mark.by_launch = true;
    hipError_t e = prismdb::dev::launch_direct(a, verify, ctx.cus, d, s, w->done[w->gen & 1u]);
    return e == hipSuccess ? 0 : FailHip(e, "direct kernel launch");
  }
  // Bulk descriptor batches: windows of the one-launch kernel.  By default
  // (wmode 2) only batches of <= 2 windows that seal or verify block
  // trailers: TableBuilder / ReadBlock batches, whose spans are block_size-
  // bounded data blocks plus one index block per file (uniform: the windows'
  // static runs balance them).  A plain checksum batch has no such shape and
  // takes the planner's task-balanced slices: 200 000 config-3 spans (1-64
  // KiB) ran at 57.5 % of the roofline as windows against 70.5 % on the
  // planner path (profiles/r06/r06s_configs.json, config3_band).
  const uint64_t wmax = g_direct_max.load(std::memory_order_relaxed);
  if (desc && route == kRouteAuto && wmax > 0 && a.n > wmax &&
      (wmode == 1 || (wmode == 2 && a.n <= 2 * wmax && block_trailers)) && !(a.flags & prismdb::dev::kFlagLogHeader))
    return RunWindows(ctx, base_args, verify, s, wmax);
  // The span kernel indexes records with 32 bits: cut larger batches.
  if (a.n > prismdb::dev::kMaxGenericSpans) {
    for (uint64_t i = 0; i < a.n; i += prismdb::dev::kMaxGenericSpans) {
      SpanBatch p = base_args;
      p.n = a.n - i < prismdb::dev::kMaxGenericSpans ? a.n - i : prismdb::dev::kMaxGenericSpans;
      if (desc) {
        p.off += i;
        p.len += i;
        if (p.init != nullptr) p.init += i;
      } else {
        p.base += i * a.stride;
      }
      if (p.out != nullptr) p.out += i;
      if (p.mismatch != nullptr) p.mismatch += i;
      if ((rc = RunBatch(ctx, p, desc, verify, s, kRoutePlanner)) != 0) return rc;
    }
    return 0;
  }
  SplitWs ws{};
  // Short spans first, one per lane (crc32c_lane_kernel); the generic path
  // below then runs over the list of the others only.
  const int lane_mode = g_lane_mode.load(std::memory_order_relaxed);
  const bool lane = desc && (lane_mode > 0 || (lane_mode == 0 && (a.flags & prismdb::dev::kFlagLogHeader)));
  // The span kernel's record streams: two per wave of its persistent grid.
  // (Round 4 tried one task sequence per wave here, the one-launch kernel's
  // ring: within +-2 % on the bulk rows, profiles/r04/r04i_configs_*.json;
  // its kernels are in git history: crc32c_kernels.hip at 36498f1.)
  const uint32_t streams = 2u * (uint32_t)ctx.cus * prismdb::dev::kWavesPerGroup;
  if ((rc = PlannerWorkspace(*w, s, a.n, streams, lane, &ws)) != 0) return rc;
  // Counters: the block of this call's parity, zeroed by the previous
  // planner call's plan kernel (or at the workspace's creation) -- no fill
  // kernel in front of the call (it and its gap took 6.7 us of a config-5
  // call, profiles/r05/r05aa_c5_seal/one_call_timeline.csv).
  static_assert(sizeof(SplitCounters) <= 256, "SplitCounters fills the first 256 B of a counter block");
  {
    char* const cb = reinterpret_cast<char*>(w->ws.counters);
    ws.counters = reinterpret_cast<SplitCounters*>(cb + prismdb::dev::kCounterBlock * (w->pcall & 1u));
    ws.zero_next = reinterpret_cast<SplitCounters*>(cb + prismdb::dev::kCounterBlock * ((w->pcall + 1u) & 1u));
  }
  hipError_t e = hipSuccess;
  if (w->dirty) {  // the last call failed after using this block, before its plan kernel
    e = hipMemsetAsync(ws.counters, 0, prismdb::dev::kCounterBlock, s);
    if (e != hipSuccess) return FailHip(e, "hipMemsetAsync");
  }
  w->dirty = true;  // until this call's plan kernel is enqueued
  t_last_counters = ws.counters;
  t_last_stream = s;
  t_last_direct = false;
  t_last_owned = w->owned;
  t_last_epoch = g_release_epoch.load(std::memory_order_acquire);
  // Sealing: the span kernels leave the trailers to one pass after them
  // (crc32c_trailer_kernel), which reads the results back -- from scratch
  // when the caller passed no `out`.  Not behind the lane kernel: it stores
  // each log record's header crc as the record finishes, and that measured
  // 5 % faster on ~1 KB WAL records than the pass (3931 against 3739 GB/s,
  // profiles/r05/r05g_variants_lane_seal.json) -- a lane's store is one of
  // 64 records' in flight, not a wave-wide stall.
  const bool trailer_pass = (a.flags & prismdb::dev::kFlagWriteTrailer) != 0 && !lane;
  if (trailer_pass) {
    a.flags &= ~prismdb::dev::kFlagWriteTrailer;
    if (a.out == nullptr) {
      if (w->cap_s < a.n) {
        const size_t cap = a.n < 4096 ? 4096 : a.n + a.n / 4;
        w->cap_s = 0;
        if ((rc = GrowBlock(&w->sgrow, cap * 4, s, "trailer result workspace")) != 0) return rc;
        w->cap_s = cap;
      }
      a.out = reinterpret_cast<uint32_t*>(w->sgrow);
    }
  }
  uint32_t* const res_out = a.out;  // the caller's out, or the trailer pass's scratch
  uint8_t* const caller_mm = a.mismatch;
  if (lane) {
    // The list of the spans the lane kernel does not own is built on the
    // side stream while the lane kernel runs; the generic path below waits
    // for it.
    if ((rc = SideStream(w)) != 0) return rc;
    e = hipEventRecord(w->fork, s);
    if (e == hipSuccess) e = hipStreamWaitEvent(w->side, w->fork, 0);
    side_join.armed = e == hipSuccess;
    if (e == hipSuccess) e = prismdb::dev::launch_long_list(a, ws, w->side);
    if (e == hipSuccess) e = hipEventRecord(w->join, w->side);
    if (e != hipSuccess) return FailHip(e, "long-span list launch");
    a.claim = &ws.counters->lane_claim;  // (zeroed with the counters above)
    e = prismdb::dev::launch_lane(a, verify, ctx.cus, s);
    if (e == hipSuccess) e = hipStreamWaitEvent(s, w->join, 0);
    if (e != hipSuccess) return FailHip(e, "lane kernel launch");
    side_join.armed = false;
    a.idx = ws.list;
    a.n_dev = &ws.counters->nlist;
    if (a.out != nullptr) a.out = ws.qout;
    if (a.mismatch != nullptr) a.mismatch = ws.qmm;
  }
  a.skip_above = prismdb::dev::kLongSpan;
  // span records for the kernel launch_span picks (its chunk size)
  a.chunk_lg = (a.flags & prismdb::dev::kFlagLogHeader) ? prismdb::dev::kLgChunkWordsLog : 10u;
  a.overflow = &ws.counters->overflow;
  a.rec = ws.rec;
  // The segment pass (long spans' 32 KiB pieces) needs only the plan: it
  // runs on the workspace's side stream from the plan kernel's end (the
  // fork: that kernel's stop event, not a marker after it -- a marker held
  // the next kernel back ~6.5 us, profiles/r05/r05aa_c5_seal), next to the
  // slice kernels and the span kernel, whose groups take the CUs as its
  // groups leave them.  The combine waits for both.  (Forked after the slice
  // mark, it got CUs only as span-kernel groups left: once the pair-run
  // kernel's tail balanced its waves they all left together, and a config-5
  // call's 2145 segments ran after it, 30-140 us; profiles/r06/r06ag.)
  if ((rc = SideStream(w)) != 0) return rc;
  // Task-balanced slices need more records than span streams: with n <= the
  // stream count every stream holds at most one record either way, and the
  // two slice kernels' launches are ~9 us of a file-sized call.
  const bool sliced = a.n > streams;
  e = prismdb::dev::launch_plan(a, desc, ws, s, w->fork);
  if (e != hipSuccess) return FailHip(e, "plan kernel launch");
  w->pcall++;  // the next call's block is the one this plan kernel zeroes
  w->dirty = false;
  e = hipStreamWaitEvent(w->side, w->fork, 0);
  if (e != hipSuccess) return FailHip(e, "side stream fork");
  side_join.armed = true;
  SpanBatch seg{};
  seg.base = a.base;
  seg.n = ws.cap_seg;
  seg.n_dev = &ws.counters->nseg;
  seg.out = ws.seg_out;
  seg.skip_above = 0xFFFFFFFFu;
  seg.overflow = &ws.counters->overflow;
  seg.role = prismdb::dev::kRoleSegments;
  seg.tabs = ctx.tabs;
  seg.rec = ws.seg_rec;
  e = prismdb::dev::launch_span(seg, false, ctx.cus, w->side, w->join);  // the join: its stop event
  if (e != hipSuccess) return FailHip(e, "segment kernel launch");
  if (sliced) {
    e = prismdb::dev::launch_slices(a, ws, s);
    if (e != hipSuccess) return FailHip(e, "slice kernels launch");
    a.slice_start = ws.slice_start;
    a.nslices_dev = &ws.counters->nslices;
    a.tasks_dev = &ws.counters->tasks;
  }
  // Large batches of one-task records take the pair-run kernel (its two
  // streams read adjacent spans); it is launched next to the general one,
  // and the one whose schedule the scan did not pick leaves at once.
  a.pair_kernel = a.slice_start != nullptr && a.n >= prismdb::dev::kPairMinSpans && !lane &&
                          !(a.flags & prismdb::dev::kFlagLogHeader)
                      ? 1u
                      : 0u;
  t_last_pair = a.pair_kernel != 0u;
  a.claim = &ws.counters->claim;  // (zeroed with the counters above)
  a.claims = reinterpret_cast<uint32_t*>(reinterpret_cast<char*>(ws.counters) + 256);
  e = prismdb::dev::launch_span(a, verify, ctx.cus, s);
  if (e != hipSuccess) return FailHip(e, "span kernel launch");
  // The call's last kernel completes the workspace's done event itself (its
  // stop event) instead of a marker after it (MarkDone, on an error return).
  hipEvent_t const done = w->done[w->gen & 1u];
  if (trailer_pass) {
    // Sealing: the trailers of every span but the long ones go out first,
    // while the segment pass finishes on the side stream; then the join and
    // the combine, which stores the long spans' trailers with their results.
    // (Joined first, the pass waited for the segment pass, which ends after
    // the span kernel, and for the cross-queue wait: a config-5 seal's tail
    // after the pair-run kernel 144 -> 137.5 us, the join's own ~8 us now
    // between the pass and the combine; profiles/r06/r06ac_timeline.txt.)
    SpanBatch t = base_args;
    t.n = a.n;
    t.skip_above = prismdb::dev::kLongSpan;
    t.overflow = &ws.counters->overflow;  // (after an overflow the span pass folded them: no skip)
    e = prismdb::dev::launch_trailers(t, desc, res_out, s, nullptr);
    if (e != hipSuccess) return FailHip(e, "trailer kernel launch");
    e = hipStreamWaitEvent(s, w->join, 0);
    if (e != hipSuccess) return FailHip(e, "side stream join");
    side_join.armed = false;
    SpanBatch c = a;
    c.flags |= prismdb::dev::kFlagWriteTrailer;
    e = prismdb::dev::launch_combine(c, desc, verify, ws, s, done);
    if (e != hipSuccess) return FailHip(e, "combine kernel launch");
    mark.by_launch = true;
    return 0;
  }
  e = hipStreamWaitEvent(s, w->join, 0);
  if (e != hipSuccess) return FailHip(e, "side stream join");
  side_join.armed = false;
  e = prismdb::dev::launch_combine(a, desc, verify, ws, s, lane ? nullptr : done);
  if (e != hipSuccess) return FailHip(e, "combine kernel launch");
  if (lane) {
    SpanBatch back = a;
    back.out = res_out;
    back.mismatch = caller_mm;
    e = prismdb::dev::launch_scatter(back, ws, ws.qout, ws.qmm, s, done);
    if (e != hipSuccess) return FailHip(e, "scatter kernel launch");
  }
  mark.by_launch = true;
  return 0;
}

}  // namespace

namespace prismdb {
void SetLastError(const std::string& msg) { t_last_error = msg; }

// The prismdb_* setters below (and the pipeline's and batch_multi's) change
// process-global routing or inject failures: one PrismDB partition thread
// calling one would reroute or fail every other thread's batches.  They act
// only when the process runs with PRISMDB_ENABLE_TEST_HOOKS=1 (read at the
// first hook call; the tests, the bench and the tools set it); otherwise
// each is a no-op that reports the current setting and sets the last error.
bool TestHooksEnabled() {
  static const bool on = [] {
    const char* e = std::getenv("PRISMDB_ENABLE_TEST_HOOKS");
    return e != nullptr && e[0] == '1' && e[1] == '\0';
  }();
  if (!on) t_last_error = "test hooks are off (set PRISMDB_ENABLE_TEST_HOOKS=1)";
  return on;
}

// The engine's own streams (pipeline rings, clique streams): one workspace
// per stream, whichever thread calls on it (one at
// a time: a leased ring, the owning workspace's thread, the clique's mutex);
// released (after its last batch) by ReleaseEngineStream before the stream
// is destroyed.
void RegisterEngineStream(hipStream_t s) {
  std::lock_guard<std::mutex> lk(g_owned_mu);
  g_owned.emplace_back();
  g_owned.back().stream = s;
  for (int k = 0; k < kOwnedSlots; ++k) {
    if (g_owned_keys[k].load(std::memory_order_relaxed) == nullptr) {
      g_owned_keys[k].store(s, std::memory_order_release);
      return;
    }
  }
  g_owned_spill.fetch_add(1, std::memory_order_release);
}

void ReleaseEngineStream(hipStream_t s) {
  std::list<Workspace> gone;
  {
    std::lock_guard<std::mutex> lk(g_owned_mu);
    for (auto it = g_owned.begin(); it != g_owned.end(); ++it) {
      if (it->stream == s) {
        gone.splice(gone.begin(), g_owned, it);
        bool slot = false;
        for (int k = 0; k < kOwnedSlots && !slot; ++k) {
          if (g_owned_keys[k].load(std::memory_order_relaxed) == s) {
            g_owned_keys[k].store(nullptr, std::memory_order_release);
            slot = true;
          }
        }
        if (!slot) g_owned_spill.fetch_sub(1, std::memory_order_release);
        break;
      }
    }
  }
  // Other threads' last-batch pointers into this workspace go stale: the
  // epoch tells their hooks so.
  g_release_epoch.fetch_add(1, std::memory_order_acq_rel);
  for (Workspace& w : gone)
    if (w.mem != nullptr) SyncAndRelease(w);
}
}  // namespace prismdb

extern "C" {

int leveldb_crc32c_device_init(int device) {
  int cur = 0;
  hipError_t e = hipGetDevice(&cur);
  if (e != hipSuccess) return FailHip(e, "hipGetDevice");
  if (device != cur) {
    e = hipSetDevice(device);
    if (e != hipSuccess) return FailHip(e, "hipSetDevice");
  }
  DeviceCtx* ctx = nullptr;
  int rc = GetCtx(&ctx);
  if (device != cur) (void)hipSetDevice(cur);
  return rc;
}

int leveldb_crc32c_batch_fixed(const void* dev_base, size_t stride, size_t len, size_t nblocks,
                               uint32_t init, uint32_t* dev_out, uint8_t* dev_mismatch,
                               uint32_t flags, void* stream) {
  if (nblocks == 0) return 0;
  if (dev_base == nullptr) return Fail(PRISMDB_CRC32C_EINVAL, "dev_base is NULL");
  if (len > 0xFFFFFFFFull) return Fail(PRISMDB_CRC32C_EINVAL, "len must be < 4 GiB");
  if ((flags & ~(PRISMDB_CRC32C_MASK | PRISMDB_CRC32C_WRITE_TRAILER | PRISMDB_CRC32C_LOG_HEADER |
                 PRISMDB_CRC32C_UNORDERED)) != 0)
    return Fail(PRISMDB_CRC32C_EINVAL, "unknown flag bits");
  if ((flags & PRISMDB_CRC32C_WRITE_TRAILER) && dev_mismatch != nullptr)
    return Fail(PRISMDB_CRC32C_EINVAL, "WRITE_TRAILER and verify are exclusive");
  DeviceCtx* ctx = nullptr;
  int rc = GetCtx(&ctx);
  if (rc != 0) return rc;
  SpanBatch a{};
  a.base = static_cast<const uint8_t*>(dev_base);
  a.stride = stride;
  a.len_c = (uint32_t)len;
  a.init_c = init;
  a.n = nblocks;
  a.out = dev_out;
  a.mismatch = dev_mismatch;
  a.flags = flags;
  return RunBatch(*ctx, a, false, dev_mismatch != nullptr, static_cast<hipStream_t>(stream), 0);
}

int leveldb_crc32c_batch(const void* dev_base, const uint64_t* dev_off, const uint32_t* dev_len,
                         const uint32_t* dev_init, size_t n, uint32_t* dev_out,
                         uint8_t* dev_mismatch, uint32_t flags, void* stream) {
  if (n == 0) return 0;
  if (dev_base == nullptr || dev_off == nullptr || dev_len == nullptr)
    return Fail(PRISMDB_CRC32C_EINVAL, "dev_base/dev_off/dev_len must be non-NULL");
  if ((flags & ~(PRISMDB_CRC32C_MASK | PRISMDB_CRC32C_WRITE_TRAILER | PRISMDB_CRC32C_LOG_HEADER |
                 PRISMDB_CRC32C_UNORDERED)) != 0)
    return Fail(PRISMDB_CRC32C_EINVAL, "unknown flag bits");
  if ((flags & PRISMDB_CRC32C_WRITE_TRAILER) && dev_mismatch != nullptr)
    return Fail(PRISMDB_CRC32C_EINVAL, "WRITE_TRAILER and verify are exclusive");
  DeviceCtx* ctx = nullptr;
  int rc = GetCtx(&ctx);
  if (rc != 0) return rc;
  SpanBatch a{};
  a.base = static_cast<const uint8_t*>(dev_base);
  a.off = dev_off;
  a.len = dev_len;
  a.init = dev_init;
  a.n = n;
  a.out = dev_out;
  a.mismatch = dev_mismatch;
  a.flags = flags;
  return RunBatch(*ctx, a, true, dev_mismatch != nullptr, static_cast<hipStream_t>(stream), 0);
}

const char* leveldb_crc32c_last_error(void) { return t_last_error.c_str(); }

// 1 if the prismdb_* test and tuning setters act in this process
// (PRISMDB_ENABLE_TEST_HOOKS=1), else 0.
int prismdb_test_hooks_enabled(void) { return prismdb::TestHooksEnabled() ? 1 : 0; }

// Test hooks, not in the public header (the parity tests and the A/B harness
// pin each path with them; no-ops unless PRISMDB_ENABLE_TEST_HOOKS=1):
// fixed-stride batches through the generic span kernel too;
void prismdb_crc32c_force_generic(int on) {
  if (prismdb::TestHooksEnabled()) g_force_generic.store(on != 0, std::memory_order_relaxed);
}

// which planner-path descriptor batches take the lane kernel first (0 =
// log-record batches, the default; 1 = every batch; -1 = none);
void prismdb_crc32c_lane_mode(int mode) {
  if (!prismdb::TestHooksEnabled()) return;
  g_lane_mode.store(mode > 0 ? 1 : (mode < 0 ? -1 : 0), std::memory_order_relaxed);
}

// descriptor batches of at most this many spans take the one-launch kernel
// (clamped to kDirectMaxSpans; 0: none do; larger batches: windows of this
// many spans, see prismdb_crc32c_windows); returns the previous value.
uint64_t prismdb_crc32c_direct_max(uint64_t n) {
  if (!prismdb::TestHooksEnabled()) return g_direct_max.load(std::memory_order_relaxed);
  if (n > prismdb::dev::kDirectMaxSpans) n = prismdb::dev::kDirectMaxSpans;
  return g_direct_max.exchange(n, std::memory_order_relaxed);
}

// the one-launch path's ticket capacity (clamped to 1..kDirectTickets) and
// debug flags (bit 0: delay the pushes, see DirectWs::dbg); return the old values.
uint32_t prismdb_crc32c_direct_tickets(uint32_t cap) {
  if (!prismdb::TestHooksEnabled()) return g_direct_cap.load(std::memory_order_relaxed);
  if (cap < 1u) cap = 1u;
  if (cap > prismdb::dev::kDirectTickets) cap = prismdb::dev::kDirectTickets;
  return g_direct_cap.exchange(cap, std::memory_order_relaxed);
}
uint32_t prismdb_crc32c_direct_debug(uint32_t flags) {
  if (!prismdb::TestHooksEnabled()) return g_direct_dbg.load(std::memory_order_relaxed);
  return g_direct_dbg.exchange(flags, std::memory_order_relaxed);
}

// descriptor batches of more than prismdb_crc32c_direct_max spans (log-record
// batches aside): 1 = windows of the one-launch kernel, 0 = the planner path,
// 2 = windows up to two of them, the planner beyond (default); returns the
// previous value.
int prismdb_crc32c_windows(int mode) {
  if (!prismdb::TestHooksEnabled()) return g_windows.load(std::memory_order_relaxed);
  return g_windows.exchange(mode < 0 || mode > 2 ? 2 : mode, std::memory_order_relaxed);
}

// the call count of the calling thread's workspace for (current device,
// stream): the next one-launch call there takes gen + 1 (its tag: the low 16
// bits; gen + 1 == 0 mod 2^16 zeroes the workspace first).  Lets a test cross
// the tag wrap in a few calls.  0, or -1 if the thread has no such workspace.
int prismdb_crc32c_direct_set_gen(void* stream, uint32_t gen) {
  if (!prismdb::TestHooksEnabled()) return -1;
  int device = 0;
  if (hipGetDevice(&device) != hipSuccess) return -1;
  for (Workspace& w : ThreadWorkspaces().lru) {
    if (w.device == device && w.stream == static_cast<hipStream_t>(stream) && w.direct != nullptr) {
      w.gen = gen;
      return 0;
    }
  }
  return -1;
}

// the cumulative one-launch counters of the workspace of the calling thread's
// last one-launch batch {tickets adopted, spans folded whole, tickets claimed
// early, tickets claimed late}, after waiting for its stream.  0, or -1.
int prismdb_crc32c_direct_stats(uint64_t out[4]) {
  if (t_last_stats == nullptr || LastBatchStale()) return -1;
  uint32_t c[4] = {0, 0, 0, 0};
  hipError_t e = hipStreamSynchronize(t_last_stream);
  if (e == hipSuccess) e = hipMemcpy(c, t_last_stats, sizeof(c), hipMemcpyDeviceToHost);
  if (e != hipSuccess) return FailHip(e, "prismdb_crc32c_direct_stats");
  for (int i = 0; i < 4; ++i) out[i] = c[i];
  return 0;
}

// the split counters of the calling thread's last planner-path descriptor
// batch {long spans, segments, overflow flag, spans listed by the lane
// kernel}, after waiting for its stream.  Returns 0; -1 if the thread has run
// no such batch; -2 if its last descriptor batch took the one-launch path.
int prismdb_crc32c_last_split(uint64_t out[4]) {
  if (t_last_direct) return -2;
  if (t_last_counters == nullptr || LastBatchStale()) return -1;
  prismdb::dev::SplitCounters c{};
  hipError_t e = hipStreamSynchronize(t_last_stream);
  if (e == hipSuccess) e = hipMemcpy(&c, t_last_counters, sizeof(c), hipMemcpyDeviceToHost);
  if (e != hipSuccess) return FailHip(e, "prismdb_crc32c_last_split");
  out[0] = c.nlong;
  out[1] = c.nseg;
  out[2] = c.overflow;
  out[3] = c.nlist;
  return 0;
}

// Test hook: the span pass's schedule of this thread's last planner-path
// batch: out[0] = chunk tasks, out[1] = task-balanced slices (0: every record
// one task -- the pair-run kernel's schedule when the host launched it),
// out[2] = 1 if the host launched the pair-run kernel.  -2 after a one-launch
// batch, -1 before any planner batch.
int prismdb_crc32c_last_schedule(uint64_t out[3]) {
  if (t_last_direct) return -2;
  if (t_last_counters == nullptr || LastBatchStale()) return -1;
  prismdb::dev::SplitCounters c{};
  hipError_t e = hipStreamSynchronize(t_last_stream);
  if (e == hipSuccess) e = hipMemcpy(&c, t_last_counters, sizeof(c), hipMemcpyDeviceToHost);
  if (e != hipSuccess) return FailHip(e, "prismdb_crc32c_last_schedule");
  out[0] = c.tasks;
  out[1] = c.nslices;
  out[2] = t_last_pair ? 1u : 0u;
  return 0;
}

// Test hook: the claimed tails of this thread's last planner-path batch:
// out[0] = claims on the span / pair-run kernels' counters (slices or runs
// taken on demand past the static deal, plus one failed claim per stream at
// the end; 0 when the batch was too small for a tail), out[1] = the same for
// the lane kernel's runs.  -2 after a one-launch batch, -1 before any.
int prismdb_crc32c_last_claims(uint64_t out[2]) {
  if (t_last_direct) return -2;
  if (t_last_counters == nullptr || LastBatchStale()) return -1;
  namespace d = prismdb::dev;
  uint32_t blk[d::kCounterBlock / 4];
  hipError_t e = hipStreamSynchronize(t_last_stream);
  if (e == hipSuccess) e = hipMemcpy(blk, t_last_counters, sizeof(blk), hipMemcpyDeviceToHost);
  if (e != hipSuccess) return FailHip(e, "prismdb_crc32c_last_claims");
  d::SplitCounters c{};
  std::memcpy(&c, blk, sizeof(c));
  out[0] = c.claim;  // the span kernel's, plus the pair-run kernel's claim lines
  for (uint32_t j = 0; j < d::kClaimLines; ++j) out[0] += blk[64 + d::kClaimLineWords * j];
  out[1] = c.lane_claim;
  return 0;
}

}  // extern "C"
