// crc32c_capi.hip -- C ABI of the batch engine (include/prismdb_crc32c.h).
//
// Per-device context (tables in HBM, CU count, self-test) is created once with
// std::call_once; after that every call is lock-free.  The long-span split
// path needs a small workspace; it is cached per (thread, device, stream) so
// concurrent callers on distinct streams never share one.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <utility>

#include "../../include/prismdb_crc32c.h"
#include "crc32c_device.h"

#ifndef PRISMDB_SPAN_J0
#define PRISMDB_SPAN_J0 0
#endif
#ifndef PRISMDB_SPAN_INJ0
#define PRISMDB_SPAN_INJ0 0
#endif
#include "crc32c_gf2.h"

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
};

DeviceCtx g_ctx[kMaxDevices];

// Test hook: route fixed-stride batches through the generic span kernel.
bool g_force_generic = false;

// Which descriptor batches go through the quad kernel first (spans of
// <= kQuadMaxLen bytes; longer ones follow on the generic path):
// 0 = log-record batches (PRISMDB_CRC32C_LOG_HEADER), 1 = all, -1 = none.
#ifndef PRISMDB_QUAD_DEFAULT
#define PRISMDB_QUAD_DEFAULT 0
#endif
int g_quad_mode = PRISMDB_QUAD_DEFAULT;

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
}

int RunBatch(DeviceCtx& ctx, const SpanBatch& base_args, bool desc, bool verify, hipStream_t s);

// Device known-answer self-test (util/crc32c.cc:269-273 vector, plus a 4 KiB
// block and a > kLongSpan span checked against the host Extend).
int SelfTest(DeviceCtx& ctx) {
#ifdef PRISMDB_MEASURE_ONLY
  // measurement-only variant builds (tools/variants.py) that knowingly break
  // results on some geometries skip the self-test; the product never defines it
  return 0;
#endif
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
    hipFree(d);
    delete[] h;
    return FailHip(e, "self-test upload");
  }
  SpanBatch a{};
  a.base = d;
  a.off = d_off;
  a.len = d_len;
  a.n = 3;
  a.out = d_out;
  int rc = RunBatch(ctx, a, true, false, nullptr);
  uint32_t got[3] = {0, 0, 0};
  if (rc == 0) {
    e = hipStreamSynchronize(nullptr);
    if (e != hipSuccess) rc = FailHip(e, "self-test sync");
  }
  if (rc == 0) {
    e = hipMemcpy(got, d_out, sizeof(got), hipMemcpyDeviceToHost);
    if (e != hipSuccess) rc = FailHip(e, "self-test download");
  }
  hipFree(d);
  delete[] h;
  if (rc != 0) return rc;
  if (got[0] != want[0] || got[1] != want[1] || got[2] != want[2]) {
    char buf[200];
    std::snprintf(buf, sizeof(buf), "device self-test: got %08x %08x %08x want %08x %08x %08x", got[0],
                  got[1], got[2], want[0], want[1], want[2]);
    return Fail(PRISMDB_CRC32C_ESELFTEST, buf);
  }
  return 0;
}

void InitDevice(DeviceCtx& ctx, int device) {
  hipError_t e = hipDeviceGetAttribute(&ctx.cus, hipDeviceAttributeMultiprocessorCount, device);
  if (e != hipSuccess || ctx.cus <= 0) {
    ctx.status = FailHip(e, "hipDeviceGetAttribute(multiprocessor count)");
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
#if PRISMDB_SPAN_J0 == 0 && !PRISMDB_SPAN_INJ0  // measurement-only builds compute wrong CRCs on purpose
  ctx.status = SelfTest(ctx);
  if (ctx.status != 0) ctx.error = t_last_error;
#endif
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

// ---- generic-path workspace, per (thread, device, stream) ----
// Fixed part: split-path counters, segment records/results, long-span list,
// planner block sums.  Growing part, sized for the largest batch seen (the
// first call with a larger batch synchronises the stream and reallocates): per
// span a 16-byte record and a 4-byte task count, plus the slice starts.
struct Workspace {
  void* mem = nullptr;
  char* grow = nullptr;
  size_t cap_rec = 0;
  char* qgrow = nullptr;  // quad path: long-span list and its results (9 B per span), run flags
  size_t cap_q = 0;
  SplitWs ws{};
};

// Slice starts needed for n spans: nslices + 1 <= n/2 + 32 * streams + 2
// (crc32c_slice_scan_kernel: tau = 64 gives <= n/2 + 1 slices of <= 32-task
// spans; a smaller tau keeps tau > T / (32 * streams)).
#ifndef PRISMDB_SLICES_PER_STREAM
#define PRISMDB_SLICES_PER_STREAM 16
#endif
size_t SliceCap(size_t n, uint32_t streams) {
  return n / 2 + 2 * (size_t)PRISMDB_SLICES_PER_STREAM * streams + 4;
}

constexpr uint64_t kCapSeg = 1u << 20;   // 1 Mi segments = 32 GiB of long spans per call
constexpr uint32_t kCapLong = 1u << 18;

int GetWorkspace(hipStream_t s, size_t nspans, uint32_t streams, bool quad, SplitWs* out) {
  thread_local std::map<std::pair<int, hipStream_t>, Workspace> cache;
  int device = 0;
  hipGetDevice(&device);
  Workspace& w = cache[{device, s}];
  if (w.mem == nullptr) {
    const size_t bytes = 256 + kCapSeg * (16 + 4) + (size_t)kCapLong * (8 + 8 + 4) +
                         (size_t)prismdb::dev::kMaxPlanBlocks * 8;
    hipError_t e = hipMalloc(&w.mem, bytes);
    if (e != hipSuccess) {
      w.mem = nullptr;
      return FailHip(e, "workspace hipMalloc");
    }
    char* p = static_cast<char*>(w.mem);
    w.ws.counters = reinterpret_cast<SplitCounters*>(p);
    p += 256;
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
  }
  if (w.cap_rec < nspans) {
    if (w.grow != nullptr) {
      hipStreamSynchronize(s);  // earlier batches on this stream may still read it
      hipFree(w.grow);
      w.grow = nullptr;
      w.cap_rec = 0;
    }
    const size_t cap = nspans < 4096 ? 4096 : nspans + nspans / 4;
    const size_t bytes = cap * (16 + 4) + SliceCap(cap, streams) * 8 + 16;
    hipError_t e = hipMalloc(reinterpret_cast<void**>(&w.grow), bytes);
    if (e != hipSuccess) return FailHip(e, "span record workspace hipMalloc");
    w.cap_rec = cap;
  }
  if (quad && w.cap_q < nspans) {
    if (w.qgrow != nullptr) {
      hipStreamSynchronize(s);
      hipFree(w.qgrow);
      w.qgrow = nullptr;
      w.cap_q = 0;
    }
    const size_t cap = nspans < 4096 ? 4096 : nspans + nspans / 4;
    hipError_t e = hipMalloc(reinterpret_cast<void**>(&w.qgrow), cap * 9 + cap / 64 + 1024);
    if (e != hipSuccess) return FailHip(e, "quad list workspace hipMalloc");
    w.cap_q = cap;
  }
  w.ws.list = quad ? reinterpret_cast<uint32_t*>(w.qgrow) : nullptr;
  w.ws.qout = quad ? reinterpret_cast<uint32_t*>(w.qgrow + w.cap_q * 4) : nullptr;
  w.ws.qmm = quad ? reinterpret_cast<uint8_t*>(w.qgrow + w.cap_q * 8) : nullptr;
  w.ws.qrun = quad ? reinterpret_cast<uint8_t*>(w.qgrow + w.cap_q * 9) : nullptr;
  w.ws.rec = reinterpret_cast<prismdb::dev::SpanRec*>(w.grow);
  w.ws.slice_start = reinterpret_cast<uint64_t*>(w.grow + w.cap_rec * 16);
  w.ws.cnt = reinterpret_cast<uint32_t*>(w.grow + w.cap_rec * 16 + SliceCap(w.cap_rec, streams) * 8);
  // Planner tiles: whole multiples of its block size, at most kMaxPlanBlocks.
  namespace d = prismdb::dev;
  const uint64_t per = (nspans + d::kMaxPlanBlocks - 1) / d::kMaxPlanBlocks;
  w.ws.tile = (per + d::kPlanThreads - 1) / d::kPlanThreads * d::kPlanThreads;
  w.ws.nblocks = (uint32_t)((nspans + w.ws.tile - 1) / w.ws.tile);
  w.ws.nstreams = streams;
  *out = w.ws;
  return 0;
}

// Launch sequence.  Fast path: one kernel.  Generic path:
// plan (span records, long spans cut into segments) -> span pass (long spans
// skipped) -> segment pass -> combine.
int RunBatch(DeviceCtx& ctx, const SpanBatch& base_args, bool desc, bool verify, hipStream_t s) {
  SpanBatch a = base_args;
  a.tabs = ctx.tabs;
  a.role = prismdb::dev::kRoleSpans;
  // Fast path: fixed stride, 4-byte aligned, 4..4096-byte multiple-of-4 spans
  // (verify: up to 4092 bytes and not a multiple of 256, so that the stored
  // trailer word fits round 0's padding lanes).
  const uint32_t max_len = 4u * prismdb::dev::kChunkWords - (verify ? 4u : 0u);
  if (!desc && (verify || a.out != nullptr) && (!verify || (a.len_c & 255u) != 0) &&
      (a.flags & (prismdb::dev::kFlagWriteTrailer | prismdb::dev::kFlagLogHeader)) == 0 &&
      a.len_c >= 4 && a.len_c <= max_len && (a.len_c & 3u) == 0 &&
      (a.stride & 3u) == 0 && (reinterpret_cast<uintptr_t>(a.base) & 3u) == 0 && !g_force_generic) {
    hipError_t e = prismdb::dev::launch_fixed(a, verify, ctx.cus, s);
    return e == hipSuccess ? 0 : FailHip(e, "fixed kernel launch");
  }
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
      const int rc = RunBatch(ctx, p, desc, verify, s);
      if (rc != 0) return rc;
    }
    return 0;
  }
  SplitWs ws{};
  // The span kernel's record streams: two per wave of its persistent grid.
  const uint32_t streams = 2u * (uint32_t)ctx.cus * prismdb::dev::kWavesPerGroup;
  // Short spans first, four per wave (crc32c_quad_kernel); the generic path
  // below then runs over the list of the longer ones only.
  const bool quad = desc && (g_quad_mode > 0 || (g_quad_mode == 0 && (a.flags & prismdb::dev::kFlagLogHeader)));
  int rc = GetWorkspace(s, a.n, streams, quad, &ws);
  if (rc != 0) return rc;
  hipError_t e = hipMemsetAsync(ws.counters, 0, sizeof(SplitCounters), s);
  if (e != hipSuccess) return FailHip(e, "hipMemsetAsync");
  t_last_counters = ws.counters;
  t_last_stream = s;
  uint32_t* const caller_out = a.out;
  uint8_t* const caller_mm = a.mismatch;
  if (quad) {
    a.qrun = ws.qrun;
    e = prismdb::dev::launch_quad(a, verify, ctx.cus, ws, s);
    if (e != hipSuccess) return FailHip(e, "quad kernel launch");
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
  e = prismdb::dev::launch_plan(a, desc, ws, s);
  if (e != hipSuccess) return FailHip(e, "plan kernel launch");
  // Task-balanced slices need more records than span streams: with n <= the
  // stream count every stream holds at most one record either way, and the
  // two slice kernels' launches are ~9 us of a file-sized call.
  if (a.n > streams) {
    e = prismdb::dev::launch_slices(a, ws, s);
    if (e != hipSuccess) return FailHip(e, "slice kernels launch");
    a.slice_start = ws.slice_start;
    a.nslices_dev = &ws.counters->nslices;
  }
  // Large batches of one-task records take the pair-run kernel (its two
  // streams read adjacent spans); it is launched next to the general one,
  // and the one whose schedule the scan did not pick leaves at once.
  a.pair_kernel = PRISMDB_SPAN_PAIR_RUNS && a.slice_start != nullptr && a.n >= prismdb::dev::kPairMinSpans &&
                          !(a.flags & prismdb::dev::kFlagLogHeader)
                      ? 1u
                      : 0u;
  e = prismdb::dev::launch_span(a, verify, ctx.cus, s);
  if (e != hipSuccess) return FailHip(e, "span kernel launch");
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
  e = prismdb::dev::launch_span(seg, false, ctx.cus, s);
  if (e != hipSuccess) return FailHip(e, "segment kernel launch");
  e = prismdb::dev::launch_combine(a, desc, verify, ws, s);
  if (e != hipSuccess) return FailHip(e, "combine kernel launch");
  if (quad) {
    SpanBatch back = a;
    back.out = caller_out;
    back.mismatch = caller_mm;
    e = prismdb::dev::launch_scatter(back, ws, ws.qout, ws.qmm, s);
    if (e != hipSuccess) return FailHip(e, "scatter kernel launch");
  }
  return 0;
}

}  // namespace

namespace prismdb {
void SetLastError(const std::string& msg) { t_last_error = msg; }
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
  if (device != cur) hipSetDevice(cur);
  return rc;
}

int leveldb_crc32c_batch_fixed(const void* dev_base, size_t stride, size_t len, size_t nblocks,
                               uint32_t init, uint32_t* dev_out, uint8_t* dev_mismatch,
                               uint32_t flags, void* stream) {
  if (nblocks == 0) return 0;
  if (dev_base == nullptr) return Fail(PRISMDB_CRC32C_EINVAL, "dev_base is NULL");
  if (len > 0xFFFFFFFFull) return Fail(PRISMDB_CRC32C_EINVAL, "len must be < 4 GiB");
  if ((flags & ~(PRISMDB_CRC32C_MASK | PRISMDB_CRC32C_WRITE_TRAILER | PRISMDB_CRC32C_LOG_HEADER)) != 0)
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
  return RunBatch(*ctx, a, false, dev_mismatch != nullptr, static_cast<hipStream_t>(stream));
}

int leveldb_crc32c_batch(const void* dev_base, const uint64_t* dev_off, const uint32_t* dev_len,
                         const uint32_t* dev_init, size_t n, uint32_t* dev_out,
                         uint8_t* dev_mismatch, uint32_t flags, void* stream) {
  if (n == 0) return 0;
  if (dev_base == nullptr || dev_off == nullptr || dev_len == nullptr)
    return Fail(PRISMDB_CRC32C_EINVAL, "dev_base/dev_off/dev_len must be non-NULL");
  if ((flags & ~(PRISMDB_CRC32C_MASK | PRISMDB_CRC32C_WRITE_TRAILER | PRISMDB_CRC32C_LOG_HEADER)) != 0)
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
  return RunBatch(*ctx, a, true, dev_mismatch != nullptr, static_cast<hipStream_t>(stream));
}

const char* leveldb_crc32c_last_error(void) { return t_last_error.c_str(); }

// Not in the public header: lets the parity tests pin the generic kernel too.
void prismdb_crc32c_force_generic(int on) { g_force_generic = on != 0; }

// Not in the public header: which descriptor batches take the quad kernel
// (0 = log-record batches, the default; 1 = every batch; -1 = none), so the
// parity tests and the A/B harness can pin either path.
void prismdb_crc32c_quad_mode(int mode) { g_quad_mode = mode > 0 ? 1 : (mode < 0 ? -1 : 0); }

// Not in the public header: the split counters of the calling thread's last
// descriptor batch {long spans, segments, overflow flag, spans listed by the
// quad kernel}, after waiting for its stream, so the tests can tell which
// path a batch took.  Returns 0, or -1 if the thread has run no such batch.
int prismdb_crc32c_last_split(uint64_t out[4]) {
  if (t_last_counters == nullptr) return -1;
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

}  // extern "C"
