// crc32c_device.h -- shared between the HIP kernels and the C-ABI host code.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace prismdb {
namespace dev {

constexpr uint32_t kPolyReflected = 0x82F63B78u;
constexpr uint32_t kConditioning = 0xFFFFFFFFu;  // util/crc32c.cc:246
constexpr uint32_t kMaskDelta = 0xa282ead8u;     // util/crc32c.h:22
constexpr uint32_t kFlagMask = 0x1u;             // == PRISMDB_CRC32C_MASK
constexpr uint32_t kFlagWriteTrailer = 0x2u;     // == PRISMDB_CRC32C_WRITE_TRAILER
constexpr uint32_t kFlagLogHeader = 0x4u;        // == PRISMDB_CRC32C_LOG_HEADER
constexpr uint32_t kLogCrcBack = 6u;             // log record: crc sits 6 B before type||payload

constexpr int kWave = 64;
constexpr int kWavesPerGroup = 16;                 // 1024-thread workgroup, one per CU
constexpr int kThreads = kWave * kWavesPerGroup;
constexpr int kRounds = 16;                        // 256-B rounds per chunk
constexpr uint32_t kChunkWords = kRounds * kWave;  // 1024 words = 4 KiB per chunk
// Log-record span kernel chunk.  8 rounds (2 KiB) would make a ~1 KB record one
// task of 9 loads, but hipcc then copies the ring's in-flight registers
// (tools/check_inflight.py: 792 sites), so it stays at 16.
constexpr int kRoundsLog = 16;
constexpr uint32_t kLgChunkWordsLog = 10u;
constexpr uint32_t kStrideBytes = 4u * kWave;      // 256 B between a lane's words
constexpr int kCopies = 32;                        // LDS table replication (bank = lane % 32)
constexpr int kTabWords = 4 * 256 * kCopies;       // 128 KiB of LDS: stride tables
constexpr int kNibWords = 8 * 16 * kWave;          // 32 KiB of LDS: per-lane realignment tables
constexpr int kLdsWords = kTabWords + kNibWords;   // 160 KiB: all of a CU's LDS

constexpr uint32_t kLongSpan = 128u * 1024u;       // spans above this are split...
constexpr uint32_t kSegment = 32u * 1024u;         // ...into pieces of this size

constexpr int kZeroWords = 16384;  // DeviceTables::zero: 256 regions of 256 B
constexpr int kTicketLgMax = 14;   // one-launch tickets of up to 2^14 chunks (64 MiB)

// Tables derived on the host from the polynomial (crc32c_gf2.h) and kept in HBM.
struct DeviceTables {
  uint32_t stride[4][256];    // stride[k][b] = shift_256(b << 8k)
  uint32_t lane_nib[8][16][64];  // [n][v][l] = shift_{256-4l}(v << 4n): lane l's realignment
  uint32_t shift_seg[32];     // column i of shift_kSegment (M)
  uint32_t shift_seg64[32];   // column i of M^64
  uint32_t lane_seg[32][64];  // [i][l] = column i of M^(63-l): lane l's final shift
  uint32_t slice4[4][256];    // slice4[k][b] = shift_4(b << 8k): one record per lane (lane kernel)
  // One-launch path (crc32c_direct.hip): a long span's tickets of g = 2^lg
  // chunks (lg 0..kTicketLgMax) are combined with M = shift_{4 KiB * g}:
  uint32_t tick64[kTicketLgMax + 1][32];         // [lg][i] = column i of M^64
  uint32_t tick_lane[kTicketLgMax + 1][32][64];  // [lg][i][l] = column i of M^(63-l): lane l's final shift
  uint32_t shift_chunk[32];       // column i of shift_{4 KiB} (tests; M for lg 0)
  // 64 KiB of zeros: the lane kernel's loads of lanes without a record to
  // read land here, 2 KiB per wave (wave % 32) -- one shared line was an L2
  // hotspot when whole runs are left to the generic path
  uint32_t zero[kZeroWords];
};

// Lane kernel (log-record batches): one record per lane, 128-B tasks of eight
// 16-B loads; records of kLaneMinLen..kLaneMaxLen bytes (the rest take the
// generic path through the long-span list).
constexpr uint32_t kLaneMinLen = 8u;  // >= 3 head bytes + one body word
constexpr uint32_t kLaneMaxLen = 1280u;
__host__ __device__ constexpr bool lane_owns(uint32_t len) { return len >= kLaneMinLen && len <= kLaneMaxLen; }

enum : uint32_t { kRoleSpans = 0, kRoleSegments = 1 };

// 16-byte span record with all geometry precomputed (crc32c_kernels.hip).
typedef uint32_t SpanRec __attribute__((ext_vector_type(4)));

struct SpanBatch {
  const uint8_t* base;
  const uint64_t* off;   // descriptor mode
  const uint32_t* len;
  const uint32_t* init;  // nullable
  uint64_t stride;       // fixed mode
  uint32_t len_c;
  uint32_t init_c;
  uint64_t n;
  const unsigned long long* n_dev;  // nullable: n = min(n, *n_dev)
  uint32_t* out;                    // nullable
  uint8_t* mismatch;                // nullable (verify)
  uint32_t flags;
  uint32_t skip_above;              // spans longer than this are left to the split path
  const uint32_t* overflow;         // nullable: split-path overflow flag
  uint32_t role;
  const DeviceTables* tabs;
  const SpanRec* rec;               // span records (generic kernel)
  // Task-balanced schedule (span role): slice k is records
  // [slice_start[k], slice_start[k+1]), *nslices_dev slices; nullable: slices
  // are runs of equal record counts instead (segment role).
  const uint64_t* slice_start;
  const unsigned long long* nslices_dev;
  uint32_t chunk_lg;  // planner: log2(chunk words) of the kernel that consumes the span records
  // nullable: record i of this batch is span idx[i] of the caller's
  // descriptors and results (the generic path behind the lane kernel runs
  // over the list of spans it does not own; n_dev holds the list length)
  const uint32_t* idx;
  // Span role: the pair-run span kernel is launched too (it takes the batch
  // when the scan finds every record one task; the general kernel then leaves).
  uint32_t pair_kernel;
  // nullable, zero at launch: the span kernel's claim counter for its last
  // kTailRounds rounds of slices or runs (dealt on demand, not statically);
  // the lane kernel's for its last rounds of runs
  uint32_t* claim;
  const unsigned long long* tasks_dev;  // nullable: the span pass's chunk tasks (slice scan)
  // nullable, zero at launch: the pair-run kernel's kClaimLines claim
  // counters, one per 128-B line (word kClaimLineWords * j)
  uint32_t* claims;
};

// Below this many spans the pair-run kernel's extra launch (~5 us) costs more
// than its 3.5 % gains (break-even near 140 us of data, ~250 K spans of 4 KiB).
constexpr uint64_t kPairMinSpans = 1ull << 18;

struct SplitCounters {
  unsigned long long nseg;
  uint32_t nlong;
  uint32_t overflow;
  unsigned long long tasks;    // chunk tasks of the span pass (long spans count 1)
  unsigned long long nslices;  // task-balanced slices (0: every record one task, runs instead)
  unsigned long long nlist;             // spans the lane kernel leaves to the generic path
  unsigned long long slice_q, slice_r;  // exact slices: q = T / K, r = T % K
  uint32_t claim;                       // span kernel: tail slices claimed (SpanBatch::claim)
  uint32_t lane_claim;                  // lane kernel: tail runs claimed (its SpanBatch::claim)
};

// A planner call's counter block (two, by call parity): SplitCounters, then
// the pair-run kernel's claim counters, one per 128-B line -- eight
// counters, each taking the claims of an eighth of the groups (one address
// took every wave's claim at ~86 per us: too few for config 5's short runs).
constexpr uint32_t kClaimLines = 8;
constexpr uint32_t kClaimLineWords = 32;
constexpr uint32_t kCounterBlock = 256 + kClaimLines * 4 * kClaimLineWords;  // bytes

struct SplitWs {
  SplitCounters* counters;
  // The other call parity's counter block: the plan kernel zeroes it for the
  // workspace's next planner call (nullptr: none).
  SplitCounters* zero_next;
  SpanRec* rec;      // one per span of the batch
  SpanRec* seg_rec;  // one per segment
  uint32_t* seg_out;
  uint64_t* long_span;
  uint64_t* long_first;
  uint32_t* long_nseg;
  uint64_t cap_seg;
  uint32_t cap_long;
  // task-balanced slices of the span pass
  uint32_t* cnt;          // tasks of each span
  uint64_t* bsum;         // per planner block: task sum, then its exclusive prefix
  uint64_t* slice_start;  // nslices + 1 entries
  uint64_t tile;          // records per planner block
  uint32_t nblocks;       // planner blocks (<= kMaxPlanBlocks)
  uint32_t nstreams;      // span-kernel record streams (2 per wave)
  uint32_t* list;         // lane path: indices of the spans the lane kernel does not own
  uint32_t* qout;         // lane path: generic-path results of the listed spans (list order)
  uint8_t* qmm;
};

// One-launch path for descriptor batches of <= kDirectMaxSpans spans
// (crc32c_direct.hip): one kernel, no planner, no memset.  Spans of one chunk
// (body <= 4 KiB) are dealt to the waves in static runs; longer spans are cut
// into tickets of 2^lg chunks that any wave may claim, and the wave that
// finishes a span's last ticket combines the partial registers.
// Capacity: 64 spans per wave's static run at 12 waves x 256 CUs (host-
// checked against the device's own CU count).  The default routing sends
// plain batches here only up to kDirectPlainSpans; batches that seal or
// verify block trailers (SST files) up to the capacity: 8-10 SST files per
// call ran 2-16 % faster in one launch than as two windows
// (tools/files_per_call.py, profiles/r06/r06as_files_per_call.json).
constexpr uint64_t kDirectMaxSpans = 196608ull;
constexpr uint64_t kDirectPlainSpans = 1ull << 17;
constexpr int kDirectThreads = 768;  // per group, one group per CU: a wave's static run is <= 64 spans
                                     // while n <= 64 * 8 * CUs (host-checked)
constexpr uint32_t kDirectTickets = 1u << 19;  // tickets per workspace slot (beyond: whole spans, one wave each)
// Hand-offs between waves of the one-launch kernel carry the call's tag in
// the top 16 bits of every 8-byte word (48-bit payload): a reader polls the
// words it needs until each carries its call's tag.  Words are written and
// read with relaxed agent-scope 8-B atomics (write-through / L2-served), so
// no wave needs a release or acquire fence: those write back or invalidate
// caches and wait for every load in flight (the table fill, the first data).
constexpr uint32_t kTagShift = 48;
constexpr uint32_t kTagMask = 0xFFFFu;

struct DirectWs {
  unsigned long long* word;  // this call's supply << 32 | claimed: tickets pushed / tickets taken
  unsigned long long* next;  // the word of the call after next (four words in turn; this call zeroes it)
  uint64_t* tmap;            // per ticket, 4 tagged words: span | (T-1, lg, k) << 32, span address, len, init
  uint64_t* part;            // per ticket: tagged partial register
  uint32_t* cdone;           // per span, at its first ticket: tickets finished
  uint32_t* stats;           // cumulative: tickets adopted, spans folded whole, tickets claimed early / late
  uint32_t* help;            // 32 replicas (128 B apart) of the help flag: == tag once a large push asks
  uint32_t cap;              // tickets
  uint32_t tag;              // this call's tag (1..0xFFFF): words of earlier calls never match
  uint32_t dbg;              // test hooks: bit 0 delays every push by ~100 us, bit 1 blind worker claims
};

constexpr uint32_t kMaxPlanBlocks = 4096;
constexpr uint32_t kSlicesPerStream = 16;  // span kernel: task-balanced slices shrink until every stream gets this many
constexpr uint64_t kMaxGenericSpans = 1ull << 30;  // per generic-path launch sequence
constexpr uint32_t kPlanThreads = 256;

hipError_t launch_span(const SpanBatch& a, bool verify, int grid, hipStream_t s, hipEvent_t stop = nullptr);
hipError_t launch_fixed(const SpanBatch& a, bool verify, int grid, hipStream_t s);
hipError_t launch_plan(const SpanBatch& a, bool desc, const SplitWs& ws, hipStream_t s, hipEvent_t stop = nullptr);
hipError_t launch_slices(const SpanBatch& a, const SplitWs& ws, hipStream_t s, hipEvent_t stop = nullptr);
hipError_t launch_combine(const SpanBatch& a, bool desc, bool verify, const SplitWs& ws,
                          hipStream_t s, hipEvent_t stop = nullptr);
hipError_t launch_long_list(const SpanBatch& a, const SplitWs& ws, hipStream_t s);
hipError_t launch_lane(const SpanBatch& a, bool verify, int grid, hipStream_t s);
constexpr int kListThreads = 1024;  // crc32c_long_list_kernel block: one atomic per 16 runs
// `done` is recorded when the kernel completes (the launch's own completion
// signal: a separate hipEventRecord marker cost ~5.7 us between back-to-back
// calls).  Always an ordered launch.
hipError_t launch_direct(const SpanBatch& a, bool verify, int grid, const DirectWs& d, hipStream_t s,
                         hipEvent_t done);
hipError_t launch_scatter(const SpanBatch& a, const SplitWs& ws, const uint32_t* qout, const uint8_t* qmm,
                          hipStream_t s, hipEvent_t stop = nullptr);
// WRITE_TRAILER on the planner path: every span's trailer from res[i], after
// the span kernels (crc32c_trailer_kernel).
hipError_t launch_trailers(const SpanBatch& a, bool desc, const uint32_t* res, hipStream_t s,
                           hipEvent_t stop = nullptr);

}  // namespace dev
}  // namespace prismdb
