// crc32c_kernels.hip -- CDNA4 (gfx950) kernels of the batched CRC32C engine.
//
// What is computed: for every span i, crc32c::Extend(init_i, base+off_i, len_i)
// (util/crc32c.cc:276-377), optionally Mask()ed (util/crc32c.h:27-31, as
// TableBuilder::WriteRawBlock stores it, table/table_builder.cc:194-196),
// optionally written back as the block trailer, and/or compared against the
// stored trailer (ReadBlock verify, table/format.cc:93-95).
//
// How (HBM-bound byte reduction; no MFMA):
//   * A span is cut into head bytes (to 4-B alignment), W body words and tail
//     bytes.  Body word i goes to lane (i - W) mod 64: the wave reads 256
//     contiguous bytes per round, rounds right-aligned so that every lane's
//     last word falls in the final round.
//   * Each lane runs its own CRC stream with stride 256 B:
//         acc <- shift_256(acc) ^ word
//     shift_256 = four lookups in LDS stride tables replicated 32x so that
//     lane l always reads bank l mod 32 (ds_read_b32 never conflicts); each
//     lookup address is one v_perm_b32.
//   * Lane l's stream ends 256-4l bytes before the body end: eight lookups in
//     lane l's nibble tables apply shift_{256-4l}, then the wave XOR-reduces
//     with DPP.  The initial register (init fed the head bytes by the planner)
//     enters with body word 0.
//   * Persistent grid: one 1024-thread workgroup per CU (the 160 KiB of LDS
//     tables are loaded once per CU), runs / task-balanced slices of spans
//     dealt round-robin to the waves' span streams, two spans folded per wave
//     at a time (two independent LDS chains), loads issued with inline asm
//     one pair ahead and retired by counted vmcnt.
//
// Kernels:
//   crc32c_fixed_kernel<K, verify>  fixed stride, 4-B aligned, len <= 4 KiB (config 2);
//                           verify: the stored trailer word rides in round 0
//   crc32c_plan_kernel      one thread per span: 16-byte span records (all
//                           geometry precomputed), long spans cut into segments
//   crc32c_slice_{scan,mark}_kernel  task-balanced slices of the span records
//   crc32c_span_kernel<verify, log>  everything else, driven by the span
//                           records; the log-record variant skips chunk 0's
//                           padding rounds
//   crc32c_pair_kernel<verify>  large batches of one-task records (pair runs)
//   crc32c_combine_kernel   stitches segments back into long spans
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "crc32c_device.h"

// Tuning constants (all result-preserving; measurement-only variants are built
// by tools/variants.py from patched copies of this file, never from switches
// in the shipped source).
namespace prismdb {
namespace dev {
namespace {
constexpr int kRing = 4;               // fixed kernel: span buffers in the prefetch ring (even)
constexpr uint32_t kRunLg = 5;         // fixed kernel: log2(pair steps per run): runs of 64 spans
constexpr uint32_t kRunsPerStream = 64;  // span kernel: one-task runs shrink until every stream gets this many
// Rounds of slices / runs claimed on demand at the end of the span kernel
// (of 16 slices per stream) and the pair-run kernel (of >= 64 runs per wave).
// Against none, with 10 reps side by side (profiles/r05/r05l_variants_tail_confirm.json,
// A/A within 0.6 %): config-3 mix +3.4 %, random spans +3.3 %, SST
// descriptors +3.5 %, sealed +3.0 %, 4 KiB descriptors +2.7 %; 8 / 8 rounds
// sat between (and cost 4 KiB descriptors 2 %), 2 and 4 ran no faster.
constexpr uint32_t kTailRounds = 12;
constexpr uint32_t kPairTailRounds = 16;
// The lane kernel's last rounds of runs of 64 records, claimed on demand:
// on ~1 KB WAL records its waves left 3542-3890 us into a 3.9 ms kernel,
// rank-1 waves 1.7 % and some XCDs 4.5 % behind the others
// (profiles/r05/r05aq_lane_timeline.json).  8 rounds against none: WAL
// verify +2.9 %, seal +1.6 % (4: +1.8 %, 12: +2.6 %;
// profiles/r05/r05ar_variants_lane_tail.json).
constexpr uint32_t kLaneTailRounds = 8;
}  // namespace
}  // namespace dev
}  // namespace prismdb

#include "crc32c_fold.h"

namespace prismdb {
namespace dev {

// ---------------------------------------------------------------------------
// Record-driven span kernel: two span streams per wave (stream s takes the
// wave's spans b = wave + (2q + s) * nwaves) folded in lockstep, every load an
// inline-asm BUFFER load issued one slot ahead and retired by a counted vmcnt.
// A task is one 4 KiB chunk and always issues exactly 17 loads (16 body dwords
// + 1 edge byte): loads outside the span hit the buffer range check and return
// 0 without touching memory, which gives chunk 0 its right-aligned zero padding
// and lets invalid or skipped tasks run through the same code.  Records come
// through the scalar cache, one span ahead per stream.
// ---------------------------------------------------------------------------
template <bool kVerify, bool kSkip>
__global__ __launch_bounds__(kThreads) void crc32c_span_kernel(SpanBatch a) {
  // Chunk geometry: 4 KiB chunks of 16 rounds; kRoundsLog for the log-record
  // kernel (crc32c_device.h).
  constexpr int kR = kSkip ? kRoundsLog : kRounds;
  constexpr uint32_t kLgC = kSkip ? kLgChunkWordsLog : 10u;  // log2(chunk words)
  // The log-record kernel skips chunk 0's padding rounds (16-round chunks).
  constexpr bool kRoundSkip = kSkip;
  constexpr uint32_t kLgB = kLgC + 2u;         // log2(chunk bytes)
  // Record indices are 32-bit: the host cuts generic batches at kMaxGenericSpans.
  uint32_t n = (uint32_t)a.n;
  if (a.n_dev != nullptr) {
    const uint64_t m = *a.n_dev;
    n = m < n ? (uint32_t)m : n;
  }
  const bool hdr = (a.flags & kFlagLogHeader) != 0;
  bool skip_long = a.role == kRoleSpans;  // long spans go through segments...
  if (a.overflow != nullptr && *a.overflow != 0u) {
    if (a.role == kRoleSegments) n = 0;   // ...unless the segment workspace overflowed
    skip_long = false;
  }
  if (n == 0) return;
  const uint32_t tid = threadIdx.x;
  const uint32_t lane = tid & 63u;
  const uint32_t wave = rfl(blockIdx.x * kWavesPerGroup + (tid >> 6));
  const uint32_t nwaves = gridDim.x * kWavesPerGroup;
  // Schedule.  The records are cut into slices of consecutive records, and
  // the wave's stream s (of S = 2 * nwaves) takes slices s, s + S, s + 2S, ...
  // so all streams sweep the batch front to back together.  Span role: slices
  // of ~equal chunk-task counts (crc32c_slice_{scan,mark}_kernel), so every stream gets the
  // same work whatever the span sizes and both streams of a wave run out
  // together (dealt equal record counts, config 3's busiest stream had 26 %
  // more tasks than the mean, and a wave folds its two streams in lockstep).  Segment role: slices of kRun records (segments are all but
  // uniform; so are span-role batches whose spans are one task each), kRun =
  // 64 shortened so every stream gets >= kRunsPerStream (64) of them:
  // a stream's count is ceil or floor of the mean, and with 16 runs per
  // stream the rounding left SST-shaped batches up to 3.6 % in the tail
  // (profiles/r02p_variants_slices_runs.json; the task-balanced slices keep
  // >= 16: smaller slices cost the config-3 mix 9 %).  A slice
  // holds at most 64 records: lane i of res[s] / bad[s] collects its i-th
  // result / verify flag, stored with one coalesced nt store when the slice's
  // last record retires (scattered 4-byte stores cost 10 % of the read rate;
  // the fixed kernel's comment has the measurement).
  const uint32_t S = 2 * nwaves;
  bool sliced = a.slice_start != nullptr;
  uint32_t K = sliced ? (uint32_t)const_load(a.nslices_dev, 0) : 0u;  // <= n/2 + 32 S + 2; 0: runs
  // Pair runs: when the scan finds every record one task (nslices = 0) and
  // the host launched crc32c_pair_kernel next to this one (a.pair_kernel,
  // large batches), that kernel takes the batch and this one leaves.
  // (not after a segment-workspace overflow: long spans are then folded here
  // as chains of chunks, but the scan counted them one task each)
  const bool pair_batch = sliced && K == 0 && skip_long;
  if (pair_batch && a.pair_kernel != 0u) return;
  // Runs: K = m S runs of q or q+1 records (q <= 63, runs 0..r-1 the longer),
  // exactly m per stream; m >= kRunsPerStream while runs keep >= 1
  // record.  (Runs of 2^lg records left a stream the ceil or floor of K/S.)
  uint32_t rq = 0, rr = 0;
  if (K == 0) {
    sliced = false;
    const uint32_t rps = kRunsPerStream;
    uint32_t m = (uint32_t)(((uint64_t)n + 63ull * S - 1u) / (63ull * S));
    if (m < rps) {
      const uint32_t mr = n / S;  // runs of >= 1 record
      m = mr < rps ? (mr > m ? mr : m) : rps;
    }
    if (m < 1u) m = 1u;
    K = (uint64_t)m * S < n ? m * S : n;
    rq = n / K;
    rr = n % K;
  }
  // A group whose streams (2 per wave) are all >= K has no slice or run: it
  // leaves before loading the tables (the segment pass of a batch with a few
  // long spans launches the whole grid for a handful of streams).
  if (blockIdx.x * 2u * kWavesPerGroup >= K) return;


  __shared__ uint32_t lds[kLdsWords];
  const uint32_t kstep = S;        // a stream's next slice or run: k + kstep
  constexpr uint32_t bstep = 1u;  // its next record in a run: b + bstep
  load_tables(lds, a.tabs, tid);
  __syncthreads();
  const StrideLanes tab = stride_lanes(lane);
  const uint32_t nibtab = 4u * (kTabWords + lane);  // byte address of lane's nibble entry [0][0]
  const ShortShift ss = short_shift_cols(lane);
  // Per stream: the pending record b (the one after the stream's newest task)
  // and its slice k = [lo, hi); b = n once the stream has no records left.
  struct Cursor {
    uint32_t b, lo, hi, k;
  };
  // Dynamic tail: slices (runs) k < Kst are dealt statically, k to stream
  // k mod S; the last kTailRounds rounds go to whichever stream asks first
  // (one atomic on a per-call counter per slice; its result is waited for
  // with the ring's loads, once per tail slice).  Waves drain at different
  // times -- by XCD as well as by SIMD rank, e.g. config 3's exits 4.5-5.6 ms
  // (profiles/r05/r05e/r05h_wave_span_ts_mixed.json) -- and the early ones
  // take the tail.
  // Claims cost an atomic on one address each: the tail shrinks with the
  // slices (runs) below 32 tasks and is dropped below 16, so the short
  // slices of a small batch do not turn it into a queue on the counter (2.4 M
  // SST spans at 4.6 pairs per run: 65 K claims in 1.8 ms ran 20 % slower
  // than no tail, 8 K claims still 1.3 %; profiles/r05/r05m/r05m_bench.json,
  // r05n_variants_tail_scaled.json).
  const uint32_t per = sliced ? (a.tasks_dev != nullptr ? (uint32_t)(const_load(a.tasks_dev, 0) / K) : 32u)
                              : rq;
  const uint32_t tail = per >= 32u ? kTailRounds : (per >= 16u ? kTailRounds * per / 32u : 0u);
  const uint32_t Kst = a.claim != nullptr && K > tail * kstep ? K - tail * kstep : K;
  // first slice or run >= k of stream st with a record for it (past Kst: claimed)
  auto open = [&](Cursor& c, uint32_t k, uint32_t st) {
    for (; k < K; k = k < Kst ? k + kstep : Kst) {  // (a claimed slice without records: claim again)
      if (k >= Kst) {
        uint32_t got = 0;
        if (lane == 0u) got = __hip_atomic_fetch_add(a.claim, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        k = Kst + rfl(got);
        if (k >= K) break;
      }
      uint32_t lo, hi;
      if (sliced) {
        lo = (uint32_t)const_load(a.slice_start, k);
        hi = (uint32_t)const_load(a.slice_start, k + 1);
      } else {
        lo = k * rq + (k < rr ? k : rr);
        hi = lo + rq + (k < rr ? 1u : 0u);
      }
      hi = hi < n ? hi : n;
      const uint32_t b = lo;
      if (b < hi) {
        c.b = b;
        c.lo = lo;
        c.hi = hi;
        c.k = k;
        return;
      }
    }
    c.b = c.lo = c.hi = n;
    c.k = K;
  };
  auto advance = [&](Cursor& c, uint32_t st) {
    if (c.b + bstep < c.hi) c.b += bstep;
    else open(c, c.k + kstep, st);
  };

  auto read_rec = [&](uint32_t b) -> SpanRec {
    SpanRec r{0u, 0u, 0u, 0u};
    if (b < n) r = const_load(a.rec, b);
    return r;
  };
  auto make_task = [&](const Cursor& c, const SpanRec& r) -> Task {
    Task t;
    t.b = c.b;
    t.r = r;
    t.c = 0;
    const bool valid = c.b < n;
    const bool skip = !valid || (skip_long && t.lng());
    t.f = (c.b - c.lo) | (c.b + bstep >= c.hi ? 1u << 8 : 0u) | (valid ? 1u << 9 : 0u) | (skip ? 1u << 10 : 0u);
    return t;
  };
  Cursor cur[2];
  SpanRec pend[2];  // record of each stream's pending record
  bool refill[2] = {false, false};
  auto next_task = [&](int s, const Task& t) -> Task {
    if (!t.skip() && t.c + 1 < t.nch(kLgB)) {  // a skipped (long) span is one task
      Task u = t;
      u.c = t.c + 1;
      return u;
    }
    Task u = make_task(cur[s], pend[s]);
    refill[s] = true;
    return u;
  };
  auto refill_recs = [&]() {  // after both streams took theirs: the scalar wait covers only older loads
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      if (refill[s]) {
        refill[s] = false;
        advance(cur[s], (uint32_t)s);
        pend[s] = read_rec(cur[s].b);
      }
    }
  };
  // 17 loads, always.
  auto issue = [&](const Task& t, uint32_t (&w)[kR], uint32_t& e) {
    const bool live = !t.skip();
    const uint32_t pad = t.pad(), h = t.h(), tl = t.t(), nch = t.nch(kLgB), len = t.len();
    // Edge window: the tail bytes and the stored trailer after them, [body
    // end, + t + 4); with a log header, [start - 6, start + len) (the stored
    // crc lies before the span).  Sizes and offsets saturate at 2^32 - 1: only
    // a log-header span of more than 2^32 - 10 bytes (log records are <= 32 KiB)
    // would lose its tail bytes, and only if it is folded here at all (long
    // spans go through segments unless the segment workspace overflows).
    const bool hwin = kVerify && hdr;
    auto sat = [](uint64_t x) -> uint32_t { return x > 0xFFFFFFFFull ? 0xFFFFFFFFu : (uint32_t)x; };
    u32x4 rb = buffer_rsrc(t.body(), live ? t.r.z : 0u);
    u32x4 re = buffer_rsrc(hwin ? t.start() - kLogCrcBack : t.body() + t.r.z,
                           live ? (hwin ? sat((uint64_t)kLogCrcBack + len) : tl + (kVerify ? 4u : 0u)) : 0u);
    // A VALU write of an SGPR (v_readfirstlane) read by a VMEM instruction
    // needs 5 wait states, and hipcc inserts none before inline asm
    // (cdna_hip_programming.md 5.7 item 2).  The descriptors are built from
    // uniform record fields on the scalar unit only, so no s_nop 4 is spent
    // here (it cost 1-5 %); tools/check_asm_hazards.py, run by build(), fails
    // the build if a compile ever feeds them from the vector unit.
    asm volatile("" : "+s"(rb), "+s"(re));
    const int32_t i0 = (int32_t)((t.c << kLgC) + lane) - (int32_t)pad;
    if (t.c != 0 || pad == 0) {
      load_rounds(w, rb, (uint32_t)i0 * 4u);
    } else if (pad <= 64u) {
      // pad <= 64 (e.g. a 3988-B SST data block): only round 0 can be
      // negative; rounds 1.. share one non-negative base with immediate
      // offsets, 2 address VALUs instead of 16
      w[0] = buf_dword<0>(rb, (uint32_t)i0 * 4u);
      load_rounds_from1(w, rb, (uint32_t)(i0 + 64) * 4u);
    } else {
      // chunk 0: offsets may be negative; give every round its own voffset so
      // the range check sees the wrapped (huge) value, never a wrapped sum
#pragma unroll
      for (int j = 0; j < kR; ++j) w[j] = buf_dword<0>(rb, (uint32_t)(i0 + 64 * j) * 4u);
    }
    // Edge bytes of the last chunk: tail bytes (lanes 3-5), stored crc (6-9).
    const bool last = t.c + 1 == nch;
    uint32_t eoff = 0xFFFFFFFFu;
    if (last && lane >= 3u && lane < 3u + tl)
      eoff = hwin ? sat((uint64_t)kLogCrcBack + h + t.r.z + (lane - 3u)) : lane - 3u;
    if (kVerify && last && lane >= 6u && lane < 10u) eoff = (hwin ? 0u : tl) + (lane - 6u);
    e = buf_ubyte(re, eoff);
  };

  // Per-stream chain state.
  uint32_t acc[2] = {0u, 0u}, r[2] = {0u, 0u};

  // Start of a chunk: the initial register (chunk 0), already fed the head
  // bytes by the planner.  It enters with body word 0: lane pad%64 of round
  // J = pad/64, a wave-uniform index.  J = 0 (full chunks, pads < 64) is one
  // XOR; otherwise a block puts it into round J's word under a scalar mask
  // (v_bitop3 w ^ (inj & m)), no branches per round.  hipcc copies the 16 ring
  // registers out and back around that block on the common path (30 v_mov per
  // span).  Returning (inj, J) instead and folding it in (a second copy of
  // the round loop under masks, as kRoundSkip does) made no copies, but was
  // no faster either (4 KiB descriptors +0.4 %, config-3 mix
  // -1.1 %, profiles/r02v_variants_span_injection.json): the span kernel is
  // not bound by its VALU count.  (A 16-way switch on J compiled to a compare
  // tree with copies at its merges; an indexed w[J] made hipcc move the ring
  // to scratch.)
  auto begin = [&](int s, const Task& t, uint32_t (&w)[kR], uint32_t& Jout) -> uint32_t {
    Jout = 0;
    if (t.c != 0) return 0u;
    const uint32_t rr = t.r.w;
    r[s] = rr;
    acc[s] = 0u;
    if (t.r.z == 0) return 0u;
    const uint32_t pad = t.pad();
    const uint32_t J = pad >> 6;
    const uint32_t inj = lane == (pad & 63u) ? rr : 0u;
    if (kRoundSkip) {
      Jout = J;
      return inj;
    }
    if (J == 0) {
      w[0] ^= inj;
    } else {
#pragma unroll
      for (int j = 1; j < kR; ++j) w[j] = __builtin_amdgcn_bitop3_b32(w[j], inj, (uint32_t)j == J ? ~0u : 0u, 0x78);
    }
    return 0u;
  };
  // Slice results: store lanes [0, t.slot()] of stream s's slice ending with task t.
  // WRITE_TRAILER: lane i of ta[s] holds the trailer address of the slice's
  // i-th span (0: none -- a skipped long span's comes from the combine pass),
  // and the slice's trailers go out with its results, one store instruction
  // per slice.  (Stored by lane 0 as each span finished, 64 stores per slice
  // sat between the ring's loads, and every counted wait after one also
  // waited for its write acknowledgement: SST descriptors sealed at 61.6 %
  // of the roofline against 73.1 % unsealed, profiles/r04/r04y_*.)
  uint32_t res[2] = {0u, 0u}, bad[2] = {0u, 0u};
  uint64_t ta[2] = {0u, 0u};
  const bool seal = (a.flags & kFlagWriteTrailer) != 0;
  // Priority rotation by SIMD age rank, as in crc32c_pair_kernel: one step
  // per finished slice.
  uint32_t prio = rfl(tid >> 6) >> 2;
  auto set_prio = [&]() {
    if (prio == 0u) __builtin_amdgcn_s_setprio(0);
    else if (prio == 1u) __builtin_amdgcn_s_setprio(1);
    else if (prio == 2u) __builtin_amdgcn_s_setprio(2);
    else __builtin_amdgcn_s_setprio(3);
  };
  set_prio();
  auto flush = [&](int s, const Task& t) {
    const uint32_t base = t.b - t.slot();
    if (lane <= t.slot()) {
      if (a.out != nullptr) __builtin_nontemporal_store(res[s], a.out + base + lane);
      if (kVerify && a.mismatch != nullptr) __builtin_nontemporal_store((uint8_t)bad[s], a.mismatch + base + lane);
      if (seal && ta[s] != 0u) store_le32(reinterpret_cast<const uint8_t*>(ta[s]), res[s]);
    }
    if (seal) ta[s] = 0u;
    prio = (prio + 1u) & 3u;
    set_prio();
  };
  // End of a span: tail bytes, conditioning, outputs.
  auto finish = [&](int s, const Task& t, uint32_t e, uint32_t body) {
    const uint32_t tl = t.t();
    const uint32_t d = tl ? readlane(e, 3) | (readlane(e, 4) << 8) | (readlane(e, 5) << 16) : 0u;
    const uint32_t crc = feed_short(ss, lane, t.r.z ? body : r[s], d, tl) ^ kConditioning;
    const uint32_t v = (a.flags & kFlagMask) ? mask_crc(crc) : crc;
    const uint32_t slot = t.slot();
    res[s] = lane == slot ? v : res[s];
    if (kVerify) {
      const uint32_t stored = readlane(e, 6) | (readlane(e, 7) << 8) | (readlane(e, 8) << 16) | (readlane(e, 9) << 24);
      bad[s] = lane == slot ? (crc != unmask_crc(stored) ? 1u : 0u) : bad[s];
    }
    if (seal) {
      const uint64_t at = reinterpret_cast<uint64_t>(hdr ? t.start() - kLogCrcBack : t.body() + t.r.z + tl);
      ta[s] = lane == slot ? at : ta[s];
    }
    if (t.last()) flush(s, t);
  };
  // Fold the pair (stream 0 task tx in wx, stream 1 task ty in wy).
  auto fold = [&](const Task& tx, uint32_t (&wx)[kR], uint32_t ex, const Task& ty,
                  uint32_t (&wy)[kR], uint32_t ey) {
    uint32_t Jx = 0, Jy = 0, ix = 0, iy = 0;  // injections (register into round J's word)
    if (!tx.skip()) ix = begin(0, tx, wx, Jx);
    if (!ty.skip()) iy = begin(1, ty, wy, Jy);
    uint32_t ax = acc[0], ay = acc[1];
    // kRoundSkip: chunk 0's rounds before round pad/64 hold only padding: acc is 0
    // there and every word is 0, so shift_256(0) ^ 0 leaves acc at 0 and the
    // rounds are skipped (a ~1 KB log record folds 4-5 rounds, not 16).
    // Skipped tasks and spans without body words fold nothing.  The pair
    // starts at the earlier of its two first rounds so the two LDS chains stay
    // interleaved.  Only log-record batches get it: elsewhere the extra
    // scalar state cost config 3 2 % and gained nothing.
    auto first_round = [](const Task& t) -> uint32_t {
      return (t.skip() || t.r.z == 0u) ? (uint32_t)kR : (t.c == 0 ? t.pad() >> 6 : 0u);
    };
    const uint32_t fx = first_round(tx), fy = first_round(ty);
    const uint32_t j0 = kRoundSkip ? (fx < fy ? fx : fy) : 0u;
    if (!kRoundSkip || (j0 == 0 && (Jx | Jy) == 0)) {
      // both registers enter in round 0; the ring registers are left untouched
#pragma unroll
      for (int j = 0; j < kR; ++j) {
        ax = step256(lds, tab, ax, j == 0 ? wx[0] ^ ix : wx[j]);
        ay = step256(lds, tab, ay, j == 0 ? wy[0] ^ iy : wy[j]);
      }
    } else {
      // a padded chunk 0: rounds before j0 skipped (kRoundSkip), round j's word
      // takes the injection under a scalar mask (one v_bitop3 w ^ (inj & m))
#pragma unroll
      for (int j = 0; j < kR; ++j) {
        if ((uint32_t)j >= j0) {
          const uint32_t mx = (uint32_t)j == Jx ? ~0u : 0u, my = (uint32_t)j == Jy ? ~0u : 0u;
          ax = step256(lds, tab, ax, __builtin_amdgcn_bitop3_b32(wx[j], ix, mx, 0x78));
          ay = step256(lds, tab, ay, __builtin_amdgcn_bitop3_b32(wy[j], iy, my, 0x78));
        }
      }
    }
    acc[0] = ax;
    acc[1] = ay;
    const bool endx = !tx.skip() && tx.c + 1 == tx.nch(kLgB), endy = !ty.skip() && ty.c + 1 == ty.nch(kLgB);
    if (endx && endy) {
      const uint32_t vx = realign(lds, nibtab, ax), vy = realign(lds, nibtab, ay);
      const uint32_t bx = wave_xor(vx), by = wave_xor(vy);
      finish(0, tx, ex, bx);
      finish(1, ty, ey, by);
    } else if (endx) {
      finish(0, tx, ex, wave_xor(realign(lds, nibtab, ax)));
    } else if (endy) {
      finish(1, ty, ey, wave_xor(realign(lds, nibtab, ay)));
    }
    // A skipped long span's result comes from the combine pass, but it may
    // close its slice: the slice's other results are stored now.
    if (tx.skip() && tx.valid() && tx.last()) flush(0, tx);
    if (ty.skip() && ty.valid() && ty.last()) flush(1, ty);
  };

  // Ring: two slots x two streams, compile-time slot indices (loop unrolled
  // over the slots) so no buffer register is copied across the back-edge
  // while its loads are in flight.  Fold slot `sl` while the other slot's two
  // tasks are in flight, then refill slot `sl`.
  Task tk[2][2];
  uint32_t wb[2][2][kR];
  uint32_t eb[2][2];
#pragma unroll
  for (int st = 0; st < 2; ++st) {
    open(cur[st], 2 * wave + st, (uint32_t)st);
    tk[0][st] = make_task(cur[st], read_rec(cur[st].b));
    advance(cur[st], (uint32_t)st);
    pend[st] = read_rec(cur[st].b);
  }
  if (!tk[0][0].valid() && !tk[0][1].valid()) return;
  tk[1][0] = next_task(0, tk[0][0]);
  tk[1][1] = next_task(1, tk[0][1]);
  refill_recs();
#pragma unroll
  for (int sl = 0; sl < 2; ++sl) {
    issue(tk[sl][0], wb[sl][0], eb[sl][0]);
    issue(tk[sl][1], wb[sl][1], eb[sl][1]);
  }
  constexpr int kYounger = 2 * (kR + 1);  // the other slot's two tasks
  for (;;) {
#pragma unroll
    for (int sl = 0; sl < 2; ++sl) {
      wait_task<kYounger>(wb[sl][0], eb[sl][0]);
      wait_task<kYounger>(wb[sl][1], eb[sl][1]);
      fold(tk[sl][0], wb[sl][0], eb[sl][0], tk[sl][1], wb[sl][1], eb[sl][1]);
      if (!tk[sl ^ 1][0].valid() && !tk[sl ^ 1][1].valid()) goto drained;
      tk[sl][0] = next_task(0, tk[sl ^ 1][0]);
      tk[sl][1] = next_task(1, tk[sl ^ 1][1]);
      refill_recs();
      issue(tk[sl][0], wb[sl][0], eb[sl][0]);
      issue(tk[sl][1], wb[sl][1], eb[sl][1]);
    }
  }
drained:
  // Retire the abandoned slot's loads while their registers are live (see the
  // fixed kernel's drain).  Every slice was stored when its last record retired.
#pragma unroll
  for (int sl = 0; sl < 2; ++sl) {
    wait_task<0>(wb[sl][0], eb[sl][0]);
    wait_task<0>(wb[sl][1], eb[sl][1]);
  }
}

// ---------------------------------------------------------------------------
// Pair runs, lean (crc32c_pair_kernel): the batches the slice scan finds all
// one-task records (every span one 4 KiB chunk or a skipped long span: SST
// data blocks, 4 KiB descriptors).  The same schedule as the span kernel's
// pair runs (K = m * nwaves runs of rq or rq + 1 record pairs, run k of wave
// k mod nwaves, the two spans of a pair adjacent), folded the way the fixed
// kernel folds: a ring of two pairs, one in flight while the other folds, and
// per pair only the run arithmetic, two scalar record reads (one pair ahead)
// and the two spans' buffer descriptors on the scalar unit.  The span
// kernel's general cursor (slices, chunk chains, record refills) cost this
// shape 134 SALU, 20 branches and 171 VALU per span against the fixed
// kernel's 29 / 1 / 128, and 1046 wave-cycles per span against 822 (PMC,
// profiles/r04/r04q_*): the general kernel ran SST descriptors at 70 % of
// the roofline where the fixed kernel runs the same blocks at 80 %.
// ---------------------------------------------------------------------------
// One span of a pair step (wave-uniform): body address, body bytes, the
// register after the head bytes, and f = pad | t << 10 | valid << 12 | skip << 13
// | slot << 16 (the span's position in its run).
struct PTask {
  uint64_t body;
  uint32_t z, w, f;
  __device__ uint32_t pad() const { return f & 1023u; }
  __device__ uint32_t t() const { return (f >> 10) & 3u; }
  __device__ bool valid() const { return (f >> 12) & 1u; }
  __device__ bool live() const { return ((f >> 12) & 3u) == 1u; }  // valid, not skipped
  __device__ uint32_t slot() const { return (f >> 16) & 63u; }
};

template <bool kVerify>
__global__ __launch_bounds__(kThreads) void crc32c_pair_kernel(SpanBatch a) {
  const uint32_t n = (uint32_t)a.n;  // (span role, no list: n_dev is null)
  // The scan's verdict: pair runs only for an all-one-task batch with the long
  // spans skipped (the general kernel takes the rest and leaves these).
  if (a.slice_start == nullptr || (a.overflow != nullptr && *a.overflow != 0u)) return;
  if ((uint32_t)const_load(a.nslices_dev, 0) != 0u || n == 0u) return;
  const uint32_t nwaves = gridDim.x * kWavesPerGroup;
  const uint32_t np = (n + 1u) / 2u;  // record pairs
  uint32_t m = (uint32_t)(((uint64_t)np + 31ull * nwaves - 1u) / (31ull * nwaves));  // <= 32 pairs a run
  if (m < kRunsPerStream) {
    const uint32_t mr = np / nwaves;
    m = mr < kRunsPerStream ? (mr > m ? mr : m) : kRunsPerStream;
  }
  if (m < 1u) m = 1u;
  const uint32_t K = (uint64_t)m * nwaves < np ? m * nwaves : np;
  const uint32_t rq = np / K, rr = np % K;
  if (blockIdx.x * kWavesPerGroup >= K) return;

  __shared__ uint32_t lds[kLdsWords];
  const uint32_t tid = threadIdx.x;
  load_tables(lds, a.tabs, tid);
  __syncthreads();
  const uint32_t lane = tid & 63u;
  const uint32_t wave = rfl(blockIdx.x * kWavesPerGroup + (tid >> 6));
  const StrideLanes tab = stride_lanes(lane);
  const uint32_t nibtab = 4u * (kTabWords + lane);
  const ShortShift ss = short_shift_cols(lane);
  const bool masked = (a.flags & kFlagMask) != 0;
  const bool seal = (a.flags & kFlagWriteTrailer) != 0;

  // Priority rotation.  Waves k, k + 4, k + 8, k + 12 of a group share SIMD
  // k % 4, and at equal user priority the older wave issues first: with equal
  // runs, a bulk SST batch's waves left at 7.7 / 8.7 / 10.2 / 11.6 ms by age
  // rank, the youngest alone at the end (tools/wave_timeline.py,
  // profiles/r05/r05e/r05e_wave_pair_ts.json).  A wave's user priority is
  // (rank + runs started) mod 4 (s_setprio: user priority ranks ahead of
  // age), so every wave spends a quarter of its runs at each level: exits
  // 9.6-10.5 ms, SST descriptors +4.2 %, sealed +4.3 %, 4 KiB descriptors
  // +4.3 % (r05e_variants_simd_rank_balance.json).  (Static run weights by
  // rank gained 1.6 %; the fixed kernel, whose remaining waves keep HBM busy
  // after the oldest leave, gains nothing from either.)
  uint32_t prio = rfl(tid >> 6) >> 2;
  auto set_prio = [&]() {
    if (prio == 0u) __builtin_amdgcn_s_setprio(0);
    else if (prio == 1u) __builtin_amdgcn_s_setprio(1);
    else if (prio == 2u) __builtin_amdgcn_s_setprio(2);
    else __builtin_amdgcn_s_setprio(3);
  };
  set_prio();

  // Issue-side cursor: run k = [lo, hi) records, pair i of it.  Runs past
  // Kst (the last kPairTailRounds rounds) are claimed on demand, as in
  // crc32c_span_kernel (runs are never empty) -- but a claim's atomic goes
  // out when the wave starts the run before it, and its return is read at
  // that run's end: no wave waits for a claim.  (Read right away, each claim
  // drained the wave's ring -- hipcc's vmcnt(0) -- and a tail cost short
  // runs more than it balanced: 2.4 M SST spans at 4.6 pairs per run ran
  // 20 % slower with 65 K claims, so batches under 16 pairs per run had
  // none, and their waves left over 1505-1721 us of a 1.72 ms kernel, by
  // SIMD age rank and XCD; profiles/r05/r05m, profiles/r06/r06ad_pair_waves.
  // Prefetched claims on one counter balanced the waves but the counter took
  // only ~86 claims per us against the ~170 per us config 5's short runs ask
  // for: the kernel ran 20 % slower, r06ae_single_counter.  Eight counters:
  // exits 1721-1756 us, desc4k -3.3 %, config-5 seals -2.4 %, r06af / r06ah.)
  // The claim's return lands in lane 0 of a ring slot's edge register (lane
  // 0 takes no edge byte: its load is out of range and returns 0 first), so
  // no register is added to the ring and the ring's own counted wait for
  // that slot retires it: issued right after a take's loads when the take
  // starts a run whose successor is claimed, read after the slot's next wait
  // -- two takes on, before that run's last take when runs hold >= 3 pairs
  // (shorter runs: no tail).  tools/check_inflight.py audits the build (a
  // claim register of its own, loop-carried, cost hipcc SGPR spills and
  // failed the audit).
  // Eight claim counters (kClaimLines), counter c for the groups b with
  // (b / 8) % 8 == c (each set spans every XCD and holds every SIMD rank):
  // counter c deals the tail runs Kst + c + 8 j.
  const uint32_t ptail = rq >= 3u ? kPairTailRounds : 0u;
  const uint32_t Kst = a.claims != nullptr && K > ptail * nwaves ? K - ptail * nwaves : K;
  const uint32_t cset = (blockIdx.x >> 3) & (kClaimLines - 1u);
  uint32_t* const ctr = a.claims != nullptr ? a.claims + kClaimLineWords * cset : nullptr;
  auto claim_into = [&](uint32_t& e, uint32_t need) {
    uint64_t sv;
    asm volatile(
        "s_cmp_eq_u32 %2, 0\n\t"
        "s_cbranch_scc1 .Lno_claim%=\n\t"
        "s_mov_b64 %1, exec\n\t"
        "s_mov_b64 exec, 1\n\t"
        "global_atomic_add %0, %3, %4, %5 sc0\n\t"
        "s_mov_b64 exec, %1\n"
        ".Lno_claim%=:"
        : "+v"(e), "=&s"(sv)
        : "s"(need), "v"(0u), "v"(1u), "s"(ctr)
        : "memory", "scc");
  };
  uint32_t k = wave, lo = 0, hi = 0, i = 0;
  auto run_bounds = [&](uint32_t kk) {
    lo = 2u * (kk * rq + (kk < rr ? kk : rr));
    hi = lo + 2u * (rq + (kk < rr ? 1u : 0u));
    hi = hi < n ? hi : n;
  };
  // the wave's next run after k is a claimed one
  auto wants_claim = [&]() -> bool { return Kst < K && k < K && k + nwaves >= Kst; };
  if (k >= Kst && k < K) {  // no static run: the first claim is waited for (no loads out yet)
    uint32_t got = 0;
    if (lane == 0u) got = __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    k = Kst + cset + kClaimLines * rfl(got);
  }
  if (k < K) run_bounds(k);
  uint32_t kn = 0u;                  // the claimed successor of the current run, once read
  uint32_t need = wants_claim() ? 1u : 0u;  // claim after this take's loads (the first: after take 0's)
  // b: the pair's first record (n: none left)
  auto pair_first = [&]() -> uint32_t { return k < K ? lo + 2u * i : n; };
  auto step = [&]() {
    if (k >= K) return;
    if (lo + 2u * (i + 1u) < hi) {
      ++i;
    } else {
      k = wants_claim() ? kn : k + nwaves;  // (claimed: read two takes ago at the latest)
      i = 0;
      if (k < K) run_bounds(k);
      need = wants_claim() ? 1u : 0u;
      prio = (prio + 1u) & 3u;
      set_prio();
    }
  };
  auto read_rec = [&](uint32_t b) -> SpanRec {
    SpanRec r{0u, 0u, 0u, 0u};
    if (b < n) r = const_load(a.rec, b);
    return r;
  };
  auto make = [&](uint32_t b, const SpanRec& r, uint32_t first) -> PTask {
    PTask t;
    const bool valid = b < n && b < hi;
    t.body = ((uint64_t)(r.y & 0xffffu) << 32) | r.x;
    t.z = valid ? r.z : 0u;
    t.w = r.w;
    const uint32_t skip = valid && ((r.y >> 30) & 1u) ? 1u : 0u;
    t.f = ((r.y >> 16) & 1023u) | (((r.y >> 28) & 3u) << 10) | ((valid ? 1u : 0u) << 12) | (skip << 13) |
          ((b - first) << 16);
    return t;
  };
  // 17 loads per span, always: 16 body dwords (chunk 0 right-aligned: the
  // pad leading words read 0 through the range check) and one edge byte per
  // lane -- tail bytes (lanes 3-5) and the stored crc (6-9).
  auto issue = [&](const PTask& t, uint32_t (&w)[kRounds], uint32_t& e) {
    const bool live = t.live();
    const uint32_t pad = t.pad(), tl = t.t();
    u32x4 rb = buffer_rsrc(reinterpret_cast<const uint8_t*>(t.body), live ? t.z : 0u);
    u32x4 re = buffer_rsrc(reinterpret_cast<const uint8_t*>(t.body + t.z), live ? tl + (kVerify ? 4u : 0u) : 0u);
    asm volatile("" : "+s"(rb), "+s"(re));  // (scalar-built: tools/check_asm_hazards.py)
    const int32_t i0 = (int32_t)lane - (int32_t)pad;
    if (pad == 0) {
      load_rounds(w, rb, (uint32_t)i0 * 4u);
    } else if (pad <= 64u) {
      w[0] = buf_dword<0>(rb, (uint32_t)i0 * 4u);
      load_rounds_from1(w, rb, (uint32_t)(i0 + 64) * 4u);
    } else {
#pragma unroll
      for (int j = 0; j < kRounds; ++j) w[j] = buf_dword<0>(rb, (uint32_t)(i0 + 64 * j) * 4u);
    }
    uint32_t eoff = 0xFFFFFFFFu;
    if (lane >= 3u && lane < 3u + tl) eoff = lane - 3u;
    if (kVerify && lane >= 6u && lane < 10u) eoff = tl + (lane - 6u);
    e = buf_ubyte(re, eoff);
  };

  // WRITE_TRAILER: lane i of ta holds the trailer address of the run's i-th
  // span (0: none), stored with the run's results (the span kernel's note).
  uint32_t res = 0u, bad = 0u;
  uint64_t ta = 0u;
  auto finish = [&](const PTask& t, uint32_t e, uint32_t body) {
    const uint32_t tl = t.t();
    const uint32_t d = tl ? readlane(e, 3) | (readlane(e, 4) << 8) | (readlane(e, 5) << 16) : 0u;
    const uint32_t crc = feed_short(ss, lane, t.z ? body : t.w, d, tl) ^ kConditioning;
    const uint32_t v = masked ? mask_crc(crc) : crc;
    const uint32_t slot = t.slot();
    res = lane == slot ? v : res;
    if (kVerify) {
      const uint32_t stored = readlane(e, 6) | (readlane(e, 7) << 8) | (readlane(e, 8) << 16) | (readlane(e, 9) << 24);
      bad = lane == slot ? (crc != unmask_crc(stored) ? 1u : 0u) : bad;
    }
    if (seal) ta = lane == slot ? t.body + t.z + tl : ta;
  };
  // The register enters with body word 0: lane pad % 64 of round pad / 64.
  auto inject = [&](const PTask& t, uint32_t (&w)[kRounds]) {
    const uint32_t pad = t.pad(), J = pad >> 6;
    const uint32_t inj = lane == (pad & 63u) ? t.w : 0u;
    if (J == 0) {
      w[0] ^= inj;
    } else {
#pragma unroll
      for (int j = 1; j < kRounds; ++j) w[j] = __builtin_amdgcn_bitop3_b32(w[j], inj, (uint32_t)j == J ? ~0u : 0u, 0x78);
    }
  };
  // Fold a pair; the run's results go out with its last pair (lanes below its
  // record count: skipped long spans' lanes too, which the combine pass then
  // overwrites).
  auto fold = [&](const PTask& tx, uint32_t (&wx)[kRounds], uint32_t ex, const PTask& ty, uint32_t (&wy)[kRounds],
                  uint32_t ey, uint32_t first, uint32_t cnt, bool last) {
    const bool lx = tx.live() && tx.z != 0u, ly = ty.live() && ty.z != 0u;
    if (lx) inject(tx, wx);
    if (ly) inject(ty, wy);
    uint32_t ax = wx[0], ay = wy[0];
#pragma unroll
    for (int j = 1; j < kRounds; ++j) {
      ax = step256(lds, tab, ax, wx[j]);
      ay = step256(lds, tab, ay, wy[j]);
    }
    const uint32_t bx = wave_xor(realign(lds, nibtab, ax)), by = wave_xor(realign(lds, nibtab, ay));
    if (tx.live()) finish(tx, ex, bx);
    if (ty.live()) finish(ty, ey, by);
    if (last) {
      if (lane < cnt) {
        if (a.out != nullptr) __builtin_nontemporal_store(res, a.out + first + lane);
        if (kVerify && a.mismatch != nullptr) __builtin_nontemporal_store((uint8_t)bad, a.mismatch + first + lane);
        if (seal && ta != 0u) store_le32(reinterpret_cast<const uint8_t*>(ta), res);
      }
      if (seal) ta = 0u;
    }
  };

  // Ring: two pair slots, compile-time slot indices (the loop is unrolled over
  // them) so no buffer register is copied while its loads are in flight.
  PTask tk[2][2];
  uint32_t tfirst[2], tcnt[2], tlast[2];  // per slot: the run's first record, its record count, last pair?
  uint32_t wb[2][2][kRounds];
  uint32_t eb[2][2];
  // records of the next pair to issue (one pair ahead: scalar loads)
  uint32_t pb = pair_first();
  SpanRec p0 = read_rec(pb), p1 = read_rec(pb + 1u);
  auto take = [&](int sl) {
    const uint32_t b = pb;
    tk[sl][0] = make(b, p0, lo);
    tk[sl][1] = make(b + 1u, p1, lo);
    tfirst[sl] = lo;
    tcnt[sl] = hi - lo;
    tlast[sl] = (k < K && b + 2u >= hi) ? 1u : 0u;
    if (k >= K) {
      tk[sl][0].f = tk[sl][1].f = 0u;
      tlast[sl] = 0u;
    }
    step();
    pb = pair_first();
    p0 = read_rec(pb);
    p1 = read_rec(pb + 1u);
  };
  uint32_t cs[2];  // per slot: a claim rides in lane 0 of its edge register eb[sl][1]
#pragma unroll
  for (int sl = 0; sl < 2; ++sl) {
    take(sl);
    issue(tk[sl][0], wb[sl][0], eb[sl][0]);
    issue(tk[sl][1], wb[sl][1], eb[sl][1]);
    cs[sl] = rfl(need);  // (rfl: an SGPR operand -- hipcc takes the flag for divergent)
    claim_into(eb[sl][1], cs[sl]);
    need = 0u;
  }
  constexpr int kYounger = 2 * (kRounds + 1);  // the other slot's two spans
  for (;;) {
#pragma unroll
    for (int sl = 0; sl < 2; ++sl) {
      wait_task<kYounger>(wb[sl][0], eb[sl][0]);
      wait_task<kYounger>(wb[sl][1], eb[sl][1]);
      if (cs[sl] != 0u) kn = Kst + cset + kClaimLines * readlane(eb[sl][1], 0);
      if (tk[sl][0].valid())
        fold(tk[sl][0], wb[sl][0], eb[sl][0], tk[sl][1], wb[sl][1], eb[sl][1], tfirst[sl], tcnt[sl], tlast[sl] != 0u);
      if (!tk[sl ^ 1][0].valid()) goto drained;
      take(sl);
      issue(tk[sl][0], wb[sl][0], eb[sl][0]);
      issue(tk[sl][1], wb[sl][1], eb[sl][1]);
      cs[sl] = rfl(need);
      claim_into(eb[sl][1], cs[sl]);
      need = 0u;
    }
  }
drained:
  // the abandoned slot's loads retire while their registers are live
#pragma unroll
  for (int sl = 0; sl < 2; ++sl) {
    wait_task<0>(wb[sl][0], eb[sl][0]);
    wait_task<0>(wb[sl][1], eb[sl][1]);
  }
}

// ---------------------------------------------------------------------------
// Fixed-geometry fast path: every span is len bytes at base + i*stride with
// base, stride and len multiples of 4 and len <= 4 KiB, so a span is K rounds
// (K = ceil(len/256), a template parameter) with no head/tail bytes and the
// same padding (pk = 64K - len/4 leading zero words, all in round 0).
// Ring of four span buffers consumed in pairs (loop unrolled x2): the next
// pair's loads are in flight while a pair is folded; counted vmcnt waits only.
// ---------------------------------------------------------------------------
template <int K, bool kVerify>
__global__ __launch_bounds__(kThreads) void crc32c_fixed_kernel(SpanBatch a) {
  const uint64_t n = a.n;
  __shared__ uint32_t lds[kLdsWords];
  const uint32_t tid = threadIdx.x;
  load_tables(lds, a.tabs, tid);
  const uint32_t lane = tid & 63u;
  __syncthreads();
  const StrideLanes tab = stride_lanes(lane);
  const uint32_t nibtab = 4u * (kTabWords + lane);  // byte address of lane's nibble entry [0][0]
  const uint64_t wave = rfl(blockIdx.x * kWavesPerGroup + (tid >> 6));
  const uint64_t nwaves = (uint64_t)gridDim.x * kWavesPerGroup;

  // Spans are dealt to waves in runs of kRun consecutive spans: run r of wave
  // w is spans [(r * nwaves + w) * kRun, +kRun), two per pair step.  Lane i
  // of `res` collects the run's i-th result and the run ends with ONE
  // coalesced 256-B store.  (One 4-byte store per span, scattered over 4096
  // waves, cost 10 % of the read rate in partial-line writes -- measured
  // with tools/bwprobe.py's store-pattern probes, profiles/
  // r01_bwprobe_store_patterns.json; runs of 64 also read 2-4 % faster than
  // spans dealt one by one.)
  // kRun = 64, shortened (power of two >= 2) for batches too small to give
  // every wave a few full runs.
  static_assert(kRunLg <= 5, "a run's results fit the 64 lanes");
  uint32_t lg = kRunLg;  // log2(pair steps per run)
  while (lg > 0 && (n >> (lg + 1)) < nwaves * 4u) --lg;
  const uint64_t kRun = 2ull << lg;
  // First span of the wave's next pair step: +2 inside a run, then on to the
  // wave's next run (the other waves' runs in between).
  // (Pairing spans half a run apart instead cost 3.7 %,
  // profiles/r02af_variants_fixed_far_pair.json.)
  const uint64_t kSecond = 1u;
  const uint64_t jump = (nwaves - 1u) * kRun + 2u;
  auto adv = [&](uint64_t x) -> uint64_t { return ((x + 2u) & (kRun - 1u)) ? x + 2u : x + jump; };
  uint64_t cur = wave * kRun;  // first span of the pair being folded
  if (cur >= n) return;

  // pk: leading zero words (round 0).  Verify sizes K for len + 4, so pk >= 1
  // and lane 0 of round 0 -- padding, masked out of the fold -- loads the
  // stored trailer word right after the span (ReadBlock, table/format.cc:93-95).
  const uint32_t pk = 64u * K - (a.len_c >> 2);  // 0..63 (1..64 when verifying)
  const uint32_t r0 = a.init_c ^ kConditioning;
  const bool masked = (a.flags & kFlagMask) != 0;
  const int32_t w0 = (int32_t)lane - (int32_t)pk;   // word index of round 0
  const uint32_t off0 = kVerify && lane == 0u ? a.len_c : (uint32_t)(w0 < 0 ? 0 : w0) * 4u;
  const uint32_t off1 = (uint32_t)(w0 + 64) * 4u;   // rounds >= 1 never clamp

  // The ring's loads are issued with inline asm and retired with explicit
  // counted waits (hipcc's own waitcnt pass merges the ring's scoreboards into
  // vmcnt(0), which would drain the prefetch).  Unconditional: a span past the
  // end re-reads the last one.  Every buffer is exactly K loads.
  auto issue = [&](uint64_t b, uint32_t (&w)[kRounds]) {
    b = b < n ? b : n - 1;
    const uint8_t* p = a.base + b * a.stride;
    w[0] = asm_load_dword<0>(p, off0);
#pragma unroll
    for (int j = 1; j < K; ++j) w[j] = asm_load_dword_at<K>(p, off1, j);
  };
  uint32_t res = 0, bad = 0;
  // Two spans folded together: two independent LDS dependency chains per wave.
  // The waits count only the ring's loads (the pairs issued after the awaited
  // one); the run-end store, when younger than them, only makes a wait stricter.
  constexpr int kYounger = (kRing / 2 - 1) * 2 * K;
  auto wait2 = [&](uint32_t (&wa)[kRounds], uint32_t (&wb)[kRounds]) {
    wait_ring<kYounger>(wa);  // the younger pairs may stay in flight
    wait_ring<kYounger>(wb);
  };
  auto fold2 = [&](const uint32_t (&wa)[kRounds], const uint32_t (&wb)[kRounds]) {
    uint32_t xa = lane >= pk ? wa[0] : 0u, xb = lane >= pk ? wb[0] : 0u;
    xa ^= lane == pk ? r0 : 0u;  // initial register enters with body word 0
    xb ^= lane == pk ? r0 : 0u;
    uint32_t acc_a = xa, acc_b = xb;
#pragma unroll
    for (int j = 1; j < K; ++j) {
      acc_a = step256(lds, tab, acc_a, wa[j]);
      acc_b = step256(lds, tab, acc_b, wb[j]);
    }
    const uint32_t va = realign(lds, nibtab, acc_a), vb = realign(lds, nibtab, acc_b);
    const uint32_t ca = wave_xor(va) ^ kConditioning, cb = wave_xor(vb) ^ kConditioning;
    const uint32_t i = (uint32_t)(cur & (kRun - 1u)), i2 = i + 1u;  // the pair's lanes in the run
    res = lane == i ? (masked ? mask_crc(ca) : ca) : res;
    res = lane == i2 ? (masked ? mask_crc(cb) : cb) : res;
    if (kVerify) {
      const uint32_t ba = ca != unmask_crc(readlane(wa[0], 0)) ? 1u : 0u;
      const uint32_t bb = cb != unmask_crc(readlane(wb[0], 0)) ? 1u : 0u;
      bad = lane == i ? ba : bad;
      bad = lane == i2 ? bb : bad;
    }
  };
  // Run end (or the last pair): lanes 0..i+1 hold results of spans b0 + lane.
  auto flush = [&]() {
    const uint64_t b0 = cur & ~(kRun - 1u);
    const uint32_t last = (uint32_t)(cur & (kRun - 1u)) + 1u;
    // nt: the results are not re-read; a streaming store keeps them from
    // contending with the read stream (0.6 % of the read rate vs 2 %, probes).
    if (lane <= last && b0 + lane < n) {
      if (!kVerify || a.out != nullptr) __builtin_nontemporal_store(res, a.out + b0 + lane);
      if (kVerify && a.mismatch != nullptr) __builtin_nontemporal_store((uint8_t)bad, a.mismatch + b0 + lane);
    }
  };

  // Ring of kRing span buffers, consumed in pairs; loop unrolled so every
  // buffer has a static register name.  (Refilling a slot before its fold,
  // with a 6-buffer ring, measured no faster: profiles/r01_variants_ring_runs.json.)
  static_assert(kRing % 2 == 0 && kRing >= 4, "pairs; one pair in flight during a fold");
  static_assert(kYounger <= 63, "vmcnt is a 6-bit counter");
  uint32_t ring[kRing][kRounds];
  uint64_t ahead = cur;  // first span of the next pair to issue
#pragma unroll
  for (int d = 0; d < kRing; d += 2) {
    issue(ahead, ring[d]);
    issue(ahead + kSecond, ring[d + 1]);
    ahead = adv(ahead);
  }
  // One exit, at the bottom of a whole ring turn: steps past the wave's last
  // pair (their loads re-read span n-1) are waited for but not folded.  The
  // prefetched pairs still in flight at the exit are retired while their
  // registers are live (operands of the markers after the wait), so the
  // compiler cannot hand such a register to other code before its load lands.
  for (;;) {
#pragma unroll
    for (int s = 0; s < kRing; s += 2) {
      wait2(ring[s], ring[s + 1]);
      const uint64_t nxt = adv(cur);
      if (cur < n) {
        fold2(ring[s], ring[s + 1]);
        if (nxt >= n || (nxt & (kRun - 1u)) == 0) flush();
      }
      cur = nxt;
      issue(ahead, ring[s]);
      issue(ahead + kSecond, ring[s + 1]);
      ahead = adv(ahead);
    }
    if (cur >= n) break;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
  for (int d = 0; d < kRing; ++d) {
#pragma unroll
    for (int j = 0; j < K; ++j) asm volatile("" : "+v"(ring[d][j]));
  }
}

// ---------------------------------------------------------------------------
// Planner: one thread per span writes its record and its task count; spans
// longer than skip_above become segments [first piece of len - (nseg-1)*kSegment
// bytes with the span's init] + nseg-1 pieces of kSegment bytes with init
// 0xFFFFFFFF (Extend(~0, d) ^ ~0 is the raw register R(0, d)), each with its
// own record for the segment pass.  Block b covers records [b*tile, +tile) and
// leaves its task sum in bsum[b] for the slice scan.
// ---------------------------------------------------------------------------
// Records of the batch: n, or the device count when the batch is the lane
// kernel's list of the spans it leaves.
__device__ __forceinline__ uint64_t batch_n(const SpanBatch& a) {
  uint64_t n = a.n;
  if (a.n_dev != nullptr) {
    const uint64_t m = *a.n_dev;
    n = m < n ? m : n;
  }
  return n;
}

template <bool kDesc>
__global__ __launch_bounds__(kPlanThreads) void crc32c_plan_kernel(SpanBatch a, SplitWs ws) {
  // the next call's counters (the other parity's block, idle since the call
  // before this one): zeroed here instead of by a fill kernel in front of it
  if (blockIdx.x == 0u && ws.zero_next != nullptr) {
    uint32_t* const z = reinterpret_cast<uint32_t*>(ws.zero_next);
    if (threadIdx.x < 64u) z[threadIdx.x] = 0u;  // SplitCounters
    else if (threadIdx.x < 64u + kClaimLines) z[64u + kClaimLineWords * (threadIdx.x - 64u)] = 0u;  // claim lines
  }
  const uint64_t n = batch_n(a);
  const uint64_t lo = (uint64_t)blockIdx.x * ws.tile;
  if (lo >= n) {  // (behind the lane kernel the list is often empty: ~4000 blocks leave at once)
    if (threadIdx.x == 0) ws.bsum[blockIdx.x] = 0;
    return;
  }
  const uint64_t hi = lo + ws.tile < n ? lo + ws.tile : n;
  __shared__ unsigned long long sum;
  if (threadIdx.x == 0) sum = 0;
  __syncthreads();
  uint32_t mine = 0;  // <= tile/256 spans of <= 32 tasks each
  // Uniform trip count (the block's bounds), so the wave can write a long
  // span's segment records together below.
  for (uint64_t i0 = lo; i0 < hi; i0 += kPlanThreads) {
    const uint64_t i = i0 + threadIdx.x;
    // this lane's long span, if it has one, for the wave's segment writes
    const uint8_t* sp = nullptr;
    uint64_t spos = 0;
    uint32_t snseg = 0, sfirst = 0, sinit = 0;
    if (i < hi) do {
    const uint64_t q = a.idx != nullptr ? a.idx[i] : i;  // the caller's span
    const uint64_t off = kDesc ? a.off[q] : q * a.stride;
    const uint32_t len = kDesc ? a.len[q] : a.len_c;
    const uint32_t init = kDesc ? (a.init != nullptr ? a.init[q] : 0u) : a.init_c;
    const uint8_t* p = a.base + off;
    const bool lng = len > a.skip_above;
    const SpanRec r = make_rec(p, len, init, lng, a.chunk_lg);
    ws.rec[i] = r;
    const uint32_t lgb = a.chunk_lg + 2u;
    const uint32_t cnt = lng ? 1u : (r.z ? (r.z >> lgb) + ((r.z & ((1u << lgb) - 1u)) != 0u ? 1u : 0u) : 1u);  // Task::nch()
    ws.cnt[i] = cnt;
    mine += cnt;
    if (!lng) break;
    const uint32_t nseg = (uint32_t)(((uint64_t)len + kSegment - 1u) / kSegment);  // len up to 2^32 - 1
    const uint32_t first = len - (nseg - 1u) * kSegment;
    const uint64_t pos = atomicAdd((unsigned long long*)&ws.counters->nseg, (unsigned long long)nseg);
    const uint32_t li = atomicAdd(&ws.counters->nlong, 1u);
    if (pos + nseg > ws.cap_seg || li >= ws.cap_long) {
      atomicOr(&ws.counters->overflow, 1u);
      break;
    }
    ws.long_span[li] = i;
    ws.long_first[li] = pos;
    ws.long_nseg[li] = nseg;
    sp = p;
    spos = pos;
    snseg = nseg;
    sfirst = first;
    sinit = init;
    } while (false);
    // Segments: the general kernel (4 KiB chunks) folds them.  Their records
    // are written by the whole wave, one long span at a time, 64 segments per
    // step: each record's head bytes are a dependent global read, and one
    // thread writing a 487 KB index span's 15 records took 12 us per call
    // (the planner's whole time on one SST file).
    uint64_t lm = __ballot(sp != nullptr);
    while (lm != 0u) {
      const int src = __ffsll((long long)lm) - 1;
      lm &= lm - 1u;
      const uint8_t* bp = reinterpret_cast<const uint8_t*>(__shfl((unsigned long long)(uintptr_t)sp, src, 64));
      const uint64_t bpos = __shfl((unsigned long long)spos, src, 64);
      const uint32_t bn = __shfl(snseg, src, 64), bf = __shfl(sfirst, src, 64), bi = __shfl(sinit, src, 64);
      for (uint32_t s = threadIdx.x & 63u; s < bn; s += 64u)
        ws.seg_rec[bpos + s] = s == 0u ? make_rec(bp, bf, bi, false, 10u)
                                       : make_rec(bp + bf + (uint64_t)(s - 1u) * kSegment, kSegment, kConditioning,
                                                  false, 10u);
    }
  }
  atomicAdd(&sum, (unsigned long long)mine);
  __syncthreads();
  if (threadIdx.x == 0) ws.bsum[blockIdx.x] = sum;
}

// Exclusive prefix of v over the block's kPlanThreads threads (LDS, log steps).
__device__ uint64_t block_exclusive_scan(uint64_t v, uint64_t* sh, uint64_t& total) {
  const uint32_t t = threadIdx.x;
  sh[t] = v;
  __syncthreads();
  for (uint32_t d = 1; d < blockDim.x; d <<= 1) {
    const uint64_t x = t >= d ? sh[t - d] : 0u;
    __syncthreads();
    sh[t] += x;
    __syncthreads();
  }
  const uint64_t incl = sh[t];
  total = sh[blockDim.x - 1];
  __syncthreads();
  return incl - v;
}

// ---------------------------------------------------------------------------
// Slice schedule of the span pass.  T tasks in all, cut into K = m S slices
// (m per stream of the span kernel's S streams): slice k = tasks
// [k q + min(k, r), ...) with q = T / K, r = T % K, i.e. q or q + 1 <= 64
// tasks, so a slice holds <= 64 records (every record is >= 1 task) and
// slice_start[k] = the first record whose first task is in slice k or later.
//   scan kernel (1 block): exclusive prefix of the planner blocks' sums, T,
//                          q, r, nslices, slice_start[0] and [nslices]
//   mark kernel (planner tiles): record i with first task E and c tasks opens
//                          slices (slice(E), slice(E+c)]: slice_start[k] = i + 1
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(1024) void crc32c_slice_scan_kernel(SpanBatch a, SplitWs ws) {
  __shared__ uint64_t sh[1024];
  const uint32_t t = threadIdx.x;
  constexpr uint32_t kPer = kMaxPlanBlocks / 1024;
  uint64_t v[kPer], mine = 0;
#pragma unroll
  for (uint32_t j = 0; j < kPer; ++j) {
    const uint32_t b = t * kPer + j;
    v[j] = b < ws.nblocks ? ws.bsum[b] : 0u;
    mine += v[j];
  }
  uint64_t T = 0;
  uint64_t run = block_exclusive_scan(mine, sh, T);
#pragma unroll
  for (uint32_t j = 0; j < kPer; ++j) {
    const uint32_t b = t * kPer + j;
    if (b < ws.nblocks) ws.bsum[b] = run;
    run += v[j];
  }
  if (t == 0) {
    const uint64_t S = ws.nstreams;
    // K = m S slices, so every stream gets exactly m of them (dealt s, s+S,
    // ...): with K = ceil(T / 2^lg) a stream got ceil or floor of K/S and the
    // ceil streams set the kernel's end (config 3: 17 slices against a mean of
    // 16.6).  Slice k = tasks [k q + min(k, r), ...) with q = T / K, r = T % K.
    // At most 64 tasks per slice (q <= 63), so at most 64 records (a lane
    // per result); at least 16 slices per stream while they stay >= 32 tasks
    // (a slice of >= 32 tasks always starts a record: spans are <= 32 tasks).
    const uint64_t per = kSlicesPerStream;
    uint64_t m = (T + 63u * S - 1u) / (63u * S);
    const uint64_t m32 = T / (32u * S);
    if (m < per && m32 > m) m = m32 < per ? m32 : per;
    if (m < 1u) m = 1u;
    uint64_t K = m * S;
    if (K > T) K = T > 0 ? T : 1u;
    ws.counters->slice_q = T / K;
    ws.counters->slice_r = T % K;
    ws.counters->tasks = T;
    // Every span one task (4 KiB blocks, log records, SST data blocks): slices
    // of tau tasks are runs of tau records, which the span kernel deals
    // without slice starts -- nslices = 0 says so and the mark pass is skipped.
    const uint64_t n = batch_n(a);
    ws.counters->nslices = T == n ? 0 : K;
    ws.slice_start[0] = 0;
    ws.slice_start[K] = n;
  }
}

__global__ __launch_bounds__(kPlanThreads) void crc32c_slice_mark_kernel(SpanBatch a, SplitWs ws) {
  const uint64_t K = ws.counters->nslices;
  if (K == 0) return;  // uniform batch: runs, no slice starts
  __shared__ uint64_t sh[kPlanThreads];
  const uint64_t n = batch_n(a);
  // slice of task position x: slices 0..r-1 hold q+1 tasks, the rest q
  const uint64_t q = ws.counters->slice_q, r = ws.counters->slice_r, rq = r * (q + 1u);
  auto slice_of = [&](uint64_t x) -> uint64_t { return x < rq ? x / (q + 1u) : r + (x - rq) / q; };
  // Thread t walks its own per = tile/256 consecutive records of the block's
  // tile: one block scan per tile instead of one per 256 records.
  const uint64_t per = ws.tile / kPlanThreads;
  const uint64_t lo = (uint64_t)blockIdx.x * ws.tile + threadIdx.x * per;
  const uint64_t hi = lo + per < n ? lo + per : n;
  uint64_t mine = 0;
  for (uint64_t i = lo; i < hi; ++i) mine += ws.cnt[i];
  uint64_t total = 0;
  uint64_t e = ws.bsum[blockIdx.x] + block_exclusive_scan(mine, sh, total);
  for (uint64_t i = lo; i < hi; ++i) {
    const uint32_t c = ws.cnt[i];
    const uint64_t k1 = slice_of(e + c);
    for (uint64_t k = slice_of(e) + 1; k <= k1 && k <= K; ++k) ws.slice_start[k] = i + 1;
    e += c;
  }
}

// ---------------------------------------------------------------------------
// Long-span combine, one wave per long span.  With M = shift_kSegment and raw
// segment registers s_k = seg_out ^ ~0, the span's register is
//     R = sum_k M^(nseg-1-k) s_k.
// Padded with zero segments in front to 64 J, segment 64 j + l goes to lane l:
//     R = sum_l M^(63-l) R_l,  R_l = sum_j (M^64)^(J-1-j) s_(64j+l)
// Each lane runs J Horner steps with M^64 (columns uniform: scalar loads),
// applies its own M^(63-l) (columns [i][l]: coalesced), and the wave
// XOR-reduces.  A serial chain (one thread per span) was nseg steps: 2048 for
// a 64 MiB span, 64x more than J.
// ---------------------------------------------------------------------------

template <bool kDesc, bool kVerify>
__global__ __launch_bounds__(256) void crc32c_combine_kernel(SpanBatch a, SplitWs ws) {
  if (ws.counters->overflow != 0u) return;
  const uint32_t nlong = min(ws.counters->nlong, ws.cap_long);
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t nw = gridDim.x * (blockDim.x >> 6);
  for (uint32_t li = rfl(blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)); li < nlong; li += nw) {
    const uint64_t span = ws.long_span[li];
    const uint64_t first = ws.long_first[li];
    const uint32_t nseg = ws.long_nseg[li];
    const uint32_t J = (nseg + 63u) >> 6;
    const int32_t pad0 = (int32_t)(J * 64u - nseg);
    uint32_t r = 0;
    for (uint32_t j = 0; j < J; ++j) {
      const int32_t k = (int32_t)(j * 64u + lane) - pad0;
      const uint32_t sk = k >= 0 ? ws.seg_out[first + (uint32_t)k] ^ kConditioning : 0u;
      r = gf2_apply(a.tabs->shift_seg64, r) ^ sk;
    }
    uint32_t y = 0;
#pragma unroll
    for (int i = 0; i < 32; ++i) y ^= a.tabs->lane_seg[i][lane] & (0u - ((r >> i) & 1u));
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) y ^= __shfl_xor(y, m);
    if (lane != 0) continue;
    const uint32_t crc = y ^ kConditioning;
    const uint32_t res = (a.flags & kFlagMask) ? mask_crc(crc) : crc;
    if (a.out != nullptr) a.out[span] = res;
    const uint64_t q = a.idx != nullptr ? a.idx[span] : span;  // the caller's span
    const uint64_t off = kDesc ? a.off[q] : q * a.stride;
    const uint32_t len = kDesc ? a.len[q] : a.len_c;
    const bool hdr = (a.flags & kFlagLogHeader) != 0;
    const uint8_t* t = hdr ? a.base + off - kLogCrcBack : a.base + off + len;
    if (a.flags & kFlagWriteTrailer) store_le32(t, res);
    if (kVerify && a.mismatch != nullptr) {
      const uint32_t stored = (uint32_t)t[0] | ((uint32_t)t[1] << 8) | ((uint32_t)t[2] << 16) |
                              ((uint32_t)t[3] << 24);
      a.mismatch[span] = crc != unmask_crc(stored) ? 1 : 0;
    }
  }
}

// ---------------------------------------------------------------------------
// Short records, one per lane (crc32c_lane_kernel).  Log records (~1 KB) are
// too short for a wave-wide fold: the span kernel spends a realignment, a
// reduction and ~190 scalar instructions on each (round 2's "quad" kernel,
// four records per wave, still a quarter of that plus masked rounds).  Here lane i of a wave runs the
// reference's own serial recurrence over record i of a run of 64:
// r <- shift_4(r ^ word), one word per step, four conflict-free LDS lookups
// in the slicing tables slice4[k][b] = shift_4(b << 8k) (the same LDS image
// and v_perm addresses as the stride tables) -- the same lookups per byte as
// the wave-wide fold, with no realignment, no cross-lane reduction and no
// per-record scalar work.  A record is h <= 3 head bytes up to 4-B
// alignment, n4 body words, then tb <= 3 tail bytes.  The body is read in
// whole 128-B lines (eight 16-B loads per lane and task, line-aligned): a lane
// fetches each line of its record once, in one task.  (Loads that followed
// the record's own alignment straddled two lines per task and fetched
// 1.86 x the record bytes from HBM -- PMC FETCH_SIZE -- the lines refetched
// by the next task after L2 had evicted them.)  Words of the first and last
// lines outside the body are masked; a line holding a byte of the record
// lies in a mapped page, so reading all of it is safe.  The head bytes come
// from the aligned dword holding the record's first byte, the tail bytes are
// the top bytes of the dword ending the record; both go through byte steps
// (shift_1(y) = y >> 8 ^ slice4[3][y & 255]).
//
// A task is one 128-B line of every lane's record, issued one task ahead into
// a two-slot ring and retired by counted vmcnt waits.  Task 0 (where bodies
// start) and the lines where some lane's record ends fold under per-word
// masks; the other lines ("clean": for each lane all body words or past its
// record) fold unmasked, with one per-lane select.  (The bound used to be the
// run's shortest record: a log split at a 32 KiB block boundary leaves a
// short fragment in most runs of 64 records, and with it every later task
// masked.)  A lane past its record re-reads its last line.  The fold is not
// what bounds the kernel: clean lines XORed instead of folded (a
// measurement-only variant) ran no faster, nor did them folded as two or four
// independent chains per lane (profiles/r05/r05q_variants_lane_chains.json).
//
// Load order inside an issue: the next run's descriptors (first task of a
// run), the edge dwords (first / last task), then the eight body loads, so
// the body loads of the other slot are always the youngest eight: after a
// vmcnt(8) wait every descriptor and edge load issued so far has landed.
// ---------------------------------------------------------------------------
// Lane kernel workgroup: one group per CU either way
// (the tables take 128 KiB of LDS).  8 waves per CU read 11.7 % faster than 16
// and 4 % faster than 12 (WAL verify; profiles/r02s3n, r02s3o): each lane's
// line is read by eight 16-B loads, and fewer waves keep fewer lines in flight
// in the CU's vector L1 between them; 4 waves hide too little latency (-27 %).
constexpr uint32_t kLaneThreads = 512;

// One 128-B line (lane kernel body): eight 16-B loads at immediate offsets.
template <int J = 0>
__device__ __forceinline__ void asm_load_line(u32x4 (&w)[8], uint64_t addr) {
  if constexpr (J < 8) {
    asm volatile("global_load_dwordx4 %0, %1, off offset:%2" : "=v"(w[J]) : "v"(addr), "n"(16 * J));
    asm_load_line<J + 1>(w, addr);
  }
}
__device__ __forceinline__ uint32_t asm_load_u32(uint64_t addr) {
  uint32_t r;
  asm volatile("global_load_dword %0, %1, off" : "=v"(r) : "v"(addr));
  return r;
}
__device__ __forceinline__ uint64_t asm_load_u64(uint64_t addr) {
  uint64_t r;
  asm volatile("global_load_dwordx2 %0, %1, off" : "=v"(r) : "v"(addr));
  return r;
}

// Wait for a slot's loads (w: body line, hd: head dword, ed: the dword ending
// the record, sc: stored crc) with the other slot's eight body loads in
// flight; the slot's registers and the prefetched descriptors are in/out
// operands.
__device__ __forceinline__ void wait_lane(u32x4 (&w)[8], uint32_t& hd, uint32_t& ed, uint32_t& sc, uint64_t& noff,
                                          uint32_t& nlen, uint32_t& ninit) {
  asm volatile("s_waitcnt vmcnt(8)"
               : "+v"(w[0]), "+v"(w[1]), "+v"(w[2]), "+v"(w[3]), "+v"(w[4]), "+v"(w[5]), "+v"(w[6]),
                 "+v"(w[7]), "+v"(hd), "+v"(ed), "+v"(sc), "+v"(noff), "+v"(nlen), "+v"(ninit)
               :
               : "memory");
}

// Wave-uniform task: run of records [rb, rb + 64), its 128-B task k of K;
// bit k of pm: some lane's record ends inside line k (a masked task); nrb:
// the wave's next owned run.
struct LaneTask {
  uint32_t rb, k, pm, K, nrb;
};

template <int kOp>  // 0: max, 1: min, 2: or
__device__ __forceinline__ uint32_t wave_reduce(uint32_t v) {
  auto f = [](uint32_t x, uint32_t y) { return kOp == 0 ? (x > y ? x : y) : kOp == 1 ? (x < y ? x : y) : (x | y); };
  v = f(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0xB1, 0xF, 0xF, false));  // quad_perm 1,0,3,2
  v = f(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x4E, 0xF, 0xF, false));  // quad_perm 2,3,0,1
  v = f(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x141, 0xF, 0xF, false)); // row_half_mirror
  v = f(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x140, 0xF, 0xF, false)); // row_mirror
  return f(f(readlane(v, 0), readlane(v, 16)), f(readlane(v, 32), readlane(v, 48)));
}

// Word idx (0..31, per lane) of a line in this lane's registers: a five-level
// select tree (31 v_cndmask).
__device__ __forceinline__ uint32_t pick_word(const u32x4 (&w)[8], uint32_t idx) {
  uint32_t v[16];
  const bool b0 = (idx & 1u) != 0u;
#pragma unroll
  for (int i = 0; i < 16; ++i) v[i] = b0 ? w[(2 * i + 1) >> 2][(2 * i + 1) & 3] : w[(2 * i) >> 2][(2 * i) & 3];
#pragma unroll
  for (int l = 1; l < 5; ++l) {
    const bool b = ((idx >> l) & 1u) != 0u;
#pragma unroll
    for (int i = 0; i < (16 >> l); ++i) v[i] = b ? v[2 * i + 1] : v[2 * i];
  }
  return v[0];
}

template <bool kVerify>
__global__ __launch_bounds__(kLaneThreads) void crc32c_lane_kernel(SpanBatch a) {
  const uint32_t n = (uint32_t)a.n;  // host cuts batches at kMaxGenericSpans (2^30)
  __shared__ uint32_t lds[kTabWords];
  const uint32_t tid = threadIdx.x;
  load_stride_image<kLaneThreads>(lds, &a.tabs->slice4[0][0], tid);
  const uint32_t lane = tid & 63u;
  __syncthreads();
  const StrideLanes tab = stride_lanes(lane);
  const uint32_t wave = rfl(blockIdx.x * (kLaneThreads / 64u) + (tid >> 6));
  const uint32_t nwaves = gridDim.x * (kLaneThreads / 64u);
  // Every run of the batch, in turn: one whose spans the kernel owns none of
  // costs one task of loads from the zero region.  (Runs used to be skipped
  // by a flag from crc32c_long_list_kernel, which then had to finish first;
  // it now runs next to this kernel.)  Runs [0, Rs) are dealt round-robin;
  // the last kLaneTailRounds rounds are claimed from a per-call counter as
  // waves run out (the atomic's return drains the wave's ring once per
  // claimed run: the compiler waits for it with vmcnt(0)).
  const uint32_t R = (n + 63u) >> 6;
  const uint32_t tailr = a.claim != nullptr && R > (kLaneTailRounds + 2u) * nwaves ? kLaneTailRounds * nwaves : 0u;
  const uint32_t Rs = R - tailr;
  auto run_after = [&](uint32_t rb) -> uint32_t {  // the wave's next run after run rb (n: none)
    uint32_t nx = (rb >> 6) + nwaves;
    if (tailr != 0u && nx >= Rs) {
      uint32_t got = 0;
      if (lane == 0u) got = __hip_atomic_fetch_add(a.claim, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      nx = Rs + rfl(got);
    }
    return nx < R ? nx << 6 : n;
  };
  const uint32_t first = wave * 64u;
  if (first >= n) return;
  // Priority rotation by SIMD age rank (two waves per SIMD here), as in
  // crc32c_pair_kernel: one step per run (WAL verify +1.1-1.3 %, seal
  // +0.8-0.9 %; profiles/r05/r05f_variants_rotation.json, r05g_variants_lane_seal.json).
  uint32_t prio = rfl(tid >> 6) >> 2;
  if (prio == 0u) __builtin_amdgcn_s_setprio(0);
  else __builtin_amdgcn_s_setprio(1);
  const bool hdr = (a.flags & kFlagLogHeader) != 0;
  const bool has_init = a.init != nullptr;
  // lanes without a record of the kernel's read a 2 KiB zero region (per wave)
  const uint64_t zero = reinterpret_cast<uint64_t>(&a.tabs->zero[0]) + 2048u * (wave & 31u);
  const uint64_t base = reinterpret_cast<uint64_t>(a.base);

  // descriptors of run rb, lane's record (clamped to the last record)
  uint64_t noff = 0;
  uint32_t nlen = 0, ninit = 0;
  auto fetch_desc = [&](uint32_t rb) {
    const uint32_t i = rb < n && rb + lane < n ? rb + lane : n - 1u;
    noff = asm_load_u64(reinterpret_cast<uint64_t>(a.off + i));
    nlen = asm_load_u32(reinterpret_cast<uint64_t>(a.len + i));
    if (has_init) ninit = asm_load_u32(reinterpret_cast<uint64_t>(a.init + i));
  };
  fetch_desc(first);
  asm volatile("s_waitcnt vmcnt(0)" : "+v"(noff), "+v"(nlen), "+v"(ninit) : : "memory");

  // issue state of the run being issued: record address, the line holding
  // the body's first word, the lane's last task (line), n4 | q0 << 16 | h << 21
  // | tb << 23 | owned << 25 (q0: the body's first word in that line), init
  uint64_t vp = zero, vl = zero;
  uint32_t vlen = 0, vkend = 0, vmeta = 0, vinit = 0;
  // Per slot: the body line, head dword (first task of a run), the dword
  // ending the record (last task), stored crc (verify), and the fold's
  // per-lane copies (record address, meta, init).  Compile-time slot indices
  // only (the loop is unrolled over the slots).
  u32x4 W[2][8];
  uint32_t HD[2] = {0u, 0u}, ED[2] = {0u, 0u}, SC[2] = {0u, 0u}, META[2], INIT[2];
  uint64_t VP[2];
  auto issue = [&](LaneTask& t, int sl) {
    if (t.rb < n && t.k == 0) {
      const uint32_t rec = t.rb + lane;
      const bool owned = rec < n && lane_owns(nlen);
      vp = owned ? base + noff : zero;
      vlen = owned ? nlen : 0u;
      const uint32_t h = owned ? (0u - (uint32_t)vp) & 3u : 0u;  // head bytes up to 4-B alignment
      const uint32_t n4 = owned ? (vlen - h) >> 2 : 0u;          // >= 1
      const uint32_t tb = owned ? (vlen - h) & 3u : 0u;
      const uint64_t vb = vp + h;
      vl = vb & ~127ull;
      const uint32_t q0 = owned ? (uint32_t)(vb & 127u) >> 2 : 0u;
      const uint32_t qe = q0 + n4;  // one past the body's last word, in words from vl
      vkend = owned ? (qe + 31u) >> 5 : 1u;
      vinit = ninit;
      vmeta = n4 | (q0 << 16) | (h << 21) | (tb << 23) | ((owned ? 1u : 0u) << 25);
      t.K = wave_reduce<0>(vkend);
      // the lines holding a record's last body word short of the line's end
      // (a record ending exactly at a line's end has no such line)
      t.pm = wave_reduce<2>(owned && (qe & 31u) != 0u ? 1u << (qe >> 5) : 0u);
      t.nrb = run_after(t.rb);
      prio ^= 1u;
      if (prio == 0u) __builtin_amdgcn_s_setprio(0);
      else __builtin_amdgcn_s_setprio(1);
    }
    // Side loads: the next run's descriptors with a run's first task, the
    // head dword with it, the end dword and the stored crc with its last.
    // The verify kernel issues them only there (WAL verify +6.8 % against
    // issuing them with every task, from a zero region when unused:
    // profiles/r02s3w_*); the sealing kernel issues them with every task
    // (2.5 % faster that way in the same A/B; neutral in round 5,
    // profiles/r05/r05w_variants_lane_merged_side_load.json).  Loads written under branches:
    // at 16 waves hipcc, short of VGPRs, copied such registers at the merge
    // before their wait; the CFG audit run by build() fails on any such touch,
    // and this build has none.
    //
    // A lane reads a side dword from memory only when the line it is in is
    // not the one the task loads (see fold: the head dword precedes a body
    // that starts a line, a log header's crc lies in the line before, the
    // tail bytes follow a body that ends a line); every other lane's address
    // is the wave's zero region (WAL verify +2.1 %,
    // profiles/r05/r05s_variants_lane_side_dwords.json).
    constexpr bool kSideAlways = !kVerify;
    const bool live = t.rb < n;
    const bool owned = live && ((vmeta >> 25) & 1u);
    const bool lastk = t.k + 1u == t.K;
    const uint32_t vq0 = (vmeta >> 16) & 31u, vh = (vmeta >> 21) & 3u, vtb = (vmeta >> 23) & 3u;
    const uint32_t vqe = vq0 + (vmeta & 0xFFFFu);
    if (kSideAlways || t.k == 0) fetch_desc(t.nrb);
    VP[sl] = vp;
    META[sl] = live ? vmeta : 0u;
    INIT[sl] = vinit;
    if (kSideAlways || t.k == 0) {
      HD[sl] = asm_load_u32(owned && t.k == 0 && vq0 == 0u && vh != 0u ? vp & ~3ull : zero);
      if (kVerify && hdr) SC[sl] = asm_load_u32(owned && t.k == 0 && 4u * vq0 < vh + kLogCrcBack ? vp - kLogCrcBack : zero);
    }
    if (kSideAlways || lastk) {
      ED[sl] = asm_load_u32(owned && lastk && vtb != 0u && (vqe & 31u) == 0u ? vp + vlen - 4u : zero);
      if (kVerify && !hdr) SC[sl] = asm_load_u32(owned && lastk ? vp + vlen : zero);
    }
    // line min(k, kend - 1) of the lane's record (a finished lane re-reads its last)
    const uint32_t kl = live ? (t.k < vkend ? t.k : vkend - 1u) : 0u;
    asm_load_line(W[sl], (live ? vl : zero) + 128u * kl);
  };
  auto next = [&](const LaneTask& t) -> LaneTask {
    LaneTask u = t;
    if (t.rb >= n) return u;
    if (t.k + 1u < t.K) {
      u.k = t.k + 1u;
    } else {
      u.rb = t.nrb;
      u.k = 0;
      u.K = 1;
      u.pm = 0;
    }
    return u;
  };

  uint32_t acc = 0;
  uint32_t hsc = 0;  // a log record's stored crc (its header's), taken at task 0
  auto fold = [&](const LaneTask& t, int sl) {
    const u32x4(&w)[8] = W[sl];
    const uint32_t meta = META[sl];
    const uint32_t n4 = meta & 0xFFFFu, q0 = (meta >> 16) & 31u;
    // byte step: shift_1(r ^ b) = (r ^ b) >> 8 ^ slice4[3][(r ^ b) & 255]
    auto byte_step = [&](uint32_t r, uint32_t bt) -> uint32_t {
      const uint32_t y = r ^ bt;
      return lds_word(lds, __builtin_amdgcn_perm(y, tab.L[3], 0x0C020400u)) ^ (y >> 8);
    };
    uint32_t x = acc;
    if (t.k == 0) {
      // the head bytes, then the body from word q0 of the line: the register
      // enters with body word 0
      const uint32_t h = (meta >> 21) & 3u;
      // the dword before the body (word q0 - 1 of this line, or loaded)
      const uint32_t hd = q0 != 0u ? pick_word(w, q0 - 1u) : HD[sl];
      const uint32_t hb = hd >> (8u * ((4u - h) & 3u));  // the record's first bytes
      if (kVerify && hdr) {
        // the header's crc: bytes [o, o + 4) of this line, o = 4 q0 - h - 6
        // (or loaded when o < 0)
        const uint32_t o = 4u * q0 - h - kLogCrcBack, j = o >> 2;
        const uint32_t lo = pick_word(w, j & 31u), hi = pick_word(w, j + 1u < 32u ? j + 1u : 31u);
        hsc = 4u * q0 < h + kLogCrcBack ? SC[sl] : __builtin_amdgcn_alignbyte(hi, lo, o & 3u);
      }
      uint32_t r = INIT[sl] ^ kConditioning;
#pragma unroll
      for (uint32_t i = 0; i < 3; ++i) {
        const uint32_t v = byte_step(r, (hb >> (8u * i)) & 255u);
        r = i < h ? v : r;
      }
#pragma unroll
      for (int i = 0; i < 32; ++i) {
        const uint32_t rel = (uint32_t)i - q0;  // body word index (huge before the body)
        const uint32_t y = rel == 0u ? r ^ w[i >> 2][i & 3] : step256(lds, tab, x, w[i >> 2][i & 3]);
        x = rel < n4 ? y : x;
      }
    } else if (((t.pm >> t.k) & 1u) == 0u) {
      // No record ends inside this line: every lane's line is all body words
      // (32k + 32 <= q0 + n4), or lies past the lane's record, which keeps
      // its register.
      uint32_t y = x;
#pragma unroll
      for (int i = 0; i < 32; ++i) y = step256(lds, tab, y, w[i >> 2][i & 3]);
      x = 32u * t.k + 32u <= q0 + n4 ? y : x;
    } else {
      const uint32_t rel0 = 32u * t.k - q0;  // body word index of the line's word 0
#pragma unroll
      for (int i = 0; i < 32; ++i) {
        const uint32_t y = step256(lds, tab, x, w[i >> 2][i & 3]);
        x = rel0 + (uint32_t)i < n4 ? y : x;
      }
    }
    acc = x;
    if (t.k + 1u == t.K) {
      uint32_t r = step256(lds, tab, x, 0u);  // shift_4 after the last body word
      const uint32_t tb = (meta >> 23) & 3u;
      // the record's last tb bytes: the low bytes of word q0 + n4 of this
      // line (the lane's last), or the top bytes of the loaded end dword when
      // the body ends the line
      const uint32_t qe = q0 + n4;
      const uint32_t fw = (qe & 31u) != 0u ? pick_word(w, qe & 31u) : ED[sl] >> (8u * ((4u - tb) & 3u));
      const uint32_t fb = tb ? fw & ((1u << (8u * tb)) - 1u) : 0u;
#pragma unroll
      for (uint32_t i = 0; i < 3; ++i) {
        const uint32_t v = byte_step(r, (fb >> (8u * i)) & 255u);
        r = i < tb ? v : r;
      }
      const uint32_t crc = r ^ kConditioning;
      const uint32_t v = (a.flags & kFlagMask) ? mask_crc(crc) : crc;
      if ((meta >> 25) & 1u) {
        const uint32_t rec = t.rb + lane;
        const uint32_t len = ((meta >> 21) & 3u) + 4u * n4 + tb;
        // one (byte-unaligned) dword store instead of four byte stores (WAL seal
        // +0.6 %, within noise: profiles/r02s3k_variants_seal_dword_store.json)
        if ((a.flags & kFlagWriteTrailer)) {
          const uint64_t ta = hdr ? VP[sl] - kLogCrcBack : VP[sl] + len;
          asm volatile("global_store_dword %0, %1, off" : : "v"(ta), "v"(v) : "memory");
        }
        if (a.out != nullptr) __builtin_nontemporal_store(v, a.out + rec);
        if (kVerify && a.mismatch != nullptr)
          __builtin_nontemporal_store((uint8_t)(crc != unmask_crc(hdr ? hsc : SC[sl]) ? 1u : 0u), a.mismatch + rec);
      }
    }
  };

  LaneTask tk[2];
  tk[0] = LaneTask{first, 0u, 0u, 1u, n};  // (pm of a first task: unused)
  issue(tk[0], 0);
  // the next run's descriptors (issued before the eight body loads) may be
  // read by the second issue: retire everything but those eight loads
  asm volatile("s_waitcnt vmcnt(8)" : "+v"(noff), "+v"(nlen), "+v"(ninit), "+v"(HD[0]), "+v"(ED[0]), "+v"(SC[0]) : : "memory");
  tk[1] = next(tk[0]);
  issue(tk[1], 1);
  for (;;) {
#pragma unroll
    for (int sl = 0; sl < 2; ++sl) {
      wait_lane(W[sl], HD[sl], ED[sl], SC[sl], noff, nlen, ninit);
      if (tk[sl].rb < n) fold(tk[sl], sl);
      if (tk[sl ^ 1].rb >= n) goto drained;
      tk[sl] = next(tk[sl ^ 1]);
      issue(tk[sl], sl);
    }
  }
drained:
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
  for (int sl = 0; sl < 2; ++sl) {
#pragma unroll
    for (int j = 0; j < 8; ++j) asm volatile("" : "+v"(W[sl][j]));
    asm volatile("" : "+v"(HD[sl]), "+v"(ED[sl]), "+v"(SC[sl]));
  }
  asm volatile("" : "+v"(noff), "+v"(nlen), "+v"(ninit));
}

// The spans the lane kernel leaves to the generic path (lane_owns() false),
// listed run by run (a wave's 64 consecutive spans stay together and in
// order); ws.counters->nlist is the count.  One atomic per block of 16 runs
// (one per run serialized on the counter: 790 us for 64 Ki runs).  Launched
// on a side stream next to the lane kernel (it reads ~12 B per span, ~60 us
// of a 17 M-record WAL batch that used to sit in front of the lane kernel:
// WAL verify +2.7 %, seal +1.4 %, profiles/r05/r05v_variants_lane_side_list.json).
__global__ __launch_bounds__(kListThreads) void crc32c_long_list_kernel(SpanBatch a, SplitWs ws) {
  const uint64_t n = a.n;
  const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
  constexpr uint32_t kWaves = kListThreads / 64;
  __shared__ uint32_t cnt[kWaves];
  __shared__ unsigned long long base;
  const uint64_t step = (uint64_t)gridDim.x * kListThreads;
  for (uint64_t b0 = (uint64_t)blockIdx.x * kListThreads; b0 < n; b0 += step) {
    const uint64_t i = b0 + 64u * wv + lane;
    const bool mine = i < n && lane_owns(a.len[i < n ? i : n - 1u]);
    const bool lng = i < n && !mine;
    const uint64_t m = __ballot(lng);
    if (lane == 0) cnt[wv] = (uint32_t)__popcll(m);
    __syncthreads();
    if (threadIdx.x == 0) {
      uint32_t tot = 0;
      for (uint32_t k = 0; k < kWaves; ++k) tot += cnt[k];
      base = tot ? atomicAdd(&ws.counters->nlist, (unsigned long long)tot) : 0ull;
    }
    __syncthreads();
    uint64_t pos = base;
    for (uint32_t k = 0; k < wv; ++k) pos += cnt[k];
    if (lng) ws.list[pos + (uint64_t)__popcll(m & ((1ull << lane) - 1ull))] = (uint32_t)i;
    __syncthreads();  // cnt/base are rewritten by the next iteration
  }
}

// Generic-path results of the listed spans, back to the caller's arrays.
__global__ __launch_bounds__(256) void crc32c_scatter_kernel(SpanBatch a, SplitWs ws, const uint32_t* qout,
                                                             const uint8_t* qmm) {
  const uint64_t nl = ws.counters->nlist;
  const uint64_t step = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nl; i += step) {
    const uint32_t q = ws.list[i];
    if (a.out != nullptr) a.out[q] = qout[i];
    if (a.mismatch != nullptr) a.mismatch[q] = qmm[i];
  }
}

// ---------------------------------------------------------------------------
// Trailer pass of a sealing planner-path batch: span i's result (out[i],
// already Mask()ed with MASK) as 4 LE bytes right after it, or with
// LOG_HEADER 6 bytes before it (TableBuilder::WriteRawBlock,
// table/table_builder.cc:192-197; log::Writer, db/log_writer.cc:90-97).  The
// span and pair kernels could store each run's trailers themselves, but
// scattered 4-byte writes spread through the read stream cost the pair
// kernel 17 % on bulk SST seals (4954 against 5966 GB/s without the stores,
// whatever their cache policy: profiles/r05/r05b_variants_pair_seal.json);
// the one-launch kernel, whose trailers go out together at the end of each
// wave's run, seals almost free.  So the trailers of a bulk batch go out
// here, in one burst after the reads: one thread per span, descriptors and
// results read coalesced, non-temporal stores.  (Plain stores, four spans per
// thread, took this pass from 117 to 77 us on a config-5 call but left 2.4 M
// dirty partial lines behind, whose write-back then ran under the next call:
// six config-5 seals back to back took 2.022 ms each against 1.682 ms,
// profiles/r06/r06n_variants.json, r06l config5_one_process.)
// ---------------------------------------------------------------------------
// With a.overflow set, spans longer than a.skip_above are left to the
// combine kernel (their results are not in yet), unless the segment
// workspace overflowed and the span pass folded them.
template <bool kDesc>
__global__ __launch_bounds__(256) void crc32c_trailer_kernel(SpanBatch a, const uint32_t* res) {
  const bool hdr = (a.flags & kFlagLogHeader) != 0;
  const uint32_t skip_above = a.overflow != nullptr && *a.overflow == 0u ? a.skip_above : 0xFFFFFFFFu;
  const uint64_t step = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < a.n; i += step) {
    const uint64_t off = kDesc ? a.off[i] : i * a.stride;
    const uint32_t len = kDesc ? a.len[i] : a.len_c;
    if (len > skip_above) continue;
    const uint8_t* t = hdr ? a.base + off - kLogCrcBack : a.base + off + len;
    store_le32(t, res[i]);
  }
}

// ---------------------------------------------------------------------------
// Host-side launchers (called from crc32c_capi.hip through crc32c_device.h).
// `stop`, where a launcher takes one: an event completed by the kernel's own
// end (hipExtLaunchKernel's stop event) instead of a marker packet after it --
// the planner path's fork onto its side stream, its join and its done event
// (a marker between two kernels cost ~2.7 us of the stream's time,
// profiles/r06/r06f_percall_floor/floor.json direct_ts_plain).
// ---------------------------------------------------------------------------
template <typename... P, typename... A>
hipError_t launch_k(void (*k)(P...), dim3 grid, dim3 block, hipStream_t s, hipEvent_t stop, A... args) {
  if (stop != nullptr) hipExtLaunchKernelGGL(k, grid, block, 0, s, nullptr, stop, 0u, args...);
  else hipLaunchKernelGGL(k, grid, block, 0, s, args...);
  return hipGetLastError();
}

hipError_t launch_span(const SpanBatch& a, bool verify, int grid, hipStream_t s, hipEvent_t stop) {
  // Log records (LOG_HEADER) are short: the variant that skips padding rounds.
  const bool skip = (a.flags & kFlagLogHeader) != 0 && a.role == kRoleSpans;
  if (verify) {
    if (a.pair_kernel && !skip) crc32c_pair_kernel<true><<<grid, kThreads, 0, s>>>(a);
    if (skip) return launch_k(crc32c_span_kernel<true, true>, dim3(grid), dim3(kThreads), s, stop, a);
    return launch_k(crc32c_span_kernel<true, false>, dim3(grid), dim3(kThreads), s, stop, a);
  }
  if (a.pair_kernel && !skip) crc32c_pair_kernel<false><<<grid, kThreads, 0, s>>>(a);
  if (skip) return launch_k(crc32c_span_kernel<false, true>, dim3(grid), dim3(kThreads), s, stop, a);
  return launch_k(crc32c_span_kernel<false, false>, dim3(grid), dim3(kThreads), s, stop, a);
}

hipError_t launch_fixed(const SpanBatch& a, bool verify, int grid, hipStream_t s) {
  // rounds: ceil(len / 256), or ceil((len + 4) / 256) when the trailer rides along
  const int rounds = (int)((a.len_c + (verify ? 4u : 0u) + 255u) / 256u);  // 1..16
  switch (rounds) {
#define PRISMDB_CASE(K)                                                  \
  case K:                                                                \
    if (verify) crc32c_fixed_kernel<K, true><<<grid, kThreads, 0, s>>>(a); \
    else crc32c_fixed_kernel<K, false><<<grid, kThreads, 0, s>>>(a);       \
    break;
    PRISMDB_CASE(1) PRISMDB_CASE(2) PRISMDB_CASE(3) PRISMDB_CASE(4)
    PRISMDB_CASE(5) PRISMDB_CASE(6) PRISMDB_CASE(7) PRISMDB_CASE(8)
    PRISMDB_CASE(9) PRISMDB_CASE(10) PRISMDB_CASE(11) PRISMDB_CASE(12)
    PRISMDB_CASE(13) PRISMDB_CASE(14) PRISMDB_CASE(15) PRISMDB_CASE(16)
#undef PRISMDB_CASE
    default:
      return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

hipError_t launch_plan(const SpanBatch& a, bool desc, const SplitWs& ws, hipStream_t s, hipEvent_t stop) {
  if (desc) return launch_k(crc32c_plan_kernel<true>, dim3(ws.nblocks), dim3(kPlanThreads), s, stop, a, ws);
  return launch_k(crc32c_plan_kernel<false>, dim3(ws.nblocks), dim3(kPlanThreads), s, stop, a, ws);
}

hipError_t launch_slices(const SpanBatch& a, const SplitWs& ws, hipStream_t s, hipEvent_t stop) {
  crc32c_slice_scan_kernel<<<1, 1024, 0, s>>>(a, ws);
  return launch_k(crc32c_slice_mark_kernel, dim3(ws.nblocks), dim3(kPlanThreads), s, stop, a, ws);
}

hipError_t launch_long_list(const SpanBatch& a, const SplitWs& ws, hipStream_t s) {
  const uint64_t lb = (a.n + kListThreads - 1) / kListThreads;
  // one block per 1024 spans up to 16 Mi spans (a grid of 1024 looped and
  // took 49 us over a 4 GiB WAL batch; the atomics are per block-iteration
  // either way)
  const int lgrid = (int)(lb < 16384u ? lb : 16384u);
  crc32c_long_list_kernel<<<lgrid, kListThreads, 0, s>>>(a, ws);
  return hipGetLastError();
}

hipError_t launch_lane(const SpanBatch& a, bool verify, int grid, hipStream_t s) {
  if (verify) crc32c_lane_kernel<true><<<grid, kLaneThreads, 0, s>>>(a);
  else crc32c_lane_kernel<false><<<grid, kLaneThreads, 0, s>>>(a);
  return hipGetLastError();
}

hipError_t launch_scatter(const SpanBatch& a, const SplitWs& ws, const uint32_t* qout, const uint8_t* qmm,
                          hipStream_t s, hipEvent_t stop) {
  return launch_k(crc32c_scatter_kernel, dim3(256), dim3(256), s, stop, a, ws, qout, qmm);
}

hipError_t launch_trailers(const SpanBatch& a, bool desc, const uint32_t* res, hipStream_t s, hipEvent_t stop) {
  const uint64_t blocks = (a.n + 255u) / 256u;
  const int grid = (int)(blocks < 16384u ? blocks : 16384u);
  if (desc) return launch_k(crc32c_trailer_kernel<true>, dim3(grid), dim3(256), s, stop, a, res);
  return launch_k(crc32c_trailer_kernel<false>, dim3(grid), dim3(256), s, stop, a, res);
}

hipError_t launch_combine(const SpanBatch& a, bool desc, bool verify, const SplitWs& ws, hipStream_t s,
                          hipEvent_t stop) {
  const dim3 grid(256), block(256);  // 1024 waves, one long span each at a time
  if (desc) {
    if (verify) return launch_k(crc32c_combine_kernel<true, true>, grid, block, s, stop, a, ws);
    return launch_k(crc32c_combine_kernel<true, false>, grid, block, s, stop, a, ws);
  }
  if (verify) return launch_k(crc32c_combine_kernel<false, true>, grid, block, s, stop, a, ws);
  return launch_k(crc32c_combine_kernel<false, false>, grid, block, s, stop, a, ws);
}

}  // namespace dev
}  // namespace prismdb
