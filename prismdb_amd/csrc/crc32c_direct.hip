// crc32c_direct.hip -- descriptor batches in ONE launch (n <= kDirectMaxSpans).
//
// PrismDB checksums one SST file at a time: TableBuilder::Finish seals ~16.8 K
// data blocks and an index block (table/table_builder.cc:185-261, called from
// DoCompactionWork, db/db_impl.cc:2220-2278), and a compaction's input files
// are verified block by block (ReadBlock, table/format.cc:91-102).  The
// planner path (crc32c_kernels.hip: memset, plan, slice scan and mark, span
// pass, segment pass, combine) spends 5-7 launches of 4-6 us each on ~10 us of
// data at that size.  This kernel does a file in one launch, 12 waves per CU
// (one 768-thread group: the tables take all of LDS):
//
//   static run   wave w < K owns q or q + 1 consecutive spans (<= 64; lane j
//                holds span j's descriptor).  Its spans of up to kRingChunks
//                (32) chunks of 4 KiB -- all the data blocks of an SST -- go
//                through an inline-asm ring of two single-task slots, one
//                task sequence (run positions in order, a span's chunks one
//                after another, the register carried between them): a wave
//                waits for its older task and folds it as soon as it lands
//                (round 4; two slots of three streams before: a file's whole
//                read went out at once and the folds bunched at its end).
//                Counted vmcnt waits, one coalesced store of the run's
//                results.
//   long spans   (more than kRingChunks chunks) are found by their run's wave
//                first and cut into T tickets of g = 2^lg chunks (T <= 64, or
//                up to 4096 when the batch has fewer spans than waves; lg in
//                kTicketLgMin..14; ticket 0 takes the remainder).  The wave
//                pushes all its tickets with ONE 64-bit atomic on
//                word = supply << 32 | claimed and writes the ticket map
//                (span | ticket index, span address, len, init: four 8-B
//                words, each tagged with the call's tag, no fence).
//   workers      the last nwaves / 32 waves have no run (at most 256 of them:
//                every worker reads `word`, and same-address reads serialize
//                in one L2 channel, ~2.5 ns each).  A worker polls `word` for
//                up to ~2 us, claims tickets one at a time while any are
//                visible, and leaves.  A long span's chunks thus go out with
//                the first loads instead of on the kernel's tail.
//   late claims  a wave that pushed tickets claims, after its own run, one at
//                a time until none is left, so every pushed ticket is claimed
//                by someone.  Other static waves leave (3072 reads of `word`
//                at the end cost ~8 us) unless a push of >= 1 MiB of ticket
//                work set the help flag (32 tagged replicas); groups a small
//                batch leaves idle wait ~3 us for that flag too.

// A claim is one atomicAdd of 1 on the claimed half of `word`: ticket C below
// the supply S is the claimer's.  A claim at C >= S ("orphan": two workers
// raced for the last visible ticket) belongs to whoever pushes ticket C: the
// pusher sees claimed > its first ticket and folds those itself.  So no wave
// waits for another wave's progress, except for a ticket-map entry that a
// running wave is writing (its push came before the claim) and a partial
// whose store the counter add overtook.  Those hand-offs are tagged words
// (kTagShift), polled: no release or acquire fence anywhere (a release
// writes back the XCD's L2 and, like an acquire, waits for every load in
// flight -- at the push, the table fill).  A ticket folds
// its chunks into a partial register R_k (ticket 0 from the span's initial
// register, the others from 0) with compiler-scheduled buffer loads, the next
// two chunks' loads in flight during a fold; the wave
// that finishes a span's last ticket (per-span counter) combines
// R = sum_k M^(T-1-k) R_k, M = shift_{4 KiB g}, lane-parallel as
// crc32c_combine_kernel does, feeds the tail bytes and stores the result.
// Calls on a stream (the workspace is per (thread, device, stream)) alternate
// between two claim words: each call starts on a zeroed one and zeroes the
// other for the next call -- no end-of-kernel counter (256 groups' atomics on
// one address serialize in its L2 channel, ~35 ns each).  If the ticket
// workspace is full, the discovering wave folds its long spans whole.
// Test hooks (DirectWs::dbg): bit 0 delays every push by ~100 us, bit 1 makes
// every worker claim once blindly (orphans); stats[] counts adopted tickets,
// whole spans, worker claims and late claims.
#include <hip/hip_ext.h>

#include "crc32c_fold.h"

namespace prismdb {
namespace dev {

namespace {

// ceil(log2(x)) for x >= 1
__device__ __forceinline__ uint32_t ceil_lg(uint32_t x) { return x <= 1u ? 0u : 32u - (uint32_t)__builtin_clz(x - 1u); }
// Chunks per ticket: 2^lg, the smallest power of two that keeps a span at
// <= 2^lt tickets, and at least 2^kTicketLgMin.  2^lt = 64 (one Horner step
// in the combine) unless the batch has far fewer spans than waves: then
// ~2 nwaves / n (floor(log2(2 nwaves)) - ceil(log2(n)), up to 4096), so that
// a few huge spans still give every wave tickets (one 1 GiB span as 64
// tickets of 16 MiB kept 64 waves busy for 4.2 ms).  Tickets were <= 8
// chunks in round 3's first version: a 64 MiB span was 2048 tickets, and
// 127 such spans took 26 ms through 96 ticket workers.  Pusher and claimer
// compute it from the same (nch, n); no division.
constexpr uint32_t kTicketLgMin = 2;
__device__ __forceinline__ uint32_t ticket_lg(uint32_t nch, uint32_t n, uint32_t nwaves) {
  const int32_t l = (int32_t)(31u - (uint32_t)__builtin_clz(2u * nwaves)) - (int32_t)ceil_lg(n);
  const uint32_t lt = l < 6 ? 6u : (l > 12 ? 12u : (uint32_t)l);
  const uint32_t lg = ceil_lg((nch + (1u << lt) - 1u) >> lt);
  return lg < kTicketLgMin ? kTicketLgMin : lg;
}
static_assert(kTicketLgMax >= 14, "2^20 chunks (4 GiB) in 64 tickets");

// Tagged 8-B words (kTagShift): relaxed agent-scope atomics, i.e. sc1
// (write-through) stores and L2-served loads, no fences.
__device__ __forceinline__ void put_tagged(uint64_t* p, uint32_t tag, uint64_t v) {
  __hip_atomic_store(p, v | ((uint64_t)tag << kTagShift), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint64_t get_word(const uint64_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ bool has_tag(uint64_t w, uint32_t tag) { return (uint32_t)(w >> kTagShift) == tag; }

// Exclusive prefix sum of v over the wave; total = the sum.
__device__ __forceinline__ uint32_t wave_excl_sum(uint32_t v, uint32_t lane, uint32_t& total) {
  uint32_t x = v;
#pragma unroll
  for (int dd = 1; dd < 64; dd <<= 1) {
    const uint32_t y = (uint32_t)__shfl_up((int)x, (unsigned)dd, 64);
    x += lane >= (uint32_t)dd ? y : 0u;
  }
  total = readlane(x, 63);
  return x - v;
}

enum : uint32_t { kKindNone = 0, kKindStatic = 1 };

// Wave-uniform span geometry, and the chunks [c, c1) a group folds (a ticket
// of a long span, or all of it).  Chunk k is 4 KiB of body words; chunk 0 is
// right-aligned (pad leading zero words), so only it is short.
struct DTask {
  uint64_t body;  // first 4-B aligned byte of the span
  uint32_t z;     // body bytes (4 W)
  uint32_t f;     // pad | h << 10 | t << 12 | kind << 14 | result lane << 16 (static run)
                  //   | ring chunk << 22 | ring chunks - 1 << 27 (static run: <= kRingChunks)
  uint32_t b;     // span
  uint32_t c;     // first chunk (groups: tickets, whole spans)
  uint32_t c1;    // one past the last chunk
  __device__ uint32_t pad() const { return f & 1023u; }
  __device__ uint32_t h() const { return (f >> 10) & 3u; }
  __device__ uint32_t t() const { return (f >> 12) & 3u; }
  __device__ bool valid() const { return ((f >> 14) & 3u) != kKindNone; }
  __device__ uint32_t slot() const { return (f >> 16) & 63u; }
  __device__ uint32_t len() const { return h() + z + t(); }
  // static run (the ring): the task's chunk, and whether it is the span's last
  __device__ uint32_t rc() const { return (f >> 22) & 31u; }
  __device__ bool rlast() const { return ((f >> 22) & 31u) == (f >> 27); }
};

// Span geometry: body, body bytes, pad | h << 10 | t << 12, chunks.
__device__ __forceinline__ DTask geometry(uint64_t p, uint32_t len) {
  DTask t;
  uint32_t h = (4u - ((uint32_t)p & 3u)) & 3u;
  h = h < len ? h : len;
  const uint32_t W = (len - h) >> 2, tl = (len - h) & 3u;
  const uint32_t nch = W ? (W + 1023u) >> 10 : 1u;
  t.body = p + h;
  t.z = 4u * W;
  t.f = (((nch << 10) - W) & 1023u) | (h << 10) | (tl << 12);
  t.b = 0;
  t.c = 0;
  t.c1 = nch;
  return t;
}

}  // namespace

// 12 waves per CU (one group: the tables take all of LDS), <= 168 VGPRs per lane
// for the ring, the run's descriptors and the combine; 3072 waves keep six
// tasks x 4 KiB in flight each, 72 MiB over the chip: a whole SST file's
// reads are issued at once.
constexpr uint32_t kDirectWaves = kDirectThreads / 64u;
// How long a ticket worker polls `word`, in s_memrealtime ticks (100 MHz):
// 2 us.  Workers are the grid's last waves, which start last: pushes come
// right after the static waves' discovery, mostly before the workers run.
// A push the workers miss is claimed by its pusher after its run.
constexpr uint64_t kWorkerPoll = 200u;
// Spans of up to this many chunks (128 KiB) are folded by their run's wave in
// the static ring, chunk after chunk on one stream; longer ones are cut into
// tickets.  Tickets cost a claim on one shared word (same-address atomics
// serialize in one L2 channel) and a chain of dependent round trips each: a
// batch of 2^17 spans of 16-64 KiB as one-chunk tickets took 222 ms, as ring
// tasks 4.3 ms; 122 K spans of 0-70 000 B took 4.6 ms with 17-chunk spans
// as tickets.
constexpr uint32_t kRingChunks = 32;
static_assert(kRingChunks <= 32, "a ring task's chunk index and count take 5 bits each (DTask::f)");
// A ticket-map entry's span field (24 bits: n <= kDirectMaxSpans) marking a
// ticket nobody folds (the workspace was full: its span is folded whole).
constexpr uint32_t kNullEntry = 0xFFFFFFu;
// A push of at least this many chunks of ticket work (1 MiB) calls every
// static wave to claim tickets after its run (an SST file's index block,
// 119 chunks, stays with the ticket workers).
constexpr uint32_t kHelpChunks = 256;
// How long a wave of an idle group waits for the help flag (s_memrealtime
// ticks, 100 MHz): 3 us.  Pushes come right after the static waves' first
// descriptor loads (~1.5-2.5 us into the kernel).
constexpr uint64_t kHelpPoll = 300u;
// Static-run weights of a group's waves 0-3, 4-7 and 8-11 (one per SIMD each;
// see the run deal in the kernel).  8:7:6 against equal runs: one sealed SST
// file per call 16.4 against 17.5 us, seven files 82.9 against 87.2 us, two
// 26.8 against 28.7 (5:4:3 and 6:5:4 over-correct; profiles/r05/
// r05c_variants_trailer_pass_weights.json, r05d_variants_run_weights.json).
constexpr uint32_t kRunWeight[3] = {8u, 7u, 6u};
static_assert(kDirectWaves == 12u, "the run weights assume 12 waves per group, 3 per SIMD");
static_assert(kDirectMaxSpans < kNullEntry, "span indices fit the entry's 24-bit field");

template <bool kVerify>
__global__ __launch_bounds__(kDirectThreads) void crc32c_direct_kernel(SpanBatch a, DirectWs d) {
  const uint32_t n = (uint32_t)a.n;  // <= kDirectMaxSpans, <= 64 per wave
  const uint32_t tid = threadIdx.x;
  const uint32_t lane = tid & 63u;
  const uint32_t wave = rfl(blockIdx.x * kDirectWaves + (tid >> 6));
  const uint32_t nwaves = gridDim.x * kDirectWaves;
  const bool hdr = (a.flags & kFlagLogHeader) != 0;
  const bool has_init = a.init != nullptr;
  const uint64_t base = reinterpret_cast<uint64_t>(a.base);
  __shared__ uint32_t lds[kLdsWords];

  // ---- the wave's static run: spans [sbase, sbase + m), m <= 64 (q or
  // q + 1 of them: runs of pairs left a wave 25 % more than the mean on an
  // SST file); lane j holds span sbase + j's descriptor.  The last
  // `reserve` waves get no run: they take the long spans' tickets while the
  // others stream their runs (a ticket is a few dependent memory round trips,
  // ~5 us each under full load, too slow for the kernel's tail).
  uint32_t reserve = nwaves / 32u;
  if ((uint64_t)n + 64u * reserve > 64ull * nwaves) reserve = (64u * nwaves - n) / 64u;  // host: n <= 64 nwaves
  const uint32_t K = n < nwaves - reserve ? n : nwaves - reserve;
  // Ticket workers: the last waves without a run, at most 256 (every worker
  // reads `word`, and reads of one address serialize in its L2 channel:
  // ~2.5 ns each, 3072 of them cost ~8 us).
  const uint32_t workers = nwaves - K < 256u ? nwaves - K : 256u;
  const bool worker = wave >= nwaves - workers;
  uint32_t sbase = 0, m = 0;
  if (wave < K) {
    // Runs weighted by the wave's place in its group: wave k of a group
    // shares its SIMD (k mod 4) with two others, and the older ones issue
    // first -- a file-sized call's waves 0-3 / 4-7 / 8-11 drained at 11.5 /
    // 12.3 / 13.4 us with the same six spans each (tools/direct_timeline.py,
    // profiles/r05/r05b_timeline_groups.json).  Group g's spans stay
    // consecutive; unweighted when the groups are not all whole, a run
    // would pass 64 spans, or the waves get fewer than 4 spans each (then
    // 8:7:6 rounds to 2/1/0-span runs, and a two-span wave is the critical
    // path while another idles; the weights were measured on file-sized
    // calls, ~6 spans per wave).
    constexpr uint32_t kW0 = kRunWeight[0], kW1 = kRunWeight[1], kW2 = kRunWeight[2];
    constexpr uint32_t kWg = 4u * (kW0 + kW1 + kW2), kWmax = kW0 > kW1 ? (kW0 > kW2 ? kW0 : kW2) : (kW1 > kW2 ? kW1 : kW2);
    const uint64_t tot = (uint64_t)(K / kDirectWaves) * kWg;
    if (K % kDirectWaves == 0u && (uint64_t)n >= 4ull * K && (uint64_t)n * kWmax <= 63ull * tot) {
      const uint32_t g = wave / kDirectWaves, k = wave % kDirectWaves;
      const uint32_t wk = k < 4u ? kW0 : (k < 8u ? kW1 : kW2);
      const uint32_t cum = k < 4u ? k * kW0 : (k < 8u ? 4u * kW0 + (k - 4u) * kW1 : 4u * (kW0 + kW1) + (k - 8u) * kW2);
      const uint64_t at = (uint64_t)g * kWg + cum;
      sbase = (uint32_t)((uint64_t)n * at / tot);
      m = (uint32_t)((uint64_t)n * (at + wk) / tot) - sbase;
    } else {
      const uint32_t q = n / K, r = n % K;
      sbase = wave * q + (wave < r ? wave : r);
      m = q + (wave < r ? 1u : 0u);
    }
  }
  // A group works if any of its waves has a run or is a ticket worker
  // (adopted tickets and whole spans belong to waves with a run).  The
  // others (batches of fewer spans than waves) wait up to kHelpPoll for a
  // large push's help flag (its replica for this group; one lane polls, the
  // group meets at a barrier) and leave unless it comes: with a few huge
  // spans, 127 static waves and 256 ticket workers folded 8 GiB of tickets
  // at 1.4 TB/s.  An active group's table words are requested first,
  // before any wave of the chip has issued a data load: requested after the
  // descriptors, they queued in HBM behind ~37 MB of other waves' first
  // loads (~5 us, tools/direct_timeline.py).
  const uint32_t g0 = blockIdx.x * kDirectWaves;
  bool helper = false;  // a wave of an idle group called in by the help flag
  if (!(g0 < K || g0 + kDirectWaves > nwaves - workers)) {
    if (tid == 0) {
      uint32_t go = 0;
      const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
      for (;;) {
        if (__hip_atomic_load(d.help + 32u * (blockIdx.x & 31u), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == d.tag) {
          go = 1;
          break;
        }
        if (__builtin_amdgcn_s_memrealtime() - t0 > kHelpPoll) break;
        __builtin_amdgcn_s_sleep(16);
      }
      lds[0] = go;
    }
    __syncthreads();
    if (lds[0] == 0u) return;
    __syncthreads();  // (the table fill overwrites lds[0])
    helper = true;
  }
  TableRegs<kDirectThreads> tr;
  tables_issue(tr, a.tabs, tid);
  uint32_t voff_lo = 0, voff_hi = 0, vlen = 0, vinit = 0;
  if (lane < m) {
    const uint64_t off = a.off[sbase + lane];
    voff_lo = (uint32_t)off;
    voff_hi = (uint32_t)(off >> 32);
    vlen = a.len[sbase + lane];
    if (has_init) vinit = a.init[sbase + lane];
  }

  // ---- 1. discovery: the run's long spans (more than kRingChunks chunks) -> tickets
  uint32_t adopt_lo = 0, adopt_hi = 0;  // orphans of this wave's push: its own to do
  uint64_t whole = 0;                   // workspace full: these run spans are folded whole here
  uint64_t lm = 0;                      // the run's long spans
  // lane j's span geometry, computed here once for the whole run on the
  // vector unit: the ring's tasks read it with four readlanes instead of
  // redoing it on the scalar unit per task (body, body bytes, flags with
  // the chunk count; only ring spans use the count)
  uint32_t gb_lo = 0, gb_hi = 0, gz = 0, gf = 0;
  {
    const uint64_t p = base + (((uint64_t)voff_hi << 32) | voff_lo);
    const DTask g = geometry(p, vlen);
    gb_lo = (uint32_t)g.body;
    gb_hi = (uint32_t)(g.body >> 32);
    gz = g.z;
    gf = g.f | (((g.c1 - 1u) & 31u) << 27);
    const bool lng = lane < m && g.c1 > kRingChunks;
    uint32_t T = 0, lg = 0;
    if (lng) {
      lg = ticket_lg(g.c1, n, nwaves);
      T = (g.c1 + (1u << lg) - 1u) >> lg;
    }
    lm = __ballot(lng);
    if (lm != 0u) {
      uint32_t total = 0, chunks = 0;
      const uint32_t ex = wave_excl_sum(T, lane, total);
      (void)wave_excl_sum(lng ? g.c1 : 0u, lane, chunks);
      if (d.dbg & 1u) {  // test hook: push late, after other waves have run out of claims
        const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
        while (__builtin_amdgcn_s_memrealtime() - t0 < 10000u) __builtin_amdgcn_s_sleep(64);
      }
      uint64_t old = 0;
      if (lane == 0)
        old = __hip_atomic_fetch_add(d.word, (unsigned long long)total << 32, __ATOMIC_RELAXED,
                                     __HIP_MEMORY_SCOPE_AGENT);
      const uint32_t S0 = readlane((uint32_t)(old >> 32), 0), C0 = readlane((uint32_t)old, 0);
      if ((uint64_t)S0 + total <= d.cap) {
        // A large push (>= kHelpChunks of ticket work) calls every wave to
        // claim after its run (the 96-256 ticket workers alone took 26 ms
        // over 127 spans of 64 MiB).  Set before the map is written (a
        // claimer polls its entry until it is): idle groups wait for the
        // flag only ~3 us, and a push of 4096 entries takes longer.
        if (chunks >= kHelpChunks && lane < 32u)
          __hip_atomic_store(d.help + 32u * lane, d.tag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        // the ticket map, one long span at a time, 64 entries per step: four
        // tagged words each, in any order (a claimer polls until all four
        // carry this call's tag; no fence, so the push does not wait for the
        // table fill in flight).  The span's descriptor rides in every
        // entry: a claimer needs one read of its entry, not a second round
        // trip to the descriptors.
        uint64_t mm = lm;
        while (mm != 0u) {
          const uint32_t src = (uint32_t)__builtin_ctzll(mm);
          mm &= mm - 1u;
          const uint32_t f0 = S0 + readlane(ex, src), Ts = readlane(T, src);
          const uint64_t addr = base + (((uint64_t)readlane(voff_hi, src) << 32) | readlane(voff_lo, src));
          const uint32_t ln = readlane(vlen, src), in = readlane(vinit, src);
          for (uint32_t k = lane; k < Ts; k += 64u) {
            uint64_t* e = d.tmap + 4ull * (f0 + k);
            put_tagged(e + 0, d.tag, (uint64_t)(sbase + src) | ((uint64_t)k << 24));  // (T, lg: from len)
            put_tagged(e + 1, d.tag, addr & ((1ull << kTagShift) - 1u));
            put_tagged(e + 2, d.tag, ln);
            put_tagged(e + 3, d.tag, in);
          }
        }
        if (C0 > S0) {
          adopt_lo = S0;
          adopt_hi = C0 < S0 + total ? C0 : S0 + total;
          if (lane == 0) atomicAdd(d.stats + 0, adopt_hi - adopt_lo);
        }
      } else {
        // no room: claimers skip these tickets (null entries; those past the
        // workspace are null by position) and this wave folds the spans whole
        whole = lm;
        if (lane == 0) atomicAdd(d.stats + 1, (uint32_t)__popcll(lm));
        const uint32_t hi = (uint64_t)S0 + total < d.cap ? S0 + total : d.cap;
        for (uint32_t k = S0 + lane; k < hi; k += 64u) put_tagged(d.tmap + 4ull * k, d.tag, kNullEntry);
      }
    }
  }

  // The claim word of the call after next starts at zero (calls take four
  // words in turn and a stream's calls run in order -- every launch is
  // ordered -- so that word is idle).
  if (wave == 0 && lane == 0) __hip_atomic_store(d.next, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);

  {
    // ---- the static run's first loads go out before the table fill's LDS
    // writes and barrier: those then overlap the first data round trip.
    const uint64_t inrun = m >= 64u ? ~0ull : (1ull << m) - 1ull;
    const uint64_t shortm = inrun & ~lm;
    // The next task after `prev` (the newest one): the next chunk of prev's
    // span, or chunk 0 of the next ring span at or after run position j.
    auto static_task = [&](uint32_t& j, const DTask& prev) -> DTask {
      if (prev.valid() && !prev.rlast()) {
        DTask t = prev;
        t.f += 1u << 22;
        return t;
      }
      const uint64_t from = j >= 64u ? 0ull : ~0ull << j;
      const uint64_t avail = shortm & from;
      if (avail == 0u) {
        j = 64u;
        DTask t = geometry(base, 0u);
        t.f = 0;  // kind none
        return t;
      }
      const uint32_t p = (uint32_t)__builtin_ctzll(avail);
      DTask t;
      t.body = ((uint64_t)readlane(gb_hi, p) << 32) | readlane(gb_lo, p);
      t.z = readlane(gz, p);
      t.f = readlane(gf, p) | (kKindStatic << 14) | (p << 16);  // (nch <= kRingChunks)
      t.b = sbase + p;
      t.c = 0;  // (the ring reads the chunk from f)
      t.c1 = 1;
      j = p + 1u;
      return t;
    };
    // 17 loads per task, always: 16 body dwords of chunk t.c (the buffer
    // range check reads 0 outside the body: chunk 0's padding) and one edge
    // byte per lane -- head bytes (lanes 0-2, chunk 0), tail bytes (3-5) and
    // stored crc (6-9) (the span's last chunk).
    auto issue = [&](const DTask& t, uint32_t (&w)[kRounds], uint32_t& e) {
      const bool live = t.valid();
      // (readfirstlane: the load branches below must be scalar branches --
      // as exec-masked branches, hipcc's CFG has paths that issue no loads)
      // chunk c > 0: the buffer starts at the chunk (no padding); chunk 0 is
      // right-aligned, pad leading words read as 0 (no extra load branch:
      // hipcc lowered one as an exec-masked branch around the ring's loads)
      const uint32_t c = t.rc();
      const bool first = c == 0u, last = t.rlast();
      const uint32_t skip = first ? 0u : (c << 12) - 4u * t.pad();  // body bytes before chunk c
      const uint32_t pad = rfl(first ? t.pad() : 0u), h = t.h(), tl = t.t(), len = t.len();
      const bool hwin = kVerify && hdr;
      auto sat = [](uint64_t x) -> uint32_t { return x > 0xFFFFFFFFull ? 0xFFFFFFFFu : (uint32_t)x; };
      const uint64_t start = t.body - h;
      u32x4 rb = buffer_rsrc(reinterpret_cast<const uint8_t*>(t.body + skip), live ? t.z - skip : 0u);
      u32x4 re = buffer_rsrc(reinterpret_cast<const uint8_t*>(hwin ? start - kLogCrcBack : start),
                             live ? (hwin ? sat((uint64_t)kLogCrcBack + len) : sat((uint64_t)len + (kVerify ? 4u : 0u)))
                                  : 0u);
      // SGPRs the vector unit wrote (readlane) need 5 wait states before a
      // VMEM instruction reads them; hipcc inserts none before inline asm.
      asm volatile("s_nop 4" : "+s"(rb), "+s"(re));
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
      const uint32_t hb = hwin ? kLogCrcBack : 0u;  // edge-window offset of the span's first byte
      uint32_t eoff = 0xFFFFFFFFu;
      if (first && lane < h) eoff = hb + lane;
      if (last && lane >= 3u && lane < 3u + tl) eoff = sat((uint64_t)hb + h + t.z + (lane - 3u));
      if (kVerify && last && lane >= 6u && lane < 10u) eoff = hwin ? lane - 6u : sat((uint64_t)len + (lane - 6u));
      e = buf_ubyte(re, eoff);
    };
    // The ring: one sequence of tasks (run positions in order, a span's
    // chunks one after another) through TWO single-task slots: a wave waits
    // for its older task (the younger one's 17 loads stay in flight) and
    // folds it as soon as it has landed.  Two tasks in flight per wave are
    // 25 MB over the chip, enough to keep HBM busy; more only lengthen every
    // wave's wait for its first data (a file-sized call's whole read used to
    // go out at once), and the folds then bunch up behind the last arrivals.
    // (slots 2 and 3 stay unused: declared with two entries, hipcc copied
    // in-flight ring registers at the loop head, tools/check_inflight.py)
    DTask tk[4];
    uint32_t wb[4][kRounds];
    uint32_t eb[4];
    uint32_t jc = 0u;
    {
      DTask none = geometry(base, 0u);
      none.f = 0;
      tk[0] = static_task(jc, none);  // (none without a run)
      tk[1] = static_task(jc, tk[0]);
    }
    // Every wave runs the ring (a wave without a run: empty tasks, whose
    // range-checked loads touch no memory, and no folds), so the ring's
    // registers have one definition on every path: hipCC then never copies
    // an in-flight register at a merge (tools/check_inflight.py).  The first
    // task's loads go out before the table fill's LDS writes and barrier.
    issue(tk[0], wb[0], eb[0]);
    tables_wait<kRounds + 1>(tr);  // its 17 loads stay in flight
    tables_store<kDirectThreads>(lds, tr, tid);
    // Group barrier for the LDS image.  Not __syncthreads(): its release
    // fence waits for every outstanding load (vmcnt(0)), slot 0's included.
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    const StrideLanes tab = stride_lanes(lane);
    const uint32_t nibtab = 4u * (kTabWords + lane);
    const ShortShift ss = short_shift_cols(lane);
    uint32_t res = 0u, bad = 0u, have = 0u;  // the static run's results: lane j = span sbase + j

    // The span's crc from its body register (or, without body words, from
    // its initial register): tail bytes, conditioning, Mask; the result, the
    // verify flag and the trailer.  A span of the static run keeps its result
    // in lane `slot` for the run's one coalesced store; the others' results
    // are stored by lane 0.
    auto finish = [&](const DTask& t, uint32_t reg, uint32_t tail, uint32_t stored, bool to_run) {
      const uint32_t tl = t.t();
      const uint32_t crc = feed_short(ss, lane, reg, tail, tl) ^ kConditioning;
      const uint32_t v = (a.flags & kFlagMask) ? mask_crc(crc) : crc;
      const uint32_t mm = crc != unmask_crc(stored) ? 1u : 0u;
      if (to_run) {
        const uint32_t slot = t.slot();
        res = lane == slot ? v : res;
        if (kVerify) bad = lane == slot ? mm : bad;
        have = lane == slot ? 1u : have;
      } else if (lane == 0) {
        if (a.out != nullptr) a.out[t.b] = v;
        if (kVerify && a.mismatch != nullptr) a.mismatch[t.b] = (uint8_t)mm;
      }
      // (a ring span's trailer is stored with the run's results, after the
      // ring: a store between the slots' loads sits in the in-order vmcnt,
      // and the counted waits would wait for its write acknowledgement)
      if ((a.flags & kFlagWriteTrailer) && lane == 0 && !to_run) {
        const uint64_t start = t.body - t.h();
        store_le32(reinterpret_cast<const uint8_t*>(hdr ? start - kLogCrcBack : t.body + t.z + tl), v);
      }
    };
    // the edge bytes read by lanes 0-9 (head, tail, stored crc) as words
    auto edge_head = [&](uint32_t e, uint32_t h) -> uint32_t {
      return h ? readlane(e, 0) | (readlane(e, 1) << 8) | (readlane(e, 2) << 16) : 0u;
    };
    auto edge_tail = [&](uint32_t e, uint32_t tl) -> uint32_t {
      return tl ? readlane(e, 3) | (readlane(e, 4) << 8) | (readlane(e, 5) << 16) : 0u;
    };
    auto edge_stored = [&](uint32_t e) -> uint32_t {
      return kVerify ? readlane(e, 6) | (readlane(e, 7) << 8) | (readlane(e, 8) << 16) | (readlane(e, 9) << 24) : 0u;
    };
    // The register enters with body word 0: lane pad % 64 of round pad / 64
    // (a wave-uniform round: a masked XOR per round, no indexed access).
    auto inject = [&](uint32_t (&w)[kRounds], uint32_t pad, uint32_t rr) {
      const uint32_t J = pad >> 6;
      const uint32_t inj = lane == (pad & 63u) ? rr : 0u;
      if (J == 0) {
        w[0] ^= inj;
      } else {
#pragma unroll
        for (int j = 1; j < kRounds; ++j) w[j] = __builtin_amdgcn_bitop3_b32(w[j], inj, (uint32_t)j == J ? ~0u : 0u, 0x78);
      }
    };

    // ---- groups: tickets and whole spans.  Compiler-scheduled buffer loads
    // (outside the body they read 0: chunk 0's right-aligned padding), two
    // chunks per step.  Rare next to the static run (an SST file has one long
    // span), so this loop favours simplicity over the ring's overlap.
    // Returns the register over chunks [t.c, t.c1) -- from the span's initial
    // register when t.c == 0, else from 0 -- and in r0 the initial register.
    auto group_reg = [&](const DTask& t, uint32_t init, uint32_t& r0) -> uint32_t {
      const __amdgpu_buffer_rsrc_t rb =
          __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>(t.body), (short)0, (int)t.z, 0x00020000);
      const uint32_t pad = t.pad(), h = t.h();
      r0 = 0u;
      uint32_t hb = 0u;  // head bytes: requested before the chunk loads, used after them
      if (t.c == 0u) {
        const uint8_t* sp = reinterpret_cast<const uint8_t*>(t.body - h);
        hb = lane < h ? (uint32_t)sp[lane] : 0u;
      }
      uint32_t acc = 0u;
      // Two chunks (32 loads, 8 KiB) per step, the next step's loads issued
      // before this step's fold: two steps in flight (a 1 MiB ticket is 128
      // steps; four-chunk steps spilled VGPRs to scratch).  Chunks past t.c1
      // read as 0 (a zero count) and are not folded.
      constexpr int kG = 2;
      auto load_step = [&](uint32_t c, uint32_t (&w)[kG][kRounds]) {
        const uint32_t nin = c >= t.c1 ? 0u : (t.c1 - c < (uint32_t)kG ? t.c1 - c : (uint32_t)kG);
        const uint32_t i0 = (c << 10) + lane - pad;  // chunk 0: wraps below the body
#pragma unroll
        for (int j = 0; j < kRounds; ++j) {
          // One opaque voffset per round: folded into the instruction's
          // immediate offset, a wrapped (negative) voffset + imm is a sum past
          // 2^32, which the range check reads as out of range -- zeros where
          // chunk 0's body words are (the span kernel's note on chunk 0).
          uint32_t o0 = (i0 + 64u * (uint32_t)j) * 4u;
          asm volatile("" : "+v"(o0));
#pragma unroll
          for (int k = 0; k < kG; ++k)
            w[k][j] = (uint32_t)k < nin ? __builtin_amdgcn_raw_buffer_load_b32(rb, (int)(o0 + 4096u * k), 0, 0) : 0u;
        }
      };
      auto fold_step = [&](uint32_t c, uint32_t (&w)[kG][kRounds]) {
        const uint32_t nin = t.c1 - c < (uint32_t)kG ? t.c1 - c : (uint32_t)kG;
        if (c == 0u) {
          r0 = feed_short(ss, lane, init ^ kConditioning, edge_head(hb, h), h);
          if (t.z != 0u) inject(w[0], pad, r0);
        }
#pragma unroll
        for (int k = 0; k < kG; ++k) {
          if ((uint32_t)k < nin) {
#pragma unroll
            for (int j = 0; j < kRounds; ++j) acc = step256(lds, tab, acc, w[k][j]);
          }
        }
      };
      uint32_t wa[kG][kRounds], wb2[kG][kRounds];
      uint32_t c = t.c;
      load_step(c, wa);
      for (;;) {
        load_step(c + kG, wb2);
        fold_step(c, wa);
        c += kG;
        if (c >= t.c1) break;
        load_step(c + kG, wa);
        fold_step(c, wb2);
        c += kG;
        if (c >= t.c1) break;
      }
      return wave_xor(realign(lds, nibtab, acc));
    };
    // tail bytes and the stored crc of a span, read directly
    auto span_edges = [&](const DTask& t, uint32_t& tail, uint32_t& stored) {
      const uint32_t tl = t.t();
      const uint64_t start = t.body - t.h();
      const uint8_t* ep = nullptr;
      if (lane >= 3u && lane < 3u + tl) ep = reinterpret_cast<const uint8_t*>(t.body + t.z + (lane - 3u));
      if (kVerify && lane >= 6u && lane < 10u)
        ep = reinterpret_cast<const uint8_t*>((hdr ? start - kLogCrcBack : t.body + t.z + tl) + (lane - 6u));
      const uint32_t e = ep != nullptr ? (uint32_t)*ep : 0u;
      tail = edge_tail(e, tl);
      stored = edge_stored(e);
    };
    // Ticket tkt (< cap): spin until its map entry is this call's, fold its
    // chunks, store and count the partial; the span's last ticket combines
    // R = sum_k M^(T-1-k) R_k (M = shift_{4 KiB 2^lg}) and finishes the span.
    // Every dependent memory round trip here costs microseconds while the
    // static runs keep HBM saturated, so the path is cut to: entry (one
    // 32-B read, repeated until all four words carry the tag), chunk loads, partial +
    // counter, and for the span's last ticket one batch of loads (partials,
    // combine columns, edge bytes) before the result.
    auto run_ticket = [&](uint32_t tkt) {
      // lanes 0-3 read the entry's four words until every one carries this
      // call's tag (a null entry: word 0 alone)
      const uint64_t* e = d.tmap + 4ull * tkt;
      uint64_t ew = 0;
      for (;;) {
        ew = lane < 4u ? get_word(e + lane) : 0u;
        const uint64_t ok = __ballot(lane < 4u && has_tag(ew, d.tag));
        if ((ok & 15u) == 15u || ((ok & 1u) && (readlane((uint32_t)ew, 0) & 0xFFFFFFu) == kNullEntry)) break;
        __builtin_amdgcn_s_sleep(2);
      }
      const uint32_t w0lo = readlane((uint32_t)ew, 0), w0hi = readlane((uint32_t)(ew >> 32), 0);
      const uint32_t sb = w0lo & 0xFFFFFFu;
      if (sb == kNullEntry) return;
      const uint32_t k = (w0lo >> 24) | ((w0hi & 0xFFFFu) << 8);
      const uint64_t addr = ((uint64_t)(readlane((uint32_t)(ew >> 32), 1) & 0xFFFFu) << 32) | readlane((uint32_t)ew, 1);
      DTask t = geometry(addr, readlane((uint32_t)ew, 2));
      t.b = sb;
      const uint32_t lg = ticket_lg(t.c1, n, nwaves), T = (t.c1 + (1u << lg) - 1u) >> lg, f0 = tkt - k;
      const uint32_t first = t.c1 - ((T - 1u) << lg);  // ticket 0: the remainder
      t.c = k ? first + ((k - 1u) << lg) : 0u;
      t.c1 = k ? t.c + (1u << lg) : first;
      uint32_t r0 = 0;
      const uint32_t v = group_reg(t, (k == 0u && has_init) ? readlane((uint32_t)ew, 3) : 0u, r0);
      // the partial (tagged), then the span's counter: the wave whose add is
      // the span's last combines, polling each partial until it carries the
      // tag (the counter add may overtake another wave's partial store)
      uint32_t old = 0;
      if (lane == 0) {
        put_tagged(d.part + tkt, d.tag, v);
        old = __hip_atomic_fetch_add(d.cdone + f0, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      if (readlane(old, 0) + 1u != T) return;
      uint32_t tail = 0, stored = 0;
      span_edges(t, tail, stored);
      uint32_t cols[32];  // lane's final shift, requested with the partials
#pragma unroll
      for (int i = 0; i < 32; ++i) cols[i] = a.tabs->tick_lane[lg][i][lane];
      const uint32_t J = (T + 63u) >> 6;
      const int32_t pad0 = (int32_t)(J * 64u - T);
      uint32_t x = 0;
      for (uint32_t j = 0; j < J; ++j) {
        const int32_t kk = (int32_t)(j * 64u + lane) - pad0;
        uint64_t pw = 0;
        for (;;) {
          pw = kk >= 0 ? get_word(d.part + f0 + (uint32_t)kk) : ((uint64_t)d.tag << kTagShift);
          if (__ballot(!has_tag(pw, d.tag)) == 0u) break;
          __builtin_amdgcn_s_sleep(2);
        }
        x = gf2_apply(a.tabs->tick64[lg], x) ^ (uint32_t)pw;
      }
      uint32_t y = 0;
#pragma unroll
      for (int i = 0; i < 32; ++i) y ^= cols[i] & (0u - ((x >> i) & 1u));
      const uint32_t R = wave_xor(y);
      if (lane == 0) __hip_atomic_store(d.cdone + f0, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      finish(t, R, tail, stored, false);
    };
    // a long span of the run folded whole by this wave (ticket workspace full)
    auto run_whole = [&](uint32_t j) {
      const uint64_t off = ((uint64_t)readlane(voff_hi, j) << 32) | readlane(voff_lo, j);
      DTask t = geometry(base + off, readlane(vlen, j));
      t.b = sbase + j;
      uint32_t r0 = 0;
      const uint32_t R = group_reg(t, readlane(vinit, j), r0);
      uint32_t tail = 0, stored = 0;
      span_edges(t, tail, stored);
      finish(t, t.z ? R : r0, tail, stored, false);
    };
    auto claim = [&](uint32_t k, uint32_t& c, uint32_t& sp) {
      uint64_t old = 0;
      if (lane == 0)
        old = __hip_atomic_fetch_add(d.word, (unsigned long long)k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      sp = readlane((uint32_t)(old >> 32), 0);
      c = readlane((uint32_t)old, 0);
    };

    // ---- the static run: its ring spans in run order (long ones skipped),
    // two single-task slots (a wait leaves the younger task's 17 loads in
    // flight), inline-asm loads, counted waits, one LDS chain per fold (the
    // 12 waves of a CU interleave theirs).  Measured in one process,
    // alternating order (profiles/r04/r04b_variants_ring4_slot1late_tablesfirst.json,
    // r04g_variants.json, r04j_variants_ring_depth.json): against round 3's
    // two slots of three streams, four single-task slots gained 3-10 %
    // (config-3 spans +10.5 %); against four slots, two gain again: one
    // sealed SST file 4135 against 3865 GB/s (16.4 us), verified +9.8 %,
    // two files +10.6 %, three +9.2 %, seven +5.8 %.
    {
      uint32_t carry = 0u;  // the register between the chunks of the current span
      // The initial register, fed the head bytes, enters chunk 0 with its
      // body word 0 (a zero injection for a later chunk, which continues the
      // carried register); realigned and reduced every task, and a span's
      // last chunk finishes it.
      auto fold = [&](const DTask& t, uint32_t (&w)[kRounds], const uint32_t e) {
        const bool c0 = t.rc() == 0u;
        const uint32_t r =
            feed_short(ss, lane, readlane(vinit, t.slot()) ^ kConditioning, edge_head(e, t.h()), t.h());
        uint32_t acc = c0 ? 0u : carry;
        if (t.z) inject(w, t.pad(), c0 ? r : 0u);
#pragma unroll
        for (int j = 0; j < kRounds; ++j) acc = step256(lds, tab, acc, w[j]);
        const uint32_t v = realign(lds, nibtab, acc);
        carry = acc;
        const uint32_t bv = wave_xor(v);
        if (t.valid() && t.rlast()) finish(t, t.z ? bv : r, edge_tail(e, t.t()), edge_stored(e), true);
      };
      issue(tk[1], wb[1], eb[1]);
      constexpr int kYounger = kRounds + 1;  // the younger task
      for (;;) {
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          wait_task<kYounger>(wb[q], eb[q]);
          if (tk[q].valid()) fold(tk[q], wb[q], eb[q]);
          // tasks are made in sequence: the next one invalid, all are
          if (!tk[q ^ 1].valid()) goto drained;
          tk[q] = static_task(jc, tk[q ^ 1]);
          issue(tk[q], wb[q], eb[q]);
        }
      }
    drained:
#pragma unroll
      for (int q = 0; q < 2; ++q) wait_task<0>(wb[q], eb[q]);
    }

    // ---- workers
    // A worker polls for pushes for a bounded time (nothing ever waits for
    // another wave's progress) and claims visible tickets one at a time.  (All 2048 waves claiming at once after the table
    // load serialized ~2048 atomics on one address, ~70 us.)
    if (worker) {
      if (d.dbg & 2u) {  // test hook: one blind claim (an orphan while nothing is pushed)
        uint32_t c = 0, sp = 0;
        claim(1u, c, sp);
        if (c < sp) {
          if (lane == 0) atomicAdd(d.stats + 2, 1u);
          if (c < d.cap) run_ticket(c);
        }
      }
      const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
      for (;;) {
        uint64_t wd = 0;
        if (lane == 0) wd = __hip_atomic_load(d.word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const uint32_t S = readlane((uint32_t)(wd >> 32), 0), C = readlane((uint32_t)wd, 0);
        if (S > C) {
          uint32_t c = 0, sp = 0;
          claim(1u, c, sp);
          if (c >= sp) break;  // an orphan: its pusher does it
          if (lane == 0) atomicAdd(d.stats + 2, 1u);
          if (c < d.cap) run_ticket(c);
          continue;
        }
        if (__builtin_amdgcn_s_memrealtime() - t0 > kWorkerPoll) break;
        __builtin_amdgcn_s_sleep(32);
      }
    }

    // ---- after the run (rare: a push that found its tickets claimed, or a
    // full ticket workspace): this wave's orphans and its whole spans
    for (uint32_t tkt = adopt_lo; tkt < adopt_hi; ++tkt) run_ticket(tkt);
    for (uint64_t wm = whole; wm != 0u; wm &= wm - 1u) run_whole((uint32_t)__builtin_ctzll(wm));

    // ---- late: a wave that pushed tickets claims, one at a time, until
    // none is left -- its own included, whoever else did not take them, so
    // every pushed ticket is claimed by someone (a claim past the supply is an
    // orphan: its pusher does it).  Other static waves join only when a large
    // push called for help (one read of their replica of the help flag, 32
    // replicas on lines of their own); otherwise they leave: 3072 reads of
    // `word` at the end cost ~8 us of the kernel's tail.
    bool help = helper;
    if (lm == 0u && wave < K)
      help = __hip_atomic_load(d.help + 32u * (wave & 31u), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == d.tag;
    while ((lm != 0u || help) && whole == 0u) {
      uint64_t wd = 0;
      if (lane == 0) wd = __hip_atomic_load(d.word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (readlane((uint32_t)(wd >> 32), 0) <= readlane((uint32_t)wd, 0)) break;
      uint32_t c = 0, sp = 0;
      claim(1u, c, sp);
      if (c >= sp) break;
      if (lane == 0) atomicAdd(d.stats + 3, 1u);
      if (c < d.cap) run_ticket(c);
    }
    // the static run's results: one coalesced store (long spans' lanes are
    // their completers')
    if (lane < m && have != 0u) {
      if (a.out != nullptr) __builtin_nontemporal_store(res, a.out + sbase + lane);
      if (kVerify && a.mismatch != nullptr) __builtin_nontemporal_store((uint8_t)bad, a.mismatch + sbase + lane);
      if (!kVerify && (a.flags & kFlagWriteTrailer)) {  // each lane its span's stored crc
        const uint64_t p = base + (((uint64_t)voff_hi << 32) | voff_lo);
        const uint64_t body = ((uint64_t)gb_hi << 32) | gb_lo;
        store_le32(reinterpret_cast<const uint8_t*>(hdr ? p - kLogCrcBack : body + gz + ((gf >> 12) & 3u)), res);
      }
    }
  }

}

hipError_t launch_direct(const SpanBatch& a, bool verify, int grid, const DirectWs& d, hipStream_t s,
                         hipEvent_t done) {
  if (verify)
    hipExtLaunchKernelGGL(crc32c_direct_kernel<true>, dim3(grid), dim3(kDirectThreads), 0, s, nullptr, done, 0u, a, d);
  else
    hipExtLaunchKernelGGL(crc32c_direct_kernel<false>, dim3(grid), dim3(kDirectThreads), 0, s, nullptr, done, 0u, a, d);
  return hipGetLastError();
}

}  // namespace dev
}  // namespace prismdb
