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
//   crc32c_combine_kernel   stitches segments back into long spans
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "crc32c_device.h"

#ifndef PRISMDB_FIXED_NOSTORE  // measurement knob: no result stores (wrong results)
#define PRISMDB_FIXED_NOSTORE 0
#endif
#ifndef PRISMDB_FIXED_NOFOLD
#define PRISMDB_FIXED_NOFOLD 0
#endif
#ifndef PRISMDB_RING
#define PRISMDB_RING 4  // span buffers in the fixed kernel's prefetch ring (even)
#endif
#ifndef PRISMDB_NT_LOADS
#define PRISMDB_NT_LOADS 1  // body words are read once: non-temporal
#endif
#ifndef PRISMDB_XOR3
#define PRISMDB_XOR3 1  // three-input XORs through v_bitop3_b32
#endif
#ifndef PRISMDB_SPAN_INJ_RING  // span kernel: initial register written into the ring registers (1) or folded in (0)
#define PRISMDB_SPAN_INJ_RING 1
#endif
#ifndef PRISMDB_SPAN_REC_WAIT  // measurement knob: span kernel waits for each record read at once
#define PRISMDB_SPAN_REC_WAIT 0
#endif
#ifndef PRISMDB_FIXED_DUMMY_SALU  // measurement knob: fixed kernel issues this many extra SALU per span pair
#define PRISMDB_FIXED_DUMMY_SALU 0
#endif
#ifndef PRISMDB_FIXED_DUMMY_VALU  // measurement knob: ... and this many extra VALU per span pair
#define PRISMDB_FIXED_DUMMY_VALU 0
#endif
#ifndef PRISMDB_QUAD_UNALIGNED  // quad kernel: body words from the record's first byte (unaligned dword loads, no head bytes)
#define PRISMDB_QUAD_UNALIGNED 0
#endif
#ifndef PRISMDB_FIXED_FAR_PAIR  // measurement knob: fixed kernel pairs spans half a run apart (the span kernel's pattern)
#define PRISMDB_FIXED_FAR_PAIR 0
#endif
#ifndef PRISMDB_FIXED_SETPRIO
#define PRISMDB_FIXED_SETPRIO 0
#endif
#ifndef PRISMDB_FIXED_CHAIN  // measurement knob: the pair's second span starts from the first's register (one dependent chain; wrong results)
#define PRISMDB_FIXED_CHAIN 0
#endif
#ifndef PRISMDB_LANE_THREADS  // lane kernel workgroup size (one group per CU)
#define PRISMDB_LANE_THREADS 512
#endif
#ifndef PRISMDB_LANE_NOFOLD  // measurement knob: lane kernel XORs its words instead of folding them (wrong results)
#define PRISMDB_LANE_NOFOLD 0
#endif
#ifndef PRISMDB_SPAN_NOEDGE  // measurement knob: span kernel issues no edge-byte load (wrong with tails / verify)
#define PRISMDB_SPAN_NOEDGE 0
#endif
#ifndef PRISMDB_SPAN_WG_EXIT  // span kernel: groups without a stream leave before the table load
#define PRISMDB_SPAN_WG_EXIT 1
#endif
#ifndef PRISMDB_PLAN_SERIAL_SEG  // A/B knob: a long span's thread writes all its segment records itself
#define PRISMDB_PLAN_SERIAL_SEG 0
#endif
#ifndef PRISMDB_SPAN_J0  // measurement knob: span kernel folds rounds >= this only (wrong results)
#define PRISMDB_SPAN_J0 0
#endif
#ifndef PRISMDB_SPAN_INJ0  // measurement knob: initial register always enters round 0 (wrong if pad >= 64)
#define PRISMDB_SPAN_INJ0 0
#endif
#ifndef PRISMDB_SPAN_SNOP  // 1: s_nop 4 between the descriptors and the asm buffer loads
#define PRISMDB_SPAN_SNOP 0
#endif
#ifndef PRISMDB_LOG_ROUNDSKIP  // log-record kernel: skip chunk 0's padding rounds
#define PRISMDB_LOG_ROUNDSKIP 1
#endif
#ifndef PRISMDB_QUAD_NOREALIGN  // measurement knob: quad kernel skips the realignment (wrong results)
#define PRISMDB_QUAD_NOREALIGN 0
#endif
#ifndef PRISMDB_QUAD_NOMASK  // measurement knob: quad kernel folds masked rounds plainly (wrong results)
#define PRISMDB_QUAD_NOMASK 0
#endif
#ifndef PRISMDB_QUAD_RALIGN_GROUPS  // realignment lookups issued in this many groups (1, 2 or 4)
#define PRISMDB_QUAD_RALIGN_GROUPS 4
#endif
#ifndef PRISMDB_SLICES_PER_STREAM  // span kernel: task-balanced slices shrink until every stream gets this many
#define PRISMDB_SLICES_PER_STREAM 16
#endif
#ifndef PRISMDB_SLICE_EXACT  // task-balanced slices: exactly m per stream (1) or ceil(T / 2^lg) (0)
#define PRISMDB_SLICE_EXACT 1
#endif
#ifndef PRISMDB_RUNS_PER_STREAM  // span kernel: runs of one-task records shrink until every stream gets this many
#define PRISMDB_RUNS_PER_STREAM 64
#endif
#ifndef PRISMDB_QUAD_CLAMPED  // quad kernel body addresses: min-clamped index per load (1) or one v_max (0)
#define PRISMDB_QUAD_CLAMPED 0
#endif
#ifndef PRISMDB_QUAD_RING
#define PRISMDB_QUAD_RING 2  // tasks in the quad kernel's ring (one folded, the rest in flight)
#endif
#ifndef PRISMDB_RUN_LG
#define PRISMDB_RUN_LG 5  // fixed kernel: log2(pair steps per run); runs of 2 << PRISMDB_RUN_LG spans
#endif

namespace prismdb {
namespace dev {

namespace {

__device__ __forceinline__ uint32_t rfl(uint32_t x) { return __builtin_amdgcn_readfirstlane(x); }
__device__ __forceinline__ uint32_t readlane(uint32_t x, uint32_t l) {
  return __builtin_amdgcn_readlane(x, l);
}

// v ^ dpp(v): with every lane active and bound_ctrl set, hipcc fuses the pair
// into one v_xor_b32_dpp.
__device__ __forceinline__ uint32_t xor_dpp(uint32_t v, int ctrl) {
  switch (ctrl) {
    case 0xB1: return v ^ __builtin_amdgcn_update_dpp(0u, v, 0xB1, 0xF, 0xF, true);
    case 0x4E: return v ^ __builtin_amdgcn_update_dpp(0u, v, 0x4E, 0xF, 0xF, true);
    case 0x141: return v ^ __builtin_amdgcn_update_dpp(0u, v, 0x141, 0xF, 0xF, true);
    default: return v ^ __builtin_amdgcn_update_dpp(0u, v, 0x140, 0xF, 0xF, true);
  }
}

// XOR within each row of 16 lanes: quad_perm [1,0,3,2], quad_perm [2,3,0,1],
// row_half_mirror, row_mirror.
__device__ __forceinline__ uint32_t row_xor(uint32_t v) {
  return xor_dpp(xor_dpp(xor_dpp(xor_dpp(v, 0xB1), 0x4E), 0x141), 0x140);
}

// XOR of v over the 64 lanes (wave-uniform result).
__device__ __forceinline__ uint32_t wave_xor(uint32_t v) {
  v = row_xor(v);
  return readlane(v, 0) ^ readlane(v, 16) ^ readlane(v, 32) ^ readlane(v, 48);
}

// Short shifts on the vector unit.  Feeding t <= 3 bytes b0..b(t-1) into the
// register r is shift_t(r ^ (b0 | b1 << 8 | b2 << 16)) (the word-feed identity
// cut to t bytes), and shift_t is a 32x32 GF(2) matrix: lane i < 32 holds its
// column i for t = 1, 2, 3 (computed once per wave, 24 LFSR steps), so
// shift_t(x) for a wave-uniform x is one select per lane and a 32-lane XOR.
struct ShortShift {
  uint32_t col[3];
};

__device__ __forceinline__ ShortShift short_shift_cols(uint32_t lane) {
  ShortShift s;
  uint32_t c = lane < 32u ? 1u << lane : 0u;
#pragma unroll
  for (int t = 0; t < 3; ++t) {
#pragma unroll
    for (int k = 0; k < 8; ++k) c = (c >> 1) ^ (kPolyReflected & (0u - (c & 1u)));
    s.col[t] = c;
  }
  return s;
}

// XOR over lanes 0..31 (lanes 32..63 must hold 0 or be ignored): DPP within
// rows, then rows 0 and 1.
__device__ __forceinline__ uint32_t half_xor(uint32_t v) {
  v = row_xor(v);
  return readlane(v, 0) ^ readlane(v, 16);
}

// Feed the t (0..3) bytes of d (little-endian) into the uniform register r.
__device__ __forceinline__ uint32_t feed_short(const ShortShift& ss, uint32_t lane, uint32_t r, uint32_t d,
                                               uint32_t t) {
  if (t == 0) return r;
  const uint32_t x = r ^ d;
  const uint32_t col = t == 1 ? ss.col[0] : (t == 2 ? ss.col[1] : ss.col[2]);
  return half_xor(((x >> (lane & 31u)) & 1u) ? col : 0u);
}

// The caller owns the span's trailer bytes when it asks for them to be written
// (TableBuilder::WriteRawBlock, table/table_builder.cc:196).
__device__ __forceinline__ void store_le32(const uint8_t* p, uint32_t v) {
  uint8_t* q = const_cast<uint8_t*>(p);
  q[0] = (uint8_t)v;
  q[1] = (uint8_t)(v >> 8);
  q[2] = (uint8_t)(v >> 16);
  q[3] = (uint8_t)(v >> 24);
}

__device__ __forceinline__ uint32_t mask_crc(uint32_t c) { return ((c << 17) | (c >> 15)) + kMaskDelta; }
__device__ __forceinline__ uint32_t unmask_crc(uint32_t m) {
  const uint32_t r = m - kMaskDelta;
  return (r << 15) | (r >> 17);
}

// LDS image of the stride tables (128 KiB): table k, entry e, copy c = lane%32
// sits at byte ((k>>1) << 16) | (e << 8) | ((k&1) << 7) | (c << 2), so every
// lookup address is one v_perm_b32: byte 1 <- byte k of acc, bytes 0 and 2
// from a per-lane constant.  Bank = c: ds_read_b32 never conflicts.
struct StrideLanes {
  uint32_t L[4];  // per-lane byte-0/byte-2 constants of tables 0..3
};

__device__ __forceinline__ StrideLanes stride_lanes(uint32_t lane) {
  StrideLanes t;
#pragma unroll
  for (int k = 0; k < 4; ++k) t.L[k] = ((uint32_t)(k & 1) << 7) | ((lane & 31u) << 2) | ((uint32_t)(k >> 1) << 16);
  return t;
}

// Fill LDS: stride tables in the image above, then the per-lane nibble tables.
__device__ __forceinline__ void load_tables(uint32_t* lds, const DeviceTables* tabs, uint32_t tid) {
  for (uint32_t w = tid; w < (uint32_t)kTabWords; w += kThreads) {
    const uint32_t k = ((w >> 14) << 1) | ((w >> 5) & 1u), e = (w >> 6) & 255u;
    lds[w] = tabs->stride[k][e];
  }
  const uint32_t* nib = &tabs->lane_nib[0][0][0];
  for (uint32_t e = tid; e < (uint32_t)kNibWords; e += kThreads) lds[kTabWords + e] = nib[e];
}

__device__ __forceinline__ uint32_t lds_word(const uint32_t* lds, uint32_t byte_addr) {
  return *reinterpret_cast<const uint32_t*>(reinterpret_cast<const char*>(lds) + byte_addr);
}

// a ^ b ^ c in one VALU instruction (gfx950 v_bitop3_b32, truth table 0x96).
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
#if PRISMDB_XOR3
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
#else
  return a ^ b ^ c;
#endif
}

// One stream step: shift_256(acc) ^ w with four conflict-free LDS lookups
// (w is folded in early so only one XOR trails the last lookup).
__device__ __forceinline__ uint32_t step256(const uint32_t* lds, const StrideLanes& t, uint32_t acc,
                                            uint32_t w) {
  const uint32_t a0 = lds_word(lds, __builtin_amdgcn_perm(acc, t.L[0], 0x0C020400u));
  const uint32_t a1 = lds_word(lds, __builtin_amdgcn_perm(acc, t.L[1], 0x0C020500u));
  const uint32_t a2 = lds_word(lds, __builtin_amdgcn_perm(acc, t.L[2], 0x0C020600u));
  const uint32_t a3 = lds_word(lds, __builtin_amdgcn_perm(acc, t.L[3], 0x0C020700u));
  return xor3(xor3(w, a0, a1), a2, a3);
}

// shift_{256-4l}(acc) for this lane: eight nibble lookups in lane l's own
// tables (entry [n][v] at word 64*(16n+v)+l, so bank = l mod 32).  nib is the
// byte address of lane l's entry [0][0] (bits 2-7 and 17 only), so each
// address is one shift plus one v_and_or_b32, the table offset n*4 KiB rides
// in the instruction's offset field.
__device__ __forceinline__ uint32_t nib_addr(uint32_t acc, int n, uint32_t nib) {
  const uint32_t x = n < 2 ? acc << (8 - 4 * n) : acc >> (4 * n - 8);
  uint32_t a;  // (x & 0xF00) | nib in one instruction (hipcc prefers and + add)
  asm("v_and_or_b32 %0, %1, %2, %3" : "=v"(a) : "v"(x), "s"(0xF00u), "v"(nib));
  return a;
}

__device__ __forceinline__ uint32_t realign(const uint32_t* lds, uint32_t nib, uint32_t acc) {
  uint32_t v[8];
#pragma unroll
  for (int n = 0; n < 8; ++n) v[n] = lds_word(lds, nib_addr(acc, n, nib) + 4096u * n);
  return xor3(xor3(v[0], v[1], v[2]), xor3(v[3], v[4], v[5]), v[6] ^ v[7]);
}

}  // namespace

// Inline-asm dword load, non-temporal, SGPR base + 32-bit VGPR byte offset.
// The compiler does not track these: consumers must go through wait_ring.
template <int kImm>
__device__ __forceinline__ uint32_t asm_load_dword(const uint8_t* base, uint32_t voff) {
  uint32_t r;
#if PRISMDB_NT_LOADS
  asm volatile("global_load_dword %0, %1, %2 offset:%3 nt" : "=v"(r) : "v"(voff), "s"(base), "n"(kImm));
#else
  asm volatile("global_load_dword %0, %1, %2 offset:%3" : "=v"(r) : "v"(voff), "s"(base), "n"(kImm));
#endif
  return r;
}

// Round j (1..K-1) of a span: immediate offset 256*(j-1) from off1.
template <int K>
__device__ __forceinline__ uint32_t asm_load_dword_at(const uint8_t* base, uint32_t off1, int j) {
  switch (j) {
    case 1: return asm_load_dword<0>(base, off1);
    case 2: return asm_load_dword<256>(base, off1);
    case 3: return asm_load_dword<512>(base, off1);
    case 4: return asm_load_dword<768>(base, off1);
    case 5: return asm_load_dword<1024>(base, off1);
    case 6: return asm_load_dword<1280>(base, off1);
    case 7: return asm_load_dword<1536>(base, off1);
    case 8: return asm_load_dword<1792>(base, off1);
    case 9: return asm_load_dword<2048>(base, off1);
    case 10: return asm_load_dword<2304>(base, off1);
    case 11: return asm_load_dword<2560>(base, off1);
    case 12: return asm_load_dword<2816>(base, off1);
    case 13: return asm_load_dword<3072>(base, off1);
    case 14: return asm_load_dword<3328>(base, off1);
    default: return asm_load_dword<3584>(base, off1);
  }
}

// Wait until this buffer's loads have landed while the kYounger loads issued
// after it (the younger ring buffers) stay in flight; output stores issued in
// between only make the wait stricter, never short.  The buffer registers are
// in/out operands so no consumer can be scheduled above the wait.
template <int kYounger, int N>
__device__ __forceinline__ void wait_ring(uint32_t (&w)[N]) {
  static_assert(N == 16 || N == 8, "ring buffers of 16 (4 KiB chunks) or 8 (2 KiB) words");
  if constexpr (N == 16) {
    asm volatile("s_waitcnt vmcnt(%16)"
                 : "+v"(w[0]), "+v"(w[1]), "+v"(w[2]), "+v"(w[3]), "+v"(w[4]), "+v"(w[5]), "+v"(w[6]),
                   "+v"(w[7]), "+v"(w[8]), "+v"(w[9]), "+v"(w[10]), "+v"(w[11]), "+v"(w[12]),
                   "+v"(w[13]), "+v"(w[14]), "+v"(w[15])
                 : "n"(kYounger)
                 : "memory");
  } else {
    asm volatile("s_waitcnt vmcnt(%8)"
                 : "+v"(w[0]), "+v"(w[1]), "+v"(w[2]), "+v"(w[3]), "+v"(w[4]), "+v"(w[5]), "+v"(w[6]),
                   "+v"(w[7])
                 : "n"(kYounger)
                 : "memory");
  }
}

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// Uniform-address load through the scalar cache (constant address space).
template <typename T>
__device__ __forceinline__ T const_load(const T* p, uint64_t i) {
  typedef const __attribute__((address_space(4))) T CT;
  return ((CT*)p)[i];
}

// A byte through the scalar cache: the aligned dword holding it (s_load has
// no byte form; a plain byte read compiles to a vector load and a vmcnt(0)
// that drains the kernels' load rings).  The dword may reach 3 bytes before
// or after the array: callers' arrays have slack on both sides.
__device__ __forceinline__ uint32_t const_byte(const uint8_t* p, uint64_t i) {
  const uint64_t ad = reinterpret_cast<uint64_t>(p) + i;
  const uint32_t w = const_load(reinterpret_cast<const uint32_t*>(ad & ~3ull), 0);
  return (w >> (8u * (uint32_t)(ad & 3u))) & 255u;
}

__device__ __forceinline__ u32x4 buffer_rsrc(const uint8_t* p, uint32_t bytes) {
  const uint64_t a = reinterpret_cast<uint64_t>(p);
  u32x4 r;
  // wave-uniform by construction; readfirstlane puts it in SGPRs for the "s" operand
  r.x = rfl((uint32_t)a);
  r.y = rfl((uint32_t)(a >> 32) & 0xffffu);  // stride 0: raw buffer
  r.z = rfl(bytes);                          // num_records: offsets >= bytes read as 0
  r.w = 0x00020000u;                         // gfx950 raw-buffer word 3 (cdna_hip_programming.md T8)
  return r;
}

template <int kImm>
__device__ __forceinline__ uint32_t buf_dword(u32x4 rs, uint32_t voff) {
  uint32_t r;
#if PRISMDB_NT_LOADS
  asm volatile("buffer_load_dword %0, %1, %2, 0 offen offset:%3 nt" : "=v"(r) : "v"(voff), "s"(rs), "n"(kImm));
#else
  asm volatile("buffer_load_dword %0, %1, %2, 0 offen offset:%3" : "=v"(r) : "v"(voff), "s"(rs), "n"(kImm));
#endif
  return r;
}

__device__ __forceinline__ uint32_t buf_ubyte(u32x4 rs, uint32_t voff) {
  uint32_t r;
  asm volatile("buffer_load_ubyte %0, %1, %2, 0 offen" : "=v"(r) : "v"(voff), "s"(rs));
  return r;
}

// w[j] = round j at voff + 256 j, j = J..N-1 (immediate offsets).
template <int N, int J = 0>
__device__ __forceinline__ void load_rounds(uint32_t (&w)[N], u32x4 rs, uint32_t voff) {
  if constexpr (J < N) {
    w[J] = buf_dword<256 * J>(rs, voff);
    load_rounds<N, J + 1>(w, rs, voff);
  }
}

// w[j] = round j at v1 + 256 (j - 1), j = J..N-1 (rounds from 1 on one base).
template <int N, int J = 1>
__device__ __forceinline__ void load_rounds_from1(uint32_t (&w)[N], u32x4 rs, uint32_t v1) {
  if constexpr (J < N) {
    w[J] = buf_dword<256 * (J - 1)>(rs, v1);
    load_rounds_from1<N, J + 1>(w, rs, v1);
  }
}

// Wait for a buffer (N body words + edge) with kYounger loads left in flight.
template <int kYounger, int N>
__device__ __forceinline__ void wait_task(uint32_t (&w)[N], uint32_t& e) {
  wait_ring<kYounger>(w);
  asm volatile("" : "+v"(e));
}

// Wave-uniform task (span ordinal q, chunk c); the span's geometry is
// recomputed from (p, len) when needed to keep the SGPR footprint small.
// ---------------------------------------------------------------------------
// Span records (written by crc32c_plan_kernel, one thread per span):
//   x = body address bits 0-31          body = first 4-B aligned byte of the span
//   y = body bits 32-47 | pad << 16 | h << 26 | t << 28 | long << 30
//   z = body bytes (4W)                 W body words, h head bytes, t tail bytes
//   w = register after the head bytes: feed(init ^ ~0, head), computed here
//       bit-serially by the planner thread (the span kernel used to spend
//       3 readlanes and a cross-lane GF(2) product per span on it)
// pad = nch*C - W leading zero words of chunk 0 (nch = ceil(W/C) >= 1), C =
// the consuming kernel's chunk in words (1024; 512 for the log-record kernel).
// ---------------------------------------------------------------------------
// Reflected CRC register fed n bytes, one bit at a time (n <= 3 here).
__device__ __forceinline__ uint32_t feed_bytes(uint32_t r, const uint8_t* p, uint32_t n) {
  for (uint32_t i = 0; i < n; ++i) {
    r ^= p[i];
#pragma unroll
    for (int k = 0; k < 8; ++k) r = (r >> 1) ^ (kPolyReflected & (0u - (r & 1u)));
  }
  return r;
}

// lgc: log2 of the consuming kernel's chunk in words (10: 4 KiB, 9: 2 KiB).
__device__ __forceinline__ SpanRec make_rec(const uint8_t* p, uint32_t len, uint32_t init, bool lng,
                                            uint32_t lgc) {
  uint32_t h = (4u - ((uint32_t)(uintptr_t)p & 3u)) & 3u;
  if (h > len) h = len;
  const uint32_t W = (len - h) >> 2, t = (len - h) & 3u;
  const uint32_t C = 1u << lgc;
  const uint32_t nch = W ? (W + C - 1u) >> lgc : 1u;
  const uint32_t pad = ((nch << lgc) - W) & (C - 1u);  // W == 0: every load is out of range anyway
  const uint64_t body = reinterpret_cast<uint64_t>(p + h);
  SpanRec r;
  r.x = (uint32_t)body;
  r.y = ((uint32_t)(body >> 32) & 0xffffu) | (pad << 16) | (h << 26) | (t << 28) | ((uint32_t)lng << 30);
  r.z = 4u * W;
  r.w = feed_bytes(init ^ kConditioning, p, h);
  return r;
}

// Wave-uniform task: chunk c of the span with record r at index b, which is
// record `slot` of its slice (`last`: the slice's final record).
struct Task {
  uint32_t b;
  SpanRec r;
  uint32_t c;
  uint32_t f;  // slot | last << 8 | valid << 9 | skip << 10: one SGPR, not four
  __device__ uint32_t slot() const { return f & 255u; }
  __device__ bool last() const { return (f >> 8) & 1u; }
  __device__ bool valid() const { return (f >> 9) & 1u; }
  __device__ bool skip() const { return (f >> 10) & 1u; }
  __device__ const uint8_t* body() const {
    return reinterpret_cast<const uint8_t*>(((uint64_t)(r.y & 0xffffu) << 32) | r.x);
  }
  __device__ uint32_t pad() const { return (r.y >> 16) & 1023u; }
  __device__ uint32_t h() const { return (r.y >> 26) & 3u; }
  __device__ uint32_t t() const { return (r.y >> 28) & 3u; }
  __device__ bool lng() const { return (r.y >> 30) & 1u; }
  // ceil(z / chunk) without the 32-bit wrap of z + chunk - 1 (z up to 2^32 - 4)
  __device__ uint32_t nch(uint32_t lgb) const {
    return r.z ? (r.z >> lgb) + ((r.z & ((1u << lgb) - 1u)) != 0u ? 1u : 0u) : 1u;
  }
  __device__ uint32_t len() const { return h() + r.z + t(); }
  __device__ const uint8_t* start() const { return body() - h(); }
};

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
template <bool kVerify, bool kSkip, bool kPairs>
__global__ __launch_bounds__(kThreads) void crc32c_span_kernel(SpanBatch a) {
  // Chunk geometry: 4 KiB chunks of 16 rounds; kRoundsLog for the log-record
  // kernel (crc32c_device.h).
  constexpr int kR = kSkip ? kRoundsLog : kRounds;
  constexpr uint32_t kLgC = kSkip ? kLgChunkWordsLog : 10u;  // log2(chunk words)
  // The log-record kernel skips chunk 0's padding rounds (16-round chunks).
  constexpr bool kRoundSkip = kSkip && PRISMDB_LOG_ROUNDSKIP;
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
  // of 2^lg_tau chunk tasks each (crc32c_slice_kernel), so every stream gets the
  // same work whatever the span sizes and both streams of a wave run out
  // together (dealt equal record counts, config 3's busiest stream had 26 %
  // more tasks than the mean, and a wave folds its two streams in lockstep).  Segment role: slices of kRun records (segments are all but
  // uniform; so are span-role batches whose spans are one task each), kRun =
  // 64 shortened so every stream gets >= PRISMDB_RUNS_PER_STREAM (64) of them:
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
  // Pair runs: the scan found every record one task (nslices = 0), so the
  // wave's two streams advance one record per fold together.  Then they share
  // the wave's runs and take alternate records (stream st: lo + st, lo + st +
  // 2, ...), so a fold reads two adjacent spans, as the fixed kernel's pairs
  // do: streams a run apart (128 KiB) cost the fixed kernel 3.7 %
  // (profiles/r02af_variants_fixed_far_pair.json).  Runs are counted in
  // pairs of records (pq or pq+1 pairs, <= 32, exactly m per wave), so only
  // the batch's last run can be odd, and a run is stored once, when stream
  // 0's last record of it is folded (stream 1's last is in the same fold, or
  // the fold before in an odd last run).
  // The host launches the pair-run kernel (kPairs) next to the general one
  // for large batches (a.pair_kernel); each leaves if the scan's result is
  // the other's.  As one kernel with a runtime switch, the two paths' scalar
  // state spilled SGPRs to scratch.
  constexpr bool pairs = kPairs;
  // (not after a segment-workspace overflow: long spans are then folded here
  // as chains of chunks, but the scan counted them one task each)
  const bool pair_batch = sliced && K == 0 && skip_long;
  if (kPairs ? !pair_batch : (pair_batch && a.pair_kernel != 0u)) return;
  // Runs: K = m S runs of q or q+1 records (q <= 63, runs 0..r-1 the longer),
  // exactly m per stream; m >= PRISMDB_RUNS_PER_STREAM while runs keep >= 1
  // record.  (Runs of 2^lg records left a stream the ceil or floor of K/S.)
  uint32_t rq = 0, rr = 0;
  if (pairs) {
    sliced = false;
    const uint32_t np = (n + 1u) / 2u;  // pairs of records
    const uint32_t rps = (uint32_t)PRISMDB_RUNS_PER_STREAM;
    uint32_t m = (uint32_t)(((uint64_t)np + 31ull * nwaves - 1u) / (31ull * nwaves));  // <= 32 pairs a run
    if (m < rps) {
      const uint32_t mr = np / nwaves;
      m = mr < rps ? (mr > m ? mr : m) : rps;
    }
    if (m < 1u) m = 1u;
    K = (uint64_t)m * nwaves < np ? m * nwaves : np;
    rq = np / K;
    rr = np % K;
  } else if (K == 0) {
    sliced = false;
    const uint32_t rps = (uint32_t)PRISMDB_RUNS_PER_STREAM;
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
  if (PRISMDB_SPAN_WG_EXIT && blockIdx.x * (pairs ? 1u : 2u) * kWavesPerGroup >= K) return;


  __shared__ uint32_t lds[kLdsWords];
  const uint32_t kstep = pairs ? nwaves : S;  // a stream's next run: k + kstep
  constexpr uint32_t bstep = pairs ? 2u : 1u;  // its next record in a run: b + bstep
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
  // first slice or run >= k of stream st with a record for it
  auto open = [&](Cursor& c, uint32_t k, uint32_t st) {
    for (; k < K; k += kstep) {
      uint32_t lo, hi;
      if (sliced) {
        lo = (uint32_t)const_load(a.slice_start, k);
        hi = (uint32_t)const_load(a.slice_start, k + 1);
      } else {
        lo = k * rq + (k < rr ? k : rr);
        hi = lo + rq + (k < rr ? 1u : 0u);
        if (pairs) {  // runs of pairs: records [2 lo, 2 hi)
          lo *= 2u;
          hi *= 2u;
        }
      }
      hi = hi < n ? hi : n;
      const uint32_t b = lo + (pairs ? st : 0u);
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
    if (PRISMDB_SPAN_REC_WAIT) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
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
#if PRISMDB_SPAN_SNOP
    asm volatile("s_nop 4" : "+s"(rb), "+s"(re));
#else
    asm volatile("" : "+s"(rb), "+s"(re));
#endif
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
#if PRISMDB_SPAN_NOEDGE
    (void)re;
    (void)eoff;
    e = 0u;
#else
    e = buf_ubyte(re, eoff);
#endif
  };

  // Per-stream chain state.
  uint32_t acc[2] = {0u, 0u}, r[2] = {0u, 0u};

  // Start of a chunk: the initial register (chunk 0), already fed the head
  // bytes by the planner.  It enters with body word 0: lane pad%64 of round
  // J = pad/64, a wave-uniform index.  J = 0 (full chunks, pads < 64) is one
  // XOR; otherwise a block puts it into round J's word under a scalar mask
  // (v_bitop3 w ^ (inj & m)), no branches per round.  hipcc copies the 16 ring
  // registers out and back around that block on the common path (30 v_mov per
  // span).  PRISMDB_SPAN_INJ_RING 0 returns (inj, J) instead and folds it in
  // (a second copy of the round loop under masks, as kRoundSkip does): no
  // copies, but no faster either (4 KiB descriptors +0.4 %, config-3 mix
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
    const uint32_t J = PRISMDB_SPAN_INJ0 ? 0u : pad >> 6;
    const uint32_t inj = lane == (pad & 63u) ? rr : 0u;
    if (!PRISMDB_SPAN_INJ_RING || kRoundSkip) {
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
  uint32_t res[2] = {0u, 0u}, bad[2] = {0u, 0u};
  auto flush = [&](int s, const Task& t) {
    const uint32_t base = t.b - t.slot();
    if (lane <= t.slot()) {
      if (a.out != nullptr) __builtin_nontemporal_store(res[s], a.out + base + lane);
      if (kVerify && a.mismatch != nullptr) __builtin_nontemporal_store((uint8_t)bad[s], a.mismatch + base + lane);
    }
  };
  // Pair runs: the run ending with stream 0's task t, lanes [0, t.slot() + 1]
  // (those below n), even lanes from stream 0, odd lanes from stream 1.
  auto flush_pair = [&](const Task& t) {
    const uint32_t base = t.b - t.slot();
    if (lane <= t.slot() + 1u && base + lane < n) {
      // by masks, not `odd ? res[1] : res[0]`: hipcc folds that select into
      // res[odd], an indexed array, and moves res and bad to scratch
      const uint32_t odd = 0u - (lane & 1u);
      if (a.out != nullptr) __builtin_nontemporal_store(res[0] ^ ((res[0] ^ res[1]) & odd), a.out + base + lane);
      if (kVerify && a.mismatch != nullptr)
        __builtin_nontemporal_store((uint8_t)(bad[0] ^ ((bad[0] ^ bad[1]) & odd)), a.mismatch + base + lane);
    }
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
    if ((a.flags & kFlagWriteTrailer) && lane == 0)
      store_le32(hdr ? t.start() - kLogCrcBack : t.body() + t.r.z + tl, v);
    if (!pairs && t.last()) flush(s, t);
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
    if ((PRISMDB_SPAN_INJ_RING && !kRoundSkip) || (j0 == 0 && (Jx | Jy) == 0)) {
      // both registers enter in round 0; the ring registers are left untouched
#pragma unroll
      for (int j = PRISMDB_SPAN_J0; j < kR; ++j) {
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
    if (pairs) {
      // the run is complete once stream 0's last record of it is folded
      if (tx.valid() && tx.last()) flush_pair(tx);
    } else {
      // A skipped long span's result comes from the combine pass, but it may
      // close its slice: the slice's other results are stored now.
      if (tx.skip() && tx.valid() && tx.last()) flush(0, tx);
      if (ty.skip() && ty.valid() && ty.last()) flush(1, ty);
    }
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
    open(cur[st], pairs ? wave : 2 * wave + st, (uint32_t)st);
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
  constexpr int kYounger = 2 * (kR + (PRISMDB_SPAN_NOEDGE ? 0 : 1));  // the other slot's two tasks
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
// Fixed-geometry fast path: every span is len bytes at base + i*stride with
// base, stride and len multiples of 4 and len <= 4 KiB, so a span is K rounds
// (K = ceil(len/256), a template parameter) with no head/tail bytes and the
// same padding (pk = 64K - len/4 leading zero words, all in round 0).
// Ring of four span buffers consumed in pairs (loop unrolled x2): the next
// pair's loads are in flight while a pair is folded; counted vmcnt waits only.
// ---------------------------------------------------------------------------
template <int K, bool kVerify>
__global__ __launch_bounds__(kThreads) void crc32c_fixed_kernel(SpanBatch a) {
  constexpr int kRing = PRISMDB_RING;
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
  static_assert(PRISMDB_RUN_LG >= 0 && PRISMDB_RUN_LG <= 5, "a run's results fit the 64 lanes");
  uint32_t lg = PRISMDB_RUN_LG;  // log2(pair steps per run)
  while (lg > 0 && (n >> (lg + 1)) < nwaves * 4u) --lg;
  const uint64_t kRun = 2ull << lg;
  // First span of the wave's next pair step: +2 inside a run, then on to the
  // wave's next run (the other waves' runs in between).
#if PRISMDB_FIXED_FAR_PAIR
  // pair = spans (r0 + i, r0 + kRun/2 + i): two sequential streams half a run apart
  const uint64_t kHalf = kRun / 2u, kSecond = kHalf;
  const uint64_t jump = (nwaves - 1u) * kRun + kHalf + 1u;
  auto adv = [&](uint64_t x) -> uint64_t { return ((x + 1u) & (kHalf - 1u)) ? x + 1u : x + jump; };
#else
  const uint64_t kSecond = 1u;
  const uint64_t jump = (nwaves - 1u) * kRun + 2u;
  auto adv = [&](uint64_t x) -> uint64_t { return ((x + 2u) & (kRun - 1u)) ? x + 2u : x + jump; };
#endif
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
#if PRISMDB_FIXED_NOFOLD  // measurement knob: loads and stores only (wrong results)
#pragma unroll
    for (int j = 1; j < K; ++j) {
      acc_a ^= wa[j];
      acc_b ^= wb[j];
    }
    const uint32_t va = acc_a, vb = acc_b;
#else
#if PRISMDB_FIXED_CHAIN
#pragma unroll
    for (int j = 1; j < K; ++j) acc_a = step256(lds, tab, acc_a, wa[j]);
    acc_b ^= acc_a;  // the second span continues the first's chain (sequential rounds)
#pragma unroll
    for (int j = 1; j < K; ++j) acc_b = step256(lds, tab, acc_b, wb[j]);
#else
#pragma unroll
    for (int j = 1; j < K; ++j) {
      acc_a = step256(lds, tab, acc_a, wa[j]);
      acc_b = step256(lds, tab, acc_b, wb[j]);
    }
#endif
    const uint32_t va = realign(lds, nibtab, acc_a), vb = realign(lds, nibtab, acc_b);
#endif
    const uint32_t ca = wave_xor(va) ^ kConditioning, cb = wave_xor(vb) ^ kConditioning;
#if PRISMDB_FIXED_FAR_PAIR
    const uint32_t i = (uint32_t)(cur & (kHalf - 1u)), i2 = i + (uint32_t)kHalf;  // the pair's lanes in the run
#else
    const uint32_t i = (uint32_t)(cur & (kRun - 1u)), i2 = i + 1u;  // the pair's lanes in the run
#endif
#if PRISMDB_FIXED_DUMMY_SALU
    {  // sensitivity probe: a dependent chain of scalar ALU work
      uint32_t d = i;
      asm volatile(".rept %1\n\ts_xor_b32 %0, %0, 0x5a5a\n\t.endr" : "+s"(d) : "n"(PRISMDB_FIXED_DUMMY_SALU));
    }
#endif
#if PRISMDB_FIXED_DUMMY_VALU
    {  // sensitivity probe: vector ALU work, four independent chains
      uint32_t d0 = lane, d1 = lane + 1u, d2 = lane + 2u, d3 = lane + 3u;
      asm volatile(".rept %4\n\tv_xor_b32 %0, 0x5a5a, %0\n\tv_xor_b32 %1, 0x5a5a, %1\n\tv_xor_b32 %2, 0x5a5a, %2\n\tv_xor_b32 %3, 0x5a5a, %3\n\t.endr"
                   : "+v"(d0), "+v"(d1), "+v"(d2), "+v"(d3) : "n"(PRISMDB_FIXED_DUMMY_VALU / 4));
    }
#endif
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
    const uint32_t last = PRISMDB_FIXED_FAR_PAIR ? (uint32_t)kRun - 1u : (uint32_t)(cur & (kRun - 1u)) + 1u;
    // nt: the results are not re-read; a streaming store keeps them from
    // contending with the read stream (0.6 % of the read rate vs 2 %, probes).
    if (!PRISMDB_FIXED_NOSTORE && lane <= last && b0 + lane < n) {
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
#if PRISMDB_FIXED_SETPRIO  // A/B knob: the pair's loads issued at raised wave priority
      __builtin_amdgcn_s_setprio(PRISMDB_FIXED_SETPRIO);
#endif
      issue(ahead, ring[s]);
      issue(ahead + kSecond, ring[s + 1]);
#if PRISMDB_FIXED_SETPRIO
      __builtin_amdgcn_s_setprio(0);
#endif
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
// Records of the batch: n, or the device count when the batch is the quad
// kernel's list of long spans.
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
  const uint64_t n = batch_n(a);
  const uint64_t lo = (uint64_t)blockIdx.x * ws.tile;
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
#if PRISMDB_PLAN_SERIAL_SEG
    if (sp != nullptr) {
      ws.seg_rec[spos] = make_rec(sp, sfirst, sinit, false, 10u);
      for (uint32_t s = 1; s < snseg; ++s)
        ws.seg_rec[spos + s] = make_rec(sp + sfirst + (uint64_t)(s - 1u) * kSegment, kSegment, kConditioning, false, 10u);
    }
#else
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
#endif
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
// Slice schedule of the span pass.  T tasks in all; slices of tau = 2^lg_tau
// tasks, tau = 64 or smaller so that each of the span kernel's S streams gets
// >= 16 slices; slice k = the records whose first task falls in
// [k*tau, (k+1)*tau), so a slice holds <= tau <= 64 records (every record is
// >= 1 task) and slice_start[k] = first record whose first task is >= k*tau.
//   scan kernel (1 block): exclusive prefix of the planner blocks' sums, T,
//                          lg_tau, nslices, slice_start[0] and [nslices]
//   mark kernel (planner tiles): record i with first task E and c tasks opens
//                          slices (E/tau, (E+c)/tau]: slice_start[k] = i + 1
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
#if PRISMDB_SLICE_EXACT
    // K = m S slices, so every stream gets exactly m of them (dealt s, s+S,
    // ...): with K = ceil(T / 2^lg) a stream got ceil or floor of K/S and the
    // ceil streams set the kernel's end (config 3: 17 slices against a mean of
    // 16.6).  Slice k = tasks [k q + min(k, r), ...) with q = T / K, r = T % K.
    // At most 64 tasks per slice (q <= 63), so at most 64 records (a lane
    // per result); at least 16 slices per stream while they stay >= 32 tasks
    // (a slice of >= 32 tasks always starts a record: spans are <= 32 tasks).
    const uint64_t per = (uint64_t)PRISMDB_SLICES_PER_STREAM;
    uint64_t m = (T + 63u * S - 1u) / (63u * S);
    const uint64_t m32 = T / (32u * S);
    if (m < per && m32 > m) m = m32 < per ? m32 : per;
    if (m < 1u) m = 1u;
    uint64_t K = m * S;
    if (K > T) K = T > 0 ? T : 1u;
    ws.counters->slice_q = T / K;
    ws.counters->slice_r = T % K;
#else
    uint32_t lg = 6;
    while (lg > 0 && (T >> lg) < S * (uint64_t)PRISMDB_SLICES_PER_STREAM) --lg;
    const uint64_t K = (T + (1ull << lg) - 1) >> lg;
    ws.counters->lg_tau = lg;
#endif
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
#if PRISMDB_SLICE_EXACT
  // slice of task position x: slices 0..r-1 hold q+1 tasks, the rest q
  const uint64_t q = ws.counters->slice_q, r = ws.counters->slice_r, rq = r * (q + 1u);
  auto slice_of = [&](uint64_t x) -> uint64_t { return x < rq ? x / (q + 1u) : r + (x - rq) / q; };
#else
  const uint32_t lg = ws.counters->lg_tau;
  auto slice_of = [&](uint64_t x) -> uint64_t { return x >> lg; };
#endif
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
__device__ __forceinline__ uint32_t gf2_apply(const uint32_t* col, uint32_t x) {
  uint32_t y = 0;
#pragma unroll
  for (int i = 0; i < 32; ++i) y ^= col[i] & (0u - ((x >> i) & 1u));
  return y;
}

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
// Short records: the quad kernel (spans of len <= kQuadMaxLen, <= 320 body
// words: log records, small blocks).  The span kernel spends one wave-wide
// fold, realignment, reduction and ~190 scalar instructions per ~1 KB record
// (profiles/r01_wal_pmc); here a wave takes FOUR records at a time:
//   * DPP row g = lane >> 4 (16 lanes) takes record 4q + g of the wave's run
//     of 64 consecutive records (runs dealt round-robin to the waves);
//   * lane j of the row runs four 256-B-stride sub-streams k = 0..3: virtual
//     lane v = 16 (k ^ (g & 1)) + j of a 64-lane frame.  So the stride
//     tables, the fold and lane v's realignment tables are the other
//     kernels' (odd rows take their sub-streams in swapped pairs: the
//     realignment lookups of rows 0/1 and 2/3 then hit different banks);
//   * a frame is kQuadRounds rounds of 64 words with the record's body
//     right-aligned (word i at frame position P + i, P = 320 - W), loaded
//     with one dword per sub-stream and round: 20 loads per lane per task,
//     addresses clamped into the record; the positions before P are zeroed
//     at fold time, where the register after the head bytes enters with
//     body word 0 (position P).  Rounds before the task's longest record are
//     not folded;
//   * head bytes, tail bytes and the stored crc ride in one byte load per
//     lane (quads 0, 1, 2 of the row) and are fed with 16-lane GF(2)
//     products: shift_t is a 32x32 matrix, lane j holds columns 2j, 2j+1;
//   * the row's CRC is one DPP row reduction; lane i of the run collects
//     record i's result (ds_bpermute) for one coalesced store per run.
// Per record that is one scalar descriptor read and a quarter of the fold's
// fixed costs.  Spans longer than kQuadMaxLen are left to the generic path
// (crc32c_long_list_kernel lists them); this kernel stores a placeholder for
// them that the scatter pass overwrites.
// ---------------------------------------------------------------------------

// Columns 2j and 2j+1 of shift_1, shift_2, shift_3 (t zero bytes) for the
// row products.
struct RowShift {
  uint32_t c[3][2];
};

__device__ __forceinline__ RowShift row_shift_cols(uint32_t j) {
  RowShift s;
#pragma unroll
  for (int b = 0; b < 2; ++b) {
    uint32_t c = 1u << (2u * j + (uint32_t)b);
#pragma unroll
    for (int t = 0; t < 3; ++t) {
#pragma unroll
      for (int k = 0; k < 8; ++k) c = (c >> 1) ^ (kPolyReflected & (0u - (c & 1u)));
      s.c[t][b] = c;
    }
  }
  return s;
}

// shift_t(x), t = 0..3, for x and t uniform within each 16-lane row: lane j
// contributes columns 2j and 2j+1 of shift_t selected by bits 2j, 2j+1 of x,
// and the row XOR-reduces (every lane of the row gets the product).  One
// product, not t products of shift_1: the DPP reduction is a dependent chain,
// and the kernel stalls on such chains, not on its instruction count.
__device__ __forceinline__ uint32_t row_shift(const RowShift& s, uint32_t j, uint32_t x, uint32_t t) {
  // selected with masks: a ternary chain here compiles to an indexed (scratch) array
  const uint32_t m1 = t == 1u ? ~0u : 0u, m2 = t == 2u ? ~0u : 0u, m3 = t == 3u ? ~0u : 0u;
  const uint32_t c0 = (s.c[0][0] & m1) | (s.c[1][0] & m2) | (s.c[2][0] & m3);
  const uint32_t c1 = (s.c[0][1] & m1) | (s.c[1][1] & m2) | (s.c[2][1] & m3);
  const uint32_t b = x >> (2u * j);
  const uint32_t y = row_xor(((b & 1u) ? c0 : 0u) ^ ((b & 2u) ? c1 : 0u));
  return t ? y : x;
}

// Lane n of the row, broadcast to the row (DPP row_newbcast).
template <int kN>
__device__ __forceinline__ uint32_t row_bcast(uint32_t v) {
  return __builtin_amdgcn_update_dpp(0u, v, 0x150 + kN, 0xF, 0xF, false);
}

// Inline-asm loads at a per-task scalar base + 32-bit per-lane offset;
// retired by wait_quad.
__device__ __forceinline__ uint32_t asm_load_dword_s(const uint8_t* sbase, uint32_t voff) {
  uint32_t r;
#if PRISMDB_NT_LOADS
  asm volatile("global_load_dword %0, %1, %2 nt" : "=v"(r) : "v"(voff), "s"(sbase));
#else
  asm volatile("global_load_dword %0, %1, %2" : "=v"(r) : "v"(voff), "s"(sbase));
#endif
  return r;
}

// Body word min(i + kAdd, wm1) of the record at sbase + bw: the index clamp,
// the address and the load in one asm block, so hipcc cannot compute the 20
// addresses of a task ahead of its loads (20 live VGPRs).  A VALU-written
// VGPR read by the load right after it is interlocked (no wait states).
template <int kAdd>
__device__ __forceinline__ uint32_t asm_load_word_clamped(const uint8_t* sbase, uint32_t bw, uint32_t i,
                                                          uint32_t wm1) {
  uint32_t r, a;
#if PRISMDB_NT_LOADS
  asm volatile(
      "v_add_u32 %1, %5, %2\n\t"
      "v_min_u32 %1, %1, %3\n\t"
      "v_lshl_add_u32 %1, %1, 2, %4\n\t"
      "global_load_dword %0, %1, %6 nt"
      : "=&v"(r), "=&v"(a)
      : "v"(i), "v"(wm1), "v"(bw), "n"(kAdd), "s"(sbase));
#else
  asm volatile(
      "v_add_u32 %1, %5, %2\n\t"
      "v_min_u32 %1, %1, %3\n\t"
      "v_lshl_add_u32 %1, %1, 2, %4\n\t"
      "global_load_dword %0, %1, %6"
      : "=&v"(r), "=&v"(a)
      : "v"(i), "v"(wm1), "v"(bw), "n"(kAdd), "s"(sbase));
#endif
  return r;
}

template <int M, int K>
__device__ __forceinline__ void quad_round_loads(uint32_t (&w)[kQuadRounds][4], const uint8_t* sbase, uint32_t bw,
                                                 const uint32_t (&i0)[4], uint32_t wm1) {
  if constexpr (M < kQuadRounds) {
    w[M][K] = asm_load_word_clamped<64 * M>(sbase, bw, i0[K], wm1);
    if constexpr (K == 3) quad_round_loads<M + 1, 0>(w, sbase, bw, i0, wm1);
    else quad_round_loads<M, K + 1>(w, sbase, bw, i0, wm1);
  }
}

// Body word max(i + 64 M, 0) of the record whose body is at sbase + bw, with
// ad = bw + 4 i and lo = bw - 256 M: the address is max(ad, lo) + 256 M, one
// VALU and the load's immediate offset (a position before the body reads
// body word 0).  ad and lo never wrap: bw >= kQuadBack (quad_window).
template <int M>
__device__ __forceinline__ uint32_t asm_load_word_max(const uint8_t* sbase, uint32_t ad, uint32_t lo) {
  uint32_t r, x;
#if PRISMDB_NT_LOADS
  asm volatile(
      "v_max_u32 %1, %2, %3\n\t"
      "global_load_dword %0, %1, %4 offset:%5 nt"
      : "=&v"(r), "=&v"(x)
      : "v"(ad), "v"(lo), "s"(sbase), "n"(256 * M));
#else
  asm volatile(
      "v_max_u32 %1, %2, %3\n\t"
      "global_load_dword %0, %1, %4 offset:%5"
      : "=&v"(r), "=&v"(x)
      : "v"(ad), "v"(lo), "s"(sbase), "n"(256 * M));
#endif
  return r;
}

template <int M, int K>
__device__ __forceinline__ void quad_round_loads_max(uint32_t (&w)[kQuadRounds][4], const uint8_t* sbase,
                                                     const uint32_t (&ad)[4], const uint32_t (&lo)[kQuadRounds]) {
  if constexpr (M < kQuadRounds) {
    w[M][K] = asm_load_word_max<M>(sbase, ad[K], lo[M]);
    if constexpr (K == 3) quad_round_loads_max<M + 1, 0>(w, sbase, ad, lo);
    else quad_round_loads_max<M, K + 1>(w, sbase, ad, lo);
  }
}

__device__ __forceinline__ uint32_t asm_load_ubyte_v(uint64_t addr) {
  uint32_t r;
  asm volatile("global_load_ubyte %0, %1, off" : "=v"(r) : "v"(addr));
  return r;
}

// Wait for one task's 20 body words and its edge byte with kYounger loads
// (the younger tasks) left in flight; the registers are in/out operands so no
// consumer is scheduled above the wait.
template <int kYounger>
__device__ __forceinline__ void wait_quad(uint32_t (&w)[kQuadRounds][4], uint32_t& e) {
  static_assert(kQuadRounds == 5, "20 body words per task");
  asm volatile("s_waitcnt vmcnt(%21)"
               : "+v"(w[0][0]), "+v"(w[0][1]), "+v"(w[0][2]), "+v"(w[0][3]), "+v"(w[1][0]), "+v"(w[1][1]),
                 "+v"(w[1][2]), "+v"(w[1][3]), "+v"(w[2][0]), "+v"(w[2][1]), "+v"(w[2][2]), "+v"(w[2][3]),
                 "+v"(w[3][0]), "+v"(w[3][1]), "+v"(w[3][2]), "+v"(w[3][3]), "+v"(w[4][0]), "+v"(w[4][1]),
                 "+v"(w[4][2]), "+v"(w[4][3]), "+v"(e)
               : "n"(kYounger)
               : "memory");
}

// A task's window.  Its four records (4-aligned indices tb .. tb+3, those
// below n) are read through one scalar base sb: the first short record A
// anchors it, sb = address(A) - kQuadBack - min(2^30, address(A) - kQuadBack),
// and a short record is the quad kernel's if it starts at least kQuadBack
// bytes into the window (the body-address arithmetic reaches that far below
// a body, unsigned) and every byte it touches (trailer after) lies below
// sb + 2^31 - 2048; any other short record is listed for the generic path
// like a long one.  Offsets from sb then fit 31
// bits, so the kernel computes them in 32 bits.  The list kernel and the quad
// kernel evaluate this same function.
struct QuadWindow {
  uint64_t sb;
  uint32_t mask;  // bit q: record tb + q is the quad kernel's
};

__device__ __forceinline__ QuadWindow quad_window(const uint8_t* base, const uint64_t (&off)[4],
                                                  const uint32_t (&len)[4], uint32_t valid) {
  uint32_t sh = 0u;
#pragma unroll
  for (int q = 0; q < 4; ++q) sh |= (((valid >> q) & 1u) && len[q] <= kQuadMaxLen ? 1u : 0u) << q;
  QuadWindow w{0u, 0u};
  if (sh == 0u) return w;
  const int A = __builtin_ctz(sh);
  uint64_t oa = off[0];
#pragma unroll
  for (int q = 1; q < 4; ++q) oa = A == q ? off[q] : oa;
  const uint64_t aa = reinterpret_cast<uint64_t>(base) + oa - kQuadBack;
  w.sb = aa - (aa < (1ull << 30) ? aa : (1ull << 30));
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const uint64_t d = reinterpret_cast<uint64_t>(base) + off[q] - w.sb;  // >= kQuadBack when in the window
    if (((sh >> q) & 1u) && d >= kQuadBack && d < (1ull << 31) - 2048u) w.mask |= 1u << q;
  }
  return w;
}

// Wave-uniform task: records tb .. tb+3, the scalar base and the fold bounds.
struct QuadTask {
  uint32_t tb;
  const uint8_t* sbase;  // body-word loads: the window base, or `zero` when no row has body words
  const uint8_t* sb;     // the window base (edge bytes, trailers)
  uint32_t u;  // fold bounds and flags, below
};
// u = m0 | mp << 4 | max h << 8 | max t << 10 | any bodyless record << 12
constexpr uint32_t kQuadAnyW0 = 1u << 12;
constexpr uint32_t kQuadOwned = 1u << 13;  // the kernel owns at least one of the task's records

template <bool kVerify>
__global__ __launch_bounds__(kThreads) void crc32c_quad_kernel(SpanBatch a) {
  // record indices in 32 bits: the host cuts batches at kMaxGenericSpans (2^30)
  const uint32_t n = (uint32_t)a.n;
  __shared__ uint32_t lds[kLdsWords];
  const uint32_t tid = threadIdx.x;
  load_tables(lds, a.tabs, tid);
  const uint32_t lane = tid & 63u, g = lane >> 4, j = lane & 15u;
  __syncthreads();
  const StrideLanes tab = stride_lanes(lane);
  const RowShift rsh = row_shift_cols(j);
  // sub-stream k = virtual lane 16 (k ^ (g & 1)) + j; its realignment entry
  uint32_t nib[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) nib[k] = 4u * ((uint32_t)kTabWords + 16u * ((uint32_t)k ^ (g & 1u)) + j);
  auto vlane = [&](int k) -> uint32_t { return (nib[k] >> 2) - (uint32_t)kTabWords; };
  const uint32_t wave = rfl(blockIdx.x * kWavesPerGroup + (tid >> 6));
  const uint32_t nwaves = gridDim.x * kWavesPerGroup;
  // Runs of 64 records (16 tasks), run r of wave w = records [(r nwaves + w) 64, +64).
  // (tb < n + 64 nwaves always, far below 2^32.)
  // Runs the quad kernel owns nothing of (ws-side flags from the list
  // kernel, read through the scalar cache) are skipped whole.
  const uint8_t* const qrun = a.qrun;
  auto next_run = [&](uint32_t rb) -> uint32_t {  // first owned run at or after rb, its first record
    while (rb < n && const_byte(qrun, (uint64_t)(rb >> 6)) == 0u) rb += 64u * nwaves;
    return rb;
  };
  auto adv = [&](uint32_t tb) -> uint32_t {
    return ((tb + 4u) & 63u) ? tb + 4u : next_run((tb & ~63u) + 64u * nwaves);
  };
  uint32_t cur = next_run(wave * 64u);
  if (cur >= n) return;
  const bool hdr = (a.flags & kFlagLogHeader) != 0;
  const uint8_t* const zero = reinterpret_cast<const uint8_t*>(&a.tabs->zero[0]) + 256u * (wave & 255u);

  // The lane's row's value out of four uniform ones.
  auto sel = [&](uint32_t x0, uint32_t x1, uint32_t x2, uint32_t x3) -> uint32_t {
    const uint32_t lo = (lane & 16u) ? x1 : x0, hi = (lane & 16u) ? x3 : x2;
    return (lane & 32u) ? hi : lo;
  };
  // Issue task tb: descriptors (scalar), the lane's row geometry (vector),
  // the fold bounds (four readlanes), 21 loads.
  // vmeta = W | P << 9 | h << 18 | t << 20 | ok << 22 | edge-byte-used << 23;
  // vpo = offset of the record's first byte from sbase.  (The init values
  // are read at fold time: one VGPR less per ring slot.)
  // A task's four descriptors, read through the scalar cache one task ahead
  // (before the wait for the slot being folded, so the read's latency hides
  // behind that wait instead of stalling issue()).
  struct QuadDesc {
    uint64_t off[4];
    uint32_t len[4], valid;
  };
  auto fetch = [&](uint32_t tb) -> QuadDesc {
    QuadDesc d;
    if (tb + 4u <= n) {  // one contiguous scalar read per array
      d.valid = 15u;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        d.off[q] = const_load(a.off + tb, (uint64_t)q);
        d.len[q] = const_load(a.len + tb, (uint64_t)q);
      }
    } else {  // the batch's last task (or past it): clamped reads
      const uint32_t last = n - 1u;
      d.valid = 0u;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const uint32_t i = tb + (uint32_t)q < last ? tb + (uint32_t)q : last;
        d.off[q] = const_load(a.off, i);
        d.len[q] = const_load(a.len, i);
        d.valid |= (tb + (uint32_t)q < n ? 1u : 0u) << q;
      }
    }
    return d;
  };
  auto issue = [&](uint32_t tb, const QuadDesc& d, uint32_t (&w)[kQuadRounds][4], uint32_t& e, QuadTask& tk,
                   uint32_t& vmeta, uint32_t& vpo) {
    const uint64_t(&off)[4] = d.off;
    const uint32_t(&len)[4] = d.len;
    const QuadWindow win = quad_window(a.base, off, len, d.valid);
    tk.tb = tb;
    tk.sb = reinterpret_cast<const uint8_t*>(win.sb);
    // the row's record in 32 bits: its offset from sbase fits 31 bits
    const uint32_t base_sb = (uint32_t)reinterpret_cast<uint64_t>(a.base) - (uint32_t)win.sb;
    const uint32_t ln = sel(len[0], len[1], len[2], len[3]);
    const bool ok = (win.mask >> g) & 1u;
    vpo = ok ? base_sb + sel((uint32_t)off[0], (uint32_t)off[1], (uint32_t)off[2], (uint32_t)off[3]) : 8u;
    // head bytes up to 4-B alignment of the absolute address (none with
    // unaligned body loads: the body starts at the record's first byte)
    uint32_t h = PRISMDB_QUAD_UNALIGNED ? 0u : (0u - ((uint32_t)win.sb + vpo)) & 3u;
    h = h < ln ? h : ln;
    uint32_t W = (ln - h) >> 2, t = (ln - h) & 3u;
    if (!ok) W = h = t = 0u;
    const uint32_t P = kQuadWords - W;
    vmeta = W | (P << 9) | (h << 18) | (t << 20) | ((uint32_t)ok << 22);
    // fold bounds: rounds from 5 - Rmax, masked through mp (rows without
    // body words read someone else's bytes: all rounds masked); flags
    const uint32_t R = (W + 63u) >> 6, mpv = W ? P >> 6 : (uint32_t)kQuadRounds;
    const uint32_t pk = R | (mpv << 4) | (h << 8) | (t << 10) | (ok && W == 0u ? kQuadAnyW0 : 0u);
    const uint32_t p0 = readlane(pk, 0), p1 = readlane(pk, 16), p2 = readlane(pk, 32), p3 = readlane(pk, 48);
    auto fmax = [&](int sh, uint32_t m) {
      return max(max((p0 >> sh) & m, (p1 >> sh) & m), max((p2 >> sh) & m, (p3 >> sh) & m));
    };
    const uint32_t rmax = fmax(0, 15u), mp = fmax(4, 15u);
    tk.u = ((uint32_t)kQuadRounds - rmax) | (mp << 4) | (fmax(8, 3u) << 8) | (fmax(10, 3u) << 10) |
           ((p0 | p1 | p2 | p3) & kQuadAnyW0) | (win.mask ? kQuadOwned : 0u);
    // Body words: frame position 64 m + v is body word 64 m + v - P, clamped
    // into the record (the fold zeroes the words outside it; a frame ends at
    // its record's last body word).  A row without
    // body words reads the first body word of the first row that has some
    // (every address read is inside a record), or the zero block if none has.
    const uint32_t bo = vpo + h;  // body offset
    const uint32_t rows_w = ((p0 & 15u) ? 1u : 0u) | ((p1 & 15u) ? 2u : 0u) | ((p2 & 15u) ? 4u : 0u) |
                            ((p3 & 15u) ? 8u : 0u);
    // (no body words anywhere: every load reads the zero slot at bw = kQuadBack)
    tk.sbase = rows_w ? tk.sb : zero - kQuadBack;
    const uint32_t safe = rows_w ? readlane(bo, 16u * (uint32_t)__builtin_ctz(rows_w)) : kQuadBack;
    const uint32_t wm1 = W ? W - 1u : 0u;
    const uint32_t bw = W ? bo : safe;
    // sub-stream k's body index in round 0; opaque, so that hipcc does not
    // hoist the 20 loop-invariant v + 64 m out of the task loop (20 VGPRs)
    uint32_t i0[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      i0[k] = vlane(k) - P;
      asm volatile("" : "+v"(i0[k]));
    }
#if PRISMDB_QUAD_CLAMPED
    quad_round_loads<0, 0>(w, tk.sbase, bw, i0, wm1);
#else
    // 4 + 4 address VALUs and one v_max per load (three per load clamped)
    uint32_t ad[4], lo[kQuadRounds];
#pragma unroll
    for (int k = 0; k < 4; ++k) ad[k] = bw + 4u * i0[k];
#pragma unroll
    for (int m = 0; m < kQuadRounds; ++m) lo[m] = bw - 256u * (uint32_t)m;
    (void)wm1;
    quad_round_loads_max<0, 0>(w, tk.sbase, ad, lo);
#endif
    // Edge byte: quad 0 of the row loads head byte o (o < h), quad 1 tail
    // byte o (o < t), quad 2 stored-crc byte o (verify); the rest are masked.
    const uint32_t qd = j >> 2, o = j & 3u;
    bool ev = false;
    uint32_t eo = vpo;
    if (qd == 0u) {
      ev = o < h;
      eo = vpo + o;
    } else if (qd == 1u) {
      ev = o < t;
      eo = bo + 4u * W + o;
    } else if (qd == 2u) {
      ev = kVerify && ok;
      eo = hdr ? vpo - kLogCrcBack + o : bo + 4u * W + t + o;
    }
    vmeta |= (ev ? 1u : 0u) << 23;
    // 64-bit address: an unused lane reads the zero block, not a byte of the window
    e = asm_load_ubyte_v(ev ? reinterpret_cast<uint64_t>(tk.sb) + eo : reinterpret_cast<uint64_t>(zero));
  };

  uint32_t res = 0u, bad = 0u;
  auto fold = [&](const QuadTask& tk, const uint32_t (&w)[kQuadRounds][4], uint32_t e, uint32_t vmeta,
                  uint32_t vpo) {
    const uint32_t W = vmeta & 511u, P = (vmeta >> 9) & 511u, h = (vmeta >> 18) & 3u, t = (vmeta >> 20) & 3u;
    const bool ok = (vmeta >> 22) & 1u;
    const uint32_t m0 = tk.u & 15u, mp = (tk.u >> 4) & 15u;
    // Edge words: each quad ORs its bytes (disjoint), rows broadcast quad 0
    // (head), quad 1 (tail), quad 2 (stored crc).
    uint32_t ew = ((vmeta >> 23) & 1u) ? e << (8u * (j & 3u)) : 0u;
    ew = xor_dpp(xor_dpp(ew, 0xB1), 0x4E);
    uint32_t r = kConditioning;  // register before the head bytes: init ^ ~0
    if (a.init != nullptr) {
      uint32_t iv[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) iv[q] = const_load(a.init, tk.tb + (uint32_t)q < n ? tk.tb + (uint32_t)q : n - 1u);
      r ^= sel(iv[0], iv[1], iv[2], iv[3]);
    }
    const uint32_t hmax = (tk.u >> 8) & 3u, tmax = (tk.u >> 10) & 3u;
    if (hmax) r = row_shift(rsh, j, r ^ row_bcast<0>(ew), h);
    uint32_t acc[4] = {0u, 0u, 0u, 0u};
    uint32_t i0[4];  // as in issue(): opaque per-task indices
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      i0[k] = vlane(k) - P;
      asm volatile("" : "+v"(i0[k]));
    }
#pragma unroll
    for (int m = 0; m < kQuadRounds; ++m) {
      if ((uint32_t)m < m0) continue;
      if (!PRISMDB_QUAD_NOMASK && (uint32_t)m <= mp) {
        // positions before the body read 0, body word 0 carries the register
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const uint32_t idx = i0[k] + 64u * (uint32_t)m;
          const uint32_t inj = idx == 0u ? r : 0u;
          const uint32_t keep = idx < W ? ~0u : 0u;
          acc[k] = step256(lds, tab, acc[k], __builtin_amdgcn_bitop3_b32(w[m][k], inj, keep, 0x28));
        }
      } else {
#pragma unroll
        for (int k = 0; k < 4; ++k) acc[k] = step256(lds, tab, acc[k], w[m][k]);
      }
    }
    // one sub-stream's eight lookups at a time (the memory clobber keeps the
    // next batch of LDS reads below): 32 in flight at once cost 24 spilled VGPRs
    // A task of records all left to the generic path folds no round (its
    // rows have no body words) and skips the realignment as well.
    uint32_t x = 0u;
    if (tk.u & kQuadOwned) {
#if PRISMDB_QUAD_NOREALIGN
      x = xor3(acc[0], acc[1], acc[2]) ^ acc[3];
#else
      x = realign(lds, nib[0], acc[0]);
#pragma unroll
      for (int k = 1; k < 4; ++k) {
        if (k % (4 / PRISMDB_QUAD_RALIGN_GROUPS) == 0) asm volatile("" ::: "memory");
        x ^= realign(lds, nib[k], acc[k]);
      }
#endif
      x = row_xor(x);
    }
    if (tk.u & kQuadAnyW0) x = W == 0u ? r : x;  // no body words: the register after the head
    if (tmax) x = row_shift(rsh, j, x ^ row_bcast<4>(ew), t);
    const uint32_t crc = x ^ kConditioning;
    const uint32_t v = (a.flags & kFlagMask) ? mask_crc(crc) : crc;
    if ((a.flags & kFlagWriteTrailer) && ok && j == 0u)
      store_le32(tk.sb + (hdr ? vpo - kLogCrcBack : vpo + h + 4u * W + t), v);
    // Lane i of the run collects record i: task tir's rows go to lanes 4 tir .. 4 tir + 3.
    const uint32_t tir = (tk.tb >> 2) & 15u;
    const int src = (int)((lane & 3u) << 6);  // byte address of lane 16 (lane & 3)
    const bool mine = (lane >> 2) == tir;
    const uint32_t gv = (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)v);
    res = mine ? gv : res;
    if (kVerify) {
      const uint32_t bd = crc != unmask_crc(row_bcast<8>(ew)) ? 1u : 0u;
      const uint32_t gb = (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)bd);
      bad = mine ? gb : bad;
    }
    // Run end: one coalesced store of the run's results (placeholders for
    // listed spans, rewritten by the scatter pass).
    if (tir == 15u || tk.tb + 4u >= n) {
      // the record index is opaque so hipcc does not keep a.out + lane and
      // a.mismatch + lane live across the loop (64-bit pointers per lane)
      uint32_t rec = (tk.tb & ~63u) + lane;
      asm volatile("" : "+v"(rec));
      if (rec < n) {
        if (a.out != nullptr) __builtin_nontemporal_store(res, a.out + rec);
        if (kVerify && a.mismatch != nullptr) __builtin_nontemporal_store((uint8_t)bad, a.mismatch + rec);
      }
    }
  };

  // Ring of kRing tasks, compile-time slots: fold one while the others are in flight.
  constexpr int kRing = PRISMDB_QUAD_RING;
  constexpr int kYounger = (kRing - 1) * (4 * kQuadRounds + 1);
  static_assert(kYounger <= 63, "vmcnt is a 6-bit counter");
  uint32_t wq[kRing][kQuadRounds][4];
  uint32_t eq[kRing];
  QuadTask tq[kRing];
  uint32_t vm[kRing], vp[kRing];
  uint32_t ahead = cur;
#pragma unroll
  for (int d = 0; d < kRing; ++d) {
    issue(ahead, fetch(ahead), wq[d], eq[d], tq[d], vm[d], vp[d]);
    ahead = adv(ahead);
  }
  for (;;) {
#pragma unroll
    for (int sl = 0; sl < kRing; ++sl) {
      const QuadDesc nd = fetch(ahead);  // ahead of the wait (its memory clobber keeps it there)
      wait_quad<kYounger>(wq[sl], eq[sl]);
      if (tq[sl].tb < n) fold(tq[sl], wq[sl], eq[sl], vm[sl], vp[sl]);
      cur = adv(cur);
      issue(ahead, nd, wq[sl], eq[sl], tq[sl], vm[sl], vp[sl]);
      ahead = adv(ahead);
    }
    if (cur >= n) break;
  }
  // Retire the tasks still in flight while their registers are live.
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
  for (int d = 0; d < kRing; ++d) {
#pragma unroll
    for (int m = 0; m < kQuadRounds; ++m) {
#pragma unroll
      for (int k = 0; k < 4; ++k) asm volatile("" : "+v"(wq[d][m][k]));
    }
    asm volatile("" : "+v"(eq[d]));
  }
}

// ---------------------------------------------------------------------------
// Short records, one per lane (crc32c_lane_kernel).  Log records (~1 KB) are
// too short for a wave-wide fold: the span kernel spends a realignment, a
// reduction and ~190 scalar instructions on each, the quad kernel (above)
// still a quarter of that plus masked rounds.  Here lane i of a wave runs the
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
// start) and tasks past the run's shortest record fold under per-word masks,
// the others unmasked; a lane past its record re-reads its last line.
//
// Load order inside an issue: the next run's descriptors (first task of a
// run), the edge dwords (first / last task), then the eight body loads, so
// the body loads of the other slot are always the youngest eight: after a
// vmcnt(8) wait every descriptor and edge load issued so far has landed.
// ---------------------------------------------------------------------------
// Lane kernel workgroup (PRISMDB_LANE_THREADS): one group per CU either way
// (the tables take 128 KiB of LDS).  8 waves per CU read 11.7 % faster than 16
// and 4 % faster than 12 (WAL verify; profiles/r02s3n, r02s3o): each lane's
// line is read by eight 16-B loads, and fewer waves keep fewer lines in flight
// in the CU's vector L1 between them; 4 waves hide too little latency (-27 %).
constexpr uint32_t kLaneThreads = PRISMDB_LANE_THREADS;

__device__ __forceinline__ void load_slice_tables(uint32_t* lds, const DeviceTables* tabs, uint32_t tid) {
  for (uint32_t w = tid; w < (uint32_t)kTabWords; w += kLaneThreads) {
    const uint32_t k = ((w >> 14) << 1) | ((w >> 5) & 1u), e = (w >> 6) & 255u;
    lds[w] = tabs->slice4[k][e];
  }
}

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

// Wave-uniform task: run of records [rb, rb + 64), its 128-B task k of K, the
// first kf unmasked; nrb: the wave's next owned run.
struct LaneTask {
  uint32_t rb, k, kf, K, nrb;
};

template <int kOp>  // 0: max, 1: min
__device__ __forceinline__ uint32_t wave_reduce(uint32_t v) {
  auto f = [](uint32_t x, uint32_t y) { return kOp == 0 ? (x > y ? x : y) : (x < y ? x : y); };
  v = f(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0xB1, 0xF, 0xF, false));  // quad_perm 1,0,3,2
  v = f(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x4E, 0xF, 0xF, false));  // quad_perm 2,3,0,1
  v = f(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x141, 0xF, 0xF, false)); // row_half_mirror
  v = f(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x140, 0xF, 0xF, false)); // row_mirror
  return f(f(readlane(v, 0), readlane(v, 16)), f(readlane(v, 32), readlane(v, 48)));
}

template <bool kVerify>
__global__ __launch_bounds__(kLaneThreads) void crc32c_lane_kernel(SpanBatch a) {
  const uint32_t n = (uint32_t)a.n;  // host cuts batches at kMaxGenericSpans (2^30)
  __shared__ uint32_t lds[kTabWords];
  const uint32_t tid = threadIdx.x;
  load_slice_tables(lds, a.tabs, tid);
  const uint32_t lane = tid & 63u;
  __syncthreads();
  const StrideLanes tab = stride_lanes(lane);
  const uint32_t wave = rfl(blockIdx.x * (kLaneThreads / 64u) + (tid >> 6));
  const uint32_t nwaves = gridDim.x * (kLaneThreads / 64u);
  const uint8_t* const qrun = a.qrun;
  auto next_run = [&](uint32_t rb) -> uint32_t {  // first owned run at or after rb
    while (rb < n && const_byte(qrun, (uint64_t)(rb >> 6)) == 0u) rb += 64u * nwaves;
    return rb;
  };
  const uint32_t first = next_run(wave * 64u);
  if (first >= n) return;
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
      uint32_t K = wave_reduce<0>(vkend);
      uint32_t kf = wave_reduce<1>(owned ? qe >> 5 : 0xFFFFu);
      t.K = K;
      t.kf = kf < K ? kf : K;
      t.nrb = next_run(t.rb + 64u * nwaves);
    }
    // Side loads: the next run's descriptors with a run's first task, the
    // head dword with it, the end dword and the stored crc with its last.
    // The verify kernel issues them only there (WAL verify +6.8 % against
    // issuing them with every task, from a zero region when unused:
    // profiles/r02s3w_*); the sealing kernel issues them with every task
    // (2.5 % faster that way in the same A/B).  Loads written under branches:
    // at 16 waves hipcc, short of VGPRs, copied such registers at the merge
    // before their wait; the CFG audit run by build() fails on any such touch,
    // and this build has none.
    constexpr bool kSideAlways = !kVerify;
    const bool live = t.rb < n;
    const bool owned = live && ((vmeta >> 25) & 1u);
    const bool lastk = t.k + 1u == t.K;
    if (kSideAlways || t.k == 0) fetch_desc(t.nrb);
    VP[sl] = vp;
    META[sl] = live ? vmeta : 0u;
    INIT[sl] = vinit;
    if (kSideAlways || t.k == 0) HD[sl] = asm_load_u32(owned && t.k == 0 ? vp & ~3ull : zero);
    if (kSideAlways || lastk) {
      ED[sl] = asm_load_u32(owned && lastk ? vp + vlen - 4u : zero);
      if (kVerify) SC[sl] = asm_load_u32(owned && lastk ? (hdr ? vp - kLogCrcBack : vp + vlen) : zero);
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
      u.kf = 0;
    }
    return u;
  };

  uint32_t acc = 0;
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
    if (PRISMDB_LANE_NOFOLD) {
#pragma unroll
      for (int i = 0; i < 32; ++i) x ^= w[i >> 2][i & 3];
    } else if (t.k == 0) {
      // the head bytes, then the body from word q0 of the line: the register
      // enters with body word 0
      const uint32_t h = (meta >> 21) & 3u;
      const uint32_t hb = HD[sl] >> (8u * ((4u - h) & 3u));  // the record's first bytes
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
    } else if (t.k < t.kf) {
#pragma unroll
      for (int i = 0; i < 32; ++i) x = step256(lds, tab, x, w[i >> 2][i & 3]);
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
      const uint32_t fb = tb ? ED[sl] >> (8u * (4u - tb)) : 0u;  // the record's last tb bytes
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
          __builtin_nontemporal_store((uint8_t)(crc != unmask_crc(SC[sl]) ? 1u : 0u), a.mismatch + rec);
      }
    }
  };

  LaneTask tk[2];
  tk[0] = LaneTask{first, 0u, 0u, 1u, n};
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

// The spans the quad kernel leaves to the generic path (len > kQuadMaxLen, or
// outside their task's window), listed run by run (a wave's 64 consecutive
// spans stay together and in order); ws.counters->nlist is the count.  One
// atomic per block of 16 runs (one per run serialized on the counter: 790 us
// for 64 Ki runs).  ws.qrun[r] = 1 if the quad kernel owns a span of run r:
// it skips the other runs.
template <bool kLane>  // kLane: the lane kernel's criterion (lane_owns), else the quad kernel's window
__global__ __launch_bounds__(kListThreads) void crc32c_long_list_kernel(SpanBatch a, SplitWs ws) {
  const uint64_t n = a.n;
  const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
  constexpr uint32_t kWaves = kListThreads / 64;
  __shared__ uint32_t cnt[kWaves];
  __shared__ unsigned long long base;
  const uint64_t step = (uint64_t)gridDim.x * kListThreads;
  for (uint64_t b0 = (uint64_t)blockIdx.x * kListThreads; b0 < n; b0 += step) {
    const uint64_t i = b0 + 64u * wv + lane;
    bool mine;
    if constexpr (kLane) {
      mine = i < n && lane_owns(a.len[i < n ? i : n - 1u]);
    } else {
      // the task (4-aligned quad of records) this lane's record belongs to
      const uint64_t t0 = i & ~3ull;
      uint64_t off[4];
      uint32_t len[4], valid = 0u;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const uint64_t r = t0 + (uint64_t)q;
        const uint64_t rc = r < n ? r : n - 1u;
        off[q] = a.off[rc];
        len[q] = a.len[rc];
        valid |= (r < n ? 1u : 0u) << q;
      }
      const QuadWindow win = quad_window(a.base, off, len, valid);
      mine = i < n && ((win.mask >> (i & 3u)) & 1u);
    }
    const bool lng = i < n && !mine;
    const uint64_t m = __ballot(lng);
    const uint64_t own = __ballot(mine);
    if (lane == 0) {
      cnt[wv] = (uint32_t)__popcll(m);
      if (i < n) ws.qrun[i >> 6] = own ? 1u : 0u;
    }
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
// Host-side launchers (called from crc32c_capi.hip through crc32c_device.h).
// ---------------------------------------------------------------------------
hipError_t launch_span(const SpanBatch& a, bool verify, int grid, hipStream_t s) {
  // Log records (LOG_HEADER) are short: the variant that skips padding rounds.
  const bool skip = (a.flags & kFlagLogHeader) != 0 && a.role == kRoleSpans;
  if (verify) {
    if (a.pair_kernel && !skip) crc32c_span_kernel<true, false, true><<<grid, kThreads, 0, s>>>(a);
    if (skip) crc32c_span_kernel<true, true, false><<<grid, kThreads, 0, s>>>(a);
    else crc32c_span_kernel<true, false, false><<<grid, kThreads, 0, s>>>(a);
  } else {
    if (a.pair_kernel && !skip) crc32c_span_kernel<false, false, true><<<grid, kThreads, 0, s>>>(a);
    if (skip) crc32c_span_kernel<false, true, false><<<grid, kThreads, 0, s>>>(a);
    else crc32c_span_kernel<false, false, false><<<grid, kThreads, 0, s>>>(a);
  }
  return hipGetLastError();
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

hipError_t launch_plan(const SpanBatch& a, bool desc, const SplitWs& ws, hipStream_t s) {
  if (desc) crc32c_plan_kernel<true><<<ws.nblocks, kPlanThreads, 0, s>>>(a, ws);
  else crc32c_plan_kernel<false><<<ws.nblocks, kPlanThreads, 0, s>>>(a, ws);
  return hipGetLastError();
}

hipError_t launch_slices(const SpanBatch& a, const SplitWs& ws, hipStream_t s) {
  crc32c_slice_scan_kernel<<<1, 1024, 0, s>>>(a, ws);
  crc32c_slice_mark_kernel<<<ws.nblocks, kPlanThreads, 0, s>>>(a, ws);
  return hipGetLastError();
}

hipError_t launch_quad(const SpanBatch& a, bool verify, int grid, const SplitWs& ws, hipStream_t s) {
  const uint64_t lb = (a.n + kListThreads - 1) / kListThreads;
  // one block per 1024 spans up to 16 Mi spans (a grid of 1024 looped and
  // took 49 us over a 4 GiB WAL batch; the atomics are per block-iteration
  // either way)
  const int lgrid = (int)(lb < 16384u ? lb : 16384u);
  if (PRISMDB_LANE_KERNEL) {
    crc32c_long_list_kernel<true><<<lgrid, kListThreads, 0, s>>>(a, ws);
    if (verify) crc32c_lane_kernel<true><<<grid, kLaneThreads, 0, s>>>(a);
    else crc32c_lane_kernel<false><<<grid, kLaneThreads, 0, s>>>(a);
  } else {
    crc32c_long_list_kernel<false><<<lgrid, kListThreads, 0, s>>>(a, ws);
    if (verify) crc32c_quad_kernel<true><<<grid, kThreads, 0, s>>>(a);
    else crc32c_quad_kernel<false><<<grid, kThreads, 0, s>>>(a);
  }
  return hipGetLastError();
}

hipError_t launch_scatter(const SpanBatch& a, const SplitWs& ws, const uint32_t* qout, const uint8_t* qmm,
                          hipStream_t s) {
  crc32c_scatter_kernel<<<256, 256, 0, s>>>(a, ws, qout, qmm);
  return hipGetLastError();
}

hipError_t launch_combine(const SpanBatch& a, bool desc, bool verify, const SplitWs& ws,
                          hipStream_t s) {
  const int grid = 256;  // 1024 waves, one long span each at a time
  if (desc) {
    if (verify) crc32c_combine_kernel<true, true><<<grid, 256, 0, s>>>(a, ws);
    else crc32c_combine_kernel<true, false><<<grid, 256, 0, s>>>(a, ws);
  } else {
    if (verify) crc32c_combine_kernel<false, true><<<grid, 256, 0, s>>>(a, ws);
    else crc32c_combine_kernel<false, false><<<grid, 256, 0, s>>>(a, ws);
  }
  return hipGetLastError();
}

}  // namespace dev
}  // namespace prismdb
