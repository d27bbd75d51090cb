// crc32c_fold.h -- device helpers shared by the CRC32C kernels: cross-lane
// XOR reductions, the LDS stride/nibble tables and their conflict-free
// lookups, the 256-B stride fold step and the per-lane realignment, inline-asm
// loads retired by counted waits, span records and tasks.
//
// The arithmetic: CRC-32C (reflected Castagnoli 0x82F63B78) is linear over
// GF(2); feeding word w into register r gives shift_4(r ^ w), and shift_n (the
// register advanced over n zero bytes) is a 32x32 bit matrix (crc32c_gf2.h).
// util/crc32c.cc:276-377 computes the same function with slicing-by-4 tables.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "crc32c_device.h"

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
// (TableBuilder::WriteRawBlock, table/table_builder.cc:196): one dword store
// at any byte alignment (the hardware splits a misaligned one; as four byte
// stores each trailer was four write requests -- the lane kernel's log-header
// stores were always one).  Little-endian, so the bytes are EncodeFixed32's.
// Non-temporal: seven sealed SST files per call run 19 % faster than with
// plain stores (5407 against 4533 GB/s, as fast as not storing at all: 5520),
// two files 5.7 %, one file and the planner path the same
// (profiles/r04/r04o_variants_store_policies.json; sc1 / sc0 sc1 gained 9-10 %).
__device__ __forceinline__ void store_le32(const uint8_t* p, uint32_t v) {
  asm volatile("global_store_dword %0, %1, off nt" : : "v"(p), "v"(v) : "memory");
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

// Fill LDS with the image above.  The image is 1024 segments of 128 B, one
// per (table k, entry e): segment q = (k >> 1) << 9 | e << 1 | (k & 1) holds
// the 32 copies of stride[k][e].  Lane x of a write writes 16 B (four copies)
// of segment x / 8, so a wave writes 1 KiB of consecutive LDS: no bank
// conflicts.  (One thread per table word writing its 128 B put every lane of
// a wave 256 B apart -- all on the same four banks -- and took ~4 us per
// group; one LDS word per thread, round 2's fill, needs 4x the instructions.)
// The table words come from L1 (eight lanes read each).  The per-lane nibble
// tables (32 KiB) are copied 16 B per lane, also consecutive.  Every global
// load of a thread is issued before its first LDS store (one memory round trip
// per group at kernel start instead of one per loop step: the fill sits in
// front of every kernel's first data load).
template <int kT>
__device__ __forceinline__ void load_stride_image(uint32_t* lds, const uint32_t* tab, uint32_t tid) {
  typedef uint32_t v4 __attribute__((ext_vector_type(4)));
  constexpr int kS = (8192 + kT - 1) / kT;
  v4* dst = reinterpret_cast<v4*>(lds);
  uint32_t v[kS];
#pragma unroll
  for (int i = 0; i < kS; ++i) {
    const uint32_t x = tid + (uint32_t)(i * kT);
    const uint32_t q = x >> 3;
    const uint32_t k = ((q >> 9) << 1) | (q & 1u), e = (q >> 1) & 255u;
    v[i] = (kS * kT == 8192 || x < 8192u) ? tab[k * 256u + e] : 0u;
  }
#pragma unroll
  for (int i = 0; i < kS; ++i) {
    const uint32_t x = tid + (uint32_t)(i * kT);
    if (kS * kT == 8192 || x < 8192u) dst[x] = v4{v[i], v[i], v[i], v[i]};
  }
}

template <int kT = kThreads>
__device__ __forceinline__ void load_tables(uint32_t* lds, const DeviceTables* tabs, uint32_t tid) {
  typedef uint32_t v4 __attribute__((ext_vector_type(4)));
  constexpr int kS = (8192 + kT - 1) / kT;
  constexpr uint32_t kNib = (uint32_t)kNibWords / 4u;
  constexpr int kN = (int)((kNib + kT - 1) / kT);
  const uint32_t* tab = &tabs->stride[0][0];
  const v4* nib = reinterpret_cast<const v4*>(&tabs->lane_nib[0][0][0]);
  uint32_t v[kS];
  v4 u[kN];
#pragma unroll
  for (int i = 0; i < kS; ++i) {
    const uint32_t x = tid + (uint32_t)(i * kT);
    const uint32_t q = x >> 3;
    const uint32_t k = ((q >> 9) << 1) | (q & 1u), e = (q >> 1) & 255u;
    v[i] = (kS * kT == 8192 || x < 8192u) ? tab[k * 256u + e] : 0u;
  }
#pragma unroll
  for (int i = 0; i < kN; ++i) {
    const uint32_t e = tid + (uint32_t)(i * kT);
    u[i] = ((uint32_t)kN * kT == kNib || e < kNib) ? nib[e] : v4{0u, 0u, 0u, 0u};
  }
  v4* dst = reinterpret_cast<v4*>(lds);
#pragma unroll
  for (int i = 0; i < kS; ++i) {
    const uint32_t x = tid + (uint32_t)(i * kT);
    if (kS * kT == 8192 || x < 8192u) dst[x] = v4{v[i], v[i], v[i], v[i]};
  }
  v4* ndst = reinterpret_cast<v4*>(lds + kTabWords);
#pragma unroll
  for (int i = 0; i < kN; ++i) {
    const uint32_t e = tid + (uint32_t)(i * kT);
    if ((uint32_t)kN * kT == kNib || e < kNib) ndst[e] = u[i];
  }
}

__device__ __forceinline__ uint32_t lds_word(const uint32_t* lds, uint32_t byte_addr) {
  return *reinterpret_cast<const uint32_t*>(reinterpret_cast<const char*>(lds) + byte_addr);
}

// a ^ b ^ c in one VALU instruction (gfx950 v_bitop3_b32, truth table 0x96).
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
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
  asm volatile("global_load_dword %0, %1, %2 offset:%3 nt" : "=v"(r) : "v"(voff), "s"(base), "n"(kImm));
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
  asm volatile("buffer_load_dword %0, %1, %2, 0 offen offset:%3 nt" : "=v"(r) : "v"(voff), "s"(rs), "n"(kImm));
  return r;
}

__device__ __forceinline__ uint32_t buf_ubyte(u32x4 rs, uint32_t voff) {
  uint32_t r;
  asm volatile("buffer_load_ubyte %0, %1, %2, 0 offen" : "=v"(r) : "v"(voff), "s"(rs));
  return r;
}

// The one-launch kernel's table fill in two halves, so that a wave's first
// data loads can be issued between them: `issue` puts every table word this
// thread copies into registers with inline-asm buffer loads (one round trip;
// offsets past a table read 0, so no lane branches), the caller retires them
// with a counted wait (tables_wait: the data loads issued after them stay in
// flight), and `store` writes the LDS image load_tables writes.
template <int kT>
struct TableRegs {
  static constexpr int kS = (8192 + kT - 1) / kT;
  static constexpr int kN = (kNibWords / 4 + kT - 1) / kT;
  uint32_t v[kS];
  u32x4 u[kN];
};

template <int kT>
__device__ __forceinline__ void tables_issue(TableRegs<kT>& r, const DeviceTables* tabs, uint32_t tid) {
  u32x4 rs = buffer_rsrc(reinterpret_cast<const uint8_t*>(&tabs->stride[0][0]), 4u * 4u * 256u);
  u32x4 rn = buffer_rsrc(reinterpret_cast<const uint8_t*>(&tabs->lane_nib[0][0][0]), 4u * (uint32_t)kNibWords);
  // SGPRs the vector unit wrote (readfirstlane) need 5 wait states before a
  // VMEM instruction reads them; hipcc inserts none before inline asm.
  asm volatile("s_nop 4" : "+s"(rs), "+s"(rn));
#pragma unroll
  for (int i = 0; i < TableRegs<kT>::kS; ++i) {
    const uint32_t x = tid + (uint32_t)(i * kT);
    const uint32_t q = x >> 3;
    const uint32_t k = ((q >> 9) << 1) | (q & 1u), e = (q >> 1) & 255u;
    const uint32_t off = x < 8192u ? 4u * (k * 256u + e) : 0xFFFFFFF0u;
    asm volatile("buffer_load_dword %0, %1, %2, 0 offen" : "=v"(r.v[i]) : "v"(off), "s"(rs));
  }
#pragma unroll
  for (int i = 0; i < TableRegs<kT>::kN; ++i) {
    const uint32_t e = tid + (uint32_t)(i * kT);
    const uint32_t off = e < (uint32_t)kNibWords / 4u ? 16u * e : 0xFFFFFFF0u;
    asm volatile("buffer_load_dwordx4 %0, %1, %2, 0 offen" : "=v"(r.u[i]) : "v"(off), "s"(rn));
  }
}

// Retire the table loads with kYounger (data) loads left in flight.
template <int kYounger>
__device__ __forceinline__ void tables_wait(TableRegs<1024>& r) {
  static_assert(TableRegs<1024>::kS == 8 && TableRegs<1024>::kN == 2, "operand list below");
  asm volatile("s_waitcnt vmcnt(%10)"
               : "+v"(r.v[0]), "+v"(r.v[1]), "+v"(r.v[2]), "+v"(r.v[3]), "+v"(r.v[4]), "+v"(r.v[5]),
                 "+v"(r.v[6]), "+v"(r.v[7]), "+v"(r.u[0]), "+v"(r.u[1])
               : "n"(kYounger));
}

template <int kYounger>
__device__ __forceinline__ void tables_wait(TableRegs<768>& r) {
  static_assert(TableRegs<768>::kS == 11 && TableRegs<768>::kN == 3, "operand list below");
  asm volatile("s_waitcnt vmcnt(%14)"
               : "+v"(r.v[0]), "+v"(r.v[1]), "+v"(r.v[2]), "+v"(r.v[3]), "+v"(r.v[4]), "+v"(r.v[5]),
                 "+v"(r.v[6]), "+v"(r.v[7]), "+v"(r.v[8]), "+v"(r.v[9]), "+v"(r.v[10]), "+v"(r.u[0]),
                 "+v"(r.u[1]), "+v"(r.u[2])
               : "n"(kYounger));
}

template <int kT>
__device__ __forceinline__ void tables_store(uint32_t* lds, const TableRegs<kT>& r, uint32_t tid) {
  typedef uint32_t v4 __attribute__((ext_vector_type(4)));
  v4* dst = reinterpret_cast<v4*>(lds);
#pragma unroll
  for (int i = 0; i < TableRegs<kT>::kS; ++i) {
    const uint32_t x = tid + (uint32_t)(i * kT);
    if (x < 8192u) dst[x] = v4{r.v[i], r.v[i], r.v[i], r.v[i]};
  }
  v4* ndst = reinterpret_cast<v4*>(lds + kTabWords);
#pragma unroll
  for (int i = 0; i < TableRegs<kT>::kN; ++i) {
    const uint32_t e = tid + (uint32_t)(i * kT);
    if (e < (uint32_t)kNibWords / 4u) ndst[e] = v4{r.u[i].x, r.u[i].y, r.u[i].z, r.u[i].w};
  }
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

// y = M x for the 32x32 GF(2) matrix M given by its columns (uniform).
__device__ __forceinline__ uint32_t gf2_apply(const uint32_t* col, uint32_t x) {
  uint32_t y = 0;
#pragma unroll
  for (int i = 0; i < 32; ++i) y ^= col[i] & (0u - ((x >> i) & 1u));
  return y;
}

}  // namespace dev
}  // namespace prismdb
