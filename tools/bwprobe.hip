// bwprobe.hip -- HBM read-bandwidth probes (measurement support, not product).
// Streams a buffer once with loads of a given width and XOR-folds it so the
// loads stay live; one u32 per thread is written.  Used to find the read
// ceiling the CRC kernel is measured against, per load width and policy.
#include <hip/hip_runtime.h>
#include <stdint.h>

template <int kWidth, bool kNT>
__global__ __launch_bounds__(256) void read_kernel(const uint8_t* __restrict__ p, uint64_t nbytes,
                                                   uint32_t* __restrict__ out, int unroll_dummy) {
  typedef uint32_t v4 __attribute__((ext_vector_type(4)));
  typedef uint32_t v2 __attribute__((ext_vector_type(2)));
  uint32_t acc = 0;
  const uint64_t tid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint64_t nthreads = (uint64_t)gridDim.x * blockDim.x;
  constexpr int U = 8;
  const uint64_t step = nthreads * kWidth;
  uint64_t i = tid * kWidth;
  for (; i + (U - 1) * step < nbytes; i += U * step) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint8_t* q = p + i + u * step;
      if (kWidth == 16) {
        v4 v = kNT ? __builtin_nontemporal_load(reinterpret_cast<const v4*>(q)) : *reinterpret_cast<const v4*>(q);
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
      } else if (kWidth == 8) {
        v2 v = kNT ? __builtin_nontemporal_load(reinterpret_cast<const v2*>(q)) : *reinterpret_cast<const v2*>(q);
        acc ^= v.x ^ v.y;
      } else {
        uint32_t v = kNT ? __builtin_nontemporal_load(reinterpret_cast<const uint32_t*>(q))
                         : *reinterpret_cast<const uint32_t*>(q);
        acc ^= v;
      }
    }
  }
  for (; i < nbytes; i += step) acc ^= *reinterpret_cast<const uint32_t*>(p + i);
  out[tid] = acc;
}

extern "C" int bwprobe_read(const void* p, uint64_t nbytes, uint32_t* out, int width, int nt, int grid,
                            void* stream) {
  hipStream_t s = (hipStream_t)stream;
  const uint8_t* b = (const uint8_t*)p;
#define L(W, N) read_kernel<W, N><<<grid, 256, 0, s>>>(b, nbytes, out, 0)
  if (width == 16) { if (nt) L(16, true); else L(16, false); }
  else if (width == 8) { if (nt) L(8, true); else L(8, false); }
  else { if (nt) L(4, true); else L(4, false); }
#undef L
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

// Block pattern of the CRC kernels: each wave owns whole 4 KiB blocks
// (16 dword loads, one per 256-B round), blocks dealt round-robin over the
// grid's waves, kR blocks in flight per wave per iteration.  kXcd remaps
// waves so that each XCD (workgroup b runs on XCD b % 8) reads one contiguous
// region per step instead of 64 KiB pieces interleaved with the other XCDs.
template <int kT, int kR, bool kXcd>
__global__ __launch_bounds__(kT) void read_blocks(const uint8_t* __restrict__ p, uint64_t nblocks,
                                                  uint32_t* __restrict__ out) {
  constexpr int kWpg = kT / 64;
  const uint32_t lane = threadIdx.x & 63u;
  const uint64_t nw = (uint64_t)gridDim.x * kWpg;
  uint64_t gw;
  if (kXcd) {
    const uint32_t x = blockIdx.x % 8u, i = blockIdx.x / 8u;
    gw = (uint64_t)x * (nw / 8) + (uint64_t)i * kWpg + (threadIdx.x >> 6);
  } else {
    gw = (uint64_t)blockIdx.x * kWpg + (threadIdx.x >> 6);
  }
  uint32_t acc = 0;
  for (uint64_t k = gw; k + (uint64_t)(kR - 1) * nw < nblocks; k += (uint64_t)kR * nw) {
    uint32_t w[kR][16];
#pragma unroll
    for (int r = 0; r < kR; ++r) {
      const uint32_t* q = reinterpret_cast<const uint32_t*>(p + (k + (uint64_t)r * nw) * 4096) + lane;
#pragma unroll
      for (int j = 0; j < 16; ++j) w[r][j] = __builtin_nontemporal_load(q + 64 * j);
    }
#pragma unroll
    for (int r = 0; r < kR; ++r)
#pragma unroll
      for (int j = 0; j < 16; ++j) acc ^= w[r][j];
  }
  out[blockIdx.x * kT + threadIdx.x] = acc;
}

extern "C" int bwprobe_blocks(const void* p, uint64_t nblocks, uint32_t* out, int wg, int ring, int xcd, int grid,
                              void* stream) {
  hipStream_t s = (hipStream_t)stream;
  const uint8_t* b = (const uint8_t*)p;
#define B(T, R, X) read_blocks<T, R, X><<<grid, T, 0, s>>>(b, nblocks, out)
  if (wg == 1024) {
    if (ring == 1) { if (xcd) B(1024, 1, true); else B(1024, 1, false); }
    else if (ring == 2) { if (xcd) B(1024, 2, true); else B(1024, 2, false); }
    else { if (xcd) B(1024, 4, true); else B(1024, 4, false); }
  } else {
    if (ring == 1) { if (xcd) B(256, 1, true); else B(256, 1, false); }
    else if (ring == 2) { if (xcd) B(256, 2, true); else B(256, 2, false); }
    else { if (xcd) B(256, 4, true); else B(256, 4, false); }
  }
#undef B
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

// The same block pattern (1024-thread groups, one per CU, 2 blocks in flight
// per wave) plus one 4-byte result per block, stored in different ways:
//   mode 0: no stores (reference)
//   mode 1: lane 0 stores out[block] after each block (exec-masked)
//   mode 2: all 64 lanes store the same value to out[block]
//   mode 3: results buffered in a VGPR (lane i = i-th block of the wave),
//           one 64-lane scattered store every 64 blocks
//   mode 4: contiguous assignment (wave w owns blocks [w*m, (w+1)*m)), lane i
//           buffers block i of a 64-block run, one coalesced 256-B store per run
template <int kMode>
__global__ __launch_bounds__(1024) void read_blocks_store(const uint8_t* __restrict__ p, uint64_t nblocks,
                                                         uint32_t* __restrict__ out) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint64_t nw = (uint64_t)gridDim.x * 16;
  const uint64_t gw = (uint64_t)blockIdx.x * 16 + (threadIdx.x >> 6);
  uint32_t buf = 0, nbuf = 0;
  const uint64_t m = nblocks / nw;  // mode 4: blocks per wave (nblocks divisible by nw * 64 assumed)
  for (uint64_t q = 0; q + 1 < (kMode == 4 ? m : (kMode >= 5 ? nblocks : nblocks / nw + 1)); q += 2) {
    uint64_t b0, b1;
    if (kMode == 4) {
      b0 = gw * m + q;
      b1 = b0 + 1;
    } else if (kMode >= 5) {  // runs of 64 consecutive blocks per wave, runs dealt round-robin
      b0 = ((q / 64) * nw + gw) * 64 + (q % 64);
      b1 = b0 + 1;
      if (b1 >= nblocks) break;
    } else {
      b0 = gw + q * nw;
      b1 = b0 + nw;
      if (b1 >= nblocks) break;
    }
    uint32_t w0[16], w1[16];
    const uint32_t* q0 = reinterpret_cast<const uint32_t*>(p + b0 * 4096) + lane;
    const uint32_t* q1 = reinterpret_cast<const uint32_t*>(p + b1 * 4096) + lane;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      w0[j] = __builtin_nontemporal_load(q0 + 64 * j);
      w1[j] = __builtin_nontemporal_load(q1 + 64 * j);
    }
    uint32_t x0 = 0, x1 = 0;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      x0 ^= w0[j];
      x1 ^= w1[j];
    }
    // wave-uniform "results"
    x0 = __builtin_amdgcn_readfirstlane(x0);
    x1 = __builtin_amdgcn_readfirstlane(x1);
    if (kMode == 0 || kMode == 5) {
      buf ^= x0 ^ x1;
    } else if (kMode == 1) {
      if (lane == 0) {
        out[b0] = x0;
        out[b1] = x1;
      }
    } else if (kMode == 2) {
      out[b0] = x0;
      out[b1] = x1;
    } else if (kMode == 3 || kMode == 4 || kMode == 6) {
      if (lane == nbuf) buf = x0;
      if (lane == nbuf + 1) buf = x1;
      nbuf += 2;
      if (nbuf == 64) {
        if (kMode == 3) out[gw + (q - 62 + lane) * nw] = buf;  // lane i: block of step q-62+i... approx scatter
        else if (kMode == 4) out[gw * m + q - 62 + lane] = buf;
        else out[b0 - 62 + lane] = buf;
        nbuf = 0;
      }
    }
  }
  if (kMode == 0 || kMode == 5) out[gw] = buf;  // keep something live
}

extern "C" int bwprobe_blocks_store(const void* p, uint64_t nblocks, uint32_t* out, int mode, int grid, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  const uint8_t* b = (const uint8_t*)p;
  switch (mode) {
    case 0: read_blocks_store<0><<<grid, 1024, 0, s>>>(b, nblocks, out); break;
    case 1: read_blocks_store<1><<<grid, 1024, 0, s>>>(b, nblocks, out); break;
    case 2: read_blocks_store<2><<<grid, 1024, 0, s>>>(b, nblocks, out); break;
    case 3: read_blocks_store<3><<<grid, 1024, 0, s>>>(b, nblocks, out); break;
    case 4: read_blocks_store<4><<<grid, 1024, 0, s>>>(b, nblocks, out); break;
    case 5: read_blocks_store<5><<<grid, 1024, 0, s>>>(b, nblocks, out); break;
    default: read_blocks_store<6><<<grid, 1024, 0, s>>>(b, nblocks, out); break;
  }
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

// Store-burst probes on the run pattern (1024-thread groups, 2 blocks per step):
//   mode 0: runs of kRunB blocks, one kRunB*4-byte result store per run (kRunB/64 VGPRs)
//   mode 1: runs of 64, results of kGroup runs buffered, stored together every kGroup runs
//   mode 2: runs of 64, one 256-B store per run with the nt (streaming) hint
template <int kMode, int kRunB, int kGroup>
__global__ __launch_bounds__(1024) void read_runs_store(const uint8_t* __restrict__ p, uint64_t nblocks,
                                                       uint32_t* __restrict__ out) {
  constexpr int kV = kMode == 0 ? kRunB / 64 : (kMode == 1 ? kGroup : 1);  // result VGPRs
  const uint32_t lane = threadIdx.x & 63u;
  const uint64_t nw = (uint64_t)gridDim.x * 16;
  const uint64_t gw = (uint64_t)blockIdx.x * 16 + (threadIdx.x >> 6);
  constexpr int kRun = kMode == 0 ? kRunB : 64;
  uint32_t res[kV];
#pragma unroll
  for (int v = 0; v < kV; ++v) res[v] = 0;
  uint64_t run_base[kGroup > 0 ? kGroup : 1];
  uint32_t slot = 0;  // results collected
  for (uint64_t q = 0;; q += 2) {
    const uint64_t b0 = ((q / kRun) * nw + gw) * kRun + (q % kRun), b1 = b0 + 1;
    if (b1 >= nblocks) break;
    uint32_t w0[16], w1[16];
    const uint32_t* q0 = reinterpret_cast<const uint32_t*>(p + b0 * 4096) + lane;
    const uint32_t* q1 = reinterpret_cast<const uint32_t*>(p + b1 * 4096) + lane;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      w0[j] = __builtin_nontemporal_load(q0 + 64 * j);
      w1[j] = __builtin_nontemporal_load(q1 + 64 * j);
    }
    uint32_t x0 = 0, x1 = 0;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      x0 ^= w0[j];
      x1 ^= w1[j];
    }
    x0 = __builtin_amdgcn_readfirstlane(x0);
    x1 = __builtin_amdgcn_readfirstlane(x1);
#pragma unroll
    for (int v = 0; v < kV; ++v) {
      if (slot / 64 == (uint32_t)v) {
        if (lane == slot % 64) res[v] = x0;
        if (lane == slot % 64 + 1) res[v] = x1;
      }
    }
    if (kMode == 1 && q % kRun == 0) run_base[(slot / 64) % (kGroup > 0 ? kGroup : 1)] = b0;
    slot += 2;
    if (kMode == 0 && slot == (uint32_t)kRun) {
#pragma unroll
      for (int v = 0; v < kV; ++v) out[b1 + 1 - kRun + 64 * v + lane] = res[v];
      slot = 0;
    } else if (kMode == 1 && slot == 64u * kGroup) {
#pragma unroll
      for (int v = 0; v < kV; ++v) out[run_base[v] + lane] = res[v];
      slot = 0;
    } else if (kMode == 2 && slot == 64u) {
      __builtin_nontemporal_store(res[0], out + b1 + 1 - 64 + lane);
      slot = 0;
    }
  }
}

extern "C" int bwprobe_runs_store(const void* p, uint64_t nblocks, uint32_t* out, int mode, int param, int grid,
                                  void* stream) {
  hipStream_t s = (hipStream_t)stream;
  const uint8_t* b = (const uint8_t*)p;
#define R(M, A, G) read_runs_store<M, A, G><<<grid, 1024, 0, s>>>(b, nblocks, out)
  if (mode == 0) {
    if (param == 128) R(0, 128, 0); else if (param == 256) R(0, 256, 0); else R(0, 512, 0);
  } else if (mode == 1) {
    if (param == 2) R(1, 64, 2); else if (param == 4) R(1, 64, 4); else R(1, 64, 8);
  } else {
    R(2, 64, 0);
  }
#undef R
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
