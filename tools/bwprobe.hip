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
