// recprobe.hip -- read-pattern probes for short records (measurement support,
// not product).  N records of len bytes at a fixed stride (~1 KB apart, like
// ~1 KB WAL records behind their 7-byte headers), each read once as whole
// 128-B lines (the lines that hold a byte of the record) in one of three
// lane-to-byte mappings, XOR-folded so the loads stay live:
//   lane   (crc32c_lane_kernel): one record per lane, a wave's 64 lanes on 64
//          consecutive records; per line eight 16-B loads by the same lane
//          (one load instruction touches 64 lines, 16 B of each)
//   octx4  8 lanes per record (octets), a wave on 8 records; per line one
//          16-B load per lane (one instruction covers 8 whole lines)
//   octw   octets, per line four 4-B loads per lane at a 32-B stride (one
//          instruction covers 32 B of each of 8 lines)
// Each wave keeps kF records' lines in flight (loads of kF lines issued
// before their fold), as the kernels keep a task ahead.
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef uint32_t v4 __attribute__((ext_vector_type(4)));

template <int kMode>
__global__ __launch_bounds__(1024) void rec_kernel(const uint8_t* __restrict__ p, uint64_t nrec, uint32_t stride,
                                                  uint32_t len, uint32_t* __restrict__ out) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint64_t wave = (uint64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  const uint64_t nw = (uint64_t)gridDim.x * (blockDim.x >> 6);
  constexpr uint32_t kPer = kMode == 0 ? 64u : 8u;  // records per wave step
  uint32_t acc = 0;
  const uint32_t sub = kMode == 0 ? 0u : (lane & 7u);
  const uint32_t rec_in = kMode == 0 ? lane : (lane >> 3);
  for (uint64_t r0 = wave * kPer; r0 < nrec; r0 += nw * kPer) {
    const uint64_t r = r0 + rec_in;
    const bool live = r < nrec;
    const uint64_t s = live ? r * stride : 0u;
    const uint64_t l0 = s & ~127ull, l1 = live ? ((s + len - 1u) & ~127ull) : l0;
    // wave-uniform line count: the longest record of the step
    uint32_t nl = (uint32_t)((l1 - l0) >> 7) + 1u;
    for (int o = 32; o >= 1; o >>= 1) {
      const uint32_t y = (uint32_t)__shfl_xor((int)nl, o, 64);
      nl = y > nl ? y : nl;
    }
    // 8 KiB of loads in flight per wave per step in every mode: one line per
    // lane (mode 0) or eight lines per octet (modes 1, 2); lines past the
    // record re-read its last line (a cache hit)
    constexpr uint32_t kL = kMode == 0 ? 1u : 8u;
    for (uint32_t t = 0; t < nl; t += kL) {
      uint64_t la[kL];
#pragma unroll
      for (uint32_t u = 0; u < kL; ++u) {
        const uint64_t x = l0 + 128ull * (t + u);
        la[u] = x > l1 ? l1 : x;
      }
      if (kMode == 0) {
        v4 a[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) a[j] = *reinterpret_cast<const v4*>(p + la[0] + 16 * j);
#pragma unroll
        for (int j = 0; j < 8; ++j) acc ^= a[j].x ^ a[j].y ^ a[j].z ^ a[j].w;
      } else if (kMode == 1) {
        v4 a[kL];
#pragma unroll
        for (uint32_t u = 0; u < kL; ++u) a[u] = *reinterpret_cast<const v4*>(p + la[u] + 16u * sub);
#pragma unroll
        for (uint32_t u = 0; u < kL; ++u) acc ^= a[u].x ^ a[u].y ^ a[u].z ^ a[u].w;
      } else {
        uint32_t a[kL][4];
#pragma unroll
        for (uint32_t u = 0; u < kL; ++u)
#pragma unroll
          for (int k = 0; k < 4; ++k) a[u][k] = *reinterpret_cast<const uint32_t*>(p + la[u] + 4u * sub + 32u * k);
#pragma unroll
        for (uint32_t u = 0; u < kL; ++u) acc ^= a[u][0] ^ a[u][1] ^ a[u][2] ^ a[u][3];
      }
    }
  }
  out[wave * 64u + lane] = acc;
}

extern "C" int recprobe(const void* p, uint64_t nrec, uint32_t stride, uint32_t len, uint32_t* out, int mode,
                        int grid, int threads, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  const uint8_t* b = (const uint8_t*)p;
  if (mode == 0) rec_kernel<0><<<grid, threads, 0, s>>>(b, nrec, stride, len, out);
  else if (mode == 1) rec_kernel<1><<<grid, threads, 0, s>>>(b, nrec, stride, len, out);
  else rec_kernel<2><<<grid, threads, 0, s>>>(b, nrec, stride, len, out);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
