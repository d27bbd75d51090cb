// recfold.hip -- read + fold probes for ~1 KB records (measurement support,
// not product; tools/recfold.py drives it).  The same N records of len bytes
// at a fixed stride, read as whole 128-B lines and folded with the lane
// kernel's LDS work (four conflict-free lookups per 4-B step in a 128 KiB
// replicated table image; the table contents are arbitrary: the probe times
// the work, its sums are not CRCs), in a two-slot software pipeline (the next
// task's loads issued before the current task is folded):
//   lane   one record per lane; a task is one line of each of the wave's 64
//          records (eight 16-B loads per lane), folded as one 32-step chain
//          (modes 2 / 3: as two / four independent chains, joined by one
//          more step each)
//   octet  8 lanes per record; a task is every line of each of the wave's 8
//          records (one 16-B load per lane and line: each instruction reads 8
//          whole lines), folded as four column chains per lane, then joined
//          (4 more steps, 4 ds_bpermutes, 2 steps standing in for the
//          per-lane realignment, 3 cross-lane XORs) -- the octet kernel's work
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef uint32_t v4 __attribute__((ext_vector_type(4)));
constexpr int kTabWords = 4 * 256 * 32;
constexpr int kMaxLines = 11;

__device__ __forceinline__ uint32_t stp(const uint32_t* lds, uint32_t c, uint32_t x, uint32_t w) {
  const uint32_t a0 = lds[(((x >> 0) & 255u) << 5) + c];
  const uint32_t a1 = lds[8192u + (((x >> 8) & 255u) << 5) + c];
  const uint32_t a2 = lds[16384u + (((x >> 16) & 255u) << 5) + c];
  const uint32_t a3 = lds[24576u + ((x >> 24) << 5) + c];
  return w ^ a0 ^ a1 ^ a2 ^ a3;
}

__device__ __forceinline__ void fill(uint32_t* lds) {
  for (uint32_t i = threadIdx.x; i < (uint32_t)kTabWords; i += blockDim.x) lds[i] = i * 0x9E3779B9u;
  __syncthreads();
}

template <int kChains>  // independent chains per line (joined by one more step each)
__global__ __launch_bounds__(512) void lane_fold(const uint8_t* __restrict__ p, uint64_t nrec, uint32_t stride,
                                                 uint32_t len, uint32_t* __restrict__ out) {
  __shared__ uint32_t lds[kTabWords];
  fill(lds);
  const uint32_t lane = threadIdx.x & 63u, c = lane & 31u;
  const uint64_t wave = (uint64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  const uint64_t nw = (uint64_t)gridDim.x * (blockDim.x >> 6);
  for (uint64_t r0 = wave * 64u; r0 < nrec; r0 += nw * 64u) {
    const uint64_t r = r0 + lane < nrec ? r0 + lane : nrec - 1u;
    const uint64_t s = r * stride, l0 = s & ~127ull, l1 = (s + len - 1u) & ~127ull;
    uint32_t nl = (uint32_t)((l1 - l0) >> 7) + 1u;
    for (int o = 32; o >= 1; o >>= 1) {
      const uint32_t y = (uint32_t)__shfl_xor((int)nl, o, 64);
      nl = y > nl ? y : nl;
    }
    auto line = [&](uint32_t t) { const uint64_t x = l0 + 128ull * t; return x > l1 ? l1 : x; };
    v4 a[8], b[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) a[j] = *reinterpret_cast<const v4*>(p + line(0) + 16 * j);
    uint32_t x = (uint32_t)r;
    for (uint32_t t = 0; t < nl; ++t) {
      if (t + 1 < nl) {
#pragma unroll
        for (int j = 0; j < 8; ++j) b[j] = *reinterpret_cast<const v4*>(p + line(t + 1) + 16 * j);
      }
      constexpr int q = 32 / kChains;
      uint32_t ch[kChains];
      ch[0] = x;
#pragma unroll
      for (int k = 1; k < kChains; ++k) ch[k] = 0u;
#pragma unroll
      for (int i = 0; i < q; ++i)
#pragma unroll
        for (int k = 0; k < kChains; ++k) ch[k] = stp(lds, c, ch[k], a[(k * q + i) >> 2][(k * q + i) & 3]);
      x = ch[0];
#pragma unroll
      for (int k = 1; k < kChains; ++k) x = stp(lds, c, x, ch[k]);
#pragma unroll
      for (int j = 0; j < 8; ++j) a[j] = b[j];
    }
    out[r] = x;
  }
}

template <int kLines>  // lines read per record (all of them, every task: counted waits stay static)
__global__ __launch_bounds__(512) void octet_fold(const uint8_t* __restrict__ p, uint64_t nrec, uint32_t stride,
                                                  uint32_t len, uint32_t* __restrict__ out) {
  __shared__ uint32_t lds[kTabWords];
  fill(lds);
  const uint32_t lane = threadIdx.x & 63u, c = lane & 31u, j = lane & 7u;
  const uint64_t wave = (uint64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  const uint64_t nw = (uint64_t)gridDim.x * (blockDim.x >> 6);
  auto geom = [&](uint64_t r0, uint64_t& l0, uint64_t& l1, uint32_t& nl, uint64_t& r) {
    r = r0 + (lane >> 3) < nrec ? r0 + (lane >> 3) : nrec - 1u;
    const uint64_t s = r * stride;
    l0 = s & ~127ull;
    l1 = (s + len - 1u) & ~127ull;
    nl = (uint32_t)((l1 - l0) >> 7) + 1u;
    for (int o = 32; o >= 8; o >>= 1) {  // (lanes of an octet agree)
      const uint32_t y = (uint32_t)__shfl_xor((int)nl, o, 64);
      nl = y > nl ? y : nl;
    }
  };
  v4 a[kLines], b[kLines];
  uint64_t l0, l1, r, nl0, nl1, rn;
  uint32_t nl, nn;
  auto load = [&](v4 (&d)[kLines], uint64_t b0, uint64_t b1, uint32_t n) {
    (void)n;
#pragma unroll
    for (int t = 0; t < kLines; ++t) {
      const uint64_t x = b0 + 128ull * t;
      d[t] = *reinterpret_cast<const v4*>(p + (x > b1 ? b1 : x) + 16u * j);
    }
  };
  uint64_t r0 = wave * 8u;
  if (r0 >= nrec) return;
  geom(r0, l0, l1, nl, r);
  load(a, l0, l1, nl);
  for (; r0 < nrec; r0 += nw * 8u) {
    const uint64_t rn0 = r0 + nw * 8u;
    const bool more = rn0 < nrec;
    if (more) {
      geom(rn0, nl0, nl1, nn, rn);
      load(b, nl0, nl1, nn);
    }
    uint32_t A[4] = {(uint32_t)r, 0u, 0u, 0u};
#pragma unroll
    for (int t = 0; t < kLines; ++t) {
#pragma unroll
      for (int i = 0; i < 4; ++i) A[i] = stp(lds, c, A[i], a[t][i]);
    }
    // join: the four columns (Horner, 4 steps), the rotation across the
    // octet (4 bpermutes), the per-lane realignment (2 steps), the octet's XOR
    uint32_t y = A[0];
    y = stp(lds, c, y, A[1]);
    y = stp(lds, c, y, A[2]);
    y = stp(lds, c, y, A[3]);
    y = stp(lds, c, y, 0u);
    const int src = (int)(((lane & ~7u) | ((j + r) & 7u)) << 2);
#pragma unroll
    for (int i = 0; i < 4; ++i) y ^= (uint32_t)__builtin_amdgcn_ds_bpermute(src + 4 * i, (int)A[i]);
    y = stp(lds, c, y, 0u);
    y = stp(lds, c, y, 0u);
    y ^= (uint32_t)__shfl_xor((int)y, 1, 64);
    y ^= (uint32_t)__shfl_xor((int)y, 2, 64);
    y ^= (uint32_t)__shfl_xor((int)y, 4, 64);
    if (j == 0) out[r] = y;
    if (more) {
#pragma unroll
      for (int t = 0; t < kLines; ++t) a[t] = b[t];
      l0 = nl0;
      l1 = nl1;
      nl = nn;
      r = rn;
    }
  }
}

extern "C" int recfold(const void* p, uint64_t nrec, uint32_t stride, uint32_t len, uint32_t* out, int mode, int grid,
                       void* stream) {
  hipStream_t s = (hipStream_t)stream;
  const uint8_t* b = (const uint8_t*)p;
  if (len == 0 || len > 1280u) return -2;
  if (mode == 0) lane_fold<1><<<grid, 512, 0, s>>>(b, nrec, stride, len, out);
  else if (mode == 2) lane_fold<2><<<grid, 512, 0, s>>>(b, nrec, stride, len, out);
  else if (mode == 3) lane_fold<4><<<grid, 512, 0, s>>>(b, nrec, stride, len, out);
  else {
    const uint32_t lines = (127u + len + 127u) / 128u;  // the most lines a record of len bytes spans
    if (lines <= 3) octet_fold<3><<<grid, 512, 0, s>>>(b, nrec, stride, len, out);
    else if (lines <= 9) octet_fold<9><<<grid, 512, 0, s>>>(b, nrec, stride, len, out);
    else octet_fold<11><<<grid, 512, 0, s>>>(b, nrec, stride, len, out);
  }
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
