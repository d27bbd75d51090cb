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
