// synth.hip -- on-device synthetic block generator (bench/test support).
//
// Produces the same bytes as oracle_fill_synthetic() (oracle/crc32c_oracle.c):
// the buffer is the little-endian u64 word stream word[k] = splitmix64(seed, k),
// so every block can be regenerated on the host for bit-exact checks without
// copying 64 GiB back.  Not part of the checksum path.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/prismdb_synth.h"

namespace {

__device__ __forceinline__ uint64_t splitmix64(uint64_t seed, uint64_t k) {
  uint64_t z = seed + (k + 1u) * 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

// Two words (16 B) per thread per step, grid-stride.
__global__ __launch_bounds__(256) void fill_kernel(uint64_t* __restrict__ dst, uint64_t nwords,
                                                   uint64_t seed, uint64_t word0) {
  const uint64_t step = (uint64_t)gridDim.x * blockDim.x * 2u;
  for (uint64_t i = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) * 2u; i < nwords; i += step) {
    const uint64_t a = splitmix64(seed, word0 + i);
    if (i + 1 < nwords) {
      const uint64_t b = splitmix64(seed, word0 + i + 1);
      typedef uint64_t v2 __attribute__((ext_vector_type(2)));
      v2 v = {a, b};
      __builtin_nontemporal_store(v, reinterpret_cast<v2*>(dst + i));
    } else {
      dst[i] = a;
    }
  }
}

__global__ void fill_tail_kernel(uint8_t* dst, uint32_t nbytes, uint64_t seed, uint64_t word) {
  const uint64_t w = splitmix64(seed, word);
  for (uint32_t j = threadIdx.x; j < nbytes; j += blockDim.x) dst[j] = (uint8_t)(w >> (8u * j));
}

}  // namespace

extern "C" int prismdb_fill_synthetic(void* dev_dst, size_t nbytes, uint64_t seed,
                                      uint64_t byte_offset, void* stream) {
  if (nbytes == 0) return 0;
  if (dev_dst == nullptr || (byte_offset & 7u) != 0 || (reinterpret_cast<uintptr_t>(dev_dst) & 15u) != 0)
    return -1;
  hipStream_t s = static_cast<hipStream_t>(stream);
  const uint64_t nwords = nbytes / 8u;
  if (nwords) {
    uint64_t blocks = (nwords / 2u + 255u) / 256u;
    if (blocks > 16384u) blocks = 16384u;
    fill_kernel<<<(unsigned)(blocks ? blocks : 1u), 256, 0, s>>>(static_cast<uint64_t*>(dev_dst), nwords, seed,
                                                                 byte_offset / 8u);
  }
  const uint32_t rem = (uint32_t)(nbytes & 7u);
  if (rem) {
    fill_tail_kernel<<<1, 64, 0, s>>>(static_cast<uint8_t*>(dev_dst) + nwords * 8u, rem, seed,
                                      byte_offset / 8u + nwords);
  }
  return hipGetLastError() == hipSuccess ? 0 : -2;
}
