// floor_probe.hip -- measurement probes for the per-call floor (tools/percall_floor.py).
//
// Not part of the product library: tiny kernels that show what a launch
// costs on its own on the box's own clock (s_memrealtime, 100 MHz):
//   probe_stamp     one wave stores the clock: bracketing a call on its stream
//                   gives the call's span, start-up and completion included
//   probe_null      an empty kernel of the one-launch kernel's grid, plain
//                   launch or hipExtLaunchKernel with a stop event (as the
//                   one-launch kernel is launched)
//   probe_waves     the same grid, each wave storing its entry and exit
//   probe_record    hipEventRecord of an event made with given flags (a marker
//                   packet; system- or agent-scope release)
//   probe_scatter   one 4-byte store per thread at a stride (dirty lines left
//                   in L2 at the kernel's end, as the trailer stores leave them)
// Build: hipcc --offload-arch=gfx950 -O3 -fPIC -shared (tools/percall_floor.py build).
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace {

__global__ void probe_null_kernel() {}

__global__ void probe_stamp_kernel(uint64_t* dst) {
  if (threadIdx.x == 0) *dst = __builtin_amdgcn_s_memrealtime();
}

__global__ void probe_waves_kernel(uint64_t* dst) {
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  const uint32_t wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  if ((threadIdx.x & 63u) == 0u) {
    dst[2u * wave] = t0;
    dst[2u * wave + 1u] = __builtin_amdgcn_s_memrealtime();
  }
}

// one wave stamps its entry; the group holds `lds` bytes of dynamic LDS
__global__ void probe_lds_kernel(uint64_t* dst) {
  extern __shared__ uint32_t dyn[];
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  if (threadIdx.x == 0) {
    dyn[0] = (uint32_t)t0;
    dst[blockIdx.x] = t0 + (dyn[0] == 0xFFFFFFFFu ? 1u : 0u);
  }
}

// a plain streaming read of n 16-B vectors (grid-stride), XOR-folded per
// thread, one word per group stored: what the memory system gives a call of
// this size with no tables and no descriptors
typedef uint32_t v4u __attribute__((ext_vector_type(4)));
__global__ void probe_read_kernel(const v4u* p, uint64_t n, uint32_t* out) {
  uint32_t x = 0;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const v4u v = __builtin_nontemporal_load(p + i);
    x ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (x == 0x12345678u) out[blockIdx.x] = x;
}

__global__ void probe_scatter_kernel(uint32_t* p, uint32_t n, uint32_t stride_words) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) p[(uint64_t)i * stride_words] = i;
}

// one aligned 32-B sector per thread at byte (i * stride + at) & ~31: full-sector
// writes of the same lines the 4-byte trailer stores touch
__global__ void probe_sector_kernel(uint8_t* p, uint32_t n, uint32_t stride, uint32_t at) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) {
    v4u* q = reinterpret_cast<v4u*>(p + (((uint64_t)i * stride + at) & ~31ull));
    q[0] = v4u{i, i, i, i};
    q[1] = v4u{i, i, i, i};
  }
}

// 4-byte stores at byte i * stride + at (any alignment a dword store takes)
__global__ void probe_scatter_at_kernel(uint8_t* p, uint32_t n, uint32_t stride, uint32_t at) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) *reinterpret_cast<uint32_t*>(p + (uint64_t)i * stride + at) = i;
}

}  // namespace

extern "C" {

int probe_sector(void* p, uint32_t n, uint32_t stride, uint32_t at, void* s) {
  probe_sector_kernel<<<(n + 255u) / 256u, 256, 0, static_cast<hipStream_t>(s)>>>(static_cast<uint8_t*>(p), n, stride, at);
  return (int)hipGetLastError();
}

int probe_scatter_at(void* p, uint32_t n, uint32_t stride, uint32_t at, void* s) {
  probe_scatter_at_kernel<<<(n + 255u) / 256u, 256, 0, static_cast<hipStream_t>(s)>>>(static_cast<uint8_t*>(p), n, stride,
                                                                                      at);
  return (int)hipGetLastError();
}

int probe_stamp(void* dst, void* s) {
  probe_stamp_kernel<<<1, 64, 0, static_cast<hipStream_t>(s)>>>(static_cast<uint64_t*>(dst));
  return (int)hipGetLastError();
}

int probe_null(int grid, int threads, void* s, void* stop_event) {
  if (stop_event != nullptr)
    hipExtLaunchKernelGGL(probe_null_kernel, dim3(grid), dim3(threads), 0, static_cast<hipStream_t>(s), nullptr,
                          static_cast<hipEvent_t>(stop_event), 0u);
  else
    probe_null_kernel<<<grid, threads, 0, static_cast<hipStream_t>(s)>>>();
  return (int)hipGetLastError();
}

int probe_waves(int grid, int threads, void* dst, void* s) {
  probe_waves_kernel<<<grid, threads, 0, static_cast<hipStream_t>(s)>>>(static_cast<uint64_t*>(dst));
  return (int)hipGetLastError();
}

int probe_scatter(void* p, uint32_t n, uint32_t stride_words, void* s) {
  probe_scatter_kernel<<<(n + 255u) / 256u, 256, 0, static_cast<hipStream_t>(s)>>>(static_cast<uint32_t*>(p), n,
                                                                                   stride_words);
  return (int)hipGetLastError();
}

int probe_lds(int grid, int threads, int lds_bytes, void* dst, void* s) {
  hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(probe_lds_kernel),
                                     hipFuncAttributeMaxDynamicSharedMemorySize, lds_bytes);
  if (e != hipSuccess) return (int)e;
  probe_lds_kernel<<<grid, threads, lds_bytes, static_cast<hipStream_t>(s)>>>(static_cast<uint64_t*>(dst));
  return (int)hipGetLastError();
}

int probe_read(const void* p, uint64_t bytes, int grid, void* out, void* s) {
  probe_read_kernel<<<grid, 1024, 0, static_cast<hipStream_t>(s)>>>(static_cast<const v4u*>(p), bytes / 16u,
                                                                    static_cast<uint32_t*>(out));
  return (int)hipGetLastError();
}

int probe_event_create(void** ev) { return (int)hipEventCreateWithFlags(reinterpret_cast<hipEvent_t*>(ev), 0); }

// an event with explicit flags: hipEventDisableTiming (2) as the product's
// done events, | hipEventDisableSystemFence (0x20000000): its record releases
// at agent scope instead of system scope
int probe_event_create_flags(void** ev, unsigned flags) {
  return (int)hipEventCreateWithFlags(reinterpret_cast<hipEvent_t*>(ev), flags);
}

int probe_record(void* ev, void* s) {
  return (int)hipEventRecord(static_cast<hipEvent_t>(ev), static_cast<hipStream_t>(s));
}

}  // extern "C"
