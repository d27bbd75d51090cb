// burstprobe.hip -- what does ONE file-sized call (67 MB) cost on this
// hardware, independent of the CRC?  Back-to-back launches on one stream,
// HIP events around 100 of them:
//
//   empty      the one-launch grid (#CUs x 768 threads), nothing to do: the
//              launch floor of a call
//   lds        the same grid, each group fills 160 KiB of LDS from a 36 KiB
//              table (what every CRC kernel does first)
//   read       the same grid, every lane reads its share of a 67 MB buffer
//              with 16-B loads, all issued at once, XOR-reduced, one store
//              per wave: the streaming floor of a file-sized call
//   read_lds   read + lds, the loads issued before the fill
//
// Prints one JSON object.  Build: hipcc --offload-arch=gfx950 -O3
// tools/burstprobe.hip -o tools/_build/burstprobe
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>

#define CHECK(x)                                                                            \
  do {                                                                                      \
    hipError_t e_ = (x);                                                                    \
    if (e_ != hipSuccess) {                                                                 \
      std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      std::exit(1);                                                                         \
    }                                                                                       \
  } while (0)

typedef uint32_t v4 __attribute__((ext_vector_type(4)));
constexpr int kThreads = 768;
constexpr int kLdsWords = 40960;  // 160 KiB
constexpr int kPer = 16;          // 16-B loads per lane, all in flight

__global__ __launch_bounds__(kThreads) void k_empty(uint32_t* out) {
  if (threadIdx.x == 0 && blockIdx.x == 0xFFFFFFFu) out[0] = 1;
}

template <bool kLds, bool kRead>
__global__ __launch_bounds__(kThreads) void k_probe(const v4* __restrict__ buf, size_t n16, const uint32_t* tab,
                                                    uint32_t* out) {
  __shared__ uint32_t lds[kLdsWords];
  const size_t nthreads = (size_t)gridDim.x * kThreads;
  const size_t gt = (size_t)blockIdx.x * kThreads + threadIdx.x;
  v4 w[kPer];
  if (kRead) {
    // lane-contiguous 16-B loads: wave-instruction k of wave g reads 1 KiB at
    // (g * kPer + k) * 1 KiB -- each wave streams kPer KiB of consecutive bytes
    const size_t wave = gt >> 6, lane = gt & 63;
#pragma unroll
    for (int k = 0; k < kPer; ++k) {
      const size_t i = (wave * kPer + k) * 64 + lane;
      w[k] = i < n16 ? __builtin_nontemporal_load(buf + i) : v4{0, 0, 0, 0};
    }
  }
  uint32_t acc = 0;
  if (kLds) {
    v4* dst = reinterpret_cast<v4*>(lds);
    for (uint32_t x = threadIdx.x; x < (uint32_t)kLdsWords / 4u; x += kThreads) {
      const uint32_t v = tab[(x * 7u) % 9216u];
      dst[x] = v4{v, v, v, v};
    }
    __syncthreads();
    acc = lds[(threadIdx.x * 41u) % kLdsWords];
  }
  if (kRead) {
#pragma unroll
    for (int k = 0; k < kPer; ++k) acc ^= w[k].x ^ w[k].y ^ w[k].z ^ w[k].w;
  }
  // one store per wave (keeps the loads alive)
  for (int d = 32; d > 0; d >>= 1) acc ^= __shfl_xor((int)acc, d, 64);
  if ((threadIdx.x & 63) == 0) out[gt >> 6] = acc;
  (void)nthreads;
}

// The one-launch kernel's table fill (one round trip: 11 words + 3 x 16 B per
// thread of a 36 KiB table, then 160 KiB of LDS writes), reading either one
// shared table (every group the same addresses) or a private copy per group.
template <bool kPrivate>
__global__ __launch_bounds__(kThreads) void k_fill(const uint32_t* tab, uint32_t* out) {
  __shared__ uint32_t lds[kLdsWords];
  const uint32_t* t = tab + (kPrivate ? (size_t)blockIdx.x * 9216u : 0u);
  uint32_t v[11];
  v4 u[3];
#pragma unroll
  for (int i = 0; i < 11; ++i) {
    const uint32_t x = threadIdx.x + (uint32_t)(i * kThreads);
    const uint32_t q = x >> 3;
    v[i] = x < 8192u ? t[(((q >> 9) << 1) | (q & 1u)) * 256u + ((q >> 1) & 255u)] : 0u;
  }
  const v4* nb = reinterpret_cast<const v4*>(t + 1024);
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    const uint32_t e = threadIdx.x + (uint32_t)(i * kThreads);
    u[i] = e < 2048u ? nb[e] : v4{0, 0, 0, 0};
  }
  v4* dst = reinterpret_cast<v4*>(lds);
#pragma unroll
  for (int i = 0; i < 11; ++i) {
    const uint32_t x = threadIdx.x + (uint32_t)(i * kThreads);
    if (x < 8192u) dst[x] = v4{v[i], v[i], v[i], v[i]};
  }
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    const uint32_t e = threadIdx.x + (uint32_t)(i * kThreads);
    if (e < 2048u) dst[8192u + e] = u[i];
  }
  __syncthreads();
  const uint32_t acc = lds[(threadIdx.x * 41u) % kLdsWords];
  if (acc == 0x12345678u) out[0] = acc;
}

int main(int argc, char** argv) {
  const size_t bytes = argc > 1 ? std::strtoull(argv[1], nullptr, 0) : 67529245ull;
  int dev = 0, cus = 0;
  CHECK(hipGetDevice(&dev));
  CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  const size_t n16 = (bytes + 15) / 16;
  v4* buf = nullptr;
  uint32_t *tab = nullptr, *out = nullptr;
  CHECK(hipMalloc(&buf, n16 * 16));
  CHECK(hipMalloc(&tab, (size_t)9216 * 4 * 1024));
  CHECK(hipMalloc(&out, 1 << 20));
  CHECK(hipMemset(buf, 0x5A, n16 * 16));
  CHECK(hipMemset(tab, 0x11, (size_t)9216 * 4 * 1024));
  // grid: #CUs groups of 768 (the one-launch kernel's), or enough waves that
  // every lane's kPer loads cover the buffer, whichever is larger
  const size_t lanes = (n16 + kPer - 1) / kPer;
  int grid = cus;
  if ((size_t)grid * kThreads < lanes) grid = (int)((lanes + kThreads - 1) / kThreads);
  hipStream_t s;
  CHECK(hipStreamCreate(&s));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  auto timed = [&](auto launch) {
    for (int i = 0; i < 10; ++i) launch();
    float best = 1e30f;
    for (int r = 0; r < 5; ++r) {
      CHECK(hipEventRecord(e0, s));
      for (int i = 0; i < 100; ++i) launch();
      CHECK(hipEventRecord(e1, s));
      CHECK(hipEventSynchronize(e1));
      float ms = 0;
      CHECK(hipEventElapsedTime(&ms, e0, e1));
      if (ms < best) best = ms;
    }
    return best * 10.0f;  // us per launch (100 launches)
  };
  const float t_empty = timed([&] { k_empty<<<cus, kThreads, 0, s>>>(out); });
  const float t_lds = timed([&] { k_probe<true, false><<<cus, kThreads, 0, s>>>(buf, n16, tab, out); });
  const float t_read = timed([&] { k_probe<false, true><<<grid, kThreads, 0, s>>>(buf, n16, tab, out); });
  const float t_read_lds = timed([&] { k_probe<true, true><<<grid, kThreads, 0, s>>>(buf, n16, tab, out); });
  // the fill right after a file-sized read (the table lines evicted from L2,
  // as between back-to-back calls): read + fill pairs minus the reads alone
  const float t_fill_shared = timed([&] {
    k_probe<false, true><<<grid, kThreads, 0, s>>>(buf, n16, tab, out);
    k_fill<false><<<cus, kThreads, 0, s>>>(tab, out);
  }) - t_read;
  const float t_fill_private = timed([&] {
    k_probe<false, true><<<grid, kThreads, 0, s>>>(buf, n16, tab, out);
    k_fill<true><<<cus, kThreads, 0, s>>>(tab, out);
  }) - t_read;
  const float t_fill_hot = timed([&] { k_fill<false><<<cus, kThreads, 0, s>>>(tab, out); });
  CHECK(hipGetLastError());
  std::printf("{\"bytes\": %zu, \"cus\": %d, \"grid_read\": %d, \"empty_us\": %.2f, \"lds_fill_us\": %.2f, "
              "\"read_us\": %.2f, \"read_lds_us\": %.2f, \"read_TBps\": %.2f, \"fill_hot_us\": %.2f, "
              "\"fill_after_read_shared_us\": %.2f, \"fill_after_read_private_us\": %.2f}\n",
              bytes, cus, grid, t_empty, t_lds, t_read, t_read_lds, bytes / (t_read * 1e-6) / 1e12, t_fill_hot,
              t_fill_shared, t_fill_private);
  return 0;
}
