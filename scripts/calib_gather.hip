// Calibration of the L2 -> fabric read-request counter (TCC_EA0_RDREQ) for the access widths of
// the frontier kernel (MI355X_MICROARCH.md, HBM section: "other access widths are uncalibrated:
// calibrate on a known byte count in your own access pattern").  Each kernel below reads a KNOWN
// set of cache lines from a buffer evicted from L2 and the Infinity Cache beforehand (a 1-GiB
// write sweep); rocprofv3 --pmc TCC_EA0_RDREQ_sum gives the requests per dispatch, so
// requests / lines = requests per 128-B line for that pattern:
//   stream16   16 B per lane, fully coalesced, 256 MiB             (the guide's reference case)
//   stride128  one 8-B load per 128-B line, 4M lines              (a sparse gather, one per line)
//   stride64   one 8-B load per 64-B half line, 8M loads = 4M lines
//   random8    4M 8-B loads at random entries of a 2-GiB table     (the frontier's cv gathers)
// Build: hipcc -O3 --offload-arch=gfx950 scripts/calib_gather.hip -o <out>   (scripts/gpu_calib.sh)
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHECK(x)                                                                      \
  do {                                                                                \
    hipError_t e_ = (x);                                                              \
    if (e_ != hipSuccess) {                                                           \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                    \
      std::exit(1);                                                                   \
    }                                                                                 \
  } while (0)

__global__ void flush_kernel(uint4* p, size_t n) {   // a write sweep larger than L2 + MALL
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    p[i] = make_uint4((uint32_t)i, 0u, 0u, 0u);
}

__global__ void stream16_kernel(const uint4* p, size_t n, uint32_t* sink) {
  uint32_t acc = 0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const uint4 v = p[i];
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x12345678u) sink[0] = acc;
}

// one 8-B load every `stride` bytes
__global__ void stride_kernel(const uint2* p, size_t n, uint32_t stride8, uint32_t* sink) {
  uint32_t acc = 0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const uint2 v = p[i * stride8];
    acc ^= v.x ^ v.y;
  }
  if (acc == 0x12345678u) sink[0] = acc;
}

__global__ void random8_kernel(const uint2* p, const uint32_t* idx, size_t n, uint32_t* sink) {
  uint32_t acc = 0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const uint2 v = p[idx[i]];
    acc ^= v.x ^ v.y;
  }
  if (acc == 0x12345678u) sink[0] = acc;
}

int main() {
  const size_t big = 1ull << 30;                 // 1 GiB flush buffer
  const size_t tab = 2ull << 30;                 // 2 GiB gather table
  uint4* flush;
  uint2* t;
  uint32_t *idx, *sink;
  const size_t n_rand = 4u << 20;
  CHECK(hipMalloc(&flush, big));
  CHECK(hipMalloc(&t, tab));
  CHECK(hipMalloc(&idx, n_rand * 4));
  CHECK(hipMalloc(&sink, 4));
  CHECK(hipMemset(t, 1, tab));
  // random entries, each in a distinct 128-B line (line = entry / 16): a permutation of lines
  const size_t lines = tab / 128;
  std::vector<uint32_t> h(n_rand);
  uint64_t s = 88172645463325252ull;
  for (size_t i = 0; i < n_rand; ++i) {
    s ^= s << 13; s ^= s >> 7; s ^= s << 17;
    h[i] = (uint32_t)(((i * (lines / n_rand)) + s % (lines / n_rand)) * 16 + (s >> 40) % 16);
  }
  for (size_t i = n_rand - 1; i > 0; --i) {       // shuffle the visiting order
    s ^= s << 13; s ^= s >> 7; s ^= s << 17;
    std::swap(h[i], h[s % (i + 1)]);
  }
  CHECK(hipMemcpy(idx, h.data(), n_rand * 4, hipMemcpyHostToDevice));
  auto cold = [&]() {
    hipLaunchKernelGGL(flush_kernel, dim3(4096), dim3(256), 0, 0, flush, big / 16);
    CHECK(hipDeviceSynchronize());
  };
  const size_t n16 = (256ull << 20) / 16;
  cold();
  hipLaunchKernelGGL(stream16_kernel, dim3(4096), dim3(256), 0, 0, reinterpret_cast<const uint4*>(t), n16, sink);
  CHECK(hipDeviceSynchronize());
  std::printf("stream16  bytes %zu lines128 %zu\n", n16 * 16, n16 * 16 / 128);
  const size_t n128 = 4u << 20;
  cold();
  hipLaunchKernelGGL(stride_kernel, dim3(4096), dim3(256), 0, 0, t, n128, 16u, sink);
  CHECK(hipDeviceSynchronize());
  std::printf("stride128 loads %zu lines128 %zu\n", n128, n128);
  cold();
  hipLaunchKernelGGL(stride_kernel, dim3(4096), dim3(256), 0, 0, t, 2 * n128, 8u, sink);
  CHECK(hipDeviceSynchronize());
  std::printf("stride64  loads %zu lines128 %zu\n", 2 * n128, n128);
  cold();
  hipLaunchKernelGGL(random8_kernel, dim3(4096), dim3(256), 0, 0, t, idx, n_rand, sink);
  CHECK(hipDeviceSynchronize());
  std::printf("random8   loads %zu lines128 %zu (idx stream %zu B)\n", n_rand, n_rand, n_rand * 4);
  return 0;
}
