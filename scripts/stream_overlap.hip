// Probe: do two streams (and the two branches of a captured HIP graph) run concurrently, and
// can a few persistent workgroups launched on a second stream ahead of a 20k-workgroup grid
// see that grid's progress while it runs?  (The design question behind a concurrent overflow
// retry for the frontier's narrow grid.)  Every wait is bounded by a wall-clock limit, so a
// serialised schedule only shows up as "seen = 0" and a long time, never as a hang.
//
//   hipcc --offload-arch=gfx950 -O2 scripts/stream_overlap.hip -o /tmp/stream_overlap
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>

#define CK(x)                                                                        \
  do {                                                                               \
    hipError_t e_ = (x);                                                             \
    if (e_ != hipSuccess) {                                                          \
      std::printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
      return 1;                                                                      \
    }                                                                                \
  } while (0)

constexpr unsigned long long LIMIT_TICKS = 2000000ull;   // 20 ms at 100 MHz

__device__ unsigned long long now() { return __builtin_amdgcn_s_memrealtime(); }

// one workgroup per entry of `out`: lane 0 waits until *ctr >= target or the limit; writes
// (seen, wait ticks)
__global__ void waiter(const unsigned* ctr, unsigned target, unsigned long long* out) {
  if (threadIdx.x != 0) return;
  const unsigned long long t0 = now();
  unsigned seen = 0;
  for (;;) {
    if (__hip_atomic_load(ctr, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) >= target) { seen = 1; break; }
    if (now() - t0 > LIMIT_TICKS) break;
    __builtin_amdgcn_s_sleep(8);
  }
  out[2 * blockIdx.x] = seen;
  out[2 * blockIdx.x + 1] = now() - t0;
}

// a grid of workgroups with `lds` bytes of LDS each, ~`spin` ticks of work, counting itself done
__global__ void worker(unsigned* ctr, unsigned long long spin) {
  extern __shared__ unsigned lds[];
  lds[threadIdx.x] = threadIdx.x;
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned long long t0 = now();
    while (now() - t0 < spin) __builtin_amdgcn_s_sleep(2);
    __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
  }
}

__global__ void zero(unsigned* ctr) { if (threadIdx.x == 0) *ctr = 0; }

static double ms_since(std::chrono::steady_clock::time_point t) {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t).count();
}

int main() {
  unsigned* ctr;
  unsigned long long* out;
  CK(hipMalloc(&ctr, 4));
  CK(hipMalloc(&out, 64 * 16));
  hipStream_t s1, s2;
  CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
  hipEvent_t e0, e1;
  CK(hipEventCreateWithFlags(&e0, hipEventDisableTiming));
  CK(hipEventCreateWithFlags(&e1, hipEventDisableTiming));
  const int NW = 16, NG = 20480;
  const size_t LDS = 22 * 1024;
  const unsigned long long SPIN = 3000;   // 30 us per grid workgroup
  unsigned long long h[2 * NW];

  auto report = [&](const char* what, double ms) {
    if (hipMemcpy(h, out, sizeof h, hipMemcpyDeviceToHost) != hipSuccess) return;
    int seen = 0;
    double wmax = 0;
    for (int i = 0; i < NW; ++i) {
      seen += (int)h[2 * i];
      wmax = std::max(wmax, h[2 * i + 1] / 100.0);
    }
    std::printf("%-44s seen %2d/%d  max wait %8.1f us  host %7.3f ms\n", what, seen, NW, wmax, ms);
  };
  // enqueue: zero on s1, fork s2 (waiters), grid on s1, join
  auto enqueue = [&](bool waiters_first) -> hipError_t {
    hipLaunchKernelGGL(zero, dim3(1), dim3(64), 0, s1, ctr);
    hipError_t e = hipEventRecord(e0, s1);
    if (e != hipSuccess) return e;
    if ((e = hipStreamWaitEvent(s2, e0, 0)) != hipSuccess) return e;
    if (waiters_first) {
      hipLaunchKernelGGL(waiter, dim3(NW), dim3(64), 0, s2, ctr, (unsigned)NG, out);
      hipLaunchKernelGGL(worker, dim3(NG), dim3(256), LDS, s1, ctr, SPIN);
    } else {
      hipLaunchKernelGGL(worker, dim3(NG), dim3(256), LDS, s1, ctr, SPIN);
      hipLaunchKernelGGL(waiter, dim3(NW), dim3(64), 0, s2, ctr, (unsigned)NG, out);
    }
    if ((e = hipEventRecord(e1, s2)) != hipSuccess) return e;
    return hipStreamWaitEvent(s1, e1, 0);
  };
  // grid alone, for its duration
  for (int rep = 0; rep < 3; ++rep) {
    auto t = std::chrono::steady_clock::now();
    hipLaunchKernelGGL(zero, dim3(1), dim3(64), 0, s1, ctr);
    hipLaunchKernelGGL(worker, dim3(NG), dim3(256), LDS, s1, ctr, SPIN);
    CK(hipStreamSynchronize(s1));
    std::printf("%-44s host %7.3f ms\n", "grid alone", ms_since(t));
  }
  for (int wf = 1; wf >= 0; --wf) {
    for (int rep = 0; rep < 2; ++rep) {
      auto t = std::chrono::steady_clock::now();
      CK(enqueue(wf));
      CK(hipStreamSynchronize(s1));
      report(wf ? "streams, waiters first" : "streams, grid first", ms_since(t));
    }
  }
  for (int wf = 1; wf >= 0; --wf) {
    hipGraph_t g;
    hipGraphExec_t ge;
    CK(hipStreamBeginCapture(s1, hipStreamCaptureModeThreadLocal));
    CK(enqueue(wf));
    CK(hipStreamEndCapture(s1, &g));
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    for (int rep = 0; rep < 3; ++rep) {
      auto t = std::chrono::steady_clock::now();
      CK(hipGraphLaunch(ge, s1));
      CK(hipStreamSynchronize(s1));
      report(wf ? "graph, waiters first" : "graph, grid first", ms_since(t));
    }
    CK(hipGraphExecDestroy(ge));
    CK(hipGraphDestroy(g));
  }
  CK(hipDeviceSynchronize());
  std::printf("done\n");
  return 0;
}
