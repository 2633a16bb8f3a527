// Stand-alone per-incident top-k over explicit dense score / reach arrays (SURVEY.md §8b
// `egr_topk`; the custom op torch.ops.egraph.topk).  The engines rank inside their own state
// (egr_plan_topk, the frontier's fused top-k); this entry point ranks arrays a caller holds:
// scores row-major [V][n_cols] fp32 and reach bits [ceil(n_cols/64)][V] u64 (the layouts of
// egr_plan_read_scores / egr_plan_read_reach).  Order: score descending, vertex id ascending
// (the (score, ~id) u64 key of csrc/frontier_body.h), over the reached vertices whose label is
// not exclude_label; EGR_NO_NODE / -inf pad.
//
// Layout: one 256-thread workgroup per 64 columns.  Wave w walks the vertices v = w (mod 4);
// lane c reads scores[v][b0 + c], so a wave's 64 loads are one contiguous 256-B row segment,
// and the reach word and the label of v are one broadcast load each.  Every lane keeps its
// column's k best keys in registers (an unrolled compare-exchange chain, KMAX deep); the four
// waves' lists then meet in LDS and lane c of wave 0 merges its column's four lists.
// Bound: HBM, V * n_cols * 4 B of scores read once (+ V*(8 + 1) B per 64 columns).
#include "graph_dev.h"

using egr::DeviceGuard;

namespace {

constexpr int TK_MAX = 16;
constexpr int TK_WAVES = 4;

__device__ __forceinline__ uint64_t tk_key(float s, uint32_t v) {
  const uint32_t f = __float_as_uint(s);
  const uint32_t o = (f & 0x80000000u) ? ~f : (f | 0x80000000u);
  return ((uint64_t)o << 32) | (uint32_t)~v;
}

__device__ __forceinline__ void tk_unkey(uint64_t k, float& s, uint32_t& v) {
  if (k == 0) {
    s = -INFINITY;
    v = EGR_NO_NODE;
    return;
  }
  const uint32_t o = (uint32_t)(k >> 32);
  s = __uint_as_float((o & 0x80000000u) ? (o & 0x7FFFFFFFu) : ~o);
  v = ~(uint32_t)k;
}

// keep the TK_MAX largest keys of the stream, descending (0 = empty)
__device__ __forceinline__ void tk_push(uint64_t (&best)[TK_MAX], uint64_t key) {
#pragma unroll
  for (int j = 0; j < TK_MAX; ++j) {
    const uint64_t b = best[j];
    const bool gt = key > b;
    best[j] = gt ? key : b;
    key = gt ? b : key;
  }
}

__global__ __launch_bounds__(64 * TK_WAVES) void dense_topk_kernel(
    const float* __restrict__ scores, const uint64_t* __restrict__ reach,
    const uint8_t* __restrict__ vlabel, uint32_t V, int B, int k, int exclude,
    uint32_t* __restrict__ out_ids, float* __restrict__ out_scores) {
  __shared__ uint64_t lists[TK_WAVES][TK_MAX][64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int w = blockIdx.x;                       // reach word = 64-column group
  const int b = w * 64 + lane;
  const bool col_ok = b < B;
  uint64_t best[TK_MAX];
#pragma unroll
  for (int j = 0; j < TK_MAX; ++j) best[j] = 0;
  const uint64_t* rw = reach + (size_t)w * V;
  for (uint32_t v = wave; v < V; v += TK_WAVES) {
    const uint64_t bits = rw[v];                  // broadcast
    if (!bits) continue;                          // uniform: nobody in this group reached v
    if (exclude >= 0 && vlabel[v] == (uint8_t)exclude) continue;
    if (col_ok && ((bits >> lane) & 1ull)) tk_push(best, tk_key(scores[(size_t)v * B + b], v));
  }
#pragma unroll
  for (int j = 0; j < TK_MAX; ++j) lists[wave][j][lane] = best[j];
  __syncthreads();
  if (wave != 0 || !col_ok) return;
  int pos[TK_WAVES] = {0, 0, 0, 0};
  for (int q = 0; q < k; ++q) {
    uint64_t m = 0;
    int from = -1;
#pragma unroll
    for (int x = 0; x < TK_WAVES; ++x) {
      const uint64_t c = pos[x] < TK_MAX ? lists[x][pos[x]][lane] : 0ull;
      if (c > m) {
        m = c;
        from = x;
      }
    }
    if (from >= 0) ++pos[from];
    float s;
    uint32_t v;
    tk_unkey(m, s, v);
    out_ids[(size_t)b * k + q] = v;
    out_scores[(size_t)b * k + q] = s;
  }
}

}  // namespace

extern "C" {

int egr_topk(const egr_snapshot* s, const float* scores, const uint64_t* reach, int32_t n_cols,
             int32_t k, int32_t exclude_label, uint32_t* out_ids, float* out_scores, void* stream) {
  if (!s || !scores || !reach || !out_ids || !out_scores || n_cols <= 0 || k < 1 || k > TK_MAX)
    return egr::fail(EGR_EINVAL, "egr_topk: bad arguments (need n_cols > 0, 1 <= k <= 16)");
  DeviceGuard guard(s->device);   // (V = 0: every wave's walk is empty, all slots pad)
  const int groups = (n_cols + 63) / 64;
  hipLaunchKernelGGL(dense_topk_kernel, dim3(groups), dim3(64 * TK_WAVES), 0, (hipStream_t)stream,
                     scores, reach, s->vlabel, (uint32_t)s->V, n_cols, k, exclude_label, out_ids,
                     out_scores);
  EGR_CHECK_LAUNCH();
  return EGR_OK;
}

}  // extern "C"
