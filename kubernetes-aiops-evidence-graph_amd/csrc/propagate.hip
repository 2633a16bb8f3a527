// Graph stages on the device snapshot:
//   A8  reach  : k-hop undirected reachability from each incident vertex, 64 incidents per u64
//                word (apoc.path.subgraphAll(maxLevel=k), src/database/neo4j.py:169-202);
//   A9  hop    : typed propagation s^{h+1}_v = s0_v + sum_{(u,t,d) in row v} val_e * s^h_u,
//                val_e = w[t][d] / deg(u), fp32, accumulated with fmaf in CSR order so the
//                result is bit-identical to oracle/egraph_oracle.c;
//       topk   : per incident, top-k vertices of the final scores over its reach set, score
//                descending, vertex id ascending on ties.
//
// Layout: scores are tiled [B/TW][V][TW] fp32 (TW = 64/16/4 columns), so a
// pull-gather of one neighbour row is TW*4 contiguous bytes (256 B at TW = 64) served by G = TW/4
// lanes with one float4 each, and the whole gather working set of a launch is one tile
// (V*TW*4 B = 64 MB at 250k vertices), which the 256 MB Infinity Cache holds while the grid,
// ordered tile-major, sweeps it.  Row blocks are remapped so that each XCD streams a contiguous
// vertex range (its L2 sees the namespace locality of the snapshot's vertex order).
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <vector>

#include "egr_internal.h"

struct egr_snapshot {
  int device = 0;
  int64_t V = 0, NE = 0;
  uint32_t* row_ptr = nullptr;
  uint32_t* col = nullptr;
  uint8_t* meta = nullptr;
  float* val = nullptr;
  uint8_t* vlabel = nullptr;
};

namespace {

constexpr int KMAX = 16;              // top-k capacity per list
constexpr int TOPK_CHUNK = 1024;      // rows per wave in top-k phase 1
constexpr uint32_t NO_NODE = EGR_NO_NODE;

struct DeviceGuard {
  int prev = -1;
  explicit DeviceGuard(int dev) {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    if (prev != dev) (void)hipSetDevice(dev);
  }
  ~DeviceGuard() {
    int cur;
    if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
  }
};

// Contiguous row ranges per XCD: workgroups are dealt round-robin over the 8 XCDs, so block l
// of a tile (nrb padded to a multiple of 8) runs on XCD l % 8; give that XCD the (l/8)-th block
// of its own contiguous eighth.  Speed only -- any placement gives the same result.
__device__ __forceinline__ uint32_t xcd_remap(uint32_t l, uint32_t nrb8) {
  const uint32_t per = nrb8 >> 3;
  return (l & 7u) * per + (l >> 3);
}

__device__ __forceinline__ void fma4(float w, const float4& x, float4& a) {
  a.x = fmaf(w, x.x, a.x);
  a.y = fmaf(w, x.y, a.y);
  a.z = fmaf(w, x.z, a.z);
  a.w = fmaf(w, x.w, a.w);
}

__device__ __forceinline__ void add_comp(float4& a, int c, float s) {
  if (c == 0) a.x = a.x + s;
  else if (c == 1) a.y = a.y + s;
  else if (c == 2) a.z = a.z + s;
  else a.w = a.w + s;
}

__device__ __forceinline__ void fma_comp(float4& a, int c, float w, float s) {
  if (c == 0) a.x = fmaf(w, s, a.x);
  else if (c == 1) a.y = fmaf(w, s, a.y);
  else if (c == 2) a.z = fmaf(w, s, a.z);
  else a.w = fmaf(w, s, a.w);
}

// first index in [s0, s1) whose column is >= lo (seed lists are sorted by column); hub
// vertices can carry one seed per incident, so long lists are bisected
__device__ __forceinline__ uint32_t seed_lower(const uint32_t* __restrict__ seed_col, uint32_t s0,
                                               uint32_t s1, uint32_t lo) {
  if (s1 - s0 <= 8u) {
    while (s0 < s1 && seed_col[s0] < lo) ++s0;
    return s0;
  }
  while (s0 < s1) {
    const uint32_t mid = (s0 + s1) >> 1;
    if (seed_col[mid] < lo) s0 = mid + 1;
    else s1 = mid;
  }
  return s0;
}

// s0 of row v for this lane's 4 columns [tile*TW + 4*gl, +4)
__device__ __forceinline__ void add_seeds(float4& acc, uint32_t v, uint32_t lo,
                                          const uint32_t* __restrict__ seed_ptr,
                                          const uint32_t* __restrict__ seed_col,
                                          const float* __restrict__ seed_val) {
  const uint32_t s1 = seed_ptr[v + 1];
  for (uint32_t s = seed_lower(seed_col, seed_ptr[v], s1, lo); s < s1; ++s) {
    const uint32_t c = seed_col[s] - lo;
    if (c >= 4u) break;
    add_comp(acc, (int)c, seed_val[s]);
  }
}

// ---- hop from sparse seeds (h = 0 -> 1): gathers s0_u straight from the seed lists ---------
template <int G>
__global__ __launch_bounds__(256) void hop_from_seeds_kernel(
    const uint32_t* __restrict__ row_ptr, const uint32_t* __restrict__ col,
    const float* __restrict__ val, const uint32_t* __restrict__ seed_ptr,
    const uint32_t* __restrict__ seed_col, const float* __restrict__ seed_val,
    float* __restrict__ xout, uint32_t V, uint32_t nrb8) {
  constexpr int TW = 4 * G;
  constexpr int ROWS = 256 / G;
  const uint32_t gl = threadIdx.x % G;
  const uint32_t tile = blockIdx.x / nrb8;
  const uint32_t rb = xcd_remap(blockIdx.x % nrb8, nrb8);
  const uint32_t v = rb * ROWS + threadIdx.x / G;
  if (v >= V) return;
  const uint32_t lo = tile * TW + 4 * gl;
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  const uint32_t e1 = row_ptr[v + 1];
  for (uint32_t e = row_ptr[v]; e < e1; ++e) {
    const uint32_t u = col[e];
    const uint32_t s0 = seed_ptr[u], s1 = seed_ptr[u + 1];
    if (s0 == s1) continue;  // contribution w*0: skipping it is exact (acc is never -0.0)
    const float w = val[e];
    for (uint32_t s = seed_lower(seed_col, s0, s1, lo); s < s1; ++s) {
      const uint32_t c = seed_col[s] - lo;
      if (c >= 4u) break;
      fma_comp(acc, (int)c, w, seed_val[s]);
    }
  }
  add_seeds(acc, v, lo, seed_ptr, seed_col, seed_val);
  reinterpret_cast<float4*>(xout + (size_t)tile * V * TW)[(size_t)v * G + gl] = acc;
}

// ---- dense hop (h >= 1): pull-gather TW-wide neighbour rows, 4 entries in flight ----------
template <int G>
__global__ __launch_bounds__(256) void hop_kernel(
    const uint32_t* __restrict__ row_ptr, const uint32_t* __restrict__ col,
    const float* __restrict__ val, const uint32_t* __restrict__ seed_ptr,
    const uint32_t* __restrict__ seed_col, const float* __restrict__ seed_val,
    const float* __restrict__ xin, float* __restrict__ xout, uint32_t V, uint32_t nrb8) {
  constexpr int TW = 4 * G;
  constexpr int ROWS = 256 / G;
  const uint32_t gl = threadIdx.x % G;
  const uint32_t tile = blockIdx.x / nrb8;
  const uint32_t rb = xcd_remap(blockIdx.x % nrb8, nrb8);
  const uint32_t v = rb * ROWS + threadIdx.x / G;
  if (v >= V) return;
  const size_t toff = (size_t)tile * V * TW;
  const float4* __restrict__ X = reinterpret_cast<const float4*>(xin + toff);
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  uint32_t e = row_ptr[v];
  const uint32_t e1 = row_ptr[v + 1];
  for (; e + 4 <= e1; e += 4) {
    const uint32_t u0 = col[e], u1 = col[e + 1], u2 = col[e + 2], u3 = col[e + 3];
    const float w0 = val[e], w1 = val[e + 1], w2 = val[e + 2], w3 = val[e + 3];
    const float4 a0 = X[(size_t)u0 * G + gl];
    const float4 a1 = X[(size_t)u1 * G + gl];
    const float4 a2 = X[(size_t)u2 * G + gl];
    const float4 a3 = X[(size_t)u3 * G + gl];
    fma4(w0, a0, acc);
    fma4(w1, a1, acc);
    fma4(w2, a2, acc);
    fma4(w3, a3, acc);
  }
  for (; e < e1; ++e) fma4(val[e], X[(size_t)col[e] * G + gl], acc);
  add_seeds(acc, v, tile * TW + 4 * gl, seed_ptr, seed_col, seed_val);
  reinterpret_cast<float4*>(xout + toff)[(size_t)v * G + gl] = acc;
}

// ---- reachability ----------------------------------------------------------------------------
__global__ void reach_sources_kernel(const uint32_t* __restrict__ src, int B, uint64_t* R,
                                     uint32_t V) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  const uint32_t v = src[b];
  if (v < V) atomicOr((unsigned long long*)&R[(size_t)(b >> 6) * V + v], 1ull << (b & 63));
}

__global__ __launch_bounds__(256) void reach_hop_kernel(const uint32_t* __restrict__ row_ptr,
                                                        const uint32_t* __restrict__ col,
                                                        const uint64_t* __restrict__ rin,
                                                        uint64_t* __restrict__ rout, uint32_t V,
                                                        uint32_t nrb8) {
  const uint32_t w = blockIdx.x / nrb8;
  const uint32_t v = xcd_remap(blockIdx.x % nrb8, nrb8) * 256 + threadIdx.x;
  if (v >= V) return;
  const uint64_t* R = rin + (size_t)w * V;
  uint64_t acc = R[v];
  const uint32_t e1 = row_ptr[v + 1];
  for (uint32_t e = row_ptr[v]; e < e1; ++e) acc |= R[col[e]];
  rout[(size_t)w * V + v] = acc;
}

// ---- seeds: (vertex, column, value) triples -> unique per-vertex lists (max-combined) ----------
__global__ void seed_keys_kernel(const uint32_t* __restrict__ sv, const uint32_t* __restrict__ sc,
                                 const float* __restrict__ sval, int64_t n, uint32_t V, int B,
                                 uint32_t Bpad, uint64_t* keys, float* vals) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t v = sv[i], c = sc[i];
  const bool ok = v < V && c < (uint32_t)B;
  keys[i] = ok ? (uint64_t)v * Bpad + c : ~0ull;
  vals[i] = sval[i];
}

__global__ void seed_head_kernel(const uint64_t* __restrict__ keys, int64_t n, uint32_t* head) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint64_t k = keys[i];
  head[i] = (k != ~0ull && (i == 0 || keys[i - 1] != k)) ? 1u : 0u;
}

__global__ void seed_compact_kernel(const uint64_t* __restrict__ keys,
                                    const float* __restrict__ vals,
                                    const uint32_t* __restrict__ head,
                                    const uint32_t* __restrict__ pos, int64_t n, uint32_t Bpad,
                                    uint64_t* ukeys, uint32_t* ucol, float* uval,
                                    uint32_t* n_unique) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  if (i == n - 1) *n_unique = pos[i] + head[i];
  if (!head[i]) return;
  const uint64_t k = keys[i];
  float m = vals[i];
  for (int64_t j = i + 1; j < n && keys[j] == k; ++j) m = fmaxf(m, vals[j]);
  const uint32_t p = pos[i];
  ukeys[p] = k;
  ucol[p] = (uint32_t)(k % Bpad);
  uval[p] = m;
}

__global__ void seed_ptr_kernel(const uint64_t* __restrict__ ukeys,
                                const uint32_t* __restrict__ n_unique, uint32_t V, uint32_t Bpad,
                                uint32_t* seed_ptr) {
  const uint32_t v = blockIdx.x * blockDim.x + threadIdx.x;
  if (v > V) return;
  const uint64_t target = (uint64_t)v * Bpad;
  uint32_t lo = 0, hi = *n_unique;
  while (lo < hi) {
    const uint32_t mid = (lo + hi) >> 1;
    if (ukeys[mid] < target) lo = mid + 1;
    else hi = mid;
  }
  seed_ptr[v] = lo;
}

__global__ void zero_seed_ptr_kernel(uint32_t* seed_ptr, uint32_t V) {
  const uint32_t v = blockIdx.x * blockDim.x + threadIdx.x;
  if (v <= V) seed_ptr[v] = 0;
}

// ---- top-k -----------------------------------------------------------------------------------
struct Cand {
  float s;
  uint32_t v;
};

__device__ __forceinline__ bool better(float s, uint32_t v, float ls, uint32_t lv) {
  return lv == NO_NODE || s > ls || (s == ls && v < lv);
}

// insert (s, v) into the sorted (best-first) register list L[0..KMAX); walking down from the
// tail, each slot takes its predecessor, the new entry, or keeps its value
__device__ __forceinline__ void list_insert(float (&Ls)[KMAX], uint32_t (&Lv)[KMAX], float s,
                                            uint32_t v) {
  if (!better(s, v, Ls[KMAX - 1], Lv[KMAX - 1])) return;
#pragma unroll
  for (int i = KMAX - 1; i > 0; --i) {
    const bool up = better(s, v, Ls[i - 1], Lv[i - 1]);
    const bool here = better(s, v, Ls[i], Lv[i]);
    Ls[i] = up ? Ls[i - 1] : (here ? s : Ls[i]);
    Lv[i] = up ? Lv[i - 1] : (here ? v : Lv[i]);
  }
  if (better(s, v, Ls[0], Lv[0])) {
    Ls[0] = s;
    Lv[0] = v;
  }
}

__global__ __launch_bounds__(256) void topk_partial_kernel(
    const float* __restrict__ X, const uint64_t* __restrict__ R,
    const uint8_t* __restrict__ vlabel, int exclude_label, uint32_t V, int TW, int B,
    int n_chunks, float* __restrict__ part_s, uint32_t* __restrict__ part_v) {
  const int lane = threadIdx.x & 63;
  const int wid = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int ntiles = (B + TW - 1) / TW;
  if (wid >= ntiles * n_chunks) return;
  const int tile = wid / n_chunks, ch = wid % n_chunks;
  const int c = lane % TW, rp = lane / TW, rps = 64 / TW;
  const int b = tile * TW + c;
  float Ls[KMAX];
  uint32_t Lv[KMAX];
#pragma unroll
  for (int i = 0; i < KMAX; ++i) {
    Ls[i] = -INFINITY;
    Lv[i] = NO_NODE;
  }
  if (b < B) {
    const float* Xt = X + (size_t)tile * V * TW;
    const uint64_t* Rw = R + (size_t)(b >> 6) * V;
    const uint64_t bit = 1ull << (b & 63);
    const uint32_t v0 = (uint32_t)ch * TOPK_CHUNK;
    const uint32_t v1 = min(V, v0 + TOPK_CHUNK);
    for (uint32_t v = v0 + rp; v < v1; v += rps) {
      if (!(Rw[v] & bit)) continue;
      if (exclude_label >= 0 && vlabel[v] == (uint8_t)exclude_label) continue;
      list_insert(Ls, Lv, Xt[(size_t)v * TW + c], v);
    }
  }
  const size_t o = ((size_t)wid * 64 + lane) * KMAX;
#pragma unroll
  for (int i = 0; i < KMAX; ++i) {
    part_s[o + i] = Ls[i];
    part_v[o + i] = Lv[i];
  }
}

__global__ __launch_bounds__(256) void topk_merge_kernel(
    const float* __restrict__ part_s, const uint32_t* __restrict__ part_v, int TW, int B,
    int n_chunks, int k, uint32_t* __restrict__ out_ids, float* __restrict__ out_scores) {
  const int lane = threadIdx.x & 63;
  const int b = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (b >= B) return;
  const int tile = b / TW, c = b % TW, rps = 64 / TW;
  float Ls[KMAX];
  uint32_t Lv[KMAX];
#pragma unroll
  for (int i = 0; i < KMAX; ++i) {
    Ls[i] = -INFINITY;
    Lv[i] = NO_NODE;
  }
  // candidate lists of column b: chunks x (lanes with lane % TW == c), KMAX entries each
  const int n_lists = n_chunks * rps;
  for (int li = lane; li < n_lists; li += 64) {
    const int ch = li / rps, rp = li % rps;
    const size_t o = (((size_t)(tile * n_chunks + ch)) * 64 + rp * TW + c) * KMAX;
    for (int i = 0; i < k; ++i) {
      const uint32_t v = part_v[o + i];
      if (v == NO_NODE) break;
      list_insert(Ls, Lv, part_s[o + i], v);
    }
  }
  // k rounds of a wave-wide arg-best over the list heads
  for (int q = 0; q < k; ++q) {
    float bs = Ls[0];
    uint32_t bv = Lv[0];
    int bl = lane;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
      const float os = __shfl_xor(bs, off, 64);
      const uint32_t ov = __shfl_xor(bv, off, 64);
      const int ol = __shfl_xor(bl, off, 64);
      if (ov != NO_NODE && better(os, ov, bs, bv)) {
        bs = os;
        bv = ov;
        bl = ol;
      }
    }
    if (lane == 0) {
      out_ids[(size_t)b * k + q] = bv;
      out_scores[(size_t)b * k + q] = bv == NO_NODE ? -INFINITY : bs;
    }
    if (bv != NO_NODE && lane == bl) {
#pragma unroll
      for (int i = 0; i < KMAX - 1; ++i) {
        Ls[i] = Ls[i + 1];
        Lv[i] = Lv[i + 1];
      }
      Ls[KMAX - 1] = -INFINITY;
      Lv[KMAX - 1] = NO_NODE;
    }
  }
}

__global__ void scores_rowmajor_kernel(const float* __restrict__ X, uint32_t V, int TW, int B,
                                       float* __restrict__ out) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (size_t)V * B) return;
  const uint32_t v = (uint32_t)(i / B);
  const int b = (int)(i % B);
  out[i] = X[((size_t)(b / TW) * V + v) * TW + (b % TW)];
}

__global__ void induced_kernel(const uint32_t* __restrict__ row_ptr,
                               const uint32_t* __restrict__ col, const uint8_t* __restrict__ meta,
                               const uint64_t* __restrict__ Rw, uint64_t bit, uint32_t V,
                               uint32_t* osrc, uint32_t* odst, uint8_t* otype, int64_t cap,
                               unsigned long long* counter) {
  const uint32_t v = blockIdx.x * blockDim.x + threadIdx.x;
  if (v >= V || !(Rw[v] & bit)) return;
  for (uint32_t e = row_ptr[v]; e < row_ptr[v + 1]; ++e) {
    const uint8_t m = meta[e];
    if (m & 1u) continue;  // dir 1 duplicates: each edge is listed once, in its target's row
    const uint32_t u = col[e];
    if (!(Rw[u] & bit)) continue;
    const unsigned long long slot = atomicAdd(counter, 1ull);
    if ((int64_t)slot < cap) {
      osrc[slot] = u;
      odst[slot] = v;
      otype[slot] = m >> 1;
    }
  }
}

}  // namespace

struct egr_plan {
  const egr_snapshot* s = nullptr;
  int B = 0, TW = 0, Bpad = 0, ntiles = 0, W = 0, k = 0;
  int64_t max_seeds = 0;
  int n_chunks = 0;
  uint32_t nrb8_hop = 0, nrb8_reach = 0;
  float* x[2] = {nullptr, nullptr};
  int xcur = 0;
  uint64_t* reach[2] = {nullptr, nullptr};
  int rcur = 0;
  int reach_hops = -1;  // -1: sources not set
  // seeds
  uint64_t *skeys_in = nullptr, *skeys = nullptr, *ukeys = nullptr;
  float *svals_in = nullptr, *svals = nullptr, *uval = nullptr;
  uint32_t *head = nullptr, *pos = nullptr, *ucol = nullptr, *seed_ptr = nullptr,
           *n_unique = nullptr;
  void* cub_tmp = nullptr;
  size_t cub_tmp_bytes = 0;
  int end_bit = 64;
  // top-k partials
  float* part_s = nullptr;
  uint32_t* part_v = nullptr;
  unsigned long long* counter = nullptr;
  int hops_done = -1;  // -1: seeds not set
  bool sources_set = false;
};

namespace {

template <typename T>
int dalloc(T** p, size_t count) {
  if (count == 0) count = 1;
  if (hipMalloc((void**)p, count * sizeof(T)) != hipSuccess) {
    (void)hipGetLastError();
    *p = nullptr;
    return egr::fail(EGR_ENOMEM, "hipMalloc failed (" + std::to_string(count * sizeof(T)) + " B)");
  }
  return EGR_OK;
}

template <typename T>
void dfree(T*& p) {
  if (p) (void)hipFree((void*)p);
  p = nullptr;
}

#define EGR_TRY(x)              \
  do {                          \
    int rc_ = (x);              \
    if (rc_ != EGR_OK) return rc_; \
  } while (0)

}  // namespace

extern "C" {

int egr_snapshot_create(const egr_graph* g, const float* weights, int32_t n_types, int32_t device,
                        egr_snapshot** out) {
  if (!g || !out) return egr::fail(EGR_EINVAL, "egr_snapshot_create: NULL argument");
  *out = nullptr;
  const int64_t V = egr_graph_num_vertices(g), E = egr_graph_num_edges(g);
  if (V <= 0) return egr::fail(EGR_EINVAL, "egr_snapshot_create: empty graph");
  int ndev = 0;
  EGR_HIP(hipGetDeviceCount(&ndev));
  if (device < 0 || device >= ndev) return egr::fail(EGR_EINVAL, "egr_snapshot_create: bad device");
  std::vector<uint32_t> row_ptr(V + 1), col(2 * E + 1);
  std::vector<uint8_t> meta(2 * E + 1), vlabel(V);
  std::vector<float> val(2 * E + 1);
  EGR_TRY(egr_graph_csr(g, weights, n_types, row_ptr.data(), col.data(), meta.data(), val.data()));
  EGR_TRY(egr_graph_export(g, vlabel.data(), nullptr, nullptr, nullptr));
  DeviceGuard guard(device);
  auto* s = new egr_snapshot();
  s->device = device;
  s->V = V;
  s->NE = 2 * E;
  int rc = EGR_OK;
  if ((rc = dalloc(&s->row_ptr, V + 1)) || (rc = dalloc(&s->col, 2 * E)) ||
      (rc = dalloc(&s->meta, 2 * E)) || (rc = dalloc(&s->val, 2 * E)) ||
      (rc = dalloc(&s->vlabel, V))) {
    egr_snapshot_free(s);
    return rc;
  }
  hipError_t e = hipMemcpy(s->row_ptr, row_ptr.data(), (V + 1) * 4, hipMemcpyHostToDevice);
  if (e == hipSuccess && E) e = hipMemcpy(s->col, col.data(), 2 * E * 4, hipMemcpyHostToDevice);
  if (e == hipSuccess && E) e = hipMemcpy(s->meta, meta.data(), 2 * E, hipMemcpyHostToDevice);
  if (e == hipSuccess && E) e = hipMemcpy(s->val, val.data(), 2 * E * 4, hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMemcpy(s->vlabel, vlabel.data(), V, hipMemcpyHostToDevice);
  if (e != hipSuccess) {
    egr_snapshot_free(s);
    return egr::fail(EGR_EDEVICE, std::string("snapshot upload: ") + hipGetErrorString(e));
  }
  *out = s;
  return EGR_OK;
}

void egr_snapshot_free(egr_snapshot* s) {
  if (!s) return;
  DeviceGuard guard(s->device);
  dfree(s->row_ptr);
  dfree(s->col);
  dfree(s->meta);
  dfree(s->val);
  dfree(s->vlabel);
  delete s;
}

int egr_snapshot_info(const egr_snapshot* s, int64_t* n_vertices, int64_t* n_entries) {
  if (!s) return egr::fail(EGR_EINVAL, "egr_snapshot_info: NULL snapshot");
  if (n_vertices) *n_vertices = s->V;
  if (n_entries) *n_entries = s->NE;
  return EGR_OK;
}

int egr_plan_create(const egr_snapshot* s, int32_t n_cols, int64_t max_seeds, int32_t k,
                    egr_plan** out) {
  if (!s || !out || n_cols <= 0 || max_seeds < 0 || k < 1 || k > KMAX)
    return egr::fail(EGR_EINVAL, "egr_plan_create: bad arguments (need n_cols > 0, 1 <= k <= 16)");
  *out = nullptr;
  DeviceGuard guard(s->device);
  auto* p = new egr_plan();
  p->s = s;
  p->B = n_cols;
  p->TW = n_cols >= 64 ? 64 : (n_cols >= 16 ? 16 : 4);
  p->Bpad = (n_cols + p->TW - 1) / p->TW * p->TW;
  p->ntiles = p->Bpad / p->TW;
  p->W = (n_cols + 63) / 64;
  p->k = k;
  p->max_seeds = max_seeds;
  const uint32_t V = (uint32_t)s->V;
  const uint32_t rows_per_block = 256 / (p->TW / 4);
  p->nrb8_hop = ((V + rows_per_block - 1) / rows_per_block + 7) / 8 * 8;
  p->nrb8_reach = ((V + 255) / 256 + 7) / 8 * 8;
  p->n_chunks = (int)((V + TOPK_CHUNK - 1) / TOPK_CHUNK);
  const uint64_t keyspace = (uint64_t)V * p->Bpad;
  p->end_bit = 1;
  while (p->end_bit < 64 && (1ull << p->end_bit) <= keyspace) ++p->end_bit;
  const size_t ms = (size_t)std::max<int64_t>(max_seeds, 1);
  int rc = EGR_OK;
  const size_t xs = (size_t)V * p->Bpad;
  const size_t parts = (size_t)p->ntiles * p->n_chunks * 64 * KMAX;
  if ((rc = dalloc(&p->x[0], xs)) || (rc = dalloc(&p->x[1], xs)) ||
      (rc = dalloc(&p->reach[0], (size_t)p->W * V)) || (rc = dalloc(&p->reach[1], (size_t)p->W * V)) ||
      (rc = dalloc(&p->skeys_in, ms)) || (rc = dalloc(&p->skeys, ms)) || (rc = dalloc(&p->ukeys, ms)) ||
      (rc = dalloc(&p->svals_in, ms)) || (rc = dalloc(&p->svals, ms)) || (rc = dalloc(&p->uval, ms)) ||
      (rc = dalloc(&p->head, ms)) || (rc = dalloc(&p->pos, ms)) || (rc = dalloc(&p->ucol, ms)) ||
      (rc = dalloc(&p->seed_ptr, (size_t)V + 1)) || (rc = dalloc(&p->n_unique, 1)) ||
      (rc = dalloc(&p->part_s, parts)) || (rc = dalloc(&p->part_v, parts)) ||
      (rc = dalloc(&p->counter, 1))) {
    egr_plan_free(p);
    return rc;
  }
  size_t b1 = 0, b2 = 0;
  if (hipcub::DeviceRadixSort::SortPairs(nullptr, b1, p->skeys_in, p->skeys, p->svals_in, p->svals,
                                         (int)ms, 0, p->end_bit) != hipSuccess ||
      hipcub::DeviceScan::ExclusiveSum(nullptr, b2, p->head, p->pos, (int)ms) != hipSuccess) {
    egr_plan_free(p);
    return egr::fail(EGR_EDEVICE, "hipcub temp-size query failed");
  }
  p->cub_tmp_bytes = std::max(b1, b2);
  if (hipMalloc(&p->cub_tmp, p->cub_tmp_bytes) != hipSuccess) {
    egr_plan_free(p);
    return egr::fail(EGR_ENOMEM, "hipMalloc (hipcub temp) failed");
  }
  *out = p;
  return EGR_OK;
}

void egr_plan_free(egr_plan* p) {
  if (!p) return;
  DeviceGuard guard(p->s->device);
  dfree(p->x[0]);
  dfree(p->x[1]);
  dfree(p->reach[0]);
  dfree(p->reach[1]);
  dfree(p->skeys_in);
  dfree(p->skeys);
  dfree(p->ukeys);
  dfree(p->svals_in);
  dfree(p->svals);
  dfree(p->uval);
  dfree(p->head);
  dfree(p->pos);
  dfree(p->ucol);
  dfree(p->seed_ptr);
  dfree(p->n_unique);
  dfree(p->part_s);
  dfree(p->part_v);
  dfree(p->counter);
  if (p->cub_tmp) (void)hipFree(p->cub_tmp);
  delete p;
}

int egr_plan_tile_width(const egr_plan* p) { return p ? p->TW : -1; }

int egr_plan_set_seeds(egr_plan* p, const uint32_t* seed_vertex, const uint32_t* seed_col,
                       const float* seed_val, int64_t n_seeds, void* stream) {
  if (!p || n_seeds < 0 || n_seeds > p->max_seeds || (n_seeds > 0 && (!seed_vertex || !seed_col || !seed_val)))
    return egr::fail(EGR_EINVAL, "egr_plan_set_seeds: bad arguments (n_seeds above plan capacity?)");
  DeviceGuard guard(p->s->device);
  hipStream_t st = (hipStream_t)stream;
  const uint32_t V = (uint32_t)p->s->V;
  p->hops_done = 0;
  p->xcur = 0;
  if (n_seeds == 0) {
    hipLaunchKernelGGL(zero_seed_ptr_kernel, dim3((V + 256) / 256), dim3(256), 0, st, p->seed_ptr, V);
    EGR_CHECK_LAUNCH();
    return EGR_OK;
  }
  const int n = (int)n_seeds;
  const dim3 g1((n + 255) / 256);
  hipLaunchKernelGGL(seed_keys_kernel, g1, dim3(256), 0, st, seed_vertex, seed_col, seed_val,
                     (int64_t)n, V, p->B, (uint32_t)p->Bpad, p->skeys_in, p->svals_in);
  EGR_CHECK_LAUNCH();
  size_t tb = p->cub_tmp_bytes;
  EGR_HIP(hipcub::DeviceRadixSort::SortPairs(p->cub_tmp, tb, p->skeys_in, p->skeys, p->svals_in,
                                             p->svals, n, 0, p->end_bit, st));
  // invalid keys (~0) sort last only if their low end_bit bits are all ones, which they are
  hipLaunchKernelGGL(seed_head_kernel, g1, dim3(256), 0, st, p->skeys, (int64_t)n, p->head);
  EGR_CHECK_LAUNCH();
  tb = p->cub_tmp_bytes;
  EGR_HIP(hipcub::DeviceScan::ExclusiveSum(p->cub_tmp, tb, p->head, p->pos, n, st));
  hipLaunchKernelGGL(seed_compact_kernel, g1, dim3(256), 0, st, p->skeys, p->svals, p->head,
                     p->pos, (int64_t)n, (uint32_t)p->Bpad, p->ukeys, p->ucol, p->uval,
                     p->n_unique);
  EGR_CHECK_LAUNCH();
  hipLaunchKernelGGL(seed_ptr_kernel, dim3((V + 256) / 256), dim3(256), 0, st, p->ukeys,
                     p->n_unique, V, (uint32_t)p->Bpad, p->seed_ptr);
  EGR_CHECK_LAUNCH();
  return EGR_OK;
}

int egr_plan_set_sources(egr_plan* p, const uint32_t* source_vertex, void* stream) {
  if (!p || !source_vertex) return egr::fail(EGR_EINVAL, "egr_plan_set_sources: NULL argument");
  DeviceGuard guard(p->s->device);
  hipStream_t st = (hipStream_t)stream;
  const uint32_t V = (uint32_t)p->s->V;
  p->rcur = 0;
  EGR_HIP(hipMemsetAsync(p->reach[0], 0, (size_t)p->W * V * 8, st));
  hipLaunchKernelGGL(reach_sources_kernel, dim3((p->B + 255) / 256), dim3(256), 0, st,
                     source_vertex, p->B, p->reach[0], V);
  EGR_CHECK_LAUNCH();
  p->sources_set = true;
  p->reach_hops = 0;
  return EGR_OK;
}

int egr_plan_hop(egr_plan* p, void* stream) {
  if (!p) return egr::fail(EGR_EINVAL, "egr_plan_hop: NULL plan");
  if (p->hops_done < 0) return egr::fail(EGR_ESTATE, "egr_plan_hop: seeds not set");
  DeviceGuard guard(p->s->device);
  hipStream_t st = (hipStream_t)stream;
  const egr_snapshot* s = p->s;
  const uint32_t V = (uint32_t)s->V;
  const dim3 grid(p->nrb8_hop * p->ntiles), block(256);
  float* xo = p->x[p->hops_done == 0 ? 0 : 1 - p->xcur];
  if (p->hops_done == 0) {
#define LAUNCH_SEED_HOP(G)                                                                   \
  hipLaunchKernelGGL(hop_from_seeds_kernel<G>, grid, block, 0, st, s->row_ptr, s->col, s->val, \
                     p->seed_ptr, p->ucol, p->uval, xo, V, p->nrb8_hop)
    if (p->TW == 64) LAUNCH_SEED_HOP(16);
    else if (p->TW == 16) LAUNCH_SEED_HOP(4);
    else LAUNCH_SEED_HOP(1);
#undef LAUNCH_SEED_HOP
    p->xcur = 0;
  } else {
    const float* xi = p->x[p->xcur];
#define LAUNCH_HOP(G)                                                                          \
  hipLaunchKernelGGL(hop_kernel<G>, grid, block, 0, st, s->row_ptr, s->col, s->val, p->seed_ptr, \
                     p->ucol, p->uval, xi, xo, V, p->nrb8_hop)
    if (p->TW == 64) LAUNCH_HOP(16);
    else if (p->TW == 16) LAUNCH_HOP(4);
    else LAUNCH_HOP(1);
#undef LAUNCH_HOP
    p->xcur = 1 - p->xcur;
  }
  EGR_CHECK_LAUNCH();
  ++p->hops_done;
  return EGR_OK;
}

int egr_plan_reach_hop(egr_plan* p, void* stream) {
  if (!p) return egr::fail(EGR_EINVAL, "egr_plan_reach_hop: NULL plan");
  if (!p->sources_set) return egr::fail(EGR_ESTATE, "egr_plan_reach_hop: sources not set");
  DeviceGuard guard(p->s->device);
  const uint32_t V = (uint32_t)p->s->V;
  hipLaunchKernelGGL(reach_hop_kernel, dim3(p->nrb8_reach * p->W), dim3(256), 0,
                     (hipStream_t)stream, p->s->row_ptr, p->s->col, p->reach[p->rcur],
                     p->reach[1 - p->rcur], V, p->nrb8_reach);
  EGR_CHECK_LAUNCH();
  p->rcur = 1 - p->rcur;
  ++p->reach_hops;
  return EGR_OK;
}

int egr_plan_topk(egr_plan* p, int32_t exclude_label, uint32_t* out_ids, float* out_scores,
                  void* stream) {
  if (!p || !out_ids || !out_scores) return egr::fail(EGR_EINVAL, "egr_plan_topk: NULL argument");
  if (p->hops_done < 1) return egr::fail(EGR_ESTATE, "egr_plan_topk: run at least one hop first");
  if (!p->sources_set) return egr::fail(EGR_ESTATE, "egr_plan_topk: sources not set");
  DeviceGuard guard(p->s->device);
  hipStream_t st = (hipStream_t)stream;
  const uint32_t V = (uint32_t)p->s->V;
  const int waves = p->ntiles * p->n_chunks;
  hipLaunchKernelGGL(topk_partial_kernel, dim3((waves + 3) / 4), dim3(256), 0, st,
                     p->x[p->xcur], p->reach[p->rcur], p->s->vlabel, exclude_label, V, p->TW,
                     p->B, p->n_chunks, p->part_s, p->part_v);
  EGR_CHECK_LAUNCH();
  hipLaunchKernelGGL(topk_merge_kernel, dim3((p->B + 3) / 4), dim3(256), 0, st, p->part_s,
                     p->part_v, p->TW, p->B, p->n_chunks, p->k, out_ids, out_scores);
  EGR_CHECK_LAUNCH();
  return EGR_OK;
}

int egr_plan_run(egr_plan* p, int32_t hops, int32_t exclude_label, uint32_t* out_ids,
                 float* out_scores, void* stream) {
  if (!p || hops < 1) return egr::fail(EGR_EINVAL, "egr_plan_run: need hops >= 1");
  if (p->hops_done != 0 || p->reach_hops != 0)
    return egr::fail(EGR_ESTATE, "egr_plan_run: set seeds and sources first");
  for (int h = 0; h < hops; ++h) {
    EGR_TRY(egr_plan_hop(p, stream));
    EGR_TRY(egr_plan_reach_hop(p, stream));
  }
  return egr_plan_topk(p, exclude_label, out_ids, out_scores, stream);
}

int egr_plan_read_scores(const egr_plan* p, float* out, void* stream) {
  if (!p || !out) return egr::fail(EGR_EINVAL, "egr_plan_read_scores: NULL argument");
  if (p->hops_done < 1) return egr::fail(EGR_ESTATE, "egr_plan_read_scores: no hop run yet");
  DeviceGuard guard(p->s->device);
  const size_t n = (size_t)p->s->V * p->B;
  hipLaunchKernelGGL(scores_rowmajor_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, p->x[p->xcur], (uint32_t)p->s->V, p->TW, p->B, out);
  EGR_CHECK_LAUNCH();
  return EGR_OK;
}

int egr_plan_read_reach(const egr_plan* p, uint64_t* out, void* stream) {
  if (!p || !out) return egr::fail(EGR_EINVAL, "egr_plan_read_reach: NULL argument");
  if (!p->sources_set) return egr::fail(EGR_ESTATE, "egr_plan_read_reach: sources not set");
  DeviceGuard guard(p->s->device);
  EGR_HIP(hipMemcpyAsync(out, p->reach[p->rcur], (size_t)p->W * p->s->V * 8,
                         hipMemcpyDeviceToDevice, (hipStream_t)stream));
  return EGR_OK;
}

int egr_plan_induced_edges(const egr_plan* p, int32_t col, uint32_t* out_src, uint32_t* out_dst,
                           uint8_t* out_type, int64_t cap, int64_t* out_n, void* stream) {
  if (!p || !out_n || col < 0 || col >= p->B || cap < 0 || (cap > 0 && (!out_src || !out_dst || !out_type)))
    return egr::fail(EGR_EINVAL, "egr_plan_induced_edges: bad arguments");
  if (!p->sources_set) return egr::fail(EGR_ESTATE, "egr_plan_induced_edges: sources not set");
  DeviceGuard guard(p->s->device);
  hipStream_t st = (hipStream_t)stream;
  const uint32_t V = (uint32_t)p->s->V;
  EGR_HIP(hipMemsetAsync(p->counter, 0, sizeof(unsigned long long), st));
  hipLaunchKernelGGL(induced_kernel, dim3((V + 255) / 256), dim3(256), 0, st, p->s->row_ptr,
                     p->s->col, p->s->meta, p->reach[p->rcur] + (size_t)(col >> 6) * V,
                     1ull << (col & 63), V, out_src, out_dst, out_type, cap, p->counter);
  EGR_CHECK_LAUNCH();
  unsigned long long n = 0;
  EGR_HIP(hipMemcpyAsync(&n, p->counter, sizeof(n), hipMemcpyDeviceToHost, st));
  EGR_HIP(hipStreamSynchronize(st));
  *out_n = (int64_t)n;
  return EGR_OK;
}

}  // extern "C"
