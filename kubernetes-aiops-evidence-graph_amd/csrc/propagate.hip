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

// ---- propagation hop ---------------------------------------------------------------------
// One block = ROWS consecutive rows of one column tile.  The block stages its rows' row_ptr,
// own seed-tile masks, labels and CSR segment (col, val) in LDS with coalesced loads.  Each
// lane group (G lanes x float4 = the row's TW columns) then walks its rows with a two-row
// software pipeline: the next row's first NB neighbour gathers (and reach words) are in flight
// while the current row runs its fmaf chain in CSR order (bit-exact with the oracle).
//   FROM_SEEDS (h = 0 -> 1): neighbour values come from the sparse seed lists, filtered by a
//              per-vertex seed-tile mask, so s0 is never materialised densely;
//   REACH      (TW >= 64): the same walk ORs the neighbours' reach words (one pass per hop);
//   CAND       (last hop): reached, non-excluded (vertex, column) pairs are appended to the
//              column's candidate list for the top-k merge, so top-k never rescans the scores.
template <int G>
struct HopGeo {
  static constexpr int ROWS = G == 1 ? 256 : 128;
};
constexpr uint32_t CSR_CAP = 2048;   // staged entries per block (longer segments read global)
constexpr int NB = 4;                // neighbour gathers per batch

struct HopArgs {
  const uint32_t* row_ptr;
  const uint32_t* col;
  const float* val;
  const uint32_t* seed_ptr;
  const uint32_t* seed_col;
  const float* seed_val;
  const uint32_t* seed_tiles;
  const uint8_t* vlabel;
  const float* xin;
  float* xout;
  const uint64_t* rin;
  uint64_t* rout;
  uint32_t* cand_count;
  uint32_t* cand_list;
  uint32_t V;
  uint32_t nchunks;
  int32_t B;
  int32_t exclude_label;
};

template <bool SEEDS, bool REACH>
struct Batch {
  float4 x[NB];
  uint64_t rw[NB];
  uint32_t m[NB];
  uint32_t u[NB];
  float w[NB];
  uint32_t n;
};

template <int G, bool FROM_SEEDS, bool REACH, bool CAND>
__global__ __launch_bounds__(256) void hop_kernel(const HopArgs A) {
  constexpr int TW = 4 * G, GROUPS = 256 / G, ROWS = HopGeo<G>::ROWS;
  __shared__ uint32_t s_rp[ROWS + 1];
  __shared__ uint32_t s_mask[ROWS];
  __shared__ uint8_t s_lab[ROWS];
  __shared__ uint32_t s_col[CSR_CAP];
  __shared__ float s_val[CSR_CAP];
  const uint32_t tid = threadIdx.x, gl = tid % G, grp = tid / G;
  const uint32_t V = A.V;
  const uint32_t tile = blockIdx.x / A.nchunks;
  const uint32_t v0 = (blockIdx.x % A.nchunks) * ROWS;
  if (v0 >= V) return;  // block-uniform, before any barrier
  const uint32_t nrows = min((uint32_t)ROWS, V - v0);
  for (uint32_t i = tid; i <= nrows; i += 256) s_rp[i] = A.row_ptr[v0 + i];
  for (uint32_t i = tid; i < nrows; i += 256) {
    s_mask[i] = A.seed_tiles[v0 + i];
    if constexpr (CAND) s_lab[i] = A.vlabel[v0 + i];
  }
  __syncthreads();
  const uint32_t e0 = s_rp[0];
  const uint32_t nst = min(s_rp[nrows] - e0, CSR_CAP);
  for (uint32_t i = tid; i < nst; i += 256) {
    s_col[i] = A.col[e0 + i];
    s_val[i] = A.val[e0 + i];
  }
  __syncthreads();
  uint32_t r = grp;
  if (r >= nrows) return;  // no barrier below

  const uint32_t lo = tile * TW + 4 * gl;  // first column of this lane
  const uint32_t tbit = tile & 31u;
  const size_t toff = (size_t)tile * V * TW;
  const float4* __restrict__ X = reinterpret_cast<const float4*>(A.xin + toff);
  const uint32_t word = lo >> 6;
  const uint64_t* __restrict__ R = A.rin + (size_t)word * V;

  auto issue = [&](uint32_t ja, uint32_t jb, Batch<FROM_SEEDS, REACH>& bt) {
    bt.n = jb > ja ? min(jb - ja, (uint32_t)NB) : 0u;
#pragma unroll
    for (int t = 0; t < NB; ++t) {
      const uint32_t jj = ja + t;
      const bool ok = (uint32_t)t < bt.n;
      uint32_t u = 0u;
      float w = 0.f;
      if (ok) {
        u = jj < CSR_CAP ? s_col[jj] : A.col[e0 + jj];
        w = jj < CSR_CAP ? s_val[jj] : A.val[e0 + jj];
      }
      bt.u[t] = u;
      bt.w[t] = w;
      if constexpr (FROM_SEEDS) {
        bt.m[t] = ok ? A.seed_tiles[u] : 0u;
      } else {
        bt.x[t] = make_float4(0.f, 0.f, 0.f, 0.f);
        if (ok) bt.x[t] = X[(size_t)u * G + gl];
      }
      if constexpr (REACH) bt.rw[t] = ok ? R[u] : 0ull;
    }
  };
  auto consume = [&](const Batch<FROM_SEEDS, REACH>& bt, float4& acc, uint64_t& rr) {
#pragma unroll
    for (int t = 0; t < NB; ++t) {
      if ((uint32_t)t < bt.n) {
        if constexpr (FROM_SEEDS) {
          if ((bt.m[t] >> tbit) & 1u) {  // w * 0 otherwise: skipping the fmaf is exact
            const uint32_t u = bt.u[t];
            const uint32_t s1 = A.seed_ptr[u + 1];
            for (uint32_t q = seed_lower(A.seed_col, A.seed_ptr[u], s1, lo); q < s1; ++q) {
              const uint32_t c = A.seed_col[q] - lo;
              if (c >= 4u) break;
              fma_comp(acc, (int)c, bt.w[t], A.seed_val[q]);
            }
          }
        } else {
          fma4(bt.w[t], bt.x[t], acc);
        }
        if constexpr (REACH) rr |= bt.rw[t];
      }
    }
  };

  Batch<FROM_SEEDS, REACH> cur, nxt;
  issue(s_rp[r] - e0, s_rp[r + 1] - e0, cur);
  uint64_t own = 0;
  if constexpr (REACH) own = R[v0 + r];
  while (true) {
    const uint32_t rn = r + GROUPS;
    const bool more = rn < nrows;
    uint64_t own_n = 0;
    if (more) {
      issue(s_rp[rn] - e0, s_rp[rn + 1] - e0, nxt);
      if constexpr (REACH) own_n = R[v0 + rn];
    }
    const uint32_t v = v0 + r;
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    uint64_t rr = own;
    consume(cur, acc, rr);
    const uint32_t b = s_rp[r + 1] - e0;
    for (uint32_t j = s_rp[r] - e0 + NB; j < b; j += NB) {  // rows longer than NB
      Batch<FROM_SEEDS, REACH> tail;
      issue(j, b, tail);
      consume(tail, acc, rr);
    }
    if ((s_mask[r] >> tbit) & 1u) add_seeds(acc, v, lo, A.seed_ptr, A.seed_col, A.seed_val);
    reinterpret_cast<float4*>(A.xout + toff)[(size_t)v * G + gl] = acc;
    if constexpr (REACH) {
      if ((lo & 63u) == 0u) A.rout[(size_t)word * V + v] = rr;
    }
    if constexpr (CAND) {
      const uint32_t bits = (uint32_t)(rr >> (lo & 63u)) & 0xFu;
      if (bits && !(A.exclude_label >= 0 && s_lab[r] == (uint8_t)A.exclude_label)) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const uint32_t bcol = lo + i;
          if (((bits >> i) & 1u) && bcol < (uint32_t)A.B) {
            const uint32_t slot = atomicAdd(&A.cand_count[bcol], 1u);
            A.cand_list[(size_t)bcol * V + slot] = v;
          }
        }
      }
    }
    if (!more) break;
    cur = nxt;
    own = own_n;
    r = rn;
  }
}

__global__ void seed_tiles_kernel(const uint64_t* __restrict__ ukeys,
                                  const uint32_t* __restrict__ n_unique, uint32_t Bpad,
                                  uint32_t TW, uint32_t* seed_tiles) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= *n_unique) return;
  const uint64_t k = ukeys[i];
  const uint32_t v = (uint32_t)(k / Bpad), tile = (uint32_t)(k % Bpad) / TW;
  atomicOr(&seed_tiles[v], 1u << (tile & 31u));
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

// k rounds of a wave-wide arg-best over the per-lane list heads; lane 0 writes the result.
// Every vertex appears in at most one lane's list, so (score desc, id asc) is a strict order
// and all lanes agree on each round's winner.
__device__ __forceinline__ void wave_emit_topk(float (&Ls)[KMAX], uint32_t (&Lv)[KMAX], int k,
                                               int lane, uint32_t* out_ids, float* out_scores) {
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
      out_ids[q] = bv;
      out_scores[q] = bv == NO_NODE ? -INFINITY : bs;
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

// A wave covers CW = min(TW, 64) columns of one tile: lane -> (column c, row phase rp); the
// wave index enumerates (tile, 64-column slice, row chunk).
__global__ __launch_bounds__(256) void topk_partial_kernel(
    const float* __restrict__ X, const uint64_t* __restrict__ R,
    const uint8_t* __restrict__ vlabel, int exclude_label, uint32_t V, int TW, int B,
    int n_chunks, float* __restrict__ part_s, uint32_t* __restrict__ part_v) {
  const int lane = threadIdx.x & 63;
  const int wid = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int CW = TW < 64 ? TW : 64, nsub = TW / CW;
  const int ntiles = (B + TW - 1) / TW;
  if (wid >= ntiles * nsub * n_chunks) return;
  const int ch = wid % n_chunks, ts = wid / n_chunks, tile = ts / nsub, sub = ts % nsub;
  const int c = lane % CW, rp = lane / CW, rps = 64 / CW;
  const int b = tile * TW + sub * CW + c;
  const int cx = sub * CW + c;   // column inside the tile
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
    // eight rows per step: all reach words and labels, then the reached scores, are loaded
    // before any insertion, so a wave keeps 8-16 loads in flight instead of one
    for (uint32_t vb = v0 + rp; vb < v1; vb += 8u * rps) {
      uint64_t wd[8];
      uint8_t lab[8];
      float xs[8];
#pragma unroll
      for (int t = 0; t < 8; ++t) {
        const uint32_t v = vb + t * rps;
        wd[t] = v < v1 ? Rw[v] : 0ull;
        lab[t] = v < v1 ? vlabel[v] : 0;
      }
#pragma unroll
      for (int t = 0; t < 8; ++t) {
        const uint32_t v = vb + t * rps;
        const bool cand = (wd[t] & bit) && !(exclude_label >= 0 && lab[t] == (uint8_t)exclude_label);
        wd[t] = cand;
        xs[t] = cand ? Xt[(size_t)v * TW + cx] : 0.f;
      }
#pragma unroll
      for (int t = 0; t < 8; ++t)
        if (wd[t]) list_insert(Ls, Lv, xs[t], vb + t * rps);
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
  const int CW = TW < 64 ? TW : 64, nsub = TW / CW;
  const int tile = b / TW, sub = (b % TW) / CW, c = b % CW, rps = 64 / CW;
  float Ls[KMAX];
  uint32_t Lv[KMAX];
#pragma unroll
  for (int i = 0; i < KMAX; ++i) {
    Ls[i] = -INFINITY;
    Lv[i] = NO_NODE;
  }
  // candidate lists of column b: chunks x (lanes with lane % CW == c), KMAX entries each
  const int n_lists = n_chunks * rps;
  for (int li = lane; li < n_lists; li += 64) {
    const int ch = li / rps, rp = li % rps;
    const size_t o = (((size_t)((tile * nsub + sub) * n_chunks + ch)) * 64 + rp * CW + c) * KMAX;
    for (int i = 0; i < k; ++i) {
      const uint32_t v = part_v[o + i];
      if (v == NO_NODE) break;
      list_insert(Ls, Lv, part_s[o + i], v);
    }
  }
  wave_emit_topk(Ls, Lv, k, lane, out_ids + (size_t)b * k, out_scores + (size_t)b * k);
}

// top-k from the candidate lists the CAND hop appended: one wave per column
__global__ __launch_bounds__(256) void topk_cand_kernel(
    const float* __restrict__ X, const uint32_t* __restrict__ cand_count,
    const uint32_t* __restrict__ cand_list, uint32_t V, int TW, int B, int k,
    uint32_t* __restrict__ out_ids, float* __restrict__ out_scores) {
  const int lane = threadIdx.x & 63;
  const int b = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (b >= B) return;
  float Ls[KMAX];
  uint32_t Lv[KMAX];
#pragma unroll
  for (int i = 0; i < KMAX; ++i) {
    Ls[i] = -INFINITY;
    Lv[i] = NO_NODE;
  }
  const uint32_t n = min(cand_count[b], V);
  const float* __restrict__ Xc = X + (size_t)(b / TW) * V * TW + (b % TW);
  const uint32_t* __restrict__ Lb = cand_list + (size_t)b * V;
  for (uint32_t i0 = lane; i0 < n; i0 += 64u * 4u) {
    uint32_t vv[4];
    float ss[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) vv[t] = i0 + t * 64u < n ? Lb[i0 + t * 64u] : NO_NODE;
#pragma unroll
    for (int t = 0; t < 4; ++t) ss[t] = vv[t] != NO_NODE ? Xc[(size_t)vv[t] * TW] : 0.f;
#pragma unroll
    for (int t = 0; t < 4; ++t)
      if (vv[t] != NO_NODE) list_insert(Ls, Lv, ss[t], vv[t]);
  }
  wave_emit_topk(Ls, Lv, k, lane, out_ids + (size_t)b * k, out_scores + (size_t)b * k);
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
  int Wa = 0;                // reach words allocated: padded columns of 128-wide tiles too
  int64_t max_seeds = 0;
  int n_chunks = 0;          // top-k full-scan chunks
  uint32_t nchunks = 0;      // hop row chunks per tile
  uint32_t nrb8_reach = 0;
  float* x[2] = {nullptr, nullptr};
  int xcur = 0;
  uint64_t* reach[2] = {nullptr, nullptr};
  int rcur = 0;
  int reach_hops = -1;  // -1: sources not set
  int hops_done = -1;   // -1: seeds not set
  bool sources_set = false;
  // seeds
  uint64_t *skeys_in = nullptr, *skeys = nullptr, *ukeys = nullptr;
  float *svals_in = nullptr, *svals = nullptr, *uval = nullptr;
  uint32_t *head = nullptr, *pos = nullptr, *ucol = nullptr, *seed_ptr = nullptr,
           *n_unique = nullptr, *seed_tiles = nullptr;
  void* cub_tmp = nullptr;
  size_t cub_tmp_bytes = 0;
  int end_bit = 64;
  // top-k: full-scan partials, and the candidate lists of the fused last hop
  float* part_s = nullptr;
  uint32_t* part_v = nullptr;
  uint32_t* cand_count = nullptr;
  uint32_t* cand_list = nullptr;
  bool cand_valid = false;
  int cand_exclude = -1;
  unsigned long long* counter = nullptr;
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

#define EGR_TRY(x)                 \
  do {                             \
    int rc_ = (x);                 \
    if (rc_ != EGR_OK) return rc_; \
  } while (0)

int choose_tile_width(int n_cols) {
  // 128-wide tiles (512-B gathers, two reach words) unless overridden; a tile must not
  // exceed the batch by more than padding, so narrow batches use narrower tiles
  int cap = 128;
  if (const char* e = getenv("EGRAPH_TILE_WIDTH")) {
    const int t = atoi(e);
    if (t == 4 || t == 16 || t == 64 || t == 128) cap = t;
  }
  int tw = n_cols >= 128 ? 128 : (n_cols >= 64 ? 64 : (n_cols >= 16 ? 16 : 4));
  return tw < cap ? tw : cap;
}

uint32_t hop_rows(int TW) {
  switch (TW) {
    case 128: return HopGeo<32>::ROWS;
    case 64: return HopGeo<16>::ROWS;
    case 16: return HopGeo<4>::ROWS;
    default: return HopGeo<1>::ROWS;
  }
}

template <int G, bool SEEDS, bool REACH, bool CAND>
void launch_hop_t(const HopArgs& a, dim3 grid, hipStream_t st) {
  hipLaunchKernelGGL((hop_kernel<G, SEEDS, REACH, CAND>), grid, dim3(256), 0, st, a);
}

template <int G>
void launch_hop_g(const HopArgs& a, dim3 grid, hipStream_t st, bool seeds, bool reach, bool cand) {
  if constexpr (G >= 16) {
    if (seeds) {
      if (cand) launch_hop_t<G, true, true, true>(a, grid, st);
      else if (reach) launch_hop_t<G, true, true, false>(a, grid, st);
      else launch_hop_t<G, true, false, false>(a, grid, st);
    } else {
      if (cand) launch_hop_t<G, false, true, true>(a, grid, st);
      else if (reach) launch_hop_t<G, false, true, false>(a, grid, st);
      else launch_hop_t<G, false, false, false>(a, grid, st);
    }
  } else {
    if (seeds) launch_hop_t<G, true, false, false>(a, grid, st);
    else launch_hop_t<G, false, false, false>(a, grid, st);
  }
}

// One propagation hop.  reach: also one reachability hop in the same pass (TW >= 64);
// cand: also append the top-k candidates of this (last) hop.
int plan_hop(egr_plan* p, void* stream, bool reach, bool cand, int exclude_label) {
  if (!p) return egr::fail(EGR_EINVAL, "egr_plan_hop: NULL plan");
  if (p->hops_done < 0) return egr::fail(EGR_ESTATE, "egr_plan_hop: seeds not set");
  if ((reach || cand) && (p->TW < 64 || !p->sources_set))
    return egr::fail(EGR_ESTATE, "fused reach needs TW >= 64 and sources set");
  DeviceGuard guard(p->s->device);
  hipStream_t st = (hipStream_t)stream;
  const egr_snapshot* s = p->s;
  const bool seeds = p->hops_done == 0;
  if (cand) EGR_HIP(hipMemsetAsync(p->cand_count, 0, (size_t)p->Bpad * 4, st));
  HopArgs a;
  a.row_ptr = s->row_ptr;
  a.col = s->col;
  a.val = s->val;
  a.seed_ptr = p->seed_ptr;
  a.seed_col = p->ucol;
  a.seed_val = p->uval;
  a.seed_tiles = p->seed_tiles;
  a.vlabel = s->vlabel;
  a.xin = seeds ? nullptr : p->x[p->xcur];
  a.xout = p->x[seeds ? 0 : 1 - p->xcur];
  a.rin = p->reach[p->rcur];
  a.rout = p->reach[1 - p->rcur];
  a.cand_count = p->cand_count;
  a.cand_list = p->cand_list;
  a.V = (uint32_t)s->V;
  a.nchunks = p->nchunks;
  a.B = p->B;
  a.exclude_label = exclude_label;
  const dim3 grid(p->nchunks * p->ntiles);
  switch (p->TW) {
    case 128: launch_hop_g<32>(a, grid, st, seeds, reach, cand); break;
    case 64: launch_hop_g<16>(a, grid, st, seeds, reach, cand); break;
    case 16: launch_hop_g<4>(a, grid, st, seeds, false, false); break;
    default: launch_hop_g<1>(a, grid, st, seeds, false, false); break;
  }
  EGR_CHECK_LAUNCH();
  p->xcur = seeds ? 0 : 1 - p->xcur;
  ++p->hops_done;
  if (reach || cand) {
    p->rcur = 1 - p->rcur;
    ++p->reach_hops;
  }
  p->cand_valid = cand;
  p->cand_exclude = exclude_label;
  return EGR_OK;
}

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
  p->TW = choose_tile_width(n_cols);
  p->Bpad = (n_cols + p->TW - 1) / p->TW * p->TW;
  p->ntiles = p->Bpad / p->TW;
  p->W = (n_cols + 63) / 64;
  p->Wa = std::max(p->W, p->Bpad / 64);
  p->k = k;
  p->max_seeds = max_seeds;
  const uint32_t V = (uint32_t)s->V;
  const uint32_t rows = hop_rows(p->TW);
  p->nchunks = (V + rows - 1) / rows;
  p->nrb8_reach = ((V + 255) / 256 + 7) / 8 * 8;
  p->n_chunks = (int)((V + TOPK_CHUNK - 1) / TOPK_CHUNK);
  const uint64_t keyspace = (uint64_t)V * p->Bpad;
  p->end_bit = 1;
  while (p->end_bit < 64 && (1ull << p->end_bit) <= keyspace) ++p->end_bit;
  const size_t ms = (size_t)std::max<int64_t>(max_seeds, 1);
  int rc = EGR_OK;
  const size_t xs = (size_t)V * p->Bpad;
  const size_t parts = (size_t)p->ntiles * (p->TW > 64 ? p->TW / 64 : 1) * p->n_chunks * 64 * KMAX;
  const bool fused = p->TW >= 64;
  if ((rc = dalloc(&p->x[0], xs)) || (rc = dalloc(&p->x[1], xs)) ||
      (rc = dalloc(&p->reach[0], (size_t)p->Wa * V)) || (rc = dalloc(&p->reach[1], (size_t)p->Wa * V)) ||
      (rc = dalloc(&p->skeys_in, ms)) || (rc = dalloc(&p->skeys, ms)) || (rc = dalloc(&p->ukeys, ms)) ||
      (rc = dalloc(&p->svals_in, ms)) || (rc = dalloc(&p->svals, ms)) || (rc = dalloc(&p->uval, ms)) ||
      (rc = dalloc(&p->head, ms)) || (rc = dalloc(&p->pos, ms)) || (rc = dalloc(&p->ucol, ms)) ||
      (rc = dalloc(&p->seed_ptr, (size_t)V + 1)) || (rc = dalloc(&p->n_unique, 1)) ||
      (rc = dalloc(&p->seed_tiles, (size_t)V)) ||
      (rc = dalloc(&p->part_s, parts)) || (rc = dalloc(&p->part_v, parts)) ||
      (rc = dalloc(&p->cand_count, (size_t)p->Bpad)) ||
      (rc = dalloc(&p->cand_list, fused ? (size_t)V * p->B : 1)) ||
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
  for (auto* q : {&p->x[0], &p->x[1]}) dfree(*q);
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
  dfree(p->seed_tiles);
  dfree(p->part_s);
  dfree(p->part_v);
  dfree(p->cand_count);
  dfree(p->cand_list);
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
  p->cand_valid = false;
  EGR_HIP(hipMemsetAsync(p->seed_tiles, 0, (size_t)V * 4, st));
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
  // invalid keys (~0) sort last: their low end_bit bits are all ones, above every valid key
  EGR_HIP(hipcub::DeviceRadixSort::SortPairs(p->cub_tmp, tb, p->skeys_in, p->skeys, p->svals_in,
                                             p->svals, n, 0, p->end_bit, st));
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
  hipLaunchKernelGGL(seed_tiles_kernel, g1, dim3(256), 0, st, p->ukeys, p->n_unique,
                     (uint32_t)p->Bpad, (uint32_t)p->TW, p->seed_tiles);
  EGR_CHECK_LAUNCH();
  return EGR_OK;
}

int egr_plan_set_sources(egr_plan* p, const uint32_t* source_vertex, void* stream) {
  if (!p || !source_vertex) return egr::fail(EGR_EINVAL, "egr_plan_set_sources: NULL argument");
  DeviceGuard guard(p->s->device);
  hipStream_t st = (hipStream_t)stream;
  const uint32_t V = (uint32_t)p->s->V;
  p->rcur = 0;
  p->cand_valid = false;
  EGR_HIP(hipMemsetAsync(p->reach[0], 0, (size_t)p->Wa * V * 8, st));
  hipLaunchKernelGGL(reach_sources_kernel, dim3((p->B + 255) / 256), dim3(256), 0, st,
                     source_vertex, p->B, p->reach[0], V);
  EGR_CHECK_LAUNCH();
  p->sources_set = true;
  p->reach_hops = 0;
  return EGR_OK;
}

int egr_plan_hop(egr_plan* p, void* stream) { return plan_hop(p, stream, false, false, -1); }

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
  p->cand_valid = false;
  return EGR_OK;
}

int egr_plan_step(egr_plan* p, void* stream) {
  if (!p) return egr::fail(EGR_EINVAL, "egr_plan_step: NULL plan");
  if (!p->sources_set) return egr::fail(EGR_ESTATE, "egr_plan_step: sources not set");
  if (p->TW >= 64) return plan_hop(p, stream, true, false, -1);
  EGR_TRY(plan_hop(p, stream, false, false, -1));
  return egr_plan_reach_hop(p, stream);
}

int egr_plan_final_step(egr_plan* p, int32_t exclude_label, void* stream) {
  if (!p) return egr::fail(EGR_EINVAL, "egr_plan_final_step: NULL plan");
  if (!p->sources_set) return egr::fail(EGR_ESTATE, "egr_plan_final_step: sources not set");
  if (p->TW >= 64) return plan_hop(p, stream, true, true, exclude_label);
  return egr_plan_step(p, stream);
}

int egr_plan_topk(egr_plan* p, int32_t exclude_label, uint32_t* out_ids, float* out_scores,
                  void* stream) {
  if (!p || !out_ids || !out_scores) return egr::fail(EGR_EINVAL, "egr_plan_topk: NULL argument");
  if (p->hops_done < 1) return egr::fail(EGR_ESTATE, "egr_plan_topk: run at least one hop first");
  if (!p->sources_set) return egr::fail(EGR_ESTATE, "egr_plan_topk: sources not set");
  DeviceGuard guard(p->s->device);
  hipStream_t st = (hipStream_t)stream;
  const uint32_t V = (uint32_t)p->s->V;
  if (p->cand_valid && p->cand_exclude == exclude_label) {
    hipLaunchKernelGGL(topk_cand_kernel, dim3((p->B + 3) / 4), dim3(256), 0, st, p->x[p->xcur],
                       p->cand_count, p->cand_list, V, p->TW, p->B, p->k, out_ids, out_scores);
    EGR_CHECK_LAUNCH();
    return EGR_OK;
  }
  const int waves = p->ntiles * (p->TW > 64 ? p->TW / 64 : 1) * p->n_chunks;
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
  for (int h = 0; h + 1 < hops; ++h) EGR_TRY(egr_plan_step(p, stream));
  EGR_TRY(egr_plan_final_step(p, exclude_label, stream));
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
