// Graph stages on the device snapshot:
//   A8  reach  : k-hop undirected reachability from each incident vertex, 64 incidents per u64
//                word (apoc.path.subgraphAll(maxLevel=k), src/database/neo4j.py:169-202);
//   A9  hop    : typed propagation s^{h+1}_v = s0_v + sum_{(u,t,d) in row v} val_e * s^h_u,
//                val_e = w[t][d] / deg(u), fp32, accumulated with fmaf in CSR order so the
//                result is bit-identical to oracle/egraph_oracle.c;
//       topk   : per incident, top-k vertices of the final scores over its reach set, score
//                descending, vertex id ascending on ties.
//
// Layout: scores are tiled [B/TW][V][TW] fp32 (TW = 128/64/16/4 columns), so a
// pull-gather of one neighbour row is TW*4 contiguous bytes (512 B at TW = 128) served by
// G = TW/4 lanes with one float4 each, and the gather working set of one tile sweep
// (V*TW*4 B = 117 MB at 229k vertices) fits the 256 MB Infinity Cache.  Reach words are
// row-major [V][RS] u64 (RS = 2*RG words, RG a power of two): a vertex's words for all
// incidents are one contiguous row, so a reach hop is the same staged gather as a propagation
// hop at 1/32 of its bytes (RG lanes x 16 B per row).
#include <algorithm>
#include <vector>

#include "graph_dev.h"

using egr::DeviceGuard;
using egr::dalloc;
using egr::dfree;

namespace {

constexpr int KMAX = 16;              // top-k capacity per list
constexpr int TOPK_CHUNK = 1024;      // rows per wave in top-k phase 1
constexpr uint32_t NO_NODE = EGR_NO_NODE;

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
// One block = one row chunk of one column tile.  Chunks come from a per-plan table built so
// that a chunk's CSR segment fits the LDS stage (CSR_CAP entries; only a lone row longer than
// that spills, into the cold tail loop).  The block stages row_ptr and (col, val) in LDS with
// all loads issued before the first wait, then every lane group (G lanes x float4 = the row's
// TW columns) walks its rows with a two-buffer software pipeline: the next row's NB gathers
// are in flight while the current row runs its fmaf chain in CSR order.
// The hot loop is branch-free: a row with fewer than NB entries fills the batch with its own
// last neighbour at weight 0 (fmaf(0, x, acc) == acc exactly: acc is never -0.0), so the
// compiler's vmcnt accounting keeps the next row's loads in flight.
//   FROM_SEEDS (h = 0 -> 1): neighbour values come from the sparse seed lists, filtered by a
//              per-vertex seed-tile mask, so s0 is never materialised densely.
// The own-row seed term s0_v is added afterwards by seed_add_kernel (out = acc + s0, the same
// single rounding as the oracle).  Reachability is a separate pass (reach_kernel): folding
// its words into this walk costs more TA cycles than the reach pass itself (PMC, round 1).
constexpr uint32_t CSR_CAP = 2048;
// sparse halo exchange: mask words per send row (32-column groups; EGR_MAX_COLS columns)
#define EGR_SX_MASK_WORDS ((EGR_MAX_COLS / 32 + 31) / 32)
constexpr int NB = 4;

template <int G>
struct HopGeo {
  static constexpr int ROWS = G == 1 ? 256 : 128;   // max rows per chunk
};

struct HopArgs {
  const uint32_t* row_ptr;
  const uint32_t* col;
  const float* val;
  const uint32_t* chunk_start;
  const uint32_t* seed_ptr;
  const uint32_t* seed_col;
  const float* seed_val;
  const uint32_t* seed_tiles;
  const float* xin;
  float* xout;
  uint8_t* nzout;     // [V][ntiles] per row tile of xout: its non-zero count (the sparse halo pack
  uint32_t ntiles;    // reads only non-zero tiles; the next hop skips gathers of zero tiles)
  // [V][ntiles] the same flags of xin (0 = the tile is all +0), read by the zero-tile skip
  // (hop_kernel<G, false, true>); xbytes = V * TW * 4, the buffer range of one tile of xin
  const uint8_t* nzin;
  uint32_t xbytes;
  uint32_t V;
  uint32_t nchunks;
  // the chunks of one row longer than CSR_CAP (egr_plan::long_chunk): with SKIP they run in a
  // launch of their own (hop_kernel<G, *, true, true>), so the main launch's chunks all compact
  const uint32_t* long_chunks;
  uint32_t nlong;
};

template <bool SEEDS>
struct Batch {
  float4 x[NB];
  uint32_t m[NB];
  uint32_t u[NB];
  float w[NB];
  uint32_t n;
  uint32_t la, lb;   // the row's (live) entry range [la, lb): n = lb - la
};

// Stage a chunk's row offsets (relative to its first entry) and up to CSR_CAP column ids (and
// values) in LDS: every global load is issued before the first LDS store.
// With nz (the hop's input tile flags, [V][ntiles]; a chunk of at most CSR_CAP entries): each
// staged entry's neighbour tile flag is loaded once the column ids have arrived, and the LIVE
// entries (flag != 0: x[col][tile] may hold a non-zero) are compacted in entry order into
// s_live, with the per-64-entry live masks s_segm and their exclusive prefix counts s_segp --
// live_before(x) = s_segp[x / 64] + popc(s_segm[x / 64] below bit x % 64).
constexpr uint32_t NSEG = CSR_CAP / 64;
template <int ROWS, bool VAL>
__device__ __forceinline__ void stage_chunk(const uint32_t* __restrict__ row_ptr,
                                            const uint32_t* __restrict__ col,
                                            const float* __restrict__ val, uint32_t v0,
                                            uint32_t nrows, uint32_t e0, uint32_t e1,
                                            uint32_t* s_rp, uint32_t* s_col, float* s_val,
                                            const uint8_t* __restrict__ nz = nullptr,
                                            uint32_t ntiles = 0, uint32_t tile = 0,
                                            uint16_t* s_live = nullptr, uint64_t* s_segm = nullptr,
                                            uint32_t* s_segp = nullptr,
                                            const uint32_t* __restrict__ seed_tiles = nullptr) {
  constexpr int PER = CSR_CAP / 256;
  const uint32_t tid = threadIdx.x;
  const uint32_t nst = min(e1 - e0, CSR_CAP);
  uint32_t rp_t = 0;
  if (tid < nrows) rp_t = row_ptr[v0 + tid];
  uint32_t cc[PER];
  float ww[PER];
  if (nst > 0) {
#pragma unroll
    for (int k = 0; k < PER; ++k) {
      const uint32_t i = min(tid + k * 256u, nst - 1u);
      cc[k] = col[e0 + i];
      if constexpr (VAL) ww[k] = val[e0 + i];
    }
  }
  if (nz || seed_tiles) {
    // (the first hop: live = the neighbour has a seed in this tile, its per-vertex tile mask)
    uint8_t ff[PER];
#pragma unroll
    for (int k = 0; k < PER; ++k)
      ff[k] = tid + k * 256u >= nst ? 0
            : nz ? nz[(size_t)cc[k] * ntiles + tile]
                 : (uint8_t)((seed_tiles[cc[k]] >> (tile & 31u)) & 1u);
    // entry i = tid + 256 k: wave w of pass k covers the 64 entries of segment 4 k + w
    const uint32_t lane = tid & 63u, wv = tid >> 6;
    uint64_t mk[PER];
#pragma unroll
    for (int k = 0; k < PER; ++k) {
      mk[k] = __ballot(ff[k] != 0);
      if (lane == 0) s_segm[4 * k + wv] = mk[k];
    }
    __syncthreads();
    if (tid < 64) {                          // exclusive prefix of the NSEG segment counts
      uint32_t c = tid < NSEG ? (uint32_t)__popcll(s_segm[tid]) : 0u, inc = c;
#pragma unroll
      for (int o = 1; o < (int)NSEG; o <<= 1) {
        const uint32_t y = __shfl_up(inc, o, 64);
        if ((int)tid >= o) inc += y;
      }
      if (tid < NSEG) s_segp[tid + 1] = inc;
      if (tid == 0) s_segp[0] = 0;
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < PER; ++k) {
      if (ff[k] != 0) {
        const uint32_t r = __builtin_amdgcn_mbcnt_hi((uint32_t)(mk[k] >> 32),
                                                     __builtin_amdgcn_mbcnt_lo((uint32_t)mk[k], 0u));
        s_live[s_segp[4 * k + wv] + r] = (uint16_t)(tid + k * 256u);
      }
    }
  }
  if (tid < nrows) s_rp[tid] = rp_t - e0;
  if (tid == 0) s_rp[nrows] = e1 - e0;       // nrows may equal the block size
  if (nst > 0) {
#pragma unroll
    for (int k = 0; k < PER; ++k) {
      const uint32_t i = tid + k * 256u;
      if (i < nst) {
        s_col[i] = cc[k];
        if constexpr (VAL) s_val[i] = ww[k];
      }
    }
  }
  __syncthreads();
}

#ifndef EGR_HOP_NT_STORE
#define EGR_HOP_NT_STORE 1
#endif
#ifndef EGR_HOP_XCD_REMAP
#define EGR_HOP_XCD_REMAP 0
#endif
#ifndef EGR_HOP_STORE_SKIP
#define EGR_HOP_STORE_SKIP 1
#endif

// SKIP (not FROM_SEEDS): the zero-tile skip -- a row's fmaf chain runs over its LIVE entries
// only, those whose neighbour tile of xin may hold a non-zero (tile flags A.nzin, compacted per
// chunk by stage_chunk), in CSR order: a skipped entry's x are all +0 and fmaf(w, +0, acc) ==
// acc (acc != -0), so the result is bit-identical.  A row with no live entry gathers nothing (its
// batch loads go through a buffer descriptor at an out-of-range offset: zeros, no fetch, and the
// loop keeps its branch-free form).  Hops 2 and 3 of a 3-hop C3 batch gather a non-zero tile
// for 9 % / 34 % of their entries, C4 2 % / 15 % (scripts/tile_sparsity.py).
// SKIP also skips the STORE of a row tile that came out all +0 and holds no seed of the row
// (seed_add_kernel adds into the tiles the seed tile mask marks, so those are always written):
// its flag (count 0) is the tile's value, and every reader of the scores goes through the flags
// (the next hop's gathers, top-k, the read-back, the packs: egr_plan::xsparse).
// LONG (with SKIP): the launch over the chunks of a lone row longer than CSR_CAP, which the main
// SKIP launch leaves out -- their entries are not compacted, and each gather of a neighbour tile
// goes through its flag (a zero tile's memory may be stale since the store skip); the main launch's
// chunks then all take the compacted path, with no per-gather flag test in the hot loop.
template <int G, bool FROM_SEEDS, bool SKIP = false, bool LONG = false>
__global__ __launch_bounds__(256) void hop_kernel(const HopArgs A) {
  constexpr int TW = 4 * G, GROUPS = 256 / G, ROWS = HopGeo<G>::ROWS;
  __shared__ uint32_t s_rp[ROWS + 1];
  __shared__ uint32_t s_col[CSR_CAP];
  __shared__ float s_val[CSR_CAP];
  __shared__ uint16_t s_live[SKIP ? CSR_CAP : 1];        // the chunk's live entries (SKIP)
  __shared__ uint64_t s_segm[SKIP ? NSEG : 1];
  __shared__ uint32_t s_segp[SKIP ? NSEG + 1 : 1];
  const uint32_t tid = threadIdx.x, gl = tid % G, grp = tid / G;
  const uint32_t V = A.V;
#if EGR_HOP_XCD_REMAP
  // workgroups are dealt to the 8 XCDs round-robin (block b -> XCD b % 8): give XCD x one
  // contiguous run of (tile, chunk) blocks, so that the chunks running at once on an XCD are
  // neighbours whose gathers share that XCD's L2
  const uint32_t nb = gridDim.x, xcd = blockIdx.x % 8u, q8 = nb / 8u, r8 = nb % 8u;
  const uint32_t lb = xcd * q8 + min(xcd, r8) + blockIdx.x / 8u;
#else
  const uint32_t lb = blockIdx.x;
#endif
  const uint32_t tile = LONG ? lb / A.nlong : lb / A.nchunks;
  const uint32_t chunk = LONG ? A.long_chunks[lb % A.nlong] : lb % A.nchunks;
  const uint32_t v0 = A.chunk_start[chunk], v1 = A.chunk_start[chunk + 1];
  const uint32_t nrows = v1 - v0;
  const uint32_t e0 = A.row_ptr[v0], e1 = A.row_ptr[v1];
  // (a lone row longer than CSR_CAP -- its own chunk -- gathers every entry; with SKIP it is the
  // LONG launch's, and the main launch leaves it: uniform in the block, before any barrier)
  if constexpr (SKIP && !LONG) {
    if (e1 - e0 > CSR_CAP) return;
  }
  constexpr bool live_on = SKIP && !LONG;
  stage_chunk<ROWS, true>(A.row_ptr, A.col, A.val, v0, nrows, e0, e1, s_rp, s_col, s_val,
                          live_on && !FROM_SEEDS ? A.nzin : nullptr, A.ntiles, tile, s_live, s_segm,
                          s_segp, live_on && FROM_SEEDS ? A.seed_tiles : nullptr);
  if (grp >= nrows) return;  // no barrier below

  const uint32_t lo = tile * TW + 4 * gl;  // first column of this lane
  const uint32_t tbit = tile & 31u;
  const size_t toff = (size_t)tile * V * TW;
  const float4* __restrict__ X = reinterpret_cast<const float4*>(A.xin + toff);
  float4* __restrict__ Y = reinterpret_cast<float4*>(A.xout + toff);
  // one gather of neighbour u's tile; SKIP: through a buffer descriptor, `none` = an
  // out-of-range offset (zeros, nothing fetched)
  const auto xr = __builtin_amdgcn_make_buffer_rsrc((void*)(A.xin + (SKIP ? toff : 0)), 0,
                                                    SKIP ? (int)A.xbytes : 0, 0x00020000);
  auto gather = [&](uint32_t u, bool none) -> float4 {
    if constexpr (SKIP) {
      const uint32_t off = none ? 0x80000000u : (u * (uint32_t)G + gl) * 16u;
      const auto q = __builtin_amdgcn_raw_buffer_load_b128(xr, (int)off, 0, 0);
      return make_float4(__uint_as_float(q[0]), __uint_as_float(q[1]), __uint_as_float(q[2]),
                         __uint_as_float(q[3]));
    } else {
      return X[(size_t)u * G + gl];
    }
  };
  // a lone row longer than CSR_CAP (not compacted): its zero tiles are not gathered either -- since
  // the store skip, a zero tile's memory may be stale, so its flag is what it holds
  auto dead = [&](uint32_t u) -> bool {
    if constexpr (SKIP && LONG) return A.nzin[(size_t)u * A.ntiles + tile] == 0;
    return false;
  };
  // live entries before staged entry x (live_on), and the entry of live index i
  auto live_before = [&](uint32_t x) -> uint32_t {
    const uint32_t sg = x >> 6, bt = x & 63u;
    return s_segp[sg] + (bt ? (uint32_t)__popcll(s_segm[sg] & ((1ull << bt) - 1ull)) : 0u);
  };
  auto entry = [&](uint32_t i) -> uint32_t {
    if constexpr (live_on) return (uint32_t)s_live[min(i, CSR_CAP - 1u)];
    return i;
  };

  // NB (live) entries of row r; slots past the row's end repeat its last one at weight 0
  auto issue = [&](uint32_t r, Batch<FROM_SEEDS>& bt) {
    const uint32_t a = s_rp[r], b = s_rp[r + 1];
    uint32_t la = a, lb = b;
    if constexpr (SKIP) {
      if constexpr (live_on) {
        la = live_before(a);
        lb = live_before(b);
      }
    }
    const uint32_t n = lb - la;
    bt.n = n;
    bt.la = la;
    bt.lb = lb;
#pragma unroll
    for (int t = 0; t < NB; ++t) {
      const uint32_t jj = entry(la + min((uint32_t)t, n > 0u ? n - 1u : 0u));
      const uint32_t u = n > 0u ? s_col[min(jj, CSR_CAP - 1u)] : v0 + r;
      bt.u[t] = u;
      bt.w[t] = (uint32_t)t < n ? s_val[min(jj, CSR_CAP - 1u)] : 0.f;
      if constexpr (FROM_SEEDS) bt.m[t] = A.seed_tiles[u];
      else bt.x[t] = gather(u, n == 0u || dead(u));
    }
  };
  auto seed_gather = [&](uint32_t u, float w, float4& acc) {
    const uint32_t s1 = A.seed_ptr[u + 1];
    for (uint32_t q = seed_lower(A.seed_col, A.seed_ptr[u], s1, lo); q < s1; ++q) {
      const uint32_t c = A.seed_col[q] - lo;
      if (c >= 4u) break;
      fma_comp(acc, (int)c, w, A.seed_val[q]);
    }
  };
  auto process = [&](uint32_t r, const Batch<FROM_SEEDS>& bt) {
    const uint32_t v = v0 + r;
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int t = 0; t < NB; ++t) {
      if constexpr (FROM_SEEDS) {
        // w * 0 unless the neighbour has a seed in this tile: skipping the fmaf is exact
        if ((uint32_t)t < bt.n && ((bt.m[t] >> tbit) & 1u)) seed_gather(bt.u[t], bt.w[t], acc);
      } else {
        fma4(bt.w[t], bt.x[t], acc);
      }
    }
    // tail of rows with more than NB entries, NT gathers per batch (deployments, services,
    // Node hubs); slots past the end repeat the last entry at weight 0
    constexpr int NT = 4;
    const uint32_t b = bt.lb;
    for (uint32_t j = bt.la + NB; j < b; j += NT) {
      uint32_t u[NT];
      float w[NT];
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        const uint32_t jj = entry(min(j + t, b - 1u));
        u[t] = jj < CSR_CAP ? s_col[jj] : A.col[e0 + jj];
        w[t] = j + t < b ? (jj < CSR_CAP ? s_val[jj] : A.val[e0 + jj]) : 0.f;
      }
      if constexpr (FROM_SEEDS) {
        uint32_t m[NT];
#pragma unroll
        for (int t = 0; t < NT; ++t) m[t] = A.seed_tiles[u[t]];
#pragma unroll
        for (int t = 0; t < NT; ++t)
          if (j + t < b && ((m[t] >> tbit) & 1u)) seed_gather(u[t], w[t], acc);
      } else {
        float4 x[NT];
#pragma unroll
        for (int t = 0; t < NT; ++t) x[t] = gather(u[t], dead(u[t]));
#pragma unroll
        for (int t = 0; t < NT; ++t) fma4(w[t], x[t], acc);
      }
    }
    // the row's non-zero count in this tile -- for the sparse halo pack, the next hop's zero-tile
    // skip and the readers of a skipped store (TW = 4G <= 128 columns: a byte): summed over the
    // G lanes of the row's group (contiguous lanes, all active for the same row); -0.0 counts
    // as non-zero
    int c = (__float_as_uint(acc.x) != 0u) + (__float_as_uint(acc.y) != 0u) +
            (__float_as_uint(acc.z) != 0u) + (__float_as_uint(acc.w) != 0u);
#pragma unroll
    for (int o = 1; o < G; o <<= 1) c += __shfl_xor(c, o, 64);
    // (SKIP: an all-+0 tile without a seed of this row is not written; c is uniform in the group)
    if (!SKIP || !EGR_HOP_STORE_SKIP || c != 0 || ((A.seed_tiles[v] >> tbit) & 1u)) {
#if EGR_HOP_NT_STORE
      // streaming store: the output tile is not re-read in this hop, so keep it from evicting
      // the input tile the gathers re-read from the Infinity Cache
      typedef float f4v __attribute__((ext_vector_type(4)));
      __builtin_nontemporal_store(f4v{acc.x, acc.y, acc.z, acc.w},
                                  reinterpret_cast<f4v*>(&Y[(size_t)v * G + gl]));
#else
      Y[(size_t)v * G + gl] = acc;
#endif
    }
    if (gl == 0) A.nzout[(size_t)v * A.ntiles + tile] = (uint8_t)c;
  };

  Batch<FROM_SEEDS> ba, bb;
  uint32_t r = grp;
  issue(r, ba);
  while (true) {
    const uint32_t r1 = r + GROUPS;
    issue(r1 < nrows ? r1 : r, bb);           // unconditional: keeps vmcnt exact
    process(r, ba);
    if (r1 >= nrows) break;
    const uint32_t r2 = r1 + GROUPS;
    issue(r2 < nrows ? r2 : r1, ba);
    process(r1, bb);
    if (r2 >= nrows) break;
    r = r2;
  }
}

// out[v, b] = acc + s0[v, b] for every unique seed (after the hop wrote acc)
// partitioned plans' per-(row, tile) byte: the hop's non-zero count of the tile (0..TW <= 128),
// or NZ_UNKNOWN once a seed was added into it (non-zero, count not kept)
constexpr uint8_t NZ_UNKNOWN = 0xFF;

__global__ void seed_add_kernel(const uint64_t* __restrict__ ukeys,
                                const float* __restrict__ uval,
                                const uint32_t* __restrict__ n_unique, uint32_t Bpad,
                                uint32_t TW, uint32_t V, float* __restrict__ X,
                                uint8_t* __restrict__ nz, uint32_t ntiles) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= *n_unique) return;
  const uint64_t k = ukeys[i];
  const uint32_t v = (uint32_t)(k / Bpad), b = (uint32_t)(k % Bpad);
  float* p = X + ((size_t)(b / TW) * V + v) * TW + (b % TW);
  *p = *p + uval[i];
  // (s0 > 0 or NaN: the entry is non-zero.)  The tile's count is no longer known without reading
  // it: NZ_UNKNOWN makes the pack count that tile from the scores
  if (nz) nz[(size_t)v * ntiles + b / TW] = NZ_UNKNOWN;
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
// R is row-major [V][RS] u64, RS = 2 * RG: word b/64 of row v holds incident b's bit.
__global__ void reach_sources_kernel(const uint32_t* __restrict__ src, int B, uint64_t* R,
                                     uint32_t V, uint32_t RS) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  const uint32_t v = src[b];
  if (v < V) atomicOr((unsigned long long*)&R[(size_t)v * RS + (b >> 6)], 1ull << (b & 63));
}

template <int RG>
struct ReachGeo {
  static constexpr int ROWS = RG == 1 ? 256 : 128;
};

__device__ __forceinline__ uint4 or4(uint4 a, const uint4& b) {
  a.x |= b.x;
  a.y |= b.y;
  a.z |= b.z;
  a.w |= b.w;
  return a;
}

// One reach hop R' = R | A R over one row chunk: the chunk's columns are staged in LDS like
// hop_kernel's, each lane group (RG lanes x 16 B = the row's RS words) ORs its rows' neighbour
// rows with the same two-buffer, branch-free pipeline (a short row repeats its last neighbour:
// OR is idempotent).
template <int RG>
__global__ __launch_bounds__(256) void reach_kernel(const uint32_t* __restrict__ row_ptr,
                                                    const uint32_t* __restrict__ col,
                                                    const uint32_t* __restrict__ chunk_start,
                                                    const uint4* __restrict__ rin,
                                                    uint4* __restrict__ rout) {
  constexpr int GROUPS = 256 / RG, ROWS = ReachGeo<RG>::ROWS;
  __shared__ uint32_t s_rp[ROWS + 1];
  __shared__ uint32_t s_col[CSR_CAP];
  const uint32_t tid = threadIdx.x, gl = tid % RG, grp = tid / RG;
  const uint32_t v0 = chunk_start[blockIdx.x], v1 = chunk_start[blockIdx.x + 1];
  const uint32_t nrows = v1 - v0;
  const uint32_t e0 = row_ptr[v0], e1 = row_ptr[v1];
  stage_chunk<ROWS, false>(row_ptr, col, nullptr, v0, nrows, e0, e1, s_rp, s_col, nullptr);
  if (grp >= nrows) return;  // no barrier below

  struct RB {
    uint4 x[NB];
    uint4 own;
  };
  auto issue = [&](uint32_t r, RB& bt) {
    const uint32_t a = s_rp[r], n = s_rp[r + 1] - a;
#pragma unroll
    for (int t = 0; t < NB; ++t) {
      const uint32_t jj = a + min((uint32_t)t, n > 0u ? n - 1u : 0u);
      const uint32_t u = n > 0u ? s_col[min(jj, CSR_CAP - 1u)] : v0 + r;
      bt.x[t] = rin[(size_t)u * RG + gl];
    }
    bt.own = rin[(size_t)(v0 + r) * RG + gl];
  };
  auto process = [&](uint32_t r, const RB& bt) {
    uint4 acc = bt.own;
#pragma unroll
    for (int t = 0; t < NB; ++t) acc = or4(acc, bt.x[t]);
    constexpr int NT = 4;
    const uint32_t b = s_rp[r + 1];
    for (uint32_t j = s_rp[r] + NB; j < b; j += NT) {
      uint4 x[NT];
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        const uint32_t jj = min(j + t, b - 1u);
        const uint32_t u = jj < CSR_CAP ? s_col[jj] : col[e0 + jj];
        x[t] = rin[(size_t)u * RG + gl];
      }
#pragma unroll
      for (int t = 0; t < NT; ++t) acc = or4(acc, x[t]);
    }
    rout[(size_t)(v0 + r) * RG + gl] = acc;
  };

  RB ba, bb;
  uint32_t r = grp;
  issue(r, ba);
  while (true) {
    const uint32_t r1 = r + GROUPS;
    issue(r1 < nrows ? r1 : r, bb);
    process(r, ba);
    if (r1 >= nrows) break;
    const uint32_t r2 = r1 + GROUPS;
    issue(r2 < nrows ? r2 : r1, ba);
    process(r1, bb);
    if (r2 >= nrows) break;
    r = r2;
  }
}

// ---- top-k candidates: deterministic count -> scan -> fill over the final reach rows --------
// A wave owns 64 vertices (lane = row) of group g.  For each word, ballots over the columns
// present in the wave give every column's count; lane c stores column (64w + c)'s count at
// cnt[col * NG + g].  One exclusive scan over cnt (column-major) yields each (column, group)
// slot, so every column's candidates end up contiguous and in vertex order, with no atomics.
// Excluded-label vertices (Incident) are never candidates.
__device__ __forceinline__ uint64_t cand_word(const uint64_t* __restrict__ R, uint32_t RS,
                                              uint32_t v, bool ok, int w, int B) {
  uint64_t word = ok ? R[(size_t)v * RS + w] : 0ull;
  const int cmax = min(64, B - w * 64);
  if (cmax < 64) word &= (1ull << cmax) - 1ull;
  return word;
}

__device__ __forceinline__ uint64_t wave_or(uint64_t x) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) x |= __shfl_xor(x, off, 64);
  return x;
}

__global__ __launch_bounds__(256) void cand_count_kernel(
    const uint64_t* __restrict__ R, uint32_t RS, const uint8_t* __restrict__ vlabel,
    int exclude_label, uint32_t V, int B, uint32_t NG, uint32_t* __restrict__ cnt) {
  const int lane = threadIdx.x & 63;
  const uint32_t g = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (g >= NG) return;
  const uint32_t v = g * 64 + lane;
  const bool ok = v < V && !(exclude_label >= 0 && vlabel[v] == (uint8_t)exclude_label);
  const int W = (B + 63) / 64;
  for (int w0 = 0; w0 < W; w0 += 4) {
    uint64_t wd[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) wd[t] = w0 + t < W ? cand_word(R, RS, v, ok, w0 + t, B) : 0ull;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int w = w0 + t;
      if (w >= W) break;
      uint32_t mycnt = 0;
      for (uint64_t m = wave_or(wd[t]); m; m &= m - 1) {
        const int c = __ffsll((long long)m) - 1;
        const uint32_t n = (uint32_t)__popcll(__ballot((wd[t] >> c) & 1ull));
        if (lane == c) mycnt = n;
      }
      if (lane < min(64, B - w * 64)) cnt[(size_t)(w * 64 + lane) * NG + g] = mycnt;
    }
  }
}

__global__ __launch_bounds__(256) void cand_fill_kernel(
    const uint64_t* __restrict__ R, uint32_t RS, const uint8_t* __restrict__ vlabel,
    int exclude_label, uint32_t V, int B, uint32_t NG, const uint32_t* __restrict__ off,
    uint32_t* __restrict__ cand_list) {
  const int lane = threadIdx.x & 63;
  const uint32_t g = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (g >= NG) return;
  const uint32_t v = g * 64 + lane;
  const bool ok = v < V && !(exclude_label >= 0 && vlabel[v] == (uint8_t)exclude_label);
  const uint64_t lt = (1ull << lane) - 1ull;
  const int W = (B + 63) / 64;
  for (int w = 0; w < W; ++w) {
    const uint64_t word = cand_word(R, RS, v, ok, w, B);
    const uint64_t cols = wave_or(word);
    if (!cols) continue;
    const uint32_t mybase = lane < min(64, B - w * 64) ? off[(size_t)(w * 64 + lane) * NG + g] : 0u;
    for (uint64_t m = cols; m; m &= m - 1) {
      const int c = __ffsll((long long)m) - 1;
      const uint64_t bits = __ballot((word >> c) & 1ull);
      const uint32_t base = __shfl(mybase, c, 64);
      if ((word >> c) & 1ull) cand_list[base + __popcll(bits & lt)] = v;
    }
  }
}

// [V][RS] -> [W][V] for egr_plan_read_reach (the header's layout)
__global__ void reach_export_kernel(const uint64_t* __restrict__ R, uint32_t RS, uint32_t V,
                                    int W, uint64_t* __restrict__ out) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (size_t)W * V) return;
  const uint32_t w = (uint32_t)(i / V), v = (uint32_t)(i % V);
  out[i] = R[(size_t)v * RS + w];
}

// ---- top-k -----------------------------------------------------------------------------------
// One score of the tiled buffer; nz (the buffer's tile flags when its last hop skipped the stores
// of all-+0 tiles, egr_plan::xsparse; else nullptr): a tile flagged 0 reads as +0 without a load.
__device__ __forceinline__ float x_at(const float* __restrict__ X, const uint8_t* __restrict__ nz,
                                      uint32_t ntiles, uint32_t V, int TW, uint32_t v, int b) {
  const uint32_t tile = (uint32_t)(b / TW);
  if (nz && nz[(size_t)v * ntiles + tile] == 0) return 0.f;
  return X[((size_t)tile * V + v) * TW + (b % TW)];
}

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
    const float* __restrict__ X, const uint64_t* __restrict__ R, uint32_t RS,
    const uint8_t* __restrict__ vlabel, int exclude_label, uint32_t V, uint32_t VC, int TW, int B,
    int n_chunks, float* __restrict__ part_s, uint32_t* __restrict__ part_v,
    const uint8_t* __restrict__ nz, uint32_t nzt) {
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
    const uint64_t* Rw = R + (b >> 6);
    const uint64_t bit = 1ull << (b & 63);
    const uint32_t v0 = (uint32_t)ch * TOPK_CHUNK;
    const uint32_t v1 = min(VC, v0 + TOPK_CHUNK);   // rows >= VC (halo) are never candidates
    // eight rows per step: all reach words and labels, then the reached scores, are loaded
    // before any insertion, so a wave keeps 8-16 loads in flight instead of one
    for (uint32_t vb = v0 + rp; vb < v1; vb += 8u * rps) {
      uint64_t wd[8];
      uint8_t lab[8];
      float xs[8];
#pragma unroll
      for (int t = 0; t < 8; ++t) {
        const uint32_t v = vb + t * rps;
        wd[t] = v < v1 ? Rw[(size_t)v * RS] : 0ull;
        lab[t] = v < v1 ? vlabel[v] : 0;
      }
#pragma unroll
      for (int t = 0; t < 8; ++t) {
        const uint32_t v = vb + t * rps;
        const bool cand = (wd[t] & bit) && !(exclude_label >= 0 && lab[t] == (uint8_t)exclude_label);
        wd[t] = cand;
        xs[t] = cand && !(nz && nz[(size_t)v * nzt + tile] == 0) ? Xt[(size_t)v * TW + cx] : 0.f;
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

// top-k over each column's candidate list (cand_fill_kernel): one wave per column
__global__ __launch_bounds__(256) void topk_cand_kernel(
    const float* __restrict__ X, const uint32_t* __restrict__ off, uint32_t NG,
    const uint32_t* __restrict__ cand_list, uint32_t V, int TW, int B, int k,
    uint32_t* __restrict__ out_ids, float* __restrict__ out_scores, const uint8_t* __restrict__ nz,
    uint32_t ntiles) {
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
  const uint32_t s0 = off[(size_t)b * NG];
  const uint32_t n = min(off[(size_t)(b + 1) * NG] - s0, V);
  const float* __restrict__ Xc = X + (size_t)(b / TW) * V * TW + (b % TW);
  const uint32_t* __restrict__ Lb = cand_list + s0;
  for (uint32_t i0 = lane; i0 < n; i0 += 64u * 4u) {
    uint32_t vv[4];
    float ss[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) vv[t] = i0 + t * 64u < n ? Lb[i0 + t * 64u] : NO_NODE;
#pragma unroll
    for (int t = 0; t < 4; ++t)
      ss[t] = vv[t] != NO_NODE && !(nz && nz[(size_t)vv[t] * ntiles + b / TW] == 0) ? Xc[(size_t)vv[t] * TW] : 0.f;
#pragma unroll
    for (int t = 0; t < 4; ++t)
      if (vv[t] != NO_NODE) list_insert(Ls, Lv, ss[t], vv[t]);
  }
  wave_emit_topk(Ls, Lv, k, lane, out_ids + (size_t)b * k, out_scores + (size_t)b * k);
}

__global__ void scores_rowmajor_kernel(const float* __restrict__ X, uint32_t V, int TW, int B,
                                       float* __restrict__ out, const uint8_t* __restrict__ nz,
                                       uint32_t ntiles) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (size_t)V * B) return;
  const uint32_t v = (uint32_t)(i / B);
  const int b = (int)(i % B);
  out[i] = x_at(X, nz, ntiles, V, TW, v, b);
}

__global__ void induced_kernel(const uint32_t* __restrict__ row_ptr,
                               const uint32_t* __restrict__ col, const uint8_t* __restrict__ meta,
                               const uint64_t* __restrict__ Rw, uint32_t RS, uint64_t bit, uint32_t V,
                               uint32_t* osrc, uint32_t* odst, uint8_t* otype, int64_t cap,
                               unsigned long long* counter) {
  const uint32_t v = blockIdx.x * blockDim.x + threadIdx.x;
  if (v >= V || !(Rw[(size_t)v * RS] & bit)) return;
  for (uint32_t e = row_ptr[v]; e < row_ptr[v + 1]; ++e) {
    const uint8_t m = meta[e];
    if (m & 1u) continue;  // dir 1 duplicates: each edge is listed once, in its target's row
    const uint32_t u = col[e];
    if (!(Rw[(size_t)u * RS] & bit)) continue;
    const unsigned long long slot = atomicAdd(counter, 1ull);
    if ((int64_t)slot < cap) {
      osrc[slot] = u;
      odst[slot] = v;
      otype[slot] = m >> 1;
    }
  }
}

// ---- halo exchange of a partitioned graph (egraph/shard.py): rows of the tiled scores and of
// the row-major reach words to / from dense [n][Bpad] / [n][W] buffers.  One block per row.
__global__ void pack_scores_kernel(const float* __restrict__ X, uint32_t V, int TW, int Bpad,
                                   const uint32_t* __restrict__ rows, float* __restrict__ out,
                                   const uint8_t* __restrict__ nz, uint32_t ntiles) {
  const uint32_t v = rows[blockIdx.x];
  for (int b = threadIdx.x; b < Bpad; b += blockDim.x)
    out[(size_t)blockIdx.x * Bpad + b] = x_at(X, nz, ntiles, V, TW, v, b);
}

__global__ void unpack_scores_kernel(float* __restrict__ X, uint32_t V, int TW, int Bpad,
                                     const uint32_t* __restrict__ rows,
                                     const uint32_t* __restrict__ src, const float* __restrict__ in,
                                     uint8_t* __restrict__ nzf) {
  const uint32_t v = rows[blockIdx.x];
  const size_t o = (size_t)src[blockIdx.x] * Bpad;
  for (int b = threadIdx.x; b < Bpad; b += blockDim.x)
    X[((size_t)(b / TW) * V + v) * TW + (b % TW)] = in[o + b];
  // a whole row written: every tile may hold a non-zero (the next hop gathers them all)
  const int ntiles = Bpad / TW;
  if (nzf)
    for (int t = threadIdx.x; t < ntiles; t += blockDim.x) nzf[(size_t)v * ntiles + t] = 0xFF;
}

__global__ void pack_reach_kernel(const uint64_t* __restrict__ R, uint32_t RS, int W,
                                  const uint32_t* __restrict__ rows, uint64_t* __restrict__ out) {
  const uint32_t v = rows[blockIdx.x];
  for (int w = threadIdx.x; w < W; w += blockDim.x) out[(size_t)blockIdx.x * W + w] = R[(size_t)v * RS + w];
}

__global__ void unpack_reach_kernel(uint64_t* __restrict__ R, uint32_t RS, int W,
                                    const uint32_t* __restrict__ rows,
                                    const uint32_t* __restrict__ src, const uint64_t* __restrict__ in) {
  const uint32_t v = rows[blockIdx.x];
  const size_t o = (size_t)src[blockIdx.x] * W;
  for (int w = threadIdx.x; w < W; w += blockDim.x) R[(size_t)v * RS + w] = in[o + w];
}

// ---- sparse halo exchange: only the non-zero entries of the boundary rows cross the link ----
// Row r of the send list (rows grouped by destination rank: seg[q] .. seg[q+1]) contributes its
// non-zero columns b as entries ((r - seg[q]) * width + b) << 32 | bits (scores, one int64) or
// ((r - seg[q]) * W + w, word) (reach, two int64), written at the row's offset of an exclusive
// scan over the per-row counts (so each peer's entries are contiguous, in (row, column) order).
// One 256-thread block per row.
__device__ __forceinline__ uint32_t sx_value(const float* X, const uint64_t* R, uint32_t V, int TW,
                                             uint32_t RS, uint32_t v, int b, bool reach,
                                             uint64_t* word) {
  if (reach) {
    *word = R[(size_t)v * RS + b];
    return *word != 0ull;
  }
  const uint32_t bits = __float_as_uint(X[((size_t)(b / TW) * V + v) * TW + (b % TW)]);
  *word = bits;
  return bits != 0u;     // -0.0 is not +0: sent (bit-exact)
}

// off[seg[q]] for q = 0..P: the entry offsets at the peer boundaries, contiguous
__global__ void sx_bounds_kernel(const int64_t* __restrict__ off, const int64_t* __restrict__ seg, int P,
                                 int64_t* __restrict__ out) {
  const int q = threadIdx.x;
  if (q <= P) out[q] = off[seg[q]];
}

// The exchange kernels run ONE WAVE PER ROW, four per 256-thread block, in a grid of at most
// SX_MAX_BLOCKS blocks that strides over the rows: a boundary row is cheap, and a block (or a
// wave) per row launched them bound by workgroup dispatch (~120k rows per C4 exchange at P = 8).
constexpr int SX_ROWS = 4;
constexpr int64_t SX_MAX_BLOCKS = 2048;      // grid-stride beyond this (8 blocks per CU)
inline dim3 sx_grid(int64_t n) { return dim3((unsigned)std::min<int64_t>((n + SX_ROWS - 1) / SX_ROWS, SX_MAX_BLOCKS)); }
// the work map is one 64-bit mask of 64-column chunks per row: rows up to 4096 columns (words)
constexpr int SX_MAP_MAX = 64 * 64;
// the work-map kernels: the same waves as sx_grid, each wave's rows strided by the wave count
// and mapped one lane each up front (a wave-per-row walk paid its row id, flags and data loads
// one after another for each of its ~15 rows)
inline dim3 sx_lane_grid(int64_t n) {
  return dim3((unsigned)std::max<int64_t>(1, std::min<int64_t>((n + SX_ROWS - 1) / SX_ROWS, SX_MAX_BLOCKS)));
}

// Sender, pass 1: the row's non-zero count, and a bit per 32-column group that holds any
// (masks [n_rows][MW] u32) so that pass 2 reads only those groups; score rows of a partitioned
// plan skip the tiles the hop wrote no non-zero to (nzf).
__global__ __launch_bounds__(256) void sx_count_kernel(const float* __restrict__ X,
    const uint64_t* __restrict__ R, uint32_t V, int TW, uint32_t RS, int width, bool reach,
    const uint32_t* __restrict__ rows, int64_t n, int64_t* __restrict__ cnt,
    uint32_t* __restrict__ masks, int MW, const uint8_t* __restrict__ nzf, uint32_t ntiles) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  for (int64_t r = (int64_t)blockIdx.x * SX_ROWS + wv; r < n; r += (int64_t)gridDim.x * SX_ROWS) {
  const uint32_t v = rows[r];
  const uint8_t* fl = nzf ? nzf + (size_t)v * ntiles : nullptr;
  // the row's tile flags in one wave-wide load (up to 64 tiles; more: read per column)
  const uint64_t fm = fl && ntiles <= 64u ? __ballot(lane < (int)ntiles && fl[lane]) : ~0ull;
  auto flagged = [&](int t) { return !fl || (ntiles <= 64u ? ((fm >> t) & 1ull) != 0ull : fl[t] != 0); };
  uint32_t mk[EGR_SX_MASK_WORDS];
#pragma unroll
  for (int i = 0; i < EGR_SX_MASK_WORDS; ++i) mk[i] = 0u;
  int c = 0;
  for (int b0 = 0; b0 < width; b0 += 64) {
    if (fl && TW >= 64 && !flagged(b0 / TW)) continue;    // (uniform: one tile per 64 columns)
    const int b = b0 + lane;
    uint64_t w;
    const bool nz = b < width && flagged(b / TW) && sx_value(X, R, V, TW, RS, v, b, reach, &w);
    const uint64_t m = __ballot(nz);
    c += __popcll(m);
    const int g = b0 >> 5;
#pragma unroll
    for (int i = 0; i < EGR_SX_MASK_WORDS; ++i) {
      if (i == (g >> 5) && (uint32_t)m) mk[i] |= 1u << (g & 31);
      if (i == ((g + 1) >> 5) && (m >> 32)) mk[i] |= 1u << ((g + 1) & 31);
    }
  }
  if (lane == 0) {
    cnt[r] = c;
    for (int i = 0; i < MW; ++i) masks[(size_t)r * MW + i] = mk[i];
  }
  }
}

// index of the k-th set bit (k from 0) of the MW-word mask m
__device__ __forceinline__ int kth_bit(const uint32_t* __restrict__ m, int MW, int k) {
  for (int i = 0; i < MW; ++i) {
    uint32_t x = m[i];
    const int c = __popc(x);
    if (k < c) {
      for (int j = 0; j < k; ++j) x &= x - 1u;
      return 32 * i + (__ffs((int)x) - 1);
    }
    k -= c;
  }
  return -1;
}

// Sender, pass 2: the non-zero entries of the row's marked groups, in column order, at the
// row's offset (the exclusive scan of pass 1's counts).  Each half-wave takes one marked group
// per round.
__global__ __launch_bounds__(256) void sx_emit_kernel(const float* __restrict__ X,
    const uint64_t* __restrict__ R, uint32_t V, int TW, uint32_t RS, int width, bool reach,
    const uint32_t* __restrict__ rows, int64_t n, const int64_t* __restrict__ seg, int P,
    const int64_t* __restrict__ off, const uint32_t* __restrict__ masks, int MW,
    int64_t* __restrict__ out, int64_t cap, const uint8_t* __restrict__ nzf, uint32_t ntiles) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, half = lane >> 5, hl = lane & 31;
  for (int64_t r = (int64_t)blockIdx.x * SX_ROWS + wv; r < n; r += (int64_t)gridDim.x * SX_ROWS) {
  uint32_t mk[EGR_SX_MASK_WORDS];
  int nset = 0;
#pragma unroll
  for (int i = 0; i < EGR_SX_MASK_WORDS; ++i) {
    mk[i] = i < MW ? masks[(size_t)r * MW + i] : 0u;
    nset += __popc(mk[i]);
  }
  if (nset == 0) continue;                                 // (uniform in the wave)
  const uint32_t v = rows[r];
  int q = 0;
  while (q + 1 < P && seg[q + 1] <= r) ++q;
  const int64_t rl = r - seg[q];
  int64_t pos = off[r];
  const int64_t lim = cap;               // entries (scores) / words (reach) the target holds
  int64_t* dst = out;
  for (int base = 0; base < nset; base += 2) {
    const int g = base + half < nset ? kth_bit(mk, MW, base + half) : -1;
    const int b = g >= 0 ? 32 * g + hl : width;
    uint64_t w = 0;
    // (a 32-column group spans several tiles below TW = 32: the count pass read only flagged
    // tiles, and a tile flagged 0 may hold stale memory since the hop's store skip)
    const bool nz = b < width && (!nzf || nzf[(size_t)v * ntiles + b / TW] != 0) &&
                    sx_value(X, R, V, TW, RS, v, b, reach, &w);
    const uint64_t m = __ballot(nz);
    const uint32_t lo = (uint32_t)m, hi = (uint32_t)(m >> 32);
    const uint32_t mine = half ? hi : lo;
    const int before = __popc(mine & ((1u << hl) - 1u)) + (half ? __popc(lo) : 0);
    // (launched before the host has checked the total against the buffer: entries past `cap`
    // words are dropped here and the call then fails)
    if (nz) {
      const int64_t idx = rl * width + b;
      if (reach) {
        if (2 * (pos + before) + 1 < lim) {
          dst[2 * (pos + before)] = idx;
          dst[2 * (pos + before) + 1] = (int64_t)w;
        }
      } else if (pos + before < lim) {
        dst[pos + before] = (idx << 32) | (int64_t)w;
      }
    }
    pos += __popcll(m);
  }
  }
}

// The work map of a wave's exchange rows, one lane per row (the fixed-capacity pack and unpack): a
// bit per 64-column chunk of the row that may hold a non-zero -- for a score row, the chunks
// over the tiles its flags mark (every chunk without flags); for a reach row, the chunks holding
// a non-zero word (the row's W <= 64 words... read by the lane: RS-word rows, 16-B loads).
// One lane per row puts the wave's rows' dependent loads (row id, then its flags) in flight at
// once; the wave then walks the rows with work, chunk by chunk.
__device__ __forceinline__ uint64_t sx_chunk_mask(const uint64_t* __restrict__ R, uint32_t RS,
                                                  int width, bool reach, uint32_t v,
                                                  const uint8_t* __restrict__ fl, uint32_t ntiles,
                                                  int TW) {
  const int nchunks = (width + 63) / 64;
  const uint64_t all = nchunks >= 64 ? ~0ull : ((1ull << nchunks) - 1ull);
  if (reach) {                                  // width = W words (one chunk while W <= 64)
    const uint64_t* row = R + (size_t)v * RS;
    uint64_t any = 0;
    for (int w = 0; w < width; ++w) any |= row[w];
    return any ? all : 0ull;
  }
  if (!fl || ntiles > 64u) return all;
  uint64_t m = 0;
  for (uint32_t t = 0; t < ntiles; ++t)
    if (fl[t]) {
      const int c0 = (int)(t * TW) / 64, c1 = (int)(t * TW + TW - 1) / 64;
      for (int c = c0; c <= c1; ++c) m |= 1ull << c;
    }
  return m;
}

// Fixed-capacity send (egr_plan_pack_sparse_cap), pass 1: every send row's non-zero count into
// cnt[r] (cnt[n] = 0 for the exclusive scan that follows).  Rows are mapped one lane each
// (sx_chunk_mask); the wave then counts only the rows with work, chunk by chunk.  (Reserving
// slot space with atomics on the peers' cursors instead of a scan serialised ~30k atomics on
// seven addresses: 0.66 ms per C4 exchange.)
__global__ __launch_bounds__(256) void sx_count_rows_kernel(const float* __restrict__ X,
    const uint64_t* __restrict__ R, uint32_t V, int TW, uint32_t RS, int width, bool reach,
    const uint32_t* __restrict__ rows, int64_t n, const uint8_t* __restrict__ nzf,
    uint32_t ntiles, int64_t* __restrict__ cnt) {
  const int lane = threadIdx.x & 63;
  const int64_t wave = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6), nw = (int64_t)gridDim.x * 4;
  if (wave == 0 && lane == 0) cnt[n] = 0;
  // score rows of a partitioned plan: the hop's per-tile counts add up on the lane; only the
  // tiles a seed add marked unknown are counted from the scores by the wave below
  const bool counted = !reach && nzf && ntiles <= 64u;
  for (int64_t g0 = wave; g0 < n; g0 += nw * 64) {   // rows g0 + j * nw, j = lane
    const int64_t rmine = g0 + (int64_t)lane * nw;
    uint32_t vm = 0;
    uint64_t cm = 0;
    if (rmine < n) {
      vm = rows[rmine];
      if (!counted)
        cm = sx_chunk_mask(R, RS, width, reach, vm, nzf ? nzf + (size_t)vm * ntiles : nullptr,
                           ntiles, TW);
    }
    int64_t mine = 0;
    if (counted && rmine < n) {
      const uint8_t* fl = nzf + (size_t)vm * ntiles;
      for (uint32_t t = 0; t < ntiles; ++t) {
        const uint8_t x = fl[t];
        if (x != NZ_UNKNOWN) {
          mine += x;
        } else {
          const int c0 = (int)(t * TW) / 64, c1 = (int)(t * TW + TW - 1) / 64;
          for (int c = c0; c <= c1; ++c) cm |= 1ull << c;
        }
      }
    }
    for (uint64_t todo = __ballot(cm != 0ull); todo; todo &= todo - 1ull) {
      const int l = __ffsll((long long)todo) - 1;
      const uint32_t v = (uint32_t)__shfl((int)vm, l, 64);
      const uint64_t m = ((uint64_t)(uint32_t)__shfl((int)(uint32_t)(cm >> 32), l, 64) << 32) |
                         (uint32_t)__shfl((int)(uint32_t)cm, l, 64);
      const uint8_t* fl = nzf ? nzf + (size_t)v * ntiles : nullptr;
      int c = 0;
      for (uint64_t cs = m; cs; cs &= cs - 1ull) {
        const int b = 64 * (__ffsll((long long)cs) - 1) + lane;
        uint64_t w = 0;
        c += __popcll(__ballot(b < width && (!fl || (counted ? fl[b / TW] == NZ_UNKNOWN : fl[b / TW] != 0)) &&
                               sx_value(X, R, V, TW, RS, v, b, reach, &w)));
      }
      if (lane == l) mine += c;
    }
    if (rmine < n) cnt[rmine] = mine;
  }
}

// Pass 2 (after the exclusive scan of cnt into off): the entries of every row with work at its
// offset within its peer's slot (off[r] - off[seg[q]]), in (row, column) order.  A slot is one
// header word -- the peer's entry count off[seg[q + 1]] - off[seg[q]], which the wave of block 0
// writes (and into counts[q] when given), flagging an overflow past the capacity -- then
// peer_cap entries (x2 words for reach): the count travels in the slot itself, so an exchange is
// ONE equal-split all-to-all.  Entries past a slot's capacity are dropped.  A row whose entries
// do not end where the scan says (its count pass and its emit disagree: the hop's tile counts
// and the scores no longer match) flags an overflow too, so the pass re-runs on the host-count
// path instead of leaving gaps or overlaps in a slot.
__global__ __launch_bounds__(256) void sx_emit_rows_kernel(const float* __restrict__ X,
    const uint64_t* __restrict__ R, uint32_t V, int TW, uint32_t RS, int width, bool reach,
    const uint32_t* __restrict__ rows, int64_t n, const int64_t* __restrict__ seg, int P,
    const uint8_t* __restrict__ nzf, uint32_t ntiles, const int64_t* __restrict__ off,
    int64_t* __restrict__ out, int64_t peer_cap, int64_t* __restrict__ counts,
    uint32_t* __restrict__ overflow) {
  const int lane = threadIdx.x & 63;
  const uint64_t lt = (1ull << lane) - 1ull;
  const int64_t wave = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6), nw = (int64_t)gridDim.x * 4;
  const int64_t stride = 1 + peer_cap * (reach ? 2 : 1);   // header word + entries
  if (wave == 0) {
    for (int q = lane; q < P; q += 64) {
      const int64_t c = off[seg[q + 1]] - off[seg[q]];
      out[(size_t)q * stride] = c;
      if (counts) counts[q] = c;
      if (c > peer_cap) atomicOr(overflow, 1u);
    }
  }
  for (int64_t g0 = wave; g0 < n; g0 += nw * 64) {   // rows g0 + j * nw, j = lane
    const int64_t rmine = g0 + (int64_t)lane * nw;
    uint32_t vm = 0;
    uint64_t cm = 0;
    if (rmine < n && off[rmine + 1] > off[rmine]) {     // (the scan says which rows have entries)
      vm = rows[rmine];
      cm = sx_chunk_mask(R, RS, width, reach, vm, nzf ? nzf + (size_t)vm * ntiles : nullptr,
                         ntiles, TW);
    }
    for (uint64_t todo = __ballot(cm != 0ull); todo; todo &= todo - 1ull) {
      const int l = __ffsll((long long)todo) - 1;
      const int64_t r = g0 + (int64_t)l * nw;
      const uint32_t v = (uint32_t)__shfl((int)vm, l, 64);
      const uint64_t m = ((uint64_t)(uint32_t)__shfl((int)(uint32_t)(cm >> 32), l, 64) << 32) |
                         (uint32_t)__shfl((int)(uint32_t)cm, l, 64);
      int q = 0;
      while (q + 1 < P && seg[q + 1] <= r) ++q;
      const int64_t rl = r - seg[q];
      int64_t pos = off[r] - off[seg[q]];
      const uint8_t* fl = nzf ? nzf + (size_t)v * ntiles : nullptr;
      int64_t* dst = out + (size_t)q * stride + 1;
      for (uint64_t cs = m; cs; cs &= cs - 1ull) {
        const int b = 64 * (__ffsll((long long)cs) - 1) + lane;
        uint64_t w = 0;
        const bool nz = b < width && (!fl || fl[b / TW]) && sx_value(X, R, V, TW, RS, v, b, reach, &w);
        const uint64_t bm = __ballot(nz);
        const int64_t p = pos + __popcll(bm & lt);
        if (nz && p < peer_cap) {
          const int64_t idx = rl * width + b;
          if (reach) {
            dst[2 * p] = idx;
            dst[2 * p + 1] = (int64_t)w;
          } else {
            dst[p] = (idx << 32) | (int64_t)w;
          }
        }
        pos += __popcll(bm);
      }
      if (lane == 0 && pos != off[r + 1] - off[seg[q]]) atomicOr(overflow, 2u);
    }
  }
}

// Receiver of the fixed-capacity exchange: zero the received halo rows (score rows: only the
// tiles written since the last unpack, once the buffer has been zeroed in full; their flags with
// them), the work map taken one lane per row as in the send.
__global__ __launch_bounds__(256) void sx_zero_rows_kernel(float* __restrict__ X,
    uint64_t* __restrict__ R, uint32_t V, int TW, uint32_t RS, int width, bool reach,
    const uint32_t* __restrict__ recv_vertex, int64_t n, uint8_t* __restrict__ nzf,
    uint32_t ntiles, bool flagged) {
  const int lane = threadIdx.x & 63;
  const int64_t wave = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6), nw = (int64_t)gridDim.x * 4;
  for (int64_t g0 = wave; g0 < n; g0 += nw * 64) {   // rows g0 + j * nw, j = lane
    const int64_t rmine = g0 + (int64_t)lane * nw;
    uint32_t vm = 0;
    uint64_t cm = 0;
    if (rmine < n) {
      vm = recv_vertex[rmine];
      if (reach) {                                   // a lane clears its own row's W words
        uint64_t* row = R + (size_t)vm * RS;
        for (int w = 0; w < width; ++w) row[w] = 0ull;
      } else {
        const int nchunks = (width + 63) / 64;
        cm = nchunks >= 64 ? ~0ull : ((1ull << nchunks) - 1ull);
        if (flagged) cm = sx_chunk_mask(R, RS, width, false, vm, nzf + (size_t)vm * ntiles, ntiles, TW);
      }
    }
    if (reach) continue;
    for (uint64_t todo = __ballot(cm != 0ull); todo; todo &= todo - 1ull) {
      const int l = __ffsll((long long)todo) - 1;
      const uint32_t v = (uint32_t)__shfl((int)vm, l, 64);
      const uint64_t m = ((uint64_t)(uint32_t)__shfl((int)(uint32_t)(cm >> 32), l, 64) << 32) |
                         (uint32_t)__shfl((int)(uint32_t)cm, l, 64);
      const uint8_t* fl = nzf ? nzf + (size_t)v * ntiles : nullptr;
      for (uint64_t cs = m; cs; cs &= cs - 1ull) {
        const int b = 64 * (__ffsll((long long)cs) - 1) + lane;
        if (b < width && (!flagged || fl[b / TW])) X[((size_t)(b / TW) * V + v) * TW + (b % TW)] = 0.f;
      }
    }
    if (nzf) {
      // every lane of the wave has read the flags of the wave's rows: clear them
      __builtin_amdgcn_wave_barrier();
      if (rmine < n)
        for (uint32_t t = 0; t < ntiles; ++t) nzf[(size_t)vm * ntiles + t] = 0;
    }
  }
}

// Receiver: zero the received halo rows, then scatter the entries (one thread per entry; the
// sender s of entry e: eseg[s] <= e < eseg[s+1]; its recv rows start at rbase[s]).
// With flags (scores of a partitioned plan whose buffer has been zeroed once): only the tiles
// a scatter (or a seed add) wrote since are cleared, and their flags with them.
__global__ __launch_bounds__(256) void sx_zero_kernel(float* __restrict__ X, uint64_t* __restrict__ R,
                               uint32_t V, int TW, uint32_t RS, int width, bool reach,
                               const uint32_t* __restrict__ recv_vertex, int64_t n,
                               uint8_t* __restrict__ nzf, uint32_t ntiles, bool flagged) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  for (int64_t r = (int64_t)blockIdx.x * SX_ROWS + wv; r < n; r += (int64_t)gridDim.x * SX_ROWS) {
  const uint32_t v = recv_vertex[r];
  uint8_t* fl = nzf ? nzf + (size_t)v * ntiles : nullptr;
  const uint64_t fm = flagged && ntiles <= 64u ? __ballot(lane < (int)ntiles && fl[lane]) : ~0ull;
  auto set = [&](int t) { return !flagged || (ntiles <= 64u ? ((fm >> t) & 1ull) != 0ull : fl[t] != 0); };
  for (int b0 = 0; b0 < width; b0 += 64) {
    if (flagged && TW >= 64 && !set(b0 / TW)) continue;    // (uniform: one tile per 64 columns)
    const int b = b0 + lane;
    if (b >= width || !set(b / TW)) continue;
    if (reach) R[(size_t)v * RS + b] = 0ull;
    else X[((size_t)(b / TW) * V + v) * TW + (b % TW)] = 0.f;
  }
  if (fl) {
    __builtin_amdgcn_wave_barrier();                       // every lane has read the flags
    for (uint32_t t = lane; t < ntiles; t += 64) fl[t] = 0;
  }
  }
}

// Fixed-capacity mode (peer_cap > 0, egr_plan_unpack_sparse_cap): sender s's slot starts at
// word s * (1 + peer_cap * per) of `in`: its entry count, then its entries, of which the first
// min(count, peer_cap) are scattered; n = P * peer_cap entry positions are scanned, and a count
// past the capacity (the sender's slot overflowed) sets *ovf.
__global__ void sx_scatter_kernel(float* __restrict__ X, uint64_t* __restrict__ R, uint32_t V,
                                  int TW, uint32_t RS, int width, bool reach,
                                  const uint32_t* __restrict__ recv_vertex,
                                  const int64_t* __restrict__ in, int64_t n,
                                  const int64_t* __restrict__ eseg,
                                  const int64_t* __restrict__ rbase, int P,
                                  uint8_t* __restrict__ nzf, uint32_t ntiles,
                                  int64_t peer_cap = 0, uint32_t* __restrict__ ovf = nullptr) {
  int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= n) return;
  int s = 0;
  if (peer_cap > 0) {
    s = (int)(e / peer_cap);
    const int64_t j = e - (int64_t)s * peer_cap;
    const int64_t base = (int64_t)s * (1 + peer_cap * (reach ? 2 : 1));
    const int64_t c = in[base];                            // the sender's header word
    if (j == 0 && c > peer_cap && ovf) atomicOr(ovf, 1u);
    if (j >= c) return;                                    // (past the count, or the slot: dropped)
    in += base + 1;                                        // entry j of this slot
    e = j;
  } else {
    while (s + 1 < P && eseg[s + 1] <= e) ++s;
  }
  int64_t idx;
  uint64_t w;
  if (reach) {
    idx = in[2 * e];
    w = (uint64_t)in[2 * e + 1];
  } else {
    const uint64_t x = (uint64_t)in[e];
    idx = (int64_t)(x >> 32);
    w = x & 0xFFFFFFFFull;
  }
  const int64_t row = rbase[s] + idx / width;     // (idx is relative to sender s's rows)
  const int b = (int)(idx % width);
  const uint32_t v = recv_vertex[row];
  if (reach) R[(size_t)v * RS + b] = w;
  else {
    X[((size_t)(b / TW) * V + v) * TW + (b % TW)] = __uint_as_float((uint32_t)w);
    if (nzf) nzf[(size_t)v * ntiles + b / TW] = 1;  // (the next unpack clears only these tiles)
  }
}

}  // namespace

struct egr_plan {
  const egr_snapshot* s = nullptr;
  uint64_t version = 0;      // snapshot version the V-sized buffers and chunk tables were built for
  int B = 0, TW = 0, Bpad = 0, ntiles = 0, W = 0, k = 0;
  int RG = 0, RS = 0;        // reach: RG lanes x 16 B per row, RS = 2*RG words per row
  int64_t max_seeds = 0;
  int n_chunks = 0;          // top-k full-scan chunks
  uint32_t nchunks = 0;      // hop row chunks per tile
  uint32_t* chunk_start = nullptr;
  uint32_t nlong = 0;        // hop chunks of one row longer than CSR_CAP, and their indices
  uint32_t* long_chunk = nullptr;
  uint32_t rnchunks = 0;     // reach row chunks
  uint32_t* rchunk_start = nullptr;
  float* x[2] = {nullptr, nullptr};
  int xcur = 0;
  // partitioned plans (egr_plan_set_owned): per x buffer, [V][ntiles] tile flags -- owned rows:
  // the hop's non-zero tiles (the sparse pack reads only those); halo rows: the tiles written
  // since the last unpack (it clears only those, once the buffer has been zeroed in full)
  uint8_t* nzf[2] = {nullptr, nullptr};
  bool xzeroed[2] = {false, false};
  bool skip_zero = true;             // hop_kernel's zero-tile skip ($EGRAPH_HOP_NO_SKIP=1: off)
  // x[i]'s last hop skipped the stores of all-+0 tiles: its flags nzf[i] say which tiles hold
  // scores, and every reader goes through them (a tile flagged 0 may hold stale memory)
  bool xsparse[2] = {false, false};
  uint64_t* reach[2] = {nullptr, nullptr};
  int rcur = 0;
  int reach_hops = -1;  // -1: sources not set
  int hops_done = -1;   // -1: seeds not set
  bool sources_set = false;
  // seeds: unique (vertex, column) keys and per-vertex lists
  egr::SeedPrep sp;
  uint32_t *seed_ptr = nullptr, *seed_tiles = nullptr;
  // top-k: full-scan partials, and the candidate lists of the final reach
  float* part_s = nullptr;
  uint32_t* part_v = nullptr;
  uint32_t NG = 0;                  // 64-vertex groups
  uint32_t* cand_cnt = nullptr;     // [B*NG + 1] per (column, group) counts
  uint32_t* cand_off = nullptr;     // exclusive scan of cand_cnt
  uint32_t* cand_list = nullptr;    // all columns' candidates, column-contiguous
  bool cand_enabled = false;
  bool cand_valid = false;
  int cand_exclude = -1;
  uint32_t owned = 0;               // rows [0, owned) are top-k candidates (partition: no halo)
  unsigned long long* counter = nullptr;
  // sparse halo exchange scratch: per-row non-zero counts / offsets, scan temp, peer totals
  int64_t* sx_off = nullptr;
  size_t sx_cap = 0;
  void* sx_tmp = nullptr;
  size_t sx_tmp_bytes = 0;
  // the fixed-capacity pack's row offsets and scan scratch, one set per kind (scores, reach):
  // the two kinds' exchanges may run at once on two streams
  int64_t* sxc_off[2] = {nullptr, nullptr};
  size_t sxc_cap[2] = {0, 0};
  void* sxc_tmp[2] = {nullptr, nullptr};
  size_t sxc_tmp_bytes[2] = {0, 0};
  int64_t* sx_tot = nullptr;        // [EGR_SX_MAX_PEERS + 1] peer bounds, then the segments
  int64_t* sx_pin = nullptr;        // pinned host: the segments up, the peer bounds down
  uint32_t* sx_mask = nullptr;      // [rows][MW] non-zero 32-column groups of each send row
  size_t sx_mask_cap = 0;
};

namespace {

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

// Row chunks of at most max_rows rows whose CSR segment fits CSR_CAP entries; a row longer
// than CSR_CAP forms a chunk of its own (its excess is read by the kernel's tail loop).
std::vector<uint32_t> build_chunks(const std::vector<uint32_t>& rp, uint32_t V, uint32_t max_rows) {
  std::vector<uint32_t> cs{0};
  uint32_t v = 0;
  while (v < V) {
    const uint32_t start = v;
    uint32_t ents = 0;
    while (v < V && v - start < max_rows) {
      const uint32_t d = rp[v + 1] - rp[v];
      if (v > start && ents + d > CSR_CAP) break;
      ents += d;
      ++v;
    }
    cs.push_back(v);
  }
  return cs;
}

// The chunks of one row longer than CSR_CAP (hop_kernel's LONG launch) -> p->long_chunk / nlong
int set_long_chunks(egr_plan* p, const std::vector<uint32_t>& cs) {
  std::vector<uint32_t> lc;
  const std::vector<uint32_t>& rp = p->s->row_ptr_host;
  for (size_t c = 0; c + 1 < cs.size(); ++c)
    if (rp[cs[c + 1]] - rp[cs[c]] > CSR_CAP) lc.push_back((uint32_t)c);
  if (lc.size() > p->nlong || !p->long_chunk) {
    dfree(p->long_chunk);
    p->long_chunk = nullptr;
    const int rc = dalloc(&p->long_chunk, std::max<size_t>(lc.size(), 1));
    if (rc != EGR_OK) return rc;
  }
  if (!lc.empty() &&
      hipMemcpy(p->long_chunk, lc.data(), lc.size() * 4, hipMemcpyHostToDevice) != hipSuccess)
    return egr::fail(EGR_EDEVICE, "long chunk table upload failed");
  p->nlong = (uint32_t)lc.size();
  return EGR_OK;
}

template <int G>
void launch_hop_g(const HopArgs& a, dim3 grid, hipStream_t st, bool seeds, bool skip, uint32_t ntiles) {
  if (seeds && skip) hipLaunchKernelGGL((hop_kernel<G, true, true>), grid, dim3(256), 0, st, a);
  else if (seeds) hipLaunchKernelGGL((hop_kernel<G, true>), grid, dim3(256), 0, st, a);
  else if (skip) hipLaunchKernelGGL((hop_kernel<G, false, true>), grid, dim3(256), 0, st, a);
  else hipLaunchKernelGGL((hop_kernel<G, false>), grid, dim3(256), 0, st, a);
  if (skip && a.nlong > 0) {                    // the lone long rows' chunks (see hop_kernel)
    const dim3 lg(a.nlong * ntiles);
    if (seeds) hipLaunchKernelGGL((hop_kernel<G, true, true, true>), lg, dim3(256), 0, st, a);
    else hipLaunchKernelGGL((hop_kernel<G, false, true, true>), lg, dim3(256), 0, st, a);
  }
}

template <int RG>
void launch_reach_g(const egr_plan* p, hipStream_t st) {
  hipLaunchKernelGGL((reach_kernel<RG>), dim3(p->rnchunks), dim3(256), 0, st, p->s->row_ptr,
                     p->s->col, p->rchunk_start, reinterpret_cast<const uint4*>(p->reach[p->rcur]),
                     reinterpret_cast<uint4*>(p->reach[1 - p->rcur]));
}

uint32_t reach_rows(int RG) { return RG == 1 ? ReachGeo<1>::ROWS : ReachGeo<2>::ROWS; }

// the current scores' tile flags for a reader, when the last hop skipped zero-tile stores
const uint8_t* x_flags(const egr_plan* p) { return p->xsparse[p->xcur] ? p->nzf[p->xcur] : nullptr; }

// One propagation hop (+ its own-row seed add).
int plan_hop(egr_plan* p, void* stream) {
  if (!p) return egr::fail(EGR_EINVAL, "egr_plan_hop: NULL plan");
  if (p->hops_done < 0) return egr::fail(EGR_ESTATE, "egr_plan_hop: seeds not set");
  DeviceGuard guard(p->s->device);
  hipStream_t st = (hipStream_t)stream;
  const egr_snapshot* s = p->s;
  const bool seeds = p->hops_done == 0;
  HopArgs a;
  a.row_ptr = s->row_ptr;
  a.col = s->col;
  a.val = s->val;
  a.chunk_start = p->chunk_start;
  a.seed_ptr = p->seed_ptr;
  a.seed_col = p->sp.uminor;
  a.seed_val = p->sp.uval;
  a.seed_tiles = p->seed_tiles;
  a.xin = seeds ? nullptr : p->x[p->xcur];
  a.xout = p->x[seeds ? 0 : 1 - p->xcur];
  a.nzout = p->nzf[seeds ? 0 : 1 - p->xcur];
  // (the skip's buffer offsets are 32-bit: one tile of xin must span < 2 GB, V < 4.2M at TW 128)
  // (the first hop skips by the seed tile masks, the others by xin's tile flags)
  const bool skip = p->skip_zero && (uint64_t)s->V * p->TW * 4 < (1ull << 31);
  a.nzin = skip && !seeds ? p->nzf[p->xcur] : nullptr;
  a.xbytes = skip && !seeds ? (uint32_t)((uint64_t)s->V * p->TW * 4) : 0u;
  a.ntiles = (uint32_t)p->ntiles;
  a.V = (uint32_t)s->V;
  a.nchunks = p->nchunks;
  a.long_chunks = p->long_chunk;
  a.nlong = p->nlong;
  const dim3 grid(p->nchunks * p->ntiles);
  switch (p->TW) {
    case 128: launch_hop_g<32>(a, grid, st, seeds, skip, a.ntiles); break;
    case 64: launch_hop_g<16>(a, grid, st, seeds, skip, a.ntiles); break;
    case 16: launch_hop_g<4>(a, grid, st, seeds, skip, a.ntiles); break;
    default: launch_hop_g<1>(a, grid, st, seeds, skip, a.ntiles); break;
  }
  EGR_CHECK_LAUNCH();
  hipLaunchKernelGGL(seed_add_kernel, dim3((unsigned)((std::max<int64_t>(p->max_seeds, 1) + 255) / 256)),
                     dim3(256), 0, st, p->sp.ukeys, p->sp.uval, p->sp.n_unique, (uint32_t)p->Bpad,
                     (uint32_t)p->TW, (uint32_t)s->V, a.xout, a.nzout, a.ntiles);
  EGR_CHECK_LAUNCH();
  p->xcur = seeds ? 0 : 1 - p->xcur;
  p->xsparse[p->xcur] = skip;
  ++p->hops_done;
  p->cand_valid = false;
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
      (rc = dalloc(&s->cv, 2 * E + 2)) || (rc = dalloc(&s->vlabel, V))) {
    egr_snapshot_free(s);
    return rc;
  }
  hipError_t e = hipMemcpy(s->row_ptr, row_ptr.data(), (V + 1) * 4, hipMemcpyHostToDevice);
  if (e == hipSuccess && E) e = hipMemcpy(s->col, col.data(), 2 * E * 4, hipMemcpyHostToDevice);
  if (e == hipSuccess && E) e = hipMemcpy(s->meta, meta.data(), 2 * E, hipMemcpyHostToDevice);
  if (e == hipSuccess && E) e = hipMemcpy(s->val, val.data(), 2 * E * 4, hipMemcpyHostToDevice);
  if (e == hipSuccess && E) {
    std::vector<uint2> cv(2 * E);
    for (int64_t i = 0; i < 2 * E; ++i) {
      uint32_t vb;
      std::memcpy(&vb, &val[i], 4);
      cv[i] = make_uint2(col[i], vb);
    }
    e = hipMemcpy(s->cv, cv.data(), 2 * E * 8, hipMemcpyHostToDevice);
  }
  if (e == hipSuccess) e = hipMemcpy(s->vlabel, vlabel.data(), V, hipMemcpyHostToDevice);
  if (e != hipSuccess) {
    egr_snapshot_free(s);
    return egr::fail(EGR_EDEVICE, std::string("snapshot upload: ") + hipGetErrorString(e));
  }
  s->cap_v = V;
  s->cap_e = 2 * E;
  if ((rc = layout_build(s, row_ptr.data(), col.data())) != EGR_OK) {
    egr_snapshot_free(s);
    return rc;
  }
  s->row_ptr_host = std::move(row_ptr);
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
  dfree(s->cv);
  dfree(s->vlabel);
  snapshot_update_free(s);
  layout_free(s);
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
  if (!s || !out || n_cols <= 0 || n_cols > EGR_MAX_COLS || max_seeds < 0 || k < 1 || k > KMAX)
    return egr::fail(EGR_EINVAL,
                     "egr_plan_create: bad arguments (need 0 < n_cols <= 8192, 1 <= k <= 16)");
  *out = nullptr;
  DeviceGuard guard(s->device);
  auto* p = new egr_plan();
  p->s = s;
  p->version = s->version;
  p->B = n_cols;
  p->TW = choose_tile_width(n_cols);
  p->Bpad = (n_cols + p->TW - 1) / p->TW * p->TW;
  p->ntiles = p->Bpad / p->TW;
  p->W = (n_cols + 63) / 64;
  p->owned = (uint32_t)s->V;
  p->RG = 1;
  while (2 * p->RG < p->W) p->RG *= 2;
  p->RS = 2 * p->RG;
  p->k = k;
  p->max_seeds = max_seeds;
  const uint32_t V = (uint32_t)s->V;
  const std::vector<uint32_t> chunks = build_chunks(s->row_ptr_host, V, hop_rows(p->TW));
  p->nchunks = (uint32_t)chunks.size() - 1;
  const std::vector<uint32_t> rchunks = build_chunks(s->row_ptr_host, V, reach_rows(p->RG));
  p->rnchunks = (uint32_t)rchunks.size() - 1;
  p->NG = (V + 63) / 64;
  // candidate lists: worst case every vertex for every column (4 B each)
  p->cand_enabled = (uint64_t)V * p->B <= (1ull << 32) - 1 &&
                    (uint64_t)V * p->B * 4 <= (16ull << 30);
  const size_t ncnt = p->cand_enabled ? (size_t)p->B * p->NG + 1 : 1;
  p->n_chunks = (int)((V + TOPK_CHUNK - 1) / TOPK_CHUNK);
  int rc = EGR_OK;
  const size_t xs = (size_t)V * p->Bpad;
  const size_t parts = (size_t)p->ntiles * (p->TW > 64 ? p->TW / 64 : 1) * p->n_chunks * 64 * KMAX;
  if ((rc = dalloc(&p->x[0], xs)) || (rc = dalloc(&p->x[1], xs)) ||
      (rc = dalloc(&p->reach[0], (size_t)p->RS * V)) || (rc = dalloc(&p->reach[1], (size_t)p->RS * V)) ||
      (rc = p->sp.alloc(max_seeds, (uint64_t)V * p->Bpad, ncnt)) ||
      (rc = dalloc(&p->seed_ptr, (size_t)V + 1)) ||
      (rc = dalloc(&p->seed_tiles, (size_t)V)) ||
      (rc = dalloc(&p->part_s, parts)) || (rc = dalloc(&p->part_v, parts)) ||
      (rc = dalloc(&p->cand_cnt, ncnt)) || (rc = dalloc(&p->cand_off, ncnt)) ||
      (rc = dalloc(&p->cand_list, p->cand_enabled ? (size_t)V * p->B : 1)) ||
      (rc = dalloc(&p->counter, 1)) || (rc = dalloc(&p->chunk_start, chunks.size())) ||
      (rc = dalloc(&p->rchunk_start, rchunks.size())) ||
      (rc = dalloc(&p->nzf[0], (size_t)V * p->ntiles)) || (rc = dalloc(&p->nzf[1], (size_t)V * p->ntiles))) {
    egr_plan_free(p);
    return rc;
  }
  p->skip_zero = getenv("EGRAPH_HOP_NO_SKIP") == nullptr;
  // every hop writes its rows' tile flags (a hop reads only flags its predecessor wrote); zero
  // them once so that no stale byte is ever read
  if (hipMemset(p->nzf[0], 0, (size_t)V * p->ntiles) != hipSuccess ||
      hipMemset(p->nzf[1], 0, (size_t)V * p->ntiles) != hipSuccess) {
    egr_plan_free(p);
    return egr::fail(EGR_EDEVICE, "plan flag init failed");
  }
  // the count pass never writes cand_cnt[B*NG], so the scan's last slot is the grand total
  if (hipMemcpy(p->chunk_start, chunks.data(), chunks.size() * 4, hipMemcpyHostToDevice) != hipSuccess ||
      hipMemcpy(p->rchunk_start, rchunks.data(), rchunks.size() * 4, hipMemcpyHostToDevice) != hipSuccess ||
      hipMemset(p->cand_cnt, 0, ncnt * 4) != hipSuccess) {
    egr_plan_free(p);
    return egr::fail(EGR_EDEVICE, "plan table upload failed");
  }
  if ((rc = set_long_chunks(p, chunks)) != EGR_OK) {
    egr_plan_free(p);
    return rc;
  }
  *out = p;
  return EGR_OK;
}

void egr_plan_free(egr_plan* p) {
  if (!p) return;
  DeviceGuard guard(p->s->device);
  for (auto* q : {&p->x[0], &p->x[1]}) dfree(*q);
  dfree(p->nzf[0]);
  dfree(p->nzf[1]);
  dfree(p->reach[0]);
  dfree(p->reach[1]);
  p->sp.free_all();
  dfree(p->seed_ptr);
  dfree(p->seed_tiles);
  dfree(p->part_s);
  dfree(p->part_v);
  dfree(p->cand_cnt);
  dfree(p->cand_off);
  dfree(p->cand_list);
  dfree(p->counter);
  dfree(p->chunk_start);
  dfree(p->long_chunk);
  dfree(p->rchunk_start);
  dfree(p->sx_off);
  for (int k = 0; k < 2; ++k) {
    dfree(p->sxc_off[k]);
    if (p->sxc_tmp[k]) (void)hipFree(p->sxc_tmp[k]);
  }
  dfree(p->sx_tot);
  if (p->sx_pin) (void)hipHostFree(p->sx_pin);
  dfree(p->sx_mask);
  if (p->sx_tmp) (void)hipFree(p->sx_tmp);
  delete p;
}

int egr_plan_tile_width(const egr_plan* p) { return p ? p->TW : -1; }

int egr_plan_shape(const egr_plan* p, int64_t* n_vertices, int32_t* n_cols) {
  if (!p) return egr::fail(EGR_EINVAL, "egr_plan_shape: NULL plan");
  if (n_vertices) *n_vertices = p->s->V;
  if (n_cols) *n_cols = p->B;
  return EGR_OK;
}


static int plan_stale(const egr_plan* p, const char* what) {
  return egr::fail(EGR_ESTATE, std::string(what) +
                   ": the snapshot was updated after this plan was created; create a new plan");
}

int egr_plan_set_seeds(egr_plan* p, const uint32_t* seed_vertex, const uint32_t* seed_col,
                       const float* seed_val, int64_t n_seeds, void* stream) {
  if (!p || n_seeds < 0 || n_seeds > p->max_seeds || (n_seeds > 0 && (!seed_vertex || !seed_col || !seed_val)))
    return egr::fail(EGR_EINVAL, "egr_plan_set_seeds: bad arguments (n_seeds above plan capacity?)");
  if (p->version != p->s->version) return plan_stale(p, "egr_plan_set_seeds");
  DeviceGuard guard(p->s->device);
  hipStream_t st = (hipStream_t)stream;
  const uint32_t V = (uint32_t)p->s->V;
  p->hops_done = 0;
  p->xcur = 0;
  p->cand_valid = false;
  EGR_HIP(hipMemsetAsync(p->seed_tiles, 0, (size_t)V * 4, st));
  EGR_TRY(p->sp.run(seed_vertex, seed_col, seed_val, n_seeds, V, p->B, false,
                    (uint64_t)p->Bpad, V, p->seed_ptr, st));
  if (n_seeds == 0) return EGR_OK;
  const dim3 g1((unsigned)((n_seeds + 255) / 256));
  hipLaunchKernelGGL(seed_tiles_kernel, g1, dim3(256), 0, st, p->sp.ukeys, p->sp.n_unique,
                     (uint32_t)p->Bpad, (uint32_t)p->TW, p->seed_tiles);
  EGR_CHECK_LAUNCH();
  return EGR_OK;
}

int egr_plan_set_sources(egr_plan* p, const uint32_t* source_vertex, void* stream) {
  if (!p || !source_vertex) return egr::fail(EGR_EINVAL, "egr_plan_set_sources: NULL argument");
  if (p->version != p->s->version) return plan_stale(p, "egr_plan_set_sources");
  DeviceGuard guard(p->s->device);
  hipStream_t st = (hipStream_t)stream;
  const uint32_t V = (uint32_t)p->s->V;
  p->rcur = 0;
  p->cand_valid = false;
  EGR_HIP(hipMemsetAsync(p->reach[0], 0, (size_t)p->RS * V * 8, st));
  hipLaunchKernelGGL(reach_sources_kernel, dim3((p->B + 255) / 256), dim3(256), 0, st,
                     source_vertex, p->B, p->reach[0], V, (uint32_t)p->RS);
  EGR_CHECK_LAUNCH();
  p->sources_set = true;
  p->reach_hops = 0;
  return EGR_OK;
}

int egr_plan_hop(egr_plan* p, void* stream) {
  if (p && p->version != p->s->version) return plan_stale(p, "egr_plan_hop");
  return plan_hop(p, stream);
}

int egr_plan_reach_hop(egr_plan* p, void* stream) {
  if (!p) return egr::fail(EGR_EINVAL, "egr_plan_reach_hop: NULL plan");
  if (!p->sources_set) return egr::fail(EGR_ESTATE, "egr_plan_reach_hop: sources not set");
  if (p->version != p->s->version) return plan_stale(p, "egr_plan_reach_hop");
  DeviceGuard guard(p->s->device);
  hipStream_t st = (hipStream_t)stream;
  switch (p->RG) {
    case 1: launch_reach_g<1>(p, st); break;
    case 2: launch_reach_g<2>(p, st); break;
    case 4: launch_reach_g<4>(p, st); break;
    case 8: launch_reach_g<8>(p, st); break;
    case 16: launch_reach_g<16>(p, st); break;
    case 32: launch_reach_g<32>(p, st); break;
    default: launch_reach_g<64>(p, st); break;
  }
  EGR_CHECK_LAUNCH();
  p->rcur = 1 - p->rcur;
  ++p->reach_hops;
  p->cand_valid = false;
  return EGR_OK;
}

int egr_plan_step(egr_plan* p, void* stream) {
  if (!p) return egr::fail(EGR_EINVAL, "egr_plan_step: NULL plan");
  if (!p->sources_set) return egr::fail(EGR_ESTATE, "egr_plan_step: sources not set");
  EGR_TRY(plan_hop(p, stream));
  return egr_plan_reach_hop(p, stream);
}

int egr_plan_final_step(egr_plan* p, int32_t exclude_label, void* stream) {
  if (!p) return egr::fail(EGR_EINVAL, "egr_plan_final_step: NULL plan");
  if (!p->sources_set) return egr::fail(EGR_ESTATE, "egr_plan_final_step: sources not set");
  EGR_TRY(egr_plan_step(p, stream));
  return egr_plan_candidates(p, exclude_label, stream);
}

int egr_plan_candidates(egr_plan* p, int32_t exclude_label, void* stream) {
  if (!p) return egr::fail(EGR_EINVAL, "egr_plan_candidates: NULL plan");
  if (!p->sources_set) return egr::fail(EGR_ESTATE, "egr_plan_candidates: sources not set");
  if (!p->cand_enabled) return EGR_OK;   // no candidate lists: top-k scans the scores
  DeviceGuard guard(p->s->device);
  hipStream_t st = (hipStream_t)stream;
  const uint32_t V = (uint32_t)p->s->V;
  const dim3 grid((p->NG + 3) / 4);
  const uint64_t* R = p->reach[p->rcur];
  (void)V;
  hipLaunchKernelGGL(cand_count_kernel, grid, dim3(256), 0, st, R, (uint32_t)p->RS,
                     p->s->vlabel, exclude_label, p->owned, p->B, p->NG, p->cand_cnt);
  EGR_CHECK_LAUNCH();
  size_t tb = p->sp.tmp_bytes;
  EGR_HIP(hipcub::DeviceScan::ExclusiveSum(p->sp.tmp, tb, p->cand_cnt, p->cand_off,
                                           (int)((size_t)p->B * p->NG + 1), st));
  hipLaunchKernelGGL(cand_fill_kernel, grid, dim3(256), 0, st, R, (uint32_t)p->RS, p->s->vlabel,
                     exclude_label, p->owned, p->B, p->NG, p->cand_off, p->cand_list);
  EGR_CHECK_LAUNCH();
  p->cand_valid = true;
  p->cand_exclude = exclude_label;
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
  if (p->cand_valid && p->cand_exclude == exclude_label) {
    hipLaunchKernelGGL(topk_cand_kernel, dim3((p->B + 3) / 4), dim3(256), 0, st, p->x[p->xcur],
                       p->cand_off, p->NG, p->cand_list, V, p->TW, p->B, p->k, out_ids, out_scores,
                       x_flags(p), (uint32_t)p->ntiles);
    EGR_CHECK_LAUNCH();
    return EGR_OK;
  }
  const int waves = p->ntiles * (p->TW > 64 ? p->TW / 64 : 1) * p->n_chunks;
  hipLaunchKernelGGL(topk_partial_kernel, dim3((waves + 3) / 4), dim3(256), 0, st,
                     p->x[p->xcur], p->reach[p->rcur], (uint32_t)p->RS, p->s->vlabel, exclude_label, V,
                     p->owned, p->TW,
                     p->B, p->n_chunks, p->part_s, p->part_v, x_flags(p), (uint32_t)p->ntiles);
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
                     (hipStream_t)stream, p->x[p->xcur], (uint32_t)p->s->V, p->TW, p->B, out,
                     x_flags(p), (uint32_t)p->ntiles);
  EGR_CHECK_LAUNCH();
  return EGR_OK;
}

int egr_plan_read_reach(const egr_plan* p, uint64_t* out, void* stream) {
  if (!p || !out) return egr::fail(EGR_EINVAL, "egr_plan_read_reach: NULL argument");
  if (!p->sources_set) return egr::fail(EGR_ESTATE, "egr_plan_read_reach: sources not set");
  DeviceGuard guard(p->s->device);
  const size_t n = (size_t)p->W * p->s->V;
  hipLaunchKernelGGL(reach_export_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, p->reach[p->rcur], (uint32_t)p->RS, (uint32_t)p->s->V,
                     p->W, out);
  EGR_CHECK_LAUNCH();
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
                     p->s->col, p->s->meta, p->reach[p->rcur] + (col >> 6), (uint32_t)p->RS,
                     1ull << (col & 63), V, out_src, out_dst, out_type, cap, p->counter);
  EGR_CHECK_LAUNCH();
  unsigned long long n = 0;
  EGR_HIP(hipMemcpyAsync(&n, p->counter, sizeof(n), hipMemcpyDeviceToHost, st));
  EGR_HIP(hipStreamSynchronize(st));
  *out_n = (int64_t)n;
  return EGR_OK;
}

int egr_snapshot_from_csr(const uint32_t* row_ptr, const uint32_t* col, const uint8_t* meta,
                          const float* val, const uint8_t* vlabel, int64_t n_vertices,
                          int32_t device, egr_snapshot** out) {
  if (!row_ptr || !out || n_vertices <= 0 || n_vertices >= (int64_t)EGR_NO_NODE || !vlabel)
    return egr::fail(EGR_EINVAL, "egr_snapshot_from_csr: bad arguments");
  *out = nullptr;
  const int64_t V = n_vertices, NE = row_ptr[V];
  if (row_ptr[0] != 0 || (NE > 0 && (!col || !meta || !val)))
    return egr::fail(EGR_EINVAL, "egr_snapshot_from_csr: row_ptr must start at 0");
  for (int64_t v = 0; v < V; ++v)
    if (row_ptr[v + 1] < row_ptr[v])
      return egr::fail(EGR_EINVAL, "egr_snapshot_from_csr: row_ptr not monotone");
  for (int64_t e = 0; e < NE; ++e)
    if (col[e] >= (uint64_t)V) return egr::fail(EGR_EINVAL, "egr_snapshot_from_csr: col out of range");
  int ndev = 0;
  EGR_HIP(hipGetDeviceCount(&ndev));
  if (device < 0 || device >= ndev) return egr::fail(EGR_EINVAL, "egr_snapshot_from_csr: bad device");
  DeviceGuard guard(device);
  auto* s = new egr_snapshot();
  s->device = device;
  s->V = V;
  s->NE = NE;
  int rc = EGR_OK;
  if ((rc = dalloc(&s->row_ptr, V + 1)) || (rc = dalloc(&s->col, NE)) || (rc = dalloc(&s->meta, NE)) ||
      (rc = dalloc(&s->val, NE)) || (rc = dalloc(&s->cv, NE + 2)) || (rc = dalloc(&s->vlabel, V))) {
    egr_snapshot_free(s);
    return rc;
  }
  hipError_t e = hipMemcpy(s->row_ptr, row_ptr, (V + 1) * 4, hipMemcpyHostToDevice);
  if (e == hipSuccess && NE) e = hipMemcpy(s->col, col, NE * 4, hipMemcpyHostToDevice);
  if (e == hipSuccess && NE) e = hipMemcpy(s->meta, meta, NE, hipMemcpyHostToDevice);
  if (e == hipSuccess && NE) e = hipMemcpy(s->val, val, NE * 4, hipMemcpyHostToDevice);
  if (e == hipSuccess && NE) {
    std::vector<uint2> cv(NE);
    for (int64_t i = 0; i < NE; ++i) {
      uint32_t vb;
      std::memcpy(&vb, &val[i], 4);
      cv[i] = make_uint2(col[i], vb);
    }
    e = hipMemcpy(s->cv, cv.data(), NE * 8, hipMemcpyHostToDevice);
  }
  if (e == hipSuccess) e = hipMemcpy(s->vlabel, vlabel, V, hipMemcpyHostToDevice);
  if (e != hipSuccess) {
    egr_snapshot_free(s);
    return egr::fail(EGR_EDEVICE, std::string("snapshot upload: ") + hipGetErrorString(e));
  }
  s->row_ptr_host.assign(row_ptr, row_ptr + V + 1);
  s->cap_v = V;
  s->cap_e = NE;
  if ((rc = layout_build(s, row_ptr, col)) != EGR_OK) {
    egr_snapshot_free(s);
    return rc;
  }
  *out = s;
  return EGR_OK;
}

int egr_plan_set_owned(egr_plan* p, int64_t n_owned) {
  if (!p || n_owned <= 0 || n_owned > p->s->V)
    return egr::fail(EGR_EINVAL, "egr_plan_set_owned: need 0 < n_owned <= n_vertices");
  // a partition's halo rows (vertices past n_owned) have no row data here: their values arrive
  // through the halo exchange, so the hop and reach sweeps run over the owned rows only
  // (fewer chunks than the plan's tables hold: they fit the allocations)
  DeviceGuard guard(p->s->device);
  const std::vector<uint32_t> chunks = build_chunks(p->s->row_ptr_host, (uint32_t)n_owned, hop_rows(p->TW));
  const std::vector<uint32_t> rchunks = build_chunks(p->s->row_ptr_host, (uint32_t)n_owned, reach_rows(p->RG));
  if (hipMemcpy(p->chunk_start, chunks.data(), chunks.size() * 4, hipMemcpyHostToDevice) != hipSuccess ||
      hipMemcpy(p->rchunk_start, rchunks.data(), rchunks.size() * 4, hipMemcpyHostToDevice) != hipSuccess)
    return egr::fail(EGR_EDEVICE, "egr_plan_set_owned: chunk table upload failed");
  p->nchunks = (uint32_t)chunks.size() - 1;
  p->rnchunks = (uint32_t)rchunks.size() - 1;
  EGR_TRY(set_long_chunks(p, chunks));
  for (int b = 0; b < 2; ++b) {
    const size_t nb = (size_t)p->s->V * p->ntiles;
    if (!p->nzf[b]) {
      const int rc = dalloc(&p->nzf[b], nb);
      if (rc != EGR_OK) return rc;
    }
    if (hipMemset(p->nzf[b], 0, nb) != hipSuccess)
      return egr::fail(EGR_EDEVICE, "egr_plan_set_owned: flag init failed");
    p->xzeroed[b] = false;
  }
  p->owned = (uint32_t)n_owned;
  p->cand_valid = false;
  return EGR_OK;
}

int egr_plan_pack_scores(const egr_plan* p, const uint32_t* rows, int64_t n, float* out, void* stream) {
  if (!p || n < 0 || (n > 0 && (!rows || !out))) return egr::fail(EGR_EINVAL, "egr_plan_pack_scores: bad arguments");
  if (p->hops_done < 0) return egr::fail(EGR_ESTATE, "egr_plan_pack_scores: seeds not set");
  if (n == 0) return EGR_OK;
  DeviceGuard guard(p->s->device);
  const float* X = p->hops_done == 0 ? nullptr : p->x[p->xcur];
  if (!X) return egr::fail(EGR_ESTATE, "egr_plan_pack_scores: run a hop first");
  hipLaunchKernelGGL(pack_scores_kernel, dim3((unsigned)n), dim3(256), 0, (hipStream_t)stream, X,
                     (uint32_t)p->s->V, p->TW, p->Bpad, rows, out, x_flags(p), (uint32_t)p->ntiles);
  EGR_CHECK_LAUNCH();
  return EGR_OK;
}

int egr_plan_unpack_scores(egr_plan* p, const uint32_t* rows, const uint32_t* src, int64_t n,
                           const float* in, void* stream) {
  if (!p || n < 0 || (n > 0 && (!rows || !src || !in)))
    return egr::fail(EGR_EINVAL, "egr_plan_unpack_scores: bad arguments");
  if (p->hops_done < 1) return egr::fail(EGR_ESTATE, "egr_plan_unpack_scores: run a hop first");
  if (n == 0) return EGR_OK;
  p->xzeroed[p->xcur] = false;              // full halo rows written: no tile tracking
  DeviceGuard guard(p->s->device);
  hipLaunchKernelGGL(unpack_scores_kernel, dim3((unsigned)n), dim3(256), 0, (hipStream_t)stream,
                     p->x[p->xcur], (uint32_t)p->s->V, p->TW, p->Bpad, rows, src, in, p->nzf[p->xcur]);
  EGR_CHECK_LAUNCH();
  p->cand_valid = false;
  return EGR_OK;
}

int egr_plan_pack_reach(const egr_plan* p, const uint32_t* rows, int64_t n, uint64_t* out, void* stream) {
  if (!p || n < 0 || (n > 0 && (!rows || !out))) return egr::fail(EGR_EINVAL, "egr_plan_pack_reach: bad arguments");
  if (!p->sources_set) return egr::fail(EGR_ESTATE, "egr_plan_pack_reach: sources not set");
  if (n == 0) return EGR_OK;
  DeviceGuard guard(p->s->device);
  hipLaunchKernelGGL(pack_reach_kernel, dim3((unsigned)n), dim3(64), 0, (hipStream_t)stream,
                     p->reach[p->rcur], (uint32_t)p->RS, p->W, rows, out);
  EGR_CHECK_LAUNCH();
  return EGR_OK;
}

int egr_plan_unpack_reach(egr_plan* p, const uint32_t* rows, const uint32_t* src, int64_t n,
                          const uint64_t* in, void* stream) {
  if (!p || n < 0 || (n > 0 && (!rows || !src || !in)))
    return egr::fail(EGR_EINVAL, "egr_plan_unpack_reach: bad arguments");
  if (!p->sources_set) return egr::fail(EGR_ESTATE, "egr_plan_unpack_reach: sources not set");
  if (n == 0) return EGR_OK;
  DeviceGuard guard(p->s->device);
  hipLaunchKernelGGL(unpack_reach_kernel, dim3((unsigned)n), dim3(64), 0, (hipStream_t)stream,
                     p->reach[p->rcur], (uint32_t)p->RS, p->W, rows, src, in);
  EGR_CHECK_LAUNCH();
  p->cand_valid = false;
  return EGR_OK;
}

int egr_plan_pack_sparse(egr_plan* p, int32_t what, const uint32_t* rows, int64_t n,
                         const int64_t* seg, int32_t P, int64_t* out, int64_t cap,
                         int64_t* counts, void* stream) {
  if (!p || (what != 0 && what != 1) || n < 0 || P < 1 || P > EGR_SX_MAX_PEERS || !seg ||
      !counts || (n > 0 && (!rows || !out)) || cap < 0 || seg[0] != 0 || seg[P] != n)
    return egr::fail(EGR_EINVAL, "egr_plan_pack_sparse: bad arguments");
  for (int q = 0; q < P; ++q)
    if (seg[q + 1] < seg[q]) return egr::fail(EGR_EINVAL, "egr_plan_pack_sparse: bad segments");
  const bool reach = what == 1;
  if (reach ? !p->sources_set : p->hops_done < 1)
    return egr::fail(EGR_ESTATE, "egr_plan_pack_sparse: nothing computed yet");
  for (int q = 0; q < P; ++q) counts[q] = 0;
  if (n == 0) return EGR_OK;
  DeviceGuard guard(p->s->device);
  hipStream_t st = (hipStream_t)stream;
  const int width = reach ? p->W : p->Bpad;
  // a score entry packs (row-in-segment * width + column) into the high 32 bits: refuse a
  // segment whose index range would wrap (the reach format keeps two words and has no limit)
  if (!reach)
    for (int q = 0; q < P; ++q)
      if ((uint64_t)(seg[q + 1] - seg[q]) * (uint64_t)width >= (1ull << 32))
        return egr::fail(EGR_EINVAL, "egr_plan_pack_sparse: a peer segment of " +
                         std::to_string(seg[q + 1] - seg[q]) + " rows x " + std::to_string(width) +
                         " columns exceeds the 2^32 entry index of the score format");
  if ((size_t)n + 1 > p->sx_cap) {
    dfree(p->sx_off);
    p->sx_cap = 0;
    int rc = dalloc(&p->sx_off, (size_t)n + 1);
    if (rc != EGR_OK) return rc;
    p->sx_cap = (size_t)n + 1;
    if (p->sx_tmp) (void)hipFree(p->sx_tmp);
    p->sx_tmp = nullptr;
    size_t tb = 0;
    EGR_HIP(hipcub::DeviceScan::ExclusiveSum(nullptr, tb, p->sx_off, p->sx_off, (int)(n + 1), st));
    EGR_HIP(hipMalloc(&p->sx_tmp, tb));
    p->sx_tmp_bytes = tb;
  }
  if (!p->sx_tot) {
    const int rc = dalloc(&p->sx_tot, (size_t)EGR_SX_MAX_PEERS + 1 + EGR_SX_MAX_PEERS + 1);
    if (rc != EGR_OK) return rc;
  }
  if (!p->sx_pin)
    EGR_HIP(hipHostMalloc(reinterpret_cast<void**>(&p->sx_pin),
                          sizeof(int64_t) * 2 * ((size_t)EGR_SX_MAX_PEERS + 1), hipHostMallocDefault));
  int64_t* dseg = p->sx_tot + EGR_SX_MAX_PEERS + 1;
  int64_t* pseg = p->sx_pin;                                  // (free: the last call synchronised)
  int64_t* pbound = p->sx_pin + EGR_SX_MAX_PEERS + 1;
  for (int q = 0; q <= P; ++q) pseg[q] = seg[q];
  EGR_HIP(hipMemcpyAsync(dseg, pseg, sizeof(int64_t) * (P + 1), hipMemcpyHostToDevice, st));
  const float* X = reach ? nullptr : p->x[p->xcur];
  const uint64_t* R = reach ? p->reach[p->rcur] : nullptr;
  const uint32_t V = (uint32_t)p->s->V;
  const int MW = (((width + 31) / 32) + 31) / 32;            // mask words per row
  if ((size_t)n * MW > p->sx_mask_cap) {
    dfree(p->sx_mask);
    p->sx_mask_cap = 0;
    const int rc = dalloc(&p->sx_mask, (size_t)n * MW);
    if (rc != EGR_OK) return rc;
    p->sx_mask_cap = (size_t)n * MW;
  }
  EGR_HIP(hipMemsetAsync(p->sx_off + n, 0, sizeof(int64_t), st));
  const dim3 sxg = sx_grid(n);
  hipLaunchKernelGGL(sx_count_kernel, sxg, dim3(256), 0, st, X, R, V, p->TW,
                     (uint32_t)p->RS, width, reach, rows, (int64_t)n, p->sx_off, p->sx_mask, MW,
                     reach ? nullptr : p->nzf[p->xcur], (uint32_t)p->ntiles);
  EGR_CHECK_LAUNCH();
  size_t tb = p->sx_tmp_bytes;
  EGR_HIP(hipcub::DeviceScan::ExclusiveSum(p->sx_tmp, tb, p->sx_off, p->sx_off, (int)(n + 1), st));
  // the entry offsets at the peer boundaries (P + 1 values) decide the all-to-all split sizes:
  // gathered on the device and read back in ONE pinned copy (one small pageable copy per peer
  // cost a staged round trip each: 288 per C4 step at P = 8)
  hipLaunchKernelGGL(sx_bounds_kernel, dim3(1), dim3(EGR_SX_MAX_PEERS + 1), 0, st, p->sx_off, dseg, P,
                     p->sx_tot);
  EGR_CHECK_LAUNCH();
  EGR_HIP(hipMemcpyAsync(pbound, p->sx_tot, sizeof(int64_t) * (P + 1), hipMemcpyDeviceToHost, st));
  // the entries go out before the host reads the sizes (the emit needs only the device offsets):
  // the device works while the copy and the host's synchronisation round trip are in flight
  hipLaunchKernelGGL(sx_emit_kernel, sxg, dim3(256), 0, st, X, R, V, p->TW,
                     (uint32_t)p->RS, width, reach, rows, (int64_t)n, dseg, P, p->sx_off, p->sx_mask,
                     MW, out, cap, reach ? nullptr : p->nzf[p->xcur], (uint32_t)p->ntiles);
  EGR_CHECK_LAUNCH();
  EGR_HIP(hipStreamSynchronize(st));
  const int64_t* bound = pbound;
  const int64_t total = bound[P];
  const int64_t words = reach ? 2 * total : total;
  if (words > cap) return egr::fail(EGR_EINVAL, "egr_plan_pack_sparse: output too small (" +
                                                    std::to_string(words) + " words)");
  for (int q = 0; q < P; ++q) counts[q] = bound[q + 1] - bound[q];
  return EGR_OK;
}

int egr_plan_unpack_sparse(egr_plan* p, int32_t what, const uint32_t* recv_vertex, int64_t n_rows,
                           const int64_t* in, int64_t n_entries, const int64_t* eseg,
                           const int64_t* rbase, int32_t P, void* stream) {
  if (!p || (what != 0 && what != 1) || n_rows < 0 || n_entries < 0 || P < 1 ||
      (n_rows > 0 && !recv_vertex) || (n_entries > 0 && (!in || !eseg || !rbase)))
    return egr::fail(EGR_EINVAL, "egr_plan_unpack_sparse: bad arguments");
  const bool reach = what == 1;
  if (reach ? !p->sources_set : p->hops_done < 1)
    return egr::fail(EGR_ESTATE, "egr_plan_unpack_sparse: nothing computed yet");
  if (n_rows == 0) return EGR_OK;
  DeviceGuard guard(p->s->device);
  hipStream_t st = (hipStream_t)stream;
  const int width = reach ? p->W : p->Bpad;
  float* X = reach ? nullptr : p->x[p->xcur];
  uint64_t* R = reach ? p->reach[p->rcur] : nullptr;
  const uint32_t V = (uint32_t)p->s->V;
  uint8_t* nzf = reach ? nullptr : p->nzf[p->xcur];
  hipLaunchKernelGGL(sx_zero_kernel, sx_grid(n_rows), dim3(256), 0,
                     st, X, R, V, p->TW, (uint32_t)p->RS, width, reach, recv_vertex, (int64_t)n_rows,
                     nzf, (uint32_t)p->ntiles,
                     nzf != nullptr && p->xzeroed[p->xcur]);
  EGR_CHECK_LAUNCH();
  if (nzf) p->xzeroed[p->xcur] = true;      // its halo rows are now tracked by their tile flags
  if (n_entries > 0) {
    hipLaunchKernelGGL(sx_scatter_kernel, dim3((unsigned)((n_entries + 255) / 256)), dim3(256), 0,
                       st, X, R, V, p->TW, (uint32_t)p->RS, width, reach, recv_vertex, in,
                       n_entries, eseg, rbase, P, nzf, (uint32_t)p->ntiles);
    EGR_CHECK_LAUNCH();
  }
  p->cand_valid = false;
  return EGR_OK;
}

int egr_plan_pack_sparse_cap(egr_plan* p, int32_t what, const uint32_t* rows, int64_t n,
                             const int64_t* seg_dev, int32_t P, int64_t* out, int64_t peer_cap,
                             int64_t* counts_dev, uint32_t* overflow_dev, void* stream) {
  if (!p || (what != 0 && what != 1) || n < 0 || P < 1 || P > EGR_SX_MAX_PEERS || !seg_dev ||
      !overflow_dev || peer_cap < 1 || !out || (n > 0 && !rows))
    return egr::fail(EGR_EINVAL, "egr_plan_pack_sparse_cap: bad arguments");
  const bool reach = what == 1;
  if (reach ? !p->sources_set : p->hops_done < 1)
    return egr::fail(EGR_ESTATE, "egr_plan_pack_sparse_cap: nothing computed yet");
  DeviceGuard guard(p->s->device);
  hipStream_t st = (hipStream_t)stream;
  const int width = reach ? p->W : p->Bpad;
  if (!reach && (uint64_t)n * (uint64_t)width >= (1ull << 32))
    return egr::fail(EGR_EINVAL, "egr_plan_pack_sparse_cap: send rows x columns exceed the 2^32 "
                                 "entry index of the score format");
  if (width > SX_MAP_MAX)
    return egr::fail(EGR_EINVAL, "egr_plan_pack_sparse_cap: more than 4096 columns (the work map "
                                 "holds 64 chunks of 64): use egr_plan_pack_sparse");
  const int kk = reach ? 1 : 0;
  if ((size_t)n + 1 > p->sxc_cap[kk]) {
    dfree(p->sxc_off[kk]);
    p->sxc_cap[kk] = 0;
    int rc = dalloc(&p->sxc_off[kk], (size_t)n + 1);
    if (rc != EGR_OK) return rc;
    p->sxc_cap[kk] = (size_t)n + 1;
    if (p->sxc_tmp[kk]) (void)hipFree(p->sxc_tmp[kk]);
    p->sxc_tmp[kk] = nullptr;
    size_t tb = 0;
    EGR_HIP(hipcub::DeviceScan::ExclusiveSum(nullptr, tb, p->sxc_off[kk], p->sxc_off[kk], (int)(n + 1), st));
    EGR_HIP(hipMalloc(&p->sxc_tmp[kk], tb));
    p->sxc_tmp_bytes[kk] = tb;
  }
  int64_t* const off = p->sxc_off[kk];
  const float* X = reach ? nullptr : p->x[p->xcur];
  const uint64_t* R = reach ? p->reach[p->rcur] : nullptr;
  const uint32_t V = (uint32_t)p->s->V;
  const uint8_t* nzf = reach ? (const uint8_t*)nullptr : p->nzf[p->xcur];
  const dim3 grid = sx_lane_grid(n);
  hipLaunchKernelGGL(sx_count_rows_kernel, grid, dim3(256), 0, st, X, R, V, p->TW, (uint32_t)p->RS,
                     width, reach, rows, n, nzf, (uint32_t)p->ntiles, off);
  EGR_CHECK_LAUNCH();
  size_t tb = p->sxc_tmp_bytes[kk];
  EGR_HIP(hipcub::DeviceScan::ExclusiveSum(p->sxc_tmp[kk], tb, off, off, (int)(n + 1), st));
  hipLaunchKernelGGL(sx_emit_rows_kernel, grid, dim3(256), 0, st, X, R, V, p->TW, (uint32_t)p->RS,
                     width, reach, rows, n, seg_dev, P, nzf, (uint32_t)p->ntiles,
                     (const int64_t*)off, out, peer_cap, counts_dev, overflow_dev);
  EGR_CHECK_LAUNCH();
  return EGR_OK;
}

int egr_plan_unpack_sparse_cap(egr_plan* p, int32_t what, const uint32_t* recv_vertex, int64_t n_rows,
                               const int64_t* in, int64_t peer_cap, uint32_t* overflow_dev,
                               const int64_t* rbase, int32_t P, void* stream) {
  if (!p || (what != 0 && what != 1) || n_rows < 0 || P < 1 || peer_cap < 1 ||
      (n_rows > 0 && (!recv_vertex || !in || !rbase)))
    return egr::fail(EGR_EINVAL, "egr_plan_unpack_sparse_cap: bad arguments");
  const bool reach = what == 1;
  if (reach ? !p->sources_set : p->hops_done < 1)
    return egr::fail(EGR_ESTATE, "egr_plan_unpack_sparse_cap: nothing computed yet");
  if (n_rows == 0) return EGR_OK;
  DeviceGuard guard(p->s->device);
  hipStream_t st = (hipStream_t)stream;
  const int width = reach ? p->W : p->Bpad;
  if (width > SX_MAP_MAX)
    return egr::fail(EGR_EINVAL, "egr_plan_unpack_sparse_cap: more than 4096 columns: use "
                                 "egr_plan_unpack_sparse");
  float* X = reach ? nullptr : p->x[p->xcur];
  uint64_t* R = reach ? p->reach[p->rcur] : nullptr;
  const uint32_t V = (uint32_t)p->s->V;
  uint8_t* nzf = reach ? nullptr : p->nzf[p->xcur];
  hipLaunchKernelGGL(sx_zero_rows_kernel, sx_lane_grid(n_rows), dim3(256), 0,
                     st, X, R, V, p->TW, (uint32_t)p->RS, width, reach, recv_vertex, (int64_t)n_rows,
                     nzf, (uint32_t)p->ntiles, nzf != nullptr && p->xzeroed[p->xcur]);
  EGR_CHECK_LAUNCH();
  if (nzf) p->xzeroed[p->xcur] = true;
  const int64_t slots = (int64_t)P * peer_cap;
  hipLaunchKernelGGL(sx_scatter_kernel, dim3((unsigned)((slots + 255) / 256)), dim3(256), 0,
                     st, X, R, V, p->TW, (uint32_t)p->RS, width, reach, recv_vertex, in,
                     slots, (const int64_t*)nullptr, rbase, P, nzf, (uint32_t)p->ntiles, peer_cap,
                     overflow_dev);
  EGR_CHECK_LAUNCH();
  p->cand_valid = false;
  return EGR_OK;
}

}  // extern "C"
