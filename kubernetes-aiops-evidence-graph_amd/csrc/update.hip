// Incremental snapshot update on the device ("incremental CSR update" of
// the alert storm, BASELINE config C5) and the snapshot download (§8f rank 2).
//
// The snapshot is the symmetric typed CSR egr_graph_csr (graph_host.cpp) derives from the
// MERGEd edge list (reference src/database/neo4j.py:95-167): every edge (s, t, d) is an entry
// (d-row: key s<<9 | t<<1 | 0) and (s-row: key d<<9 | t<<1 | 1), rows sorted by key, and
// val = w[t][dir] / deg(col).  An update appends vertices and NEW edges (the host MERGE,
// egr_graph_merge_edges, dedups them) and produces exactly the CSR egr_graph_csr would build for
// the grown graph, without the host rebuild or re-upload:
//   1. delta entries (2 per edge) + per-row added counts            delta_kernel
//   2. sort the delta entries by (row, key)                         2 x hipcub radix sort
//   3. new row_ptr = scan(old degree + added), delta row offsets    hipcub scans
//   4. per row: merge the old (sorted) row with its delta segment, recomputing every entry's
//      val from the NEW degrees (an edge changes deg of its endpoints, hence val of every entry
//      that points at them)                                         merge_kernel
// into spare buffers, then the spare and live sets are swapped.  Duplicate / out-of-range edges
// are detected on the device and the update is rejected with the snapshot unchanged.
#include <hipcub/hipcub.hpp>

#include <algorithm>

#include "graph_dev.h"

using egr::DeviceGuard;
using egr::dalloc;
using egr::dfree;

struct SnapUpdate {
  // spare CSR set (the merge target), with capacities
  uint32_t* row_ptr = nullptr;
  uint32_t* col = nullptr;
  uint8_t* meta = nullptr;
  float* val = nullptr;
  uint2* cv = nullptr;
  uint8_t* vlabel = nullptr;
  int64_t cap_v = 0, cap_e = 0;
  // scratch, grown on demand
  int64_t cap_m = 0, cap_rows = 0;
  uint32_t *drow = nullptr, *drow2 = nullptr;       // [2m]
  uint64_t *dkey = nullptr, *dkey2 = nullptr;       // [2m]
  uint32_t *add = nullptr, *deg = nullptr, *doff = nullptr;  // [V' + 1]
  void* temp = nullptr;
  size_t temp_bytes = 0;
  float* wmeta = nullptr;                           // [256]: weight by meta byte
  uint32_t* flag = nullptr;                         // [2]: bad edge, duplicate
};

void snapshot_update_free(egr_snapshot* s) {
  SnapUpdate* u = s->upd;
  if (!u) return;
  dfree(u->row_ptr);
  dfree(u->col);
  dfree(u->meta);
  dfree(u->val);
  dfree(u->cv);
  dfree(u->vlabel);
  dfree(u->drow);
  dfree(u->drow2);
  dfree(u->dkey);
  dfree(u->dkey2);
  dfree(u->add);
  dfree(u->deg);
  dfree(u->doff);
  dfree(u->temp);
  dfree(u->wmeta);
  dfree(u->flag);
  delete u;
  s->upd = nullptr;
}

namespace {

constexpr uint32_t FLAG_BAD = 0, FLAG_DUP = 1;

__global__ void __launch_bounds__(256) delta_kernel(const uint32_t* __restrict__ es,
                                                    const uint32_t* __restrict__ ed,
                                                    const uint8_t* __restrict__ et, int64_t m,
                                                    uint32_t Vn, uint32_t* __restrict__ drow,
                                                    uint64_t* __restrict__ dkey,
                                                    uint32_t* __restrict__ add,
                                                    uint32_t* __restrict__ flag) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= m) return;
  uint32_t s = es[e], d = ed[e], t = et[e];
  if (s >= Vn || d >= Vn || t >= 128u) {
    atomicOr(&flag[FLAG_BAD], 1u);
    // park the entries in row 0 with keys no real entry has; the update is rejected anyway
    s = d = 0;
    t = 0;
  }
  drow[2 * e] = d;
  dkey[2 * e] = (uint64_t)s << 9 | t << 1 | 0u;
  drow[2 * e + 1] = s;
  dkey[2 * e + 1] = (uint64_t)d << 9 | t << 1 | 1u;
  atomicAdd(&add[d], 1u);
  atomicAdd(&add[s], 1u);
}

__global__ void __launch_bounds__(256) degree_kernel(const uint32_t* __restrict__ row_ptr, uint32_t V,
                                                     uint32_t Vn, const uint32_t* __restrict__ add,
                                                     uint32_t* __restrict__ deg) {
  const uint32_t v = blockIdx.x * blockDim.x + threadIdx.x;
  if (v > Vn) return;
  deg[v] = v == Vn ? 0u : (v < V ? row_ptr[v + 1] - row_ptr[v] : 0u) + add[v];
}

// One thread per row of the grown graph: merge the old row (keys col<<9|meta, sorted) with the
// row's sorted delta segment into the new arrays; val from the new degrees.
__global__ void __launch_bounds__(256) merge_kernel(
    const uint32_t* __restrict__ rp_old, const uint32_t* __restrict__ col_old,
    const uint8_t* __restrict__ meta_old, uint32_t V, uint32_t Vn,
    const uint32_t* __restrict__ rp_new, const uint32_t* __restrict__ doff,
    const uint32_t* __restrict__ add, const uint64_t* __restrict__ dkey,
    const float* __restrict__ wmeta, uint32_t* __restrict__ col_new, uint8_t* __restrict__ meta_new,
    float* __restrict__ val_new, uint2* __restrict__ cv_new, uint32_t* __restrict__ flag) {
  const uint32_t v = blockIdx.x * blockDim.x + threadIdx.x;
  if (v >= Vn) return;
  uint32_t i = v < V ? rp_old[v] : 0u;
  const uint32_t ie = v < V ? rp_old[v + 1] : 0u;
  uint32_t j = doff[v];
  const uint32_t je = j + add[v];
  uint32_t o = rp_new[v];
  uint64_t prev = ~0ull;
  while (i < ie || j < je) {
    uint64_t k;
    const uint64_t ko = i < ie ? ((uint64_t)col_old[i] << 9 | meta_old[i]) : ~0ull;
    const uint64_t kd = j < je ? dkey[j] : ~0ull;
    if (ko < kd) {
      k = ko;
      ++i;
    } else {
      if (ko == kd) atomicOr(&flag[FLAG_DUP], 1u);
      k = kd;
      ++j;
    }
    if (k == prev) atomicOr(&flag[FLAG_DUP], 1u);
    prev = k;
    const uint32_t u = (uint32_t)(k >> 9);
    const uint32_t mt = (uint32_t)(k & 0x1FFu);
    const float deg = (float)(rp_new[u + 1] - rp_new[u]);
    const float w = wmeta[mt & 0xFFu] / deg;     // IEEE division, as egr_graph_csr on the host
    col_new[o] = u;
    meta_new[o] = (uint8_t)mt;
    val_new[o] = w;
    cv_new[o] = make_uint2(u, __float_as_uint(w));
    ++o;
  }
}

__global__ void __launch_bounds__(256) labels_kernel(const uint8_t* __restrict__ old_l, uint32_t V,
                                                     const uint8_t* __restrict__ new_l, uint32_t Vn,
                                                     uint8_t* __restrict__ out) {
  const uint32_t v = blockIdx.x * blockDim.x + threadIdx.x;
  if (v >= Vn) return;
  out[v] = v < V ? old_l[v] : new_l[v - V];
}

// multi-source BFS over the symmetric CSR: dist[v] = hops from the nearest source, 0xFF beyond
__global__ void __launch_bounds__(256) within_seed_kernel(const uint32_t* __restrict__ src, int64_t n,
                                                          uint32_t V, uint8_t* __restrict__ dist) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n && src[i] < V) dist[src[i]] = 0;
}

__global__ void __launch_bounds__(256) within_hop_kernel(const uint32_t* __restrict__ row_ptr,
                                                         const uint32_t* __restrict__ col, uint32_t V,
                                                         uint8_t h, uint8_t* __restrict__ dist) {
  const uint32_t v = blockIdx.x * blockDim.x + threadIdx.x;
  if (v >= V || dist[v] != (uint8_t)(h - 1)) return;
  for (uint32_t e = row_ptr[v], ee = row_ptr[v + 1]; e < ee; ++e) {
    const uint32_t u = col[e];
    if (dist[u] == 0xFF) dist[u] = h;   // racing writers all store h
  }
}

inline unsigned grid(int64_t n, int bs = 256) { return (unsigned)std::max<int64_t>(1, (n + bs - 1) / bs); }

int bits_for(uint64_t x) {
  int b = 1;
  while (b < 64 && (x >> b)) ++b;
  return b;
}

// grow the spare CSR set and scratch for V' vertices, NE' entries, 2m delta entries
int ensure(egr_snapshot* s, SnapUpdate* u, int64_t Vn, int64_t NEn, int64_t m2) {
  int rc = EGR_OK;
  if (u->cap_v < Vn) {
    const int64_t c = Vn + Vn / 4 + 1024;
    dfree(u->row_ptr);
    dfree(u->vlabel);
    u->cap_v = 0;
    if ((rc = dalloc(&u->row_ptr, c + 1)) || (rc = dalloc(&u->vlabel, c))) return rc;
    u->cap_v = c;
  }
  if (u->cap_e < NEn) {
    const int64_t c = NEn + NEn / 4 + 4096;
    dfree(u->col);
    dfree(u->meta);
    dfree(u->val);
    dfree(u->cv);
    u->cap_e = 0;
    if ((rc = dalloc(&u->col, c)) || (rc = dalloc(&u->meta, c)) || (rc = dalloc(&u->val, c)) ||
        (rc = dalloc(&u->cv, c + 2)))
      return rc;
    u->cap_e = c;
  }
  bool temp_stale = false;
  if (u->cap_m < m2) {
    const int64_t c = std::max<int64_t>(m2 + m2 / 2, 4096);
    dfree(u->drow);
    dfree(u->drow2);
    dfree(u->dkey);
    dfree(u->dkey2);
    u->cap_m = 0;
    if ((rc = dalloc(&u->drow, c)) || (rc = dalloc(&u->drow2, c)) || (rc = dalloc(&u->dkey, c)) ||
        (rc = dalloc(&u->dkey2, c)))
      return rc;
    u->cap_m = c;
    temp_stale = true;
  }
  if (u->cap_rows < Vn + 1) {
    const int64_t c = Vn + Vn / 4 + 1024;
    dfree(u->add);
    dfree(u->deg);
    dfree(u->doff);
    u->cap_rows = 0;
    if ((rc = dalloc(&u->add, c + 1)) || (rc = dalloc(&u->deg, c + 1)) || (rc = dalloc(&u->doff, c + 1)))
      return rc;
    u->cap_rows = c;
    temp_stale = true;
  }
  if (temp_stale || !u->temp) {
    size_t a = 0, b = 0, c = 0;
    hipcub::DoubleBuffer<uint64_t> k(u->dkey, u->dkey2);
    hipcub::DoubleBuffer<uint32_t> r(u->drow, u->drow2);
    if (hipcub::DeviceRadixSort::SortPairs(nullptr, a, k, r, (int)u->cap_m) != hipSuccess ||
        hipcub::DeviceRadixSort::SortPairs(nullptr, b, r, k, (int)u->cap_m) != hipSuccess ||
        hipcub::DeviceScan::ExclusiveSum(nullptr, c, u->deg, u->doff, (int)(u->cap_rows + 1)) != hipSuccess)
      return egr::fail(EGR_EDEVICE, "egr_snapshot_update: temp sizing failed");
    dfree(u->temp);
    u->temp_bytes = 0;
    const size_t t = std::max(a, std::max(b, c));
    if ((rc = dalloc((uint8_t**)&u->temp, t))) return rc;
    u->temp_bytes = t;
  }
  if (!u->wmeta && ((rc = dalloc(&u->wmeta, 256)) || (rc = dalloc(&u->flag, 2)))) return rc;
  (void)s;
  return EGR_OK;
}

}  // namespace

extern "C" {

int egr_snapshot_update(egr_snapshot* s, const uint8_t* new_vlabel, int64_t n_new,
                        const uint32_t* edge_src, const uint32_t* edge_dst, const uint8_t* edge_type,
                        int64_t n_edges, const float* weights, int32_t n_types, void* stream) {
  if (!s || n_new < 0 || n_edges < 0 || (n_new > 0 && !new_vlabel) ||
      (n_edges > 0 && (!edge_src || !edge_dst || !edge_type)) || n_types < 0 || n_types > 128 ||
      (n_types > 0 && !weights))
    return egr::fail(EGR_EINVAL, "egr_snapshot_update: bad arguments");
  const int64_t V = s->V, Vn = V + n_new, NEn = s->NE + 2 * n_edges;
  if (Vn >= (int64_t)EGR_NO_NODE || NEn >= 0xFFFFFFFFll)
    return egr::fail(EGR_EINVAL, "egr_snapshot_update: graph too large for u32 ids");
  if (n_new == 0 && n_edges == 0) return EGR_OK;
  DeviceGuard guard(s->device);
  hipStream_t st = (hipStream_t)stream;
  // The spare set is the previous version's arrays: a plan or frontier kernel enqueued earlier
  // on ANOTHER stream may still read them.  Drain the device before the merge (or ensure's
  // reallocation) writes into them; updates are per alert-storm tick, not per batch.
  EGR_HIP(hipDeviceSynchronize());
  if (!s->upd) s->upd = new SnapUpdate();
  SnapUpdate* u = s->upd;
  EGR_TRY(ensure(s, u, Vn, NEn, 2 * n_edges));
  // weight by meta byte (t << 1 | dir), as egr_graph_csr: types beyond n_types weigh 1
  float wm[256];
  for (int mt = 0; mt < 256; ++mt) {
    const int t = mt >> 1, dir = mt & 1;
    wm[mt] = t < n_types ? weights[t * 2 + dir] : 1.0f;
  }
  EGR_HIP(hipMemcpyAsync(u->wmeta, wm, sizeof(wm), hipMemcpyHostToDevice, st));
  EGR_HIP(hipMemsetAsync(u->flag, 0, 8, st));
  EGR_HIP(hipMemsetAsync(u->add, 0, (size_t)(Vn + 1) * 4, st));
  const int64_t m2 = 2 * n_edges;
  if (n_edges) {
    hipLaunchKernelGGL(delta_kernel, dim3(grid(n_edges)), dim3(256), 0, st, edge_src, edge_dst,
                       edge_type, n_edges, (uint32_t)Vn, u->drow, u->dkey, u->add, u->flag);
    // (row, key) order: sort by key, then stably by row
    hipcub::DoubleBuffer<uint64_t> k(u->dkey, u->dkey2);
    hipcub::DoubleBuffer<uint32_t> r(u->drow, u->drow2);
    size_t tb = u->temp_bytes;
    if (hipcub::DeviceRadixSort::SortPairs(u->temp, tb, k, r, (int)m2, 0, bits_for((uint64_t)Vn << 9), st) != hipSuccess)
      return egr::fail(EGR_EDEVICE, "egr_snapshot_update: key sort failed");
    tb = u->temp_bytes;
    if (hipcub::DeviceRadixSort::SortPairs(u->temp, tb, r, k, (int)m2, 0, bits_for((uint64_t)Vn), st) != hipSuccess)
      return egr::fail(EGR_EDEVICE, "egr_snapshot_update: row sort failed");
    if (k.Current() != u->dkey) std::swap(u->dkey, u->dkey2);
    if (r.Current() != u->drow) std::swap(u->drow, u->drow2);
  }
  hipLaunchKernelGGL(degree_kernel, dim3(grid(Vn + 1)), dim3(256), 0, st, s->row_ptr, (uint32_t)V,
                     (uint32_t)Vn, u->add, u->deg);
  size_t tb = u->temp_bytes;
  if (hipcub::DeviceScan::ExclusiveSum(u->temp, tb, u->deg, u->row_ptr, (int)(Vn + 1), st) != hipSuccess)
    return egr::fail(EGR_EDEVICE, "egr_snapshot_update: degree scan failed");
  tb = u->temp_bytes;
  if (hipcub::DeviceScan::ExclusiveSum(u->temp, tb, u->add, u->doff, (int)(Vn + 1), st) != hipSuccess)
    return egr::fail(EGR_EDEVICE, "egr_snapshot_update: delta scan failed");
  hipLaunchKernelGGL(merge_kernel, dim3(grid(Vn)), dim3(256), 0, st, s->row_ptr, s->col, s->meta,
                     (uint32_t)V, (uint32_t)Vn, u->row_ptr, u->doff, u->add, u->dkey, u->wmeta,
                     u->col, u->meta, u->val, u->cv, u->flag);
  hipLaunchKernelGGL(labels_kernel, dim3(grid(Vn)), dim3(256), 0, st, s->vlabel, (uint32_t)V,
                     new_vlabel, (uint32_t)Vn, u->vlabel);
  EGR_CHECK_LAUNCH();
  uint32_t flag[2] = {0, 0};
  EGR_HIP(hipMemcpyAsync(flag, u->flag, 8, hipMemcpyDeviceToHost, st));
  std::vector<uint32_t> rp_host((size_t)Vn + 1);
  EGR_HIP(hipMemcpyAsync(rp_host.data(), u->row_ptr, (Vn + 1) * 4, hipMemcpyDeviceToHost, st));
  EGR_HIP(hipStreamSynchronize(st));
  if (flag[FLAG_BAD]) return egr::fail(EGR_EINVAL, "egr_snapshot_update: edge endpoint or type out of range");
  if (flag[FLAG_DUP])
    return egr::fail(EGR_EINVAL, "egr_snapshot_update: edge already in the snapshot (or repeated)");
  // swap the live and spare sets
  std::swap(s->row_ptr, u->row_ptr);
  std::swap(s->col, u->col);
  std::swap(s->meta, u->meta);
  std::swap(s->val, u->val);
  std::swap(s->cv, u->cv);
  std::swap(s->vlabel, u->vlabel);
  std::swap(s->cap_v, u->cap_v);
  std::swap(s->cap_e, u->cap_e);
  s->V = Vn;
  s->NE = NEn;
  s->row_ptr_host = std::move(rp_host);
  ++s->version;
  // the frontier's locality layout follows the update (new vertices after the old ones); if it
  // cannot be rebuilt it is dropped and the frontier reads the canonical arrays (same results)
  (void)layout_extend(s, st);
  return EGR_OK;
}

int egr_snapshot_download(const egr_snapshot* s, uint32_t* row_ptr, uint32_t* col, uint8_t* meta,
                          float* val, uint8_t* vlabel) {
  if (!s) return egr::fail(EGR_EINVAL, "egr_snapshot_download: NULL snapshot");
  DeviceGuard guard(s->device);
  const size_t V = (size_t)s->V, NE = (size_t)s->NE;
  if (row_ptr) EGR_HIP(hipMemcpy(row_ptr, s->row_ptr, (V + 1) * 4, hipMemcpyDeviceToHost));
  if (col && NE) EGR_HIP(hipMemcpy(col, s->col, NE * 4, hipMemcpyDeviceToHost));
  if (meta && NE) EGR_HIP(hipMemcpy(meta, s->meta, NE, hipMemcpyDeviceToHost));
  if (val && NE) EGR_HIP(hipMemcpy(val, s->val, NE * 4, hipMemcpyDeviceToHost));
  if (vlabel) EGR_HIP(hipMemcpy(vlabel, s->vlabel, V, hipMemcpyDeviceToHost));
  return EGR_OK;
}

int64_t egr_snapshot_version(const egr_snapshot* s) { return s ? (int64_t)s->version : -1; }

int egr_snapshot_within(const egr_snapshot* s, const uint32_t* sources, int64_t n, int32_t hops,
                        uint8_t* out_dist, void* stream) {
  if (!s || n < 0 || (n > 0 && !sources) || !out_dist || hops < 0 || hops > 254)
    return egr::fail(EGR_EINVAL, "egr_snapshot_within: bad arguments (0 <= hops <= 254)");
  DeviceGuard guard(s->device);
  hipStream_t st = (hipStream_t)stream;
  const uint32_t V = (uint32_t)s->V;
  EGR_HIP(hipMemsetAsync(out_dist, 0xFF, V, st));
  if (n == 0) return EGR_OK;
  hipLaunchKernelGGL(within_seed_kernel, dim3(grid(n)), dim3(256), 0, st, sources, n, V, out_dist);
  for (int h = 1; h <= hops; ++h)
    hipLaunchKernelGGL(within_hop_kernel, dim3(grid(V)), dim3(256), 0, st, s->row_ptr, s->col, V,
                       (uint8_t)h, out_dist);
  EGR_CHECK_LAUNCH();
  return EGR_OK;
}

}  // extern "C"
