// The frontier engine's locality layout of a snapshot (graph_dev.h egr_snapshot::lay).
//
// A column's frontier walks the rows of its members three times, and a member's row is one or
// two 8-B gathers -- a 128-B cache line each, mostly for one member.  On the Kubernetes evidence
// graph the rows of a column's last hops are the pods scheduled on the incident's Nodes, which
// the collectors' creation order scatters over every namespace: ~1.2k distinct lines per C3
// column.  Renumbering the vertices so that a Node's pods (and each pod's attachments) are
// contiguous brings that to ~0.3k lines (4x fewer L2 misses per column for the same gathers).
//
// The order (locality_order below, the same rule as egraph.graph.locality_order): every vertex
// hangs under its highest-degree neighbour when that neighbour's degree is higher (ties: the
// lower id); the forest is laid out root by root, then by the subtree under the root, then by
// depth and id.  Nothing in it names a label: hubs are found by degree.
//
// Exactness: only ids change.  Each row keeps its entries in the canonical (original
// neighbour id) order with the same values, so every fmaf chain is the one the canonical CSR
// gives; the frontier maps its inputs (seed vertices, incident vertices) through `perm` and
// breaks top-k ties and writes its outputs with the original ids (`iperm`).
#include <algorithm>
#include <new>
#include <numeric>

#include "graph_dev.h"

using egr::DeviceGuard;
using egr::dalloc;
using egr::dfree;

struct FrLayout {
  uint32_t* row_ptr = nullptr;    // [cap_v + 1]
  uint2* cv = nullptr;            // [cap_e + 2] (two entries of padding, as the canonical cv)
  uint8_t* vlabel = nullptr;      // [cap_v]
  uint32_t* perm = nullptr;       // [cap_v] original -> internal
  uint32_t* iperm = nullptr;      // [cap_v] internal -> original
  uint32_t* deg = nullptr;        // [cap_v + 1] scratch
  void* temp = nullptr;           // scan scratch
  size_t temp_bytes = 0;
  int64_t cap_v = 0, cap_e = 0, V = 0;
  std::vector<uint32_t> order;    // internal -> original (host copy, extended by updates)
  int64_t v_ordered = 0;          // vertices when `order` was last computed by locality_order
};

namespace {

// order[i] = the original vertex placed at internal position i
std::vector<uint32_t> locality_order(const uint32_t* rp, const uint32_t* col, int64_t V) {
  std::vector<int64_t> parent((size_t)V, -1);
  for (int64_t v = 0; v < V; ++v) {
    int64_t best = -1;
    uint32_t bd = 0;
    for (uint32_t e = rp[v]; e < rp[v + 1]; ++e) {
      const int64_t u = col[e];
      const uint32_t du = rp[u + 1] - rp[u];
      if (best < 0 || du > bd || (du == bd && u < best)) {
        best = u;
        bd = du;
      }
    }
    if (best >= 0 && bd > rp[v + 1] - rp[v]) parent[(size_t)v] = best;
  }
  // root, the vertex right under it, and the depth of every vertex (degrees grow strictly
  // towards a root, so a chain ends)
  std::vector<int64_t> root((size_t)V), top((size_t)V), depth((size_t)V, 0);
  for (int64_t v = 0; v < V; ++v) {
    int64_t r = v, t = v, d = 0;
    for (int64_t c = parent[(size_t)v]; c >= 0; c = parent[(size_t)c]) {
      if (parent[(size_t)c] >= 0) t = c;
      r = c;
      ++d;
    }
    root[(size_t)v] = r;
    top[(size_t)v] = t;
    depth[(size_t)v] = d;
  }
  std::vector<uint32_t> order((size_t)V);
  std::iota(order.begin(), order.end(), 0u);
  std::sort(order.begin(), order.end(), [&](uint32_t a, uint32_t b) {
    if (root[a] != root[b]) return root[a] < root[b];
    if (top[a] != top[b]) return top[a] < top[b];
    if (depth[a] != depth[b]) return depth[a] < depth[b];
    return a < b;
  });
  return order;
}

__global__ void __launch_bounds__(256) lay_deg_kernel(const uint32_t* __restrict__ rp,
                                                      const uint32_t* __restrict__ iperm, uint32_t V,
                                                      uint32_t* __restrict__ deg) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i > V) return;
  deg[i] = i < V ? rp[iperm[i] + 1] - rp[iperm[i]] : 0u;
}

// one thread per internal row: the original row's entries, in their order, neighbour ids mapped
__global__ void __launch_bounds__(256) lay_rows_kernel(const uint32_t* __restrict__ rp,
                                                       const uint2* __restrict__ cv,
                                                       const uint8_t* __restrict__ vlabel,
                                                       const uint32_t* __restrict__ iperm,
                                                       const uint32_t* __restrict__ perm,
                                                       const uint32_t* __restrict__ nrp, uint32_t V,
                                                       uint2* __restrict__ out,
                                                       uint8_t* __restrict__ out_label) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= V) return;
  const uint32_t o = iperm[i];
  const uint32_t e0 = rp[o], n = rp[o + 1] - e0, d0 = nrp[i];
  for (uint32_t j = 0; j < n; ++j) {
    const uint2 c = cv[e0 + j];
    out[d0 + j] = make_uint2(perm[c.x], c.y);
  }
  out_label[i] = vlabel[o];
}

// the vertices an update appended keep their own ids: perm / iperm are the identity on [v0, V)
__global__ void __launch_bounds__(256) lay_tail_kernel(uint32_t v0, uint32_t V, uint32_t* __restrict__ perm,
                                                       uint32_t* __restrict__ iperm) {
  const uint32_t i = v0 + blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= V) return;
  perm[i] = i;
  iperm[i] = i;
}

inline unsigned lgrid(int64_t n) { return (unsigned)std::max<int64_t>(1, (n + 255) / 256); }

bool layout_enabled() {
  const char* e = getenv("EGRAPH_FRONTIER_LAYOUT");
  return !(e && e[0] == '0');
}

// (re)lay the device arrays of s->lay from the canonical snapshot for lay->order (its size is V).
// tail_from > 0: the device perm / iperm are current for [0, tail_from) and `order` only appended
// identity entries after it (an update's new vertices) -- those are filled on the device, so the
// call copies nothing from the host and does not wait for the stream; 0: both uploaded from
// `order` (and the host waits for the copy of its stack buffer).
int relayout(egr_snapshot* s, hipStream_t st, int64_t tail_from = 0) {
  FrLayout* L = s->lay;
  const int64_t V = s->V, NE = s->NE;
  int rc = EGR_OK;
  if (L->cap_v < V) {
    tail_from = 0;                          // (new arrays: nothing on the device is current)
    const int64_t c = V + V / 4 + 1024;
    dfree(L->row_ptr);
    dfree(L->vlabel);
    dfree(L->perm);
    dfree(L->iperm);
    dfree(L->deg);
    dfree(L->temp);
    L->cap_v = 0;
    L->temp_bytes = 0;
    if ((rc = dalloc(&L->row_ptr, c + 1)) || (rc = dalloc(&L->vlabel, c)) || (rc = dalloc(&L->perm, c)) ||
        (rc = dalloc(&L->iperm, c)) || (rc = dalloc(&L->deg, c + 1)))
      return rc;
    size_t tb = 0;
    EGR_HIP(hipcub::DeviceScan::ExclusiveSum(nullptr, tb, L->deg, L->row_ptr, (int)(c + 1)));
    if ((rc = dalloc((uint8_t**)&L->temp, tb))) return rc;
    L->temp_bytes = tb;
    L->cap_v = c;
  }
  if (L->cap_e < NE) {
    const int64_t c = NE + NE / 4 + 4096;
    dfree(L->cv);
    L->cap_e = 0;
    if ((rc = dalloc(&L->cv, c + 2))) return rc;
    EGR_HIP(hipMemset(L->cv, 0, (size_t)(c + 2) * sizeof(uint2)));
    L->cap_e = c;
  }
  const bool full = tail_from <= 0;
  std::vector<uint32_t> perm;
  if (full) {
    perm.resize((size_t)V);
    for (int64_t i = 0; i < V; ++i) perm[L->order[(size_t)i]] = (uint32_t)i;
    EGR_HIP(hipMemcpyAsync(L->iperm, L->order.data(), (size_t)V * 4, hipMemcpyHostToDevice, st));
    EGR_HIP(hipMemcpyAsync(L->perm, perm.data(), (size_t)V * 4, hipMemcpyHostToDevice, st));
  } else if (tail_from < V) {
    hipLaunchKernelGGL(lay_tail_kernel, dim3(lgrid(V - tail_from)), dim3(256), 0, st,
                       (uint32_t)tail_from, (uint32_t)V, L->perm, L->iperm);
  }
  hipLaunchKernelGGL(lay_deg_kernel, dim3(lgrid(V + 1)), dim3(256), 0, st, s->row_ptr, L->iperm,
                     (uint32_t)V, L->deg);
  size_t tb = L->temp_bytes;
  EGR_HIP(hipcub::DeviceScan::ExclusiveSum(L->temp, tb, L->deg, L->row_ptr, (int)(V + 1), st));
  hipLaunchKernelGGL(lay_rows_kernel, dim3(lgrid(V)), dim3(256), 0, st, s->row_ptr, s->cv, s->vlabel,
                     L->iperm, L->perm, L->row_ptr, (uint32_t)V, L->cv, L->vlabel);
  EGR_CHECK_LAUNCH();
  if (full) EGR_HIP(hipStreamSynchronize(st));   // (perm lives on the host stack until here)
  L->V = V;
  return EGR_OK;
}

}  // namespace

// The layout is an optional second copy (~1.25x the canonical cv plus row pointers, perm, iperm
// and labels): when it cannot be built -- device memory, a host allocation -- it is dropped and
// the frontier reads the canonical arrays, which give the same results bit for bit.  Neither
// function fails its caller: a graph that fits HBM without the layout still gets its snapshot
// (egr_snapshot_create / egr_snapshot_from_csr) and its updates (egr_snapshot_update).
static void layout_drop(egr_snapshot* s) {
  layout_free(s);
  (void)hipGetLastError();                  // (a failed allocation's status is not the caller's)
}

int layout_build(egr_snapshot* s, const uint32_t* row_ptr_host, const uint32_t* col_host) {
  if (!layout_enabled() || s->V <= 0) return EGR_OK;
  DeviceGuard guard(s->device);
  int rc = EGR_ENOMEM;
  try {
    if (!s->lay) s->lay = new FrLayout();
    s->lay->order = locality_order(row_ptr_host, col_host, s->V);
    s->lay->v_ordered = s->V;
    rc = relayout(s, nullptr);
  } catch (const std::bad_alloc&) {
    rc = EGR_ENOMEM;
  }
  if (rc != EGR_OK) layout_drop(s);
  return EGR_OK;
}

// After an update: the new vertices go after the old ones with their own ids (the device fills
// that tail, nothing is copied from the host and the host does not wait), every row re-laid on
// the device (the rows' offsets moved).  Appended vertices are not placed by locality, so once
// the graph has grown by a quarter since the order was computed, the order is recomputed from
// the current CSR (one column download) and uploaded whole.
int layout_extend(egr_snapshot* s, hipStream_t st) {
  if (!s->lay) return EGR_OK;
  DeviceGuard guard(s->device);
  int rc = EGR_ENOMEM;
  try {
    FrLayout* L = s->lay;
    const int64_t v0 = (int64_t)L->order.size();
    if (s->V - L->v_ordered > L->v_ordered / 4 && (int64_t)s->row_ptr_host.size() == s->V + 1) {
      std::vector<uint32_t> col((size_t)s->NE);
      EGR_HIP(hipStreamSynchronize(st));
      if (s->NE > 0)
        EGR_HIP(hipMemcpy(col.data(), s->col, (size_t)s->NE * 4, hipMemcpyDeviceToHost));
      L->order = locality_order(s->row_ptr_host.data(), col.data(), s->V);
      L->v_ordered = s->V;
      rc = relayout(s, st);
    } else {
      for (int64_t v = v0; v < s->V; ++v) L->order.push_back((uint32_t)v);
      rc = relayout(s, st, v0 > 0 ? v0 : 0);
    }
  } catch (const std::bad_alloc&) {
    rc = EGR_ENOMEM;
  }
  if (rc != EGR_OK) layout_drop(s);         // (the frontier then reads the canonical arrays)
  return EGR_OK;
}

void layout_free(egr_snapshot* s) {
  FrLayout* L = s->lay;
  if (!L) return;
  dfree(L->row_ptr);
  dfree(L->cv);
  dfree(L->vlabel);
  dfree(L->perm);
  dfree(L->iperm);
  dfree(L->deg);
  dfree(L->temp);
  delete L;
  s->lay = nullptr;
}

FrLayoutView layout_view(const egr_snapshot* s) {
  if (s->lay && s->lay->V == s->V)
    return {s->lay->row_ptr, s->lay->cv, s->lay->vlabel, s->lay->perm, s->lay->iperm};
  return {s->row_ptr, s->cv, s->vlabel, nullptr, nullptr};
}

extern "C" int egr_locality_order(const uint32_t* row_ptr, const uint32_t* col, int64_t n_vertices,
                                  uint32_t* out_order) {
  if (!row_ptr || !out_order || n_vertices < 0 || (n_vertices > 0 && row_ptr[n_vertices] > 0 && !col))
    return egr::fail(EGR_EINVAL, "egr_locality_order: bad arguments");
  for (int64_t v = 0; v < n_vertices; ++v)
    if (row_ptr[v + 1] < row_ptr[v]) return egr::fail(EGR_EINVAL, "egr_locality_order: row_ptr not monotone");
  const int64_t NE = n_vertices > 0 ? row_ptr[n_vertices] : 0;
  for (int64_t e = 0; e < NE; ++e)
    if (col[e] >= (uint64_t)n_vertices) return egr::fail(EGR_EINVAL, "egr_locality_order: col out of range");
  try {
    const std::vector<uint32_t> o = locality_order(row_ptr, col, n_vertices);
    std::copy(o.begin(), o.end(), out_order);
  } catch (...) {
    return egr::fail(EGR_ENOMEM, "egr_locality_order: allocation failed");
  }
  return EGR_OK;
}
