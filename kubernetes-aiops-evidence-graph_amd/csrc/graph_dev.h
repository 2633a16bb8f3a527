// Device-side pieces shared by the dense propagation plan (propagate.hip) and the frontier
// engine (frontier.hip): the snapshot object, device-guard / allocation helpers and the seed
// preparation kernels (triples -> sorted, max-combined unique keys).
#pragma once

#include <hipcub/hipcub.hpp>

#include <string>
#include <vector>

#include "egr_internal.h"

struct egr_snapshot {
  int device = 0;
  int64_t V = 0, NE = 0;
  std::vector<uint32_t> row_ptr_host;   // for the per-plan chunk tables
  uint32_t* row_ptr = nullptr;
  uint32_t* col = nullptr;
  uint8_t* meta = nullptr;
  float* val = nullptr;
  uint2* cv = nullptr;       // (col, val bits) per entry: one 8-B load per entry (frontier)
  uint8_t* vlabel = nullptr;
  // incremental updates (update.hip): capacities of the live arrays, a version bumped by every
  // update (plans built on an older version refuse to run), and the spare buffers / scratch
  int64_t cap_v = 0, cap_e = 0;
  uint64_t version = 0;
  struct SnapUpdate* upd = nullptr;
  // The frontier engine's locality layout (layout.hip; nullptr when off): the same CSR with its
  // vertices renumbered so that the rows a 3-hop frontier walks sit close together.  Rows keep
  // their entries in the canonical order (so every fmaf chain is unchanged); `perm` maps an
  // original vertex id to its internal one, `iperm` back.  Frontier inputs are mapped in and its
  // outputs (top-k ids, tie-break order, member pool) are original ids.
  struct FrLayout* lay = nullptr;
};

// update.hip: frees egr_snapshot::upd (called by egr_snapshot_free)
void snapshot_update_free(egr_snapshot* s);

// layout.hip: the frontier layout of a snapshot.  layout_build computes the vertex order from
// the snapshot's host CSR and lays the device arrays out (egr_snapshot_create / _from_csr);
// layout_extend re-lays them after an update, new vertices numbered after the old ones;
// layout_free releases them.  Off when $EGRAPH_FRONTIER_LAYOUT is "0".
int layout_build(egr_snapshot* s, const uint32_t* row_ptr_host, const uint32_t* col_host);
int layout_extend(egr_snapshot* s, hipStream_t st);
void layout_free(egr_snapshot* s);
struct FrLayoutView {
  const uint32_t* row_ptr;
  const uint2* cv;
  const uint8_t* vlabel;
  const uint32_t* perm;    // nullptr: identity
  const uint32_t* iperm;
};
FrLayoutView layout_view(const egr_snapshot* s);

namespace egr {

template <typename T>
inline int dalloc(T** p, size_t count) {
  if (count == 0) count = 1;
  if (hipMalloc((void**)p, count * sizeof(T)) != hipSuccess) {
    (void)hipGetLastError();
    *p = nullptr;
    return fail(EGR_ENOMEM, "hipMalloc failed (" + std::to_string(count * sizeof(T)) + " B)");
  }
  return EGR_OK;
}

template <typename T>
inline void dfree(T*& p) {
  if (p) (void)hipFree((void*)p);
  p = nullptr;
}

#define EGR_TRY(x)                 \
  do {                             \
    int rc_ = (x);                 \
    if (rc_ != EGR_OK) return rc_; \
  } while (0)

// ---- seeds: (vertex, column, value) triples -> unique keys (max-combined) -------------------
// A key is major * minor_n + minor; the dense plan uses (vertex, column) with minor_n = Bpad,
// the frontier engine (column, vertex) with minor_n = V.  Invalid triples get key ~0, which
// sorts last.
namespace seedk {

__global__ static void keys_kernel(const uint32_t* __restrict__ sv, const uint32_t* __restrict__ sc,
                                   const float* __restrict__ sval, int64_t n, uint32_t V, int B,
                                   bool col_major, uint64_t minor_n, uint64_t* keys, float* vals) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t v = sv[i], c = sc[i];
  const bool ok = v < V && c < (uint32_t)B;
  keys[i] = !ok ? ~0ull : col_major ? (uint64_t)c * minor_n + v : (uint64_t)v * minor_n + c;
  vals[i] = sval[i];
}

__global__ static void head_kernel(const uint64_t* __restrict__ keys, int64_t n, uint32_t* head) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint64_t k = keys[i];
  head[i] = (k != ~0ull && (i == 0 || keys[i - 1] != k)) ? 1u : 0u;
}

// unique keys, their minor part and the max of their values
__global__ static void compact_kernel(const uint64_t* __restrict__ keys,
                                      const float* __restrict__ vals,
                                      const uint32_t* __restrict__ head,
                                      const uint32_t* __restrict__ pos, int64_t n, uint64_t minor_n,
                                      uint64_t* ukeys, uint32_t* uminor, float* uval,
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
  uminor[p] = (uint32_t)(k % minor_n);
  uval[p] = m;
}

// ptr[m] = first unique key >= m * minor_n, for m in [0, n_major]
__global__ static void ptr_kernel(const uint64_t* __restrict__ ukeys,
                                  const uint32_t* __restrict__ n_unique, uint32_t n_major,
                                  uint64_t minor_n, uint32_t* ptr) {
  const uint32_t m = blockIdx.x * blockDim.x + threadIdx.x;
  if (m > n_major) return;
  const uint64_t target = (uint64_t)m * minor_n;
  uint32_t lo = 0, hi = *n_unique;
  while (lo < hi) {
    const uint32_t mid = (lo + hi) >> 1;
    if (ukeys[mid] < target) lo = mid + 1;
    else hi = mid;
  }
  ptr[m] = lo;
}

__global__ static void zero_kernel(uint32_t* p, uint32_t n) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) p[i] = 0;
}

}  // namespace seedk

inline int key_bits(uint64_t keyspace) {
  int b = 1;
  while (b < 64 && (1ull << b) <= keyspace) ++b;
  return b;
}

// Workspace of the seed preparation for up to `cap` triples.
struct SeedPrep {
  int64_t cap = 0;
  int end_bit = 64;
  uint64_t *keys_in = nullptr, *keys = nullptr, *ukeys = nullptr;
  float *vals_in = nullptr, *vals = nullptr, *uval = nullptr;
  uint32_t *head = nullptr, *pos = nullptr, *uminor = nullptr, *n_unique = nullptr;
  void* tmp = nullptr;
  size_t tmp_bytes = 0;

  // extra_scan_n: size of another ExclusiveSum the owner runs with `tmp`
  int alloc(int64_t max_seeds, uint64_t keyspace, size_t extra_scan_n) {
    cap = max_seeds;
    end_bit = key_bits(keyspace);
    const size_t ms = (size_t)std::max<int64_t>(max_seeds, 1);
    int rc = EGR_OK;
    if ((rc = dalloc(&keys_in, ms)) || (rc = dalloc(&keys, ms)) || (rc = dalloc(&ukeys, ms)) ||
        (rc = dalloc(&vals_in, ms)) || (rc = dalloc(&vals, ms)) || (rc = dalloc(&uval, ms)) ||
        (rc = dalloc(&head, ms)) || (rc = dalloc(&pos, ms)) || (rc = dalloc(&uminor, ms)) ||
        (rc = dalloc(&n_unique, 1)))
      return rc;
    size_t b1 = 0, b2 = 0, b3 = 0;
    uint32_t* u32 = head;
    if (hipcub::DeviceRadixSort::SortPairs(nullptr, b1, keys_in, keys, vals_in, vals, (int)ms, 0,
                                           end_bit) != hipSuccess ||
        hipcub::DeviceScan::ExclusiveSum(nullptr, b2, head, pos, (int)ms) != hipSuccess ||
        hipcub::DeviceScan::ExclusiveSum(nullptr, b3, u32, pos, (int)std::max<size_t>(extra_scan_n, 1)) !=
            hipSuccess)
      return fail(EGR_EDEVICE, "hipcub temp-size query failed");
    tmp_bytes = std::max({b1, b2, b3});
    if (hipMalloc(&tmp, tmp_bytes) != hipSuccess) {
      (void)hipGetLastError();
      tmp = nullptr;
      return fail(EGR_ENOMEM, "hipMalloc (hipcub temp) failed");
    }
    return EGR_OK;
  }

  void free_all() {
    dfree(keys_in);
    dfree(keys);
    dfree(ukeys);
    dfree(vals_in);
    dfree(vals);
    dfree(uval);
    dfree(head);
    dfree(pos);
    dfree(uminor);
    dfree(n_unique);
    if (tmp) (void)hipFree(tmp);
    tmp = nullptr;
  }

  // sort + max-combine n triples; afterwards ukeys/uminor/uval[0..*n_unique) are the unique
  // keys in ascending order and ptr[0..n_major] indexes them by major
  int run(const uint32_t* sv, const uint32_t* sc, const float* sval, int64_t n, uint32_t V, int B,
          bool col_major, uint64_t minor_n, uint32_t n_major, uint32_t* ptr, hipStream_t st) {
    EGR_HIP(hipMemsetAsync(n_unique, 0, 4, st));
    if (n == 0) {
      hipLaunchKernelGGL(seedk::zero_kernel, dim3((n_major + 256) / 256), dim3(256), 0, st, ptr,
                         n_major + 1);
      EGR_CHECK_LAUNCH();
      return EGR_OK;
    }
    const int ni = (int)n;
    const dim3 g1((ni + 255) / 256);
    hipLaunchKernelGGL(seedk::keys_kernel, g1, dim3(256), 0, st, sv, sc, sval, (int64_t)n, V, B,
                       col_major, minor_n, keys_in, vals_in);
    EGR_CHECK_LAUNCH();
    size_t tb = tmp_bytes;
    // invalid keys (~0) sort last: their low end_bit bits are all ones, above every valid key
    EGR_HIP(hipcub::DeviceRadixSort::SortPairs(tmp, tb, keys_in, keys, vals_in, vals, ni, 0,
                                               end_bit, st));
    hipLaunchKernelGGL(seedk::head_kernel, g1, dim3(256), 0, st, keys, (int64_t)n, head);
    EGR_CHECK_LAUNCH();
    tb = tmp_bytes;
    EGR_HIP(hipcub::DeviceScan::ExclusiveSum(tmp, tb, head, pos, ni, st));
    hipLaunchKernelGGL(seedk::compact_kernel, g1, dim3(256), 0, st, keys, vals, head, pos,
                       (int64_t)n, minor_n, ukeys, uminor, uval, n_unique);
    EGR_CHECK_LAUNCH();
    hipLaunchKernelGGL(seedk::ptr_kernel, dim3((n_major + 256) / 256), dim3(256), 0, st, ukeys,
                       n_unique, n_major, minor_n, ptr);
    EGR_CHECK_LAUNCH();
    return EGR_OK;
  }
};

}  // namespace egr
