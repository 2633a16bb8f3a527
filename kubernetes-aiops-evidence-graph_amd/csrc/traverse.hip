// Typed one-hop neighbours on the device snapshot: the building block of GraphService's typed
// path queries (reference src/database/neo4j.py:205-279 -- find_related_changes,
// find_affected_by_node, get_service_dependencies), each a chain of
//   MATCH (a)-[:TYPE]->(b:Label)   /   MATCH (a)<-[:TYPE]-(b:Label)
// steps over the symmetric typed CSR (graph_dev.h: entry meta = type << 1 | dir; dir 1 = the
// row vertex is the relationship's source, dir 0 = its target).
//
// Layout: one wave per query vertex walks its row 64 entries a round; the entries whose
// (type, dir) and neighbour label match are compacted by ballot rank into the query's output
// segment, in CSR order (neighbour id, type, dir), so the result is deterministic.  A first
// call without an output array counts the matches; the caller scans the counts into segment
// offsets and calls again to emit.  Bound: latency of one row read per query; the queries are
// a few vertices.
#include "graph_dev.h"

using egr::DeviceGuard;

namespace {

__global__ __launch_bounds__(256) void typed_neighbors_kernel(
    const uint32_t* __restrict__ row_ptr, const uint32_t* __restrict__ col,
    const uint8_t* __restrict__ meta, const uint8_t* __restrict__ vlabel, uint32_t V,
    const uint32_t* __restrict__ q, int64_t n, uint32_t want_meta, int32_t label,
    const int64_t* __restrict__ out_off, uint32_t* __restrict__ out_v, uint32_t* __restrict__ out_n) {
  const int64_t i = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (i >= n) return;                               // (wave-uniform)
  const uint32_t v = q[i];
  uint32_t found = 0;
  if (v < V) {
    const uint32_t e0 = row_ptr[v], e1 = row_ptr[v + 1];
    uint32_t* const dst = out_v ? out_v + out_off[i] : nullptr;
    for (uint32_t base = e0; base < e1; base += 64) {
      const uint32_t e = base + lane;
      bool hit = false;
      uint32_t u = 0;
      if (e < e1 && meta[e] == want_meta) {
        u = col[e];
        hit = label < 0 || vlabel[u] == (uint8_t)label;
      }
      const uint64_t m = __ballot(hit);
      const uint32_t r = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                                   __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
      if (hit && dst) dst[found + r] = u;
      found += (uint32_t)__popcll(m);
    }
  }
  if (lane == 0) out_n[i] = found;
}

}  // namespace

extern "C" int egr_snapshot_typed_neighbors(const egr_snapshot* s, const uint32_t* vertices,
                                            int64_t n, int32_t rel_type, int32_t dir, int32_t label,
                                            const int64_t* out_off, uint32_t* out_vertices,
                                            uint32_t* out_counts, void* stream) {
  if (!s || n < 0 || rel_type < 0 || rel_type > 127 || (dir != 0 && dir != 1) || label > 255 ||
      (n > 0 && (!vertices || !out_counts || (out_vertices && !out_off))))
    return egr::fail(EGR_EINVAL, "egr_snapshot_typed_neighbors: bad arguments");
  if (n == 0) return EGR_OK;
  DeviceGuard guard(s->device);
  const hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(typed_neighbors_kernel, dim3((unsigned)((n + 3) / 4)), dim3(256), 0, st,
                     s->row_ptr, s->col, s->meta, s->vlabel, (uint32_t)s->V, vertices, n,
                     (uint32_t)rel_type << 1 | (uint32_t)dir, label, out_off, out_vertices, out_counts);
  EGR_CHECK_LAUNCH();
  return EGR_OK;
}
