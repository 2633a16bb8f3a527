// Host side of the evidence graph: MERGE semantics of the reference's GraphService and the
// symmetric typed CSR that the device snapshot is built from.
//
// Reference: src/database/neo4j.py
//   create_entities_batch (:95-113): per entity `MERGE (n:{type} {id: $id}) SET n += $props`
//       -> a vertex is keyed by (label, id); re-merging an existing (label, id) creates nothing.
//   create_relations_batch (:145-167): per relation
//       `MATCH (source {id}) MATCH (target {id}) MERGE (source)-[r:{type}]->(target)`
//       -> label-less match: every vertex carrying the id participates (cartesian product);
//          an edge is keyed by (source vertex, type, target vertex); a missing endpoint drops
//          the relation silently.
// Properties are not stored here: the Python GraphService mirror keeps them (last write wins).
#include <algorithm>
#include <cstring>
#include <numeric>
#include <string>
#include <string_view>
#include <unordered_map>
#include <vector>

#include "egr_internal.h"

struct egr_graph {
  std::vector<std::string> labels, rtypes;
  std::vector<std::string> vid;          // vertex id strings, creation order
  std::vector<uint8_t> vlabel;
  // id -> first vertex, open addressing over the id bytes: a lookup hashes the caller's bytes in
  // place (no std::string per query) and compares them with vid[v].  Read-only between merges,
  // so concurrent finds (egr_graph_find) are safe while no merge runs.
  struct IdSlot {
    uint32_t tag;   // high hash bits | 1 (0 = empty)
    int32_t v;
  };
  std::vector<IdSlot> idx;
  size_t idx_n = 0;
  // An id carried by several vertices (one per label: MERGE keys a vertex by (label, id)) keeps
  // its vertices, creation order, under its first vertex; vmulti[first] marks such ids.  Every
  // other id has exactly the one vertex idx names.
  std::unordered_map<int32_t, std::vector<int32_t>> multi;
  std::vector<uint8_t> vmulti;
  std::vector<int32_t> esrc, edst;
  std::vector<uint8_t> etype;
  // the (source, type, target) edge set, open addressing (load <= 1/2; t = -1: empty slot)
  struct ESlot {
    int32_t s, d, t;
  };
  std::vector<ESlot> eset;
  size_t eset_n = 0;
};

namespace {

// Index of name s in names, appended if absent.  Label and relationship-type tables are tiny
// (at most 255 / 127 names), so a scan beats hashing a std::string built per call.
int intern(std::vector<std::string>& names, std::string_view s, size_t max_names, const char* what) {
  for (size_t i = 0; i < names.size(); ++i)
    if (names[i].size() == s.size() && memcmp(names[i].data(), s.data(), s.size()) == 0) return (int)i;
  if (names.size() >= max_names) return egr::fail(EGR_EINVAL, std::string("too many distinct ") + what);
  names.emplace_back(s);
  return (int)names.size() - 1;
}

inline uint64_t edge_hash(int32_t s, int32_t d, int32_t t) {
  uint64_t h = ((uint64_t)(uint32_t)s << 32 | (uint32_t)d) * 0x9E3779B97F4A7C15ull;
  h ^= (uint64_t)(uint32_t)t * 0xC2B2AE3D27D4EB4Full;
  h ^= h >> 31;
  h *= 0xD6E8FEB86659FD93ull;
  return h ^ (h >> 32);
}

// true if (s, d, t) was not in the edge set (and is now)
bool eset_insert(egr_graph* g, int32_t s, int32_t d, int32_t t) {
  if (2 * (g->eset_n + 1) > g->eset.size()) {         // grow to keep the load at most 1/2
    std::vector<egr_graph::ESlot> old;
    old.swap(g->eset);
    g->eset.assign(std::max<size_t>(4096, 2 * old.size()), egr_graph::ESlot{0, 0, -1});
    const size_t m = g->eset.size() - 1;
    for (const auto& e : old) {
      if (e.t < 0) continue;
      size_t i = (size_t)edge_hash(e.s, e.d, e.t) & m;
      while (g->eset[i].t >= 0) i = (i + 1) & m;
      g->eset[i] = e;
    }
  }
  const size_t m = g->eset.size() - 1;
  for (size_t i = (size_t)edge_hash(s, d, t) & m;; i = (i + 1) & m) {
    egr_graph::ESlot& e = g->eset[i];
    if (e.t < 0) {
      e = egr_graph::ESlot{s, d, t};
      ++g->eset_n;
      return true;
    }
    if (e.s == s && e.d == d && e.t == t) return false;
  }
}

// 64-bit hash of an id's bytes, 8 at a time (a multiply-xorshift mix per word)
inline uint64_t id_hash(const char* p, size_t n) {
  uint64_t h = 0x9E3779B97F4A7C15ull ^ (n * 0xFF51AFD7ED558CCDull);
  while (n >= 8) {
    uint64_t w;
    memcpy(&w, p, 8);
    h = (h ^ (w * 0xC4CEB9FE1A85EC53ull)) * 0x9E3779B97F4A7C15ull;
    h ^= h >> 29;
    p += 8;
    n -= 8;
  }
  if (n) {
    uint64_t w = 0;
    memcpy(&w, p, n);
    h = (h ^ (w * 0xC4CEB9FE1A85EC53ull)) * 0x9E3779B97F4A7C15ull;
  }
  h ^= h >> 32;
  h *= 0xD6E8FEB86659FD93ull;
  return h ^ (h >> 32);
}

void idx_put(egr_graph* g, const std::string& id, int32_t v) {
  if (2 * (g->idx_n + 1) > g->idx.size()) {         // grow to keep the load at most 1/2
    std::vector<egr_graph::IdSlot> old;
    old.swap(g->idx);
    g->idx.assign(std::max<size_t>(1024, 2 * old.size()), egr_graph::IdSlot{0u, -1});
    const size_t m = g->idx.size() - 1;
    for (const auto& e : old) {
      if (!e.tag) continue;
      const std::string& s = g->vid[e.v];
      size_t i = (size_t)id_hash(s.data(), s.size()) & m;
      while (g->idx[i].tag) i = (i + 1) & m;
      g->idx[i] = e;
    }
  }
  const uint64_t h = id_hash(id.data(), id.size());
  const size_t m = g->idx.size() - 1;
  size_t i = (size_t)h & m;
  while (g->idx[i].tag) i = (i + 1) & m;
  g->idx[i] = egr_graph::IdSlot{(uint32_t)(h >> 32) | 1u, v};
  ++g->idx_n;
}

inline int32_t idx_find_h(const egr_graph* g, const char* p, size_t n, uint64_t h) {
  const uint32_t tag = (uint32_t)(h >> 32) | 1u;
  const size_t m = g->idx.size() - 1;
  for (size_t i = (size_t)h & m;; i = (i + 1) & m) {
    const egr_graph::IdSlot e = g->idx[i];
    if (!e.tag) return -1;
    if (e.tag == tag) {
      const std::string& s = g->vid[e.v];
      if (s.size() == n && memcmp(s.data(), p, n) == 0) return e.v;
    }
  }
}

inline int32_t idx_find(const egr_graph* g, const char* p, size_t n) {
  if (g->idx.empty()) return -1;
  return idx_find_h(g, p, n, id_hash(p, n));
}

// idx_find of n ids (blob + offsets) into out.  A lookup is three dependent cache misses (its
// index slot, the vertex's std::string, the string's bytes) into tables far larger than the
// caches; they are software-pipelined over groups of LB ids -- every id's slot prefetched, then
// every hit's string object, then its bytes -- so the misses of a group overlap instead of
// queueing one after another.
void batch_find(const egr_graph* g, const char* blob, const int64_t* off, int64_t n, int32_t* out) {
  if (g->idx.empty()) {
    for (int64_t i = 0; i < n; ++i) out[i] = -1;
    return;
  }
  constexpr int LB = 32;
  const size_t m = g->idx.size() - 1;
  uint64_t h[LB];
  for (int64_t i0 = 0; i0 < n; i0 += LB) {
    const int c = (int)std::min<int64_t>(LB, n - i0);
    for (int j = 0; j < c; ++j) {
      const int64_t i = i0 + j;
      h[j] = id_hash(blob + off[i], (size_t)(off[i + 1] - off[i]));
      __builtin_prefetch(&g->idx[(size_t)h[j] & m]);
    }
    for (int j = 0; j < c; ++j) {
      const egr_graph::IdSlot e = g->idx[(size_t)h[j] & m];
      if (e.tag == ((uint32_t)(h[j] >> 32) | 1u)) __builtin_prefetch(&g->vid[e.v]);
    }
    for (int j = 0; j < c; ++j) {
      const egr_graph::IdSlot e = g->idx[(size_t)h[j] & m];
      if (e.tag == ((uint32_t)(h[j] >> 32) | 1u)) __builtin_prefetch(g->vid[e.v].data());
    }
    for (int j = 0; j < c; ++j) {
      const int64_t i = i0 + j;
      out[i] = idx_find_h(g, blob + off[i], (size_t)(off[i + 1] - off[i]), h[j]);
    }
  }
}

// The vertices carrying an id (creation order): none, its one vertex, or its multi list.
struct IdVerts {
  const int32_t* p;
  size_t n;
  int32_t one;
};

inline IdVerts verts_of(const egr_graph* g, int32_t v) {
  IdVerts r{nullptr, 0, -1};
  if (v < 0) return r;
  if (g->vmulti[v]) {
    const auto& vs = g->multi.at(v);
    r.p = vs.data();
    r.n = vs.size();
  } else {
    r.one = v;
    r.n = 1;
  }
  return r;
}

inline std::string_view str_at(const char* blob, const int64_t* off, int64_t i) {
  return std::string_view(blob + off[i], (size_t)(off[i + 1] - off[i]));
}

int64_t copy_out(const std::string& s, char* buf, int64_t cap) {
  if (buf && cap > 0) memcpy(buf, s.data(), (size_t)std::min<int64_t>(cap, (int64_t)s.size()));
  return (int64_t)s.size();
}

}  // namespace

extern "C" {

int egr_graph_create(egr_graph** out) {
  if (!out) return egr::fail(EGR_EINVAL, "egr_graph_create: out is NULL");
  try {
    *out = new egr_graph();
  } catch (...) {
    return egr::fail(EGR_ENOMEM, "egr_graph_create: allocation failed");
  }
  return EGR_OK;
}

void egr_graph_free(egr_graph* g) { delete g; }

int egr_graph_merge_nodes(egr_graph* g, const char* id_blob, const int64_t* id_off,
                          const char* label_blob, const int64_t* label_off, int64_t n,
                          int32_t* out_vertex) {
  if (!g || n < 0 || (n > 0 && (!id_blob || !id_off || !label_blob || !label_off)))
    return egr::fail(EGR_EINVAL, "egr_graph_merge_nodes: bad arguments");
  for (int64_t i = 0; i < n; ++i) {
    std::string_view id = str_at(id_blob, id_off, i);
    int lab = intern(g->labels, str_at(label_blob, label_off, i), 255, "labels");
    if (lab < 0) return lab;
    const int32_t first = idx_find(g, id.data(), id.size());
    int32_t v = -1;
    if (first >= 0) {
      if (g->vmulti[first]) {
        for (int32_t c : g->multi.at(first))
          if (g->vlabel[c] == lab) { v = c; break; }
      } else if (g->vlabel[first] == lab) {
        v = first;
      }
    }
    if (v < 0) {
      if (g->vid.size() >= 0x7FFFFFF0u) return egr::fail(EGR_EINVAL, "too many vertices");
      v = (int32_t)g->vid.size();
      g->vid.emplace_back(id);
      g->vlabel.push_back((uint8_t)lab);
      g->vmulti.push_back(0);
      if (first < 0) {
        idx_put(g, g->vid.back(), v);                 // the id's first vertex
      } else {                                        // another label of an existing id
        if (!g->vmulti[first]) {
          g->multi[first] = {first};
          g->vmulti[first] = 1;
        }
        g->multi[first].push_back(v);
      }
    }
    if (out_vertex) out_vertex[i] = v;
  }
  return EGR_OK;
}

int egr_graph_merge_edges(egr_graph* g, const char* src_blob, const int64_t* src_off,
                          const char* dst_blob, const int64_t* dst_off, const char* type_blob,
                          const int64_t* type_off, int64_t n, int64_t* out_new) {
  if (!g || n < 0 || (n > 0 && (!src_blob || !src_off || !dst_blob || !dst_off || !type_blob || !type_off)))
    return egr::fail(EGR_EINVAL, "egr_graph_merge_edges: bad arguments");
  int64_t created = 0;
  // MATCH never creates vertices: every endpoint id resolves up front, in pipelined batches
  std::vector<int32_t> fs((size_t)n), fd((size_t)n);
  batch_find(g, src_blob, src_off, n, fs.data());
  batch_find(g, dst_blob, dst_off, n, fd.data());
  // the types of the edges whose endpoints both exist (a MATCH that fails names no type), then
  // the MERGE loop with each edge's set slot prefetched PF edges ahead
  std::vector<int8_t> ty((size_t)n, -1);
  for (int64_t i = 0; i < n; ++i) {
    if (fs[(size_t)i] < 0 || fd[(size_t)i] < 0) continue;
    const int t = intern(g->rtypes, str_at(type_blob, type_off, i), 127, "relationship types");
    if (t < 0) return t;
    ty[(size_t)i] = (int8_t)t;
  }
  constexpr int64_t PF = 16;
  for (int64_t i = 0; i < n; ++i) {
    if (i + PF < n) {
      const size_t j = (size_t)(i + PF);
      if (ty[j] >= 0 && !g->vmulti[fs[j]] && !g->vmulti[fd[j]] && !g->eset.empty())
        __builtin_prefetch(&g->eset[(size_t)edge_hash(fs[j], fd[j], ty[j]) & (g->eset.size() - 1)]);
    }
    const int t = ty[(size_t)i];
    if (t < 0) continue;
    const IdVerts sv = verts_of(g, fs[(size_t)i]);
    const IdVerts dv = verts_of(g, fd[(size_t)i]);
    for (size_t a = 0; a < sv.n; ++a)
      for (size_t b = 0; b < dv.n; ++b) {
        const int32_t s = sv.p ? sv.p[a] : sv.one, d = dv.p ? dv.p[b] : dv.one;
        if (eset_insert(g, s, d, t)) {
          g->esrc.push_back(s);
          g->edst.push_back(d);
          g->etype.push_back((uint8_t)t);
          ++created;
        }
      }
  }
  if (out_new) *out_new = created;
  return EGR_OK;
}

int egr_graph_add_edges_indexed(egr_graph* g, const int32_t* src, const int32_t* dst,
                                const char* type_blob, const int64_t* type_off, int32_t n_types,
                                const int32_t* type_idx, int64_t n, int64_t* out_new) {
  if (!g || n < 0 || n_types < 0 || (n_types > 0 && (!type_blob || !type_off)) ||
      (n > 0 && (!src || !dst || !type_idx)))
    return egr::fail(EGR_EINVAL, "egr_graph_add_edges_indexed: bad arguments");
  std::vector<int> tmap((size_t)n_types);
  for (int32_t i = 0; i < n_types; ++i) {
    tmap[i] = intern(g->rtypes, str_at(type_blob, type_off, i), 127, "relationship types");
    if (tmap[i] < 0) return tmap[i];
  }
  const int64_t V = (int64_t)g->vid.size();
  int64_t created = 0;
  for (int64_t i = 0; i < n; ++i) {
    if (src[i] < 0 || src[i] >= V || dst[i] < 0 || dst[i] >= V || type_idx[i] < 0 || type_idx[i] >= n_types)
      return egr::fail(EGR_EINVAL, "egr_graph_add_edges_indexed: vertex or type index out of range");
    const int32_t t = tmap[type_idx[i]];
    if (eset_insert(g, src[i], dst[i], t)) {
      g->esrc.push_back(src[i]);
      g->edst.push_back(dst[i]);
      g->etype.push_back((uint8_t)t);
      ++created;
    }
  }
  if (out_new) *out_new = created;
  return EGR_OK;
}

int64_t egr_graph_num_vertices(const egr_graph* g) { return g ? (int64_t)g->vid.size() : -1; }
int64_t egr_graph_num_edges(const egr_graph* g) { return g ? (int64_t)g->esrc.size() : -1; }
int32_t egr_graph_num_labels(const egr_graph* g) { return g ? (int32_t)g->labels.size() : -1; }
int32_t egr_graph_num_rel_types(const egr_graph* g) { return g ? (int32_t)g->rtypes.size() : -1; }

int64_t egr_graph_label_name(const egr_graph* g, int32_t i, char* buf, int64_t cap) {
  if (!g || i < 0 || i >= (int32_t)g->labels.size()) return -1;
  return copy_out(g->labels[i], buf, cap);
}

int64_t egr_graph_rel_type_name(const egr_graph* g, int32_t i, char* buf, int64_t cap) {
  if (!g || i < 0 || i >= (int32_t)g->rtypes.size()) return -1;
  return copy_out(g->rtypes[i], buf, cap);
}

int64_t egr_graph_vertex_id(const egr_graph* g, int64_t v, char* buf, int64_t cap) {
  if (!g || v < 0 || v >= (int64_t)g->vid.size()) return -1;
  return copy_out(g->vid[v], buf, cap);
}

int egr_graph_lookup(const egr_graph* g, const char* blob, const int64_t* off, int64_t n,
                     int32_t* out_vertex) {
  if (!g || n < 0 || (n > 0 && (!blob || !off || !out_vertex)))
    return egr::fail(EGR_EINVAL, "egr_graph_lookup: bad arguments");
  batch_find(g, blob, off, n, out_vertex);
  return EGR_OK;
}

int egr_graph_lookup_labeled(const egr_graph* g, const char* blob, const int64_t* off, int64_t n,
                             const char* label_blob, const int64_t* label_off, int32_t* out_vertex) {
  if (!g || n < 0 || (n > 0 && (!blob || !off || !label_blob || !label_off || !out_vertex)))
    return egr::fail(EGR_EINVAL, "egr_graph_lookup_labeled: bad arguments");
  batch_find(g, blob, off, n, out_vertex);
  for (int64_t i = 0; i < n; ++i) {
    const IdVerts vs = verts_of(g, out_vertex[i]);
    out_vertex[i] = -1;
    if (!vs.n) continue;
    const std::string_view lab = str_at(label_blob, label_off, i);
    int li = -1;
    for (size_t j = 0; j < g->labels.size() && li < 0; ++j)
      if (g->labels[j] == lab) li = (int)j;
    if (li < 0) continue;
    for (size_t a = 0; a < vs.n; ++a) {
      const int32_t v = vs.p ? vs.p[a] : vs.one;
      if (g->vlabel[(size_t)v] == li) {
        out_vertex[i] = v;
        break;
      }
    }
  }
  return EGR_OK;
}

int32_t egr_graph_find(const egr_graph* g, const char* id, int64_t len) {
  if (!g || len < 0 || (len > 0 && !id)) return -1;
  return idx_find(g, id, (size_t)len);
}

int egr_graph_export(const egr_graph* g, uint8_t* vertex_label, int32_t* edge_src,
                     int32_t* edge_dst, uint8_t* edge_type) {
  if (!g) return egr::fail(EGR_EINVAL, "egr_graph_export: graph is NULL");
  if (vertex_label && !g->vlabel.empty()) memcpy(vertex_label, g->vlabel.data(), g->vlabel.size());
  const size_t E = g->esrc.size();
  if (E) {
    if (edge_src) memcpy(edge_src, g->esrc.data(), E * 4);
    if (edge_dst) memcpy(edge_dst, g->edst.data(), E * 4);
    if (edge_type) memcpy(edge_type, g->etype.data(), E);
  }
  return EGR_OK;
}

int egr_graph_export_edges(const egr_graph* g, int64_t first, int64_t n, int32_t* edge_src,
                           int32_t* edge_dst, uint8_t* edge_type) {
  if (!g || first < 0 || n < 0 || first + n > (int64_t)g->esrc.size())
    return egr::fail(EGR_EINVAL, "egr_graph_export_edges: range outside the edge list");
  if (n == 0) return EGR_OK;
  if (edge_src) memcpy(edge_src, g->esrc.data() + first, (size_t)n * 4);
  if (edge_dst) memcpy(edge_dst, g->edst.data() + first, (size_t)n * 4);
  if (edge_type) memcpy(edge_type, g->etype.data() + first, (size_t)n);
  return EGR_OK;
}

int egr_graph_csr(const egr_graph* g, const float* weights, int32_t n_types, uint32_t* row_ptr,
                  uint32_t* col, uint8_t* meta, float* val) {
  if (!g || !row_ptr || !col || !meta || !val || n_types < 0 || (n_types > 0 && !weights))
    return egr::fail(EGR_EINVAL, "egr_graph_csr: bad arguments");
  const size_t V = g->vid.size(), E = g->esrc.size();
  if (2 * E >= 0xFFFFFFFFull) return egr::fail(EGR_EINVAL, "egr_graph_csr: too many edges for u32 CSR");
  std::vector<uint32_t> cnt(V + 1, 0);
  for (size_t e = 0; e < E; ++e) {
    ++cnt[g->edst[e] + 1];  // dir 0 entry in the target's row
    ++cnt[g->esrc[e] + 1];  // dir 1 entry in the source's row
  }
  for (size_t v = 0; v < V; ++v) cnt[v + 1] += cnt[v];
  memcpy(row_ptr, cnt.data(), (V + 1) * sizeof(uint32_t));
  std::vector<uint64_t> key(2 * E);  // (u << 9 | type << 1 | dir) sorts (u, type, dir)
  std::vector<uint32_t> fill(cnt.begin(), cnt.end() - 1);
  for (size_t e = 0; e < E; ++e) {
    const uint64_t s = (uint32_t)g->esrc[e], d = (uint32_t)g->edst[e], t = g->etype[e];
    key[fill[d]++] = s << 9 | t << 1 | 0u;
    key[fill[s]++] = d << 9 | t << 1 | 1u;
  }
  for (size_t v = 0; v < V; ++v) std::sort(key.begin() + cnt[v], key.begin() + cnt[v + 1]);
  for (size_t i = 0; i < 2 * E; ++i) {
    const uint32_t u = (uint32_t)(key[i] >> 9);
    const uint32_t m = (uint32_t)(key[i] & 0x1FF);
    const uint32_t t = m >> 1, dir = m & 1u;
    const float w = ((int32_t)t < n_types) ? weights[t * 2 + dir] : 1.0f;
    const float deg = (float)(cnt[u + 1] - cnt[u]);
    col[i] = u;
    meta[i] = (uint8_t)m;
    val[i] = w / deg;
  }
  return EGR_OK;
}

}  // extern "C"
