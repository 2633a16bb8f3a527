/*
 * ORACLE (test infrastructure only) -- plain-C CPU restatement of the evidence-graph hot path.
 *
 * Used only by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg, as the checker
 * and the CPU baseline.  Never linked into or called by the product (libegraph.so).
 *
 *   orc_round         CPython round(x, nd): exact decimal formatting + correctly rounded
 *                     parse, the same two steps as Objects/floatobject.c double_round
 *   orc_rules_eval    rules_engine.py:264-455 + hypothesis_ranker.py:44-71 over the encoded
 *                     row columns of include/egraph.h (sequential, row order)
 *   orc_rank          hypothesis_ranker.py:13-80 (stable insertion sort)
 *   orc_reach         apoc.path.subgraphAll(maxLevel) node sets: per-column BFS over the
 *                     undirected graph (neo4j.py:169-202; parity unpinned by the reference,
 *                     pinned by hand-built known-answer graphs in tests/)
 *   orc_propagate     DESIGN.md §A9 (build-defined): s^{h+1}_v = s0_v + sum_e val_e s^h_u,
 *                     fmaf in CSR order, dense; parity pinned bit-for-bit with the GPU
 *   orc_topk          per column: score desc, vertex id asc, over the reach set
 *   orc_frontier      the three above per column over only the vertices the column touches
 *                     (the frontier engine's algorithm on the CPU; bench.py's CPU baseline)
 *
 * Build: oracle/Makefile -> oracle/liboracle.so (gcc, -ffp-contract=off).
 */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "egraph.h"

#ifdef _OPENMP
#include <omp.h>
#endif

double orc_round(double x, int nd) {
  if (isnan(x) || isinf(x) || x == 0.0) return x;
  char buf[400];
  snprintf(buf, sizeof buf, "%.*f", nd, x); /* glibc: exact, round-half-even on the binary value */
  double r = strtod(buf, NULL);
  if (r == 0.0) r = copysign(0.0, x);
  return r;
}

static double pymin(double a, double b) { return (b < a) ? b : a; }

static double final_score(double conf, double w, double support, double strength) {
  double score = conf;
  score *= w;
  if (support > 0) score *= 1 + (pymin(support, 5.0) * 0.05);
  score *= 1 + (strength * 0.2);
  return orc_round(score, 4);
}

static int holds(int type, uint32_t mask, double param, uint32_t flags, uint32_t vocab,
                 int n_node_rows, int max_per_node, double errors, uint32_t network_bit) {
  switch (type) {
    case EGR_C_WAITING_REASON: case EGR_C_TERMINATED_REASON: case EGR_C_LOG_PATTERN:
      return (vocab & mask) != 0;
    case EGR_C_RECENT_DEPLOY: return (flags & EGR_F_RECENT_DEPLOY) != 0;
    case EGR_C_NO_RECENT_DEPLOY: return (flags & EGR_F_RECENT_DEPLOY) == 0;
    case EGR_C_MEMORY_USAGE_HIGH: return (flags & EGR_F_MEMORY_HIGH) != 0;
    case EGR_C_HPA_AT_MAX: return (flags & EGR_F_HPA_AT_MAX) != 0;
    case EGR_C_LATENCY_HIGH: return (flags & EGR_F_LATENCY_HIGH) != 0;
    case EGR_C_NODE_UNHEALTHY: return (flags & EGR_F_NODE_ISSUE) != 0;
    case EGR_C_MULTIPLE_PODS_SAME_NODE: return n_node_rows > 0 && (double)max_per_node >= param;
    case EGR_C_POD_NOT_READY: return (flags & EGR_F_NOT_READY) != 0;
    case EGR_C_READINESS_PROBE_FAILING: return (flags & EGR_F_READINESS_FAIL) != 0;
    case EGR_C_NETWORK_ERRORS_HIGH:
      return errors >= param && network_bit < 32 && ((vocab >> network_bit) & 1u);
    default: return 0;
  }
}

/* outputs mirror egr_rules_out, host arrays */
int orc_rules_eval(const egr_rule_table* T, const uint32_t* flags, const uint32_t* vocab,
                   const uint32_t* node, const double* err, const int64_t* seg_off, int32_t B,
                   uint32_t* out_mask, uint8_t* out_n, uint8_t* out_oc, uint8_t* out_or,
                   double* out_conf, double* out_final, double* out_strength) {
  const int R = T->n_rules, S = R + 1;
  uint32_t* keys = NULL;
  int* counts = NULL;
  int64_t cap = 0;
  for (int32_t i = 0; i < B; ++i) {
    const int64_t b = seg_off[i], e = seg_off[i + 1];
    uint32_t f = 0, v = 0;
    double errors = 0.0;
    int n_node = 0, maxc = 0;
    if (e - b > cap) {
      cap = e - b;
      keys = realloc(keys, cap * sizeof *keys);
      counts = realloc(counts, cap * sizeof *counts);
    }
    int nk = 0;
    for (int64_t r = b; r < e; ++r) {
      f |= flags[r];
      v |= vocab[r];
      errors = errors + err[r];
      if (node[r] != EGR_NO_NODE) {
        ++n_node;
        int j = 0;
        while (j < nk && keys[j] != node[r]) ++j;
        if (j == nk) { keys[nk] = node[r]; counts[nk++] = 0; }
        if (++counts[j] > maxc) maxc = counts[j];
      }
    }
    int matched[EGR_MAX_RULES], nm = 0, ordc[EGR_MAX_RULES + 1], ordr[EGR_MAX_RULES + 1];
    double conf[EGR_MAX_RULES + 1], fin[EGR_MAX_RULES + 1], str[EGR_MAX_RULES + 1];
    uint32_t mask = 0;
    for (int r = 0; r < R; ++r) {
      const egr_rule* ru = &T->rules[r];
      int mc = 0;
      double ss = 0.0;
      for (int c = 0; c < ru->n_conds; ++c)
        if (holds(ru->cond_type[c], ru->cond_mask[c], ru->cond_param[c], f, v, n_node, maxc,
                  errors, T->network_vocab_bit)) {
          ++mc;
          ss += ru->cond_strength[c];
        }
      if (ru->n_conds > 0 && mc == ru->n_conds) {
        str[r] = ss / (double)(ru->n_conds > 1 ? ru->n_conds : 1);
        double cc = ru->confidence_base * 0.6 + str[r] * 0.4;
        if (mc > 2) cc = pymin(cc * 1.1, 0.99);
        conf[r] = orc_round(cc, 3);
        fin[r] = final_score(conf[r], ru->category_weight, (double)mc, str[r]);
        matched[nm++] = r;
        mask |= 1u << r;
      }
    }
    if (nm == 0) {
      conf[R] = T->unknown_confidence;
      str[R] = 0.0;
      fin[R] = final_score(conf[R], T->unknown_category_weight, 0.0, 0.0);
      ordc[0] = ordr[0] = R;
    } else {
      /* list.sort(key=confidence, reverse=True): stable insertion sort */
      for (int k = 0; k < nm; ++k) {
        int x = matched[k], j = k;
        while (j > 0 && conf[ordc[j - 1]] < conf[x]) { ordc[j] = ordc[j - 1]; --j; }
        ordc[j] = x;
      }
      for (int k = 0; k < nm; ++k) {
        int x = ordc[k], j = k;
        while (j > 0 && fin[ordr[j - 1]] < fin[x]) { ordr[j] = ordr[j - 1]; --j; }
        ordr[j] = x;
      }
    }
    const int nh = nm ? nm : 1;
    out_mask[i] = mask;
    out_n[i] = (uint8_t)nh;
    for (int p = 0; p < S; ++p) {
      out_oc[(int64_t)i * S + p] = p < nh ? (uint8_t)ordc[p] : 0xFF;
      out_or[(int64_t)i * S + p] = p < nh ? (uint8_t)ordr[p] : 0xFF;
    }
    for (int p = 0; p < nh; ++p) {
      int s = ordc[p];
      out_conf[(int64_t)i * S + s] = conf[s];
      out_final[(int64_t)i * S + s] = fin[s];
      out_strength[(int64_t)i * S + s] = str[s];
    }
  }
  free(keys);
  free(counts);
  return 0;
}

int orc_rank(const double* conf, const double* w, const double* sup, const double* str,
             const int64_t* off, int32_t n_lists, double* out_final, int32_t* out_order) {
  for (int32_t l = 0; l < n_lists; ++l) {
    const int64_t b = off[l], n = off[l + 1] - off[l];
    for (int64_t i = 0; i < n; ++i) out_final[b + i] = final_score(conf[b + i], w[b + i], sup[b + i], str[b + i]);
    for (int64_t k = 0; k < n; ++k) {
      int64_t j = k;
      while (j > 0 && out_final[b + out_order[b + j - 1]] < out_final[b + k]) {
        out_order[b + j] = out_order[b + j - 1];
        --j;
      }
      out_order[b + j] = (int32_t)k;
    }
  }
  return 0;
}

/* reach bits [ceil(B/64)][V]: BFS from src[b] to depth `hops` over the symmetric CSR */
int orc_reach(const uint32_t* row_ptr, const uint32_t* col, int64_t V, const uint32_t* src,
              int32_t B, int32_t hops, uint64_t* out, int threads) {
  const int W = (B + 63) / 64;
  memset(out, 0, (size_t)W * V * 8);
#ifdef _OPENMP
  if (threads > 0) omp_set_num_threads(threads);
#pragma omp parallel
#endif
  {
    int* depth = malloc(V * sizeof(int));
    uint32_t* queue = malloc(V * sizeof(uint32_t));
#ifdef _OPENMP
#pragma omp for schedule(dynamic)
#endif
    for (int w = 0; w < W; ++w) { /* one thread owns a whole 64-column word */
      for (int32_t b = w * 64; b < B && b < w * 64 + 64; ++b) {
        if (src[b] >= (uint64_t)V) continue;
        for (int64_t v = 0; v < V; ++v) depth[v] = -1;
        int64_t qh = 0, qt = 0;
        queue[qt++] = src[b];
        depth[src[b]] = 0;
        while (qh < qt) {
          const uint32_t v = queue[qh++];
          out[(size_t)w * V + v] |= 1ull << (b % 64);
          if (depth[v] == hops) continue;
          for (uint32_t e = row_ptr[v]; e < row_ptr[v + 1]; ++e)
            if (depth[col[e]] < 0) {
              depth[col[e]] = depth[v] + 1;
              queue[qt++] = col[e];
            }
        }
      }
    }
    free(depth);
    free(queue);
  }
  return 0;
}

/* scores out [V][B] row-major after `hops` hops; seeds max-combined per (v, b) */
int orc_propagate(const uint32_t* row_ptr, const uint32_t* col, const float* val, int64_t V,
                  const uint32_t* seed_v, const uint32_t* seed_c, const float* seed_s,
                  int64_t n_seeds, int32_t B, int32_t hops, float* out, int threads) {
  const size_t n = (size_t)V * B;
  float* s0 = calloc(n, sizeof(float));
  float* cur = calloc(n, sizeof(float));
  if (!s0 || !cur) { free(s0); free(cur); return -3; }
  unsigned char* has = calloc(n, 1);
  for (int64_t i = 0; i < n_seeds; ++i) {
    if (seed_v[i] >= (uint64_t)V || seed_c[i] >= (uint32_t)B) continue;
    const size_t k = (size_t)seed_v[i] * B + seed_c[i];
    if (!has[k] || seed_s[i] > s0[k]) s0[k] = seed_s[i];
    has[k] = 1;
  }
  free(has);
  memcpy(cur, s0, n * sizeof(float));
#ifdef _OPENMP
  if (threads > 0) omp_set_num_threads(threads);
#endif
  for (int h = 0; h < hops; ++h) {
#ifdef _OPENMP
#pragma omp parallel for schedule(dynamic, 256)
#endif
    for (int64_t v = 0; v < V; ++v) {
      for (int32_t b = 0; b < B; ++b) {
        float acc = 0.0f;
        for (uint32_t e = row_ptr[v]; e < row_ptr[v + 1]; ++e)
          acc = fmaf(val[e], cur[(size_t)col[e] * B + b], acc);
        out[(size_t)v * B + b] = acc + s0[(size_t)v * B + b];
      }
    }
    memcpy(cur, out, n * sizeof(float));
  }
  if (hops == 0) memcpy(out, s0, n * sizeof(float));
  free(s0);
  free(cur);
  return 0;
}

/* one hop of the same recurrence on given inputs (the partitioned-graph protocol tests):
 * out[v][b] = fmaf-chain over row v of val_e * xin[col_e][b], then + s0[v][b]              */
int orc_hop_step(const uint32_t* row_ptr, const uint32_t* col, const float* val, int64_t V,
                 int32_t B, const float* xin, const float* s0, float* out) {
  for (int64_t v = 0; v < V; ++v) {
    for (int32_t b = 0; b < B; ++b) {
      float acc = 0.0f;
      for (uint32_t e = row_ptr[v]; e < row_ptr[v + 1]; ++e)
        acc = fmaf(val[e], xin[(size_t)col[e] * B + b], acc);
      out[(size_t)v * B + b] = acc + s0[(size_t)v * B + b];
    }
  }
  return 0;
}

typedef struct { float s; uint32_t v; } cand;

static int cand_cmp(const void* a, const void* b) {
  const cand* x = a;
  const cand* y = b;
  if (x->s > y->s) return -1;
  if (x->s < y->s) return 1;
  return (x->v < y->v) ? -1 : (x->v > y->v);
}

int orc_topk(const float* scores, int64_t V, int32_t B, const uint64_t* reach,
             const uint8_t* vlabel, int32_t exclude_label, int32_t k, uint32_t* out_ids,
             float* out_scores) {
  cand* c = malloc(V * sizeof(cand));
  for (int32_t b = 0; b < B; ++b) {
    int64_t n = 0;
    for (int64_t v = 0; v < V; ++v) {
      if (!((reach[(size_t)(b / 64) * V + v] >> (b % 64)) & 1u)) continue;
      if (exclude_label >= 0 && vlabel[v] == (uint8_t)exclude_label) continue;
      c[n].s = scores[(size_t)v * B + b];
      c[n].v = (uint32_t)v;
      ++n;
    }
    qsort(c, n, sizeof(cand), cand_cmp);
    for (int32_t q = 0; q < k; ++q) {
      out_ids[(size_t)b * k + q] = q < n ? c[q].v : EGR_NO_NODE;
      out_scores[(size_t)b * k + q] = q < n ? c[q].s : -INFINITY;
    }
  }
  free(c);
  return 0;
}

/* ---- orc_frontier: the same results per column, touching only what the column touches -----
 * The CPU form of the frontier engine's algorithm (csrc/frontier.hip), used as the honest CPU
 * baseline of bench.py (the dense orc_propagate sweeps V x B per hop although > 99 % of the
 * values are exact zeros) and as a checker at sizes where the dense [V][B] arrays are large.
 * Per column b, with per-thread dense scratch reset through touched lists:
 *   T_0 = seeds, cur = s0 (max-combined as orc_propagate)
 *   hop h: U = seeds + neighbours of every u in T_h with cur[u] != 0; for v in U the chain
 *          acc = fmaf(val_e, cur[col_e], acc) over row v in CSR order, then acc + s0[v] --
 *          the SAME arithmetic as orc_propagate on the same dense values (cur is exact zero
 *          outside T_h); every other vertex is exactly 0 in the dense recurrence too.
 *   reach: BFS from src[b] to depth `hops` (orc_reach); top-k over it as orc_topk.
 *   prune: the last hop computes only the reach set's members (the engine's pruned last
 *          pull): the scores top-k reads are unchanged, the others are never read.
 * Bit-identical to orc_propagate + orc_reach + orc_topk (tests/test_oracle_frontier.py).
 * work_out (optional, [2]): CSR entries read by the hop chains, rows walked.              */
typedef struct { uint32_t v; float s; } seedent;

static int cand_better(float s, uint32_t v, float s2, uint32_t v2) {
  return s > s2 || (s == s2 && v < v2);
}

int orc_frontier(const uint32_t* row_ptr, const uint32_t* col, const float* val,
                 const uint8_t* vlabel, int64_t V, const uint32_t* seed_v, const uint32_t* seed_c,
                 const float* seed_s, int64_t n_seeds, const uint32_t* src, int32_t B,
                 int32_t hops, int32_t exclude_label, int32_t k, int prune, uint32_t* out_ids,
                 float* out_scores, int64_t* work_out, int threads) {
  /* seeds grouped by column (counting sort; invalid triples dropped) */
  int64_t* ptr = calloc((size_t)B + 1, sizeof(int64_t));
  seedent* grp = malloc((size_t)(n_seeds > 0 ? n_seeds : 1) * sizeof(seedent));
  if (!ptr || !grp) { free(ptr); free(grp); return -3; }
  for (int64_t i = 0; i < n_seeds; ++i)
    if (seed_v[i] < (uint64_t)V && seed_c[i] < (uint32_t)B) ++ptr[seed_c[i] + 1];
  for (int32_t b = 0; b < B; ++b) ptr[b + 1] += ptr[b];
  {
    int64_t* cur = malloc((size_t)B * sizeof(int64_t));
    memcpy(cur, ptr, (size_t)B * sizeof(int64_t));
    for (int64_t i = 0; i < n_seeds; ++i)
      if (seed_v[i] < (uint64_t)V && seed_c[i] < (uint32_t)B) {
        grp[cur[seed_c[i]]].v = seed_v[i];
        grp[cur[seed_c[i]]++].s = seed_s[i];
      }
    free(cur);
  }
  int64_t w_entries = 0, w_rows = 0;
#ifdef _OPENMP
  if (threads > 0) omp_set_num_threads(threads);
#pragma omp parallel reduction(+ : w_entries, w_rows)
#endif
  {
    float* cur = calloc((size_t)V, sizeof(float));
    float* s0 = calloc((size_t)V, sizeof(float));
    uint8_t* has = calloc((size_t)V, 1);
    uint32_t* mark = calloc((size_t)V, sizeof(uint32_t));    /* generation stamps */
    int* depth = malloc((size_t)V * sizeof(int));
    uint32_t* T = malloc((size_t)V * sizeof(uint32_t));
    uint32_t* U = malloc((size_t)V * sizeof(uint32_t));
    float* nv = malloc((size_t)V * sizeof(float));
    uint32_t* sd = malloc((size_t)V * sizeof(uint32_t));
    uint32_t* queue = malloc((size_t)V * sizeof(uint32_t));
    uint32_t gen = 0;
    for (int64_t v = 0; v < V; ++v) depth[v] = -1;
#ifdef _OPENMP
#pragma omp for schedule(dynamic, 4)
#endif
    for (int32_t b = 0; b < B; ++b) {
      /* s0: max-combine the column's seeds */
      int64_t nsd = 0;
      for (int64_t i = ptr[b]; i < ptr[b + 1]; ++i) {
        const uint32_t v = grp[i].v;
        if (!has[v]) { has[v] = 1; s0[v] = grp[i].s; sd[nsd++] = v; }
        else if (grp[i].s > s0[v]) s0[v] = grp[i].s;
      }
      /* the reach set of the incident vertex first (BFS to depth `hops`): with `prune` the
       * last hop computes only its members, the only scores top-k reads */
      int64_t qh = 0, qt = 0;
      if (src[b] < (uint64_t)V) {
        queue[qt++] = src[b];
        depth[src[b]] = 0;
      }
      while (qh < qt) {
        const uint32_t v = queue[qh++];
        if (depth[v] == hops) continue;
        for (uint32_t e = row_ptr[v]; e < row_ptr[v + 1]; ++e)
          if (depth[col[e]] < 0) {
            depth[col[e]] = depth[v] + 1;
            queue[qt++] = col[e];
          }
      }
      int64_t nT = 0;
      for (int64_t i = 0; i < nsd; ++i) { cur[sd[i]] = s0[sd[i]]; T[nT++] = sd[i]; }
      for (int32_t h = 0; h < hops; ++h) {
        const int last_pruned = prune && h == hops - 1;
        ++gen;
        int64_t nU = 0;
        for (int64_t i = 0; i < nsd; ++i)
          if (mark[sd[i]] != gen) { mark[sd[i]] = gen; U[nU++] = sd[i]; }
        for (int64_t i = 0; i < nT; ++i) {
          const uint32_t u = T[i];
          if (cur[u] == 0.0f) continue;
          for (uint32_t e = row_ptr[u]; e < row_ptr[u + 1]; ++e)
            if (mark[col[e]] != gen) { mark[col[e]] = gen; U[nU++] = col[e]; }
        }
        int64_t nW = 0;
        for (int64_t i = 0; i < nU; ++i) {
          const uint32_t v = U[i];
          if (last_pruned && depth[v] < 0) continue;   /* outside the reach set: never read */
          float acc = 0.0f;
          for (uint32_t e = row_ptr[v]; e < row_ptr[v + 1]; ++e) acc = fmaf(val[e], cur[col[e]], acc);
          w_entries += row_ptr[v + 1] - row_ptr[v];
          ++w_rows;
          nv[nW] = acc + s0[v];
          U[nW++] = v;
        }
        for (int64_t i = 0; i < nT; ++i) cur[T[i]] = 0.0f;
        for (int64_t i = 0; i < nW; ++i) { cur[U[i]] = nv[i]; T[i] = U[i]; }
        nT = nW;
      }
      /* top-k over the reach set */
      uint32_t* ids = out_ids + (size_t)b * k;
      float* scs = out_scores + (size_t)b * k;
      int32_t nk = 0;
      for (int64_t i = 0; i < qt; ++i) {
        const uint32_t v = queue[i];
        if (exclude_label >= 0 && vlabel[v] == (uint8_t)exclude_label) continue;
        const float s = cur[v];
        if (nk < k || cand_better(s, v, scs[nk - 1], ids[nk - 1])) {
          int32_t j = nk < k ? nk++ : k - 1;
          while (j > 0 && cand_better(s, v, scs[j - 1], ids[j - 1])) {
            scs[j] = scs[j - 1];
            ids[j] = ids[j - 1];
            --j;
          }
          scs[j] = s;
          ids[j] = v;
        }
      }
      for (int64_t i = 0; i < qt; ++i) depth[queue[i]] = -1;
      for (int32_t q = nk; q < k; ++q) {
        ids[q] = EGR_NO_NODE;
        scs[q] = -INFINITY;
      }
      /* reset the scratch this column touched */
      for (int64_t i = 0; i < nT; ++i) cur[T[i]] = 0.0f;
      for (int64_t i = 0; i < nsd; ++i) { has[sd[i]] = 0; s0[sd[i]] = 0.0f; }
    }
    free(cur); free(s0); free(has); free(mark); free(depth); free(T); free(U); free(nv);
    free(sd); free(queue);
  }
  if (work_out) {
    work_out[0] = w_entries;
    work_out[1] = w_rows;
  }
  free(ptr);
  free(grp);
  return 0;
}
