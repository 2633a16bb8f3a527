/*
 * egraph.h -- C-ABI of libegraph.so, the MI355X (gfx950) evidence-graph correlation engine.
 *
 * Drop-in boundary for the reference's hot path (ShreyashDarade/Kubernetes-AIOps-Evidence-Graph).
 * Plain C: pointers, sizes, status codes.  No torch / HIP types appear in any signature;
 * `stream` arguments are hipStream_t passed as void* (NULL = the null stream).
 * Device pointers are caller-owned (e.g. torch tensors) and are never retained past a call;
 * egr_snapshot / egr_plan own the device buffers they allocate.
 *
 * Reference interfaces each group replaces (paths relative to the reference repo):
 *   egr_rules_eval  <- RulesEngine.generate_hypotheses   src/services/rca/rules_engine.py:199-233
 *                      (+ _extract_signals :264-376, _match_rule :378-397, _check_condition :399-441,
 *                         _calculate_confidence :443-455, unknown fallback :457-478)
 *                      fused with HypothesisRanker.rank  src/services/rca/hypothesis_ranker.py:13-80
 *   egr_rank        <- HypothesisRanker.rank             src/services/rca/hypothesis_ranker.py:13-80
 *   egr_graph_*     <- GraphService.create_entities_batch / create_relations_batch
 *                                                        src/database/neo4j.py:95-113, :145-167
 *   egr_snapshot_*  <- the Neo4j store the Cypher queries read (docker-compose.yml:26-33)
 *   egr_plan_reach* <- GraphService.get_incident_graph -> apoc.path.subgraphAll(maxLevel=3)
 *                                                        src/database/neo4j.py:169-202
 *   egr_plan_hop / egr_plan_topk
 *                   <- build-defined typed k-hop propagation + per-incident top-k (no reference
 *                      counterpart; spec in DESIGN.md §A9)
 *
 * Every function returns EGR_OK (0) or a negative status; egr_last_error() describes the
 * last failure on the calling thread.
 */
#ifndef EGRAPH_H_
#define EGRAPH_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define EGR_OK 0
#define EGR_EINVAL (-1)   /* bad argument (Python shim raises ValueError) */
#define EGR_EDEVICE (-2)  /* HIP runtime / kernel failure (shim raises RuntimeError) */
#define EGR_ENOMEM (-3)   /* allocation failure */
#define EGR_ESTATE (-4)   /* object used in the wrong state */

#define EGR_VERSION 1

const char* egr_last_error(void);
int egr_version(void);

/* Pinned host memory mapped into the GPU address space (hipHostMalloc mapped + coherent):
 * *host is the CPU address, *dev the address kernels use.  The drop-in's small launches read
 * their inputs from and write their results to it directly (no DMA copies; egraph/batcher.py,
 * egraph/ranker.py).  Free with egr_host_free.                                              */
int egr_host_alloc(int64_t bytes, void** host, void** dev);
int egr_host_free(void* host);
/* Number of HIP devices visible (0 on a GPU-less host; never fails). */
int egr_device_count(void);

/* ------------------------------------------------------------------------------------------
 * Rules (A1-A6).  Evidence rows are pre-encoded per row by the host encoder into 20 bytes:
 *   row_flags  u32  EGR_F_* bits below (per-row predicates, rules_engine.py:315-376)
 *   row_vocab  u32  bit i set = the row's waiting reason / terminated reason / log pattern is
 *                   vocabulary entry i (vocabulary built from the rule table's value lists)
 *   row_node   u32  pods_by_node key of the row (rules_engine.py:323-330), EGR_NO_NODE if the
 *                   row does not count
 *   row_err    f64  log error_count contribution (rules_engine.py:354); integral unless
 *                   EGR_F_ERR_FLOAT is set (then the segment is summed in row order)
 * Incident i owns rows [seg_off[i], seg_off[i+1]).
 * ---------------------------------------------------------------------------------------- */
#define EGR_F_RECENT_DEPLOY   (1u << 0)  /* deploy_change: is_recent_change truthy         :342 */
#define EGR_F_IMAGE_CHANGED   (1u << 1)  /* image_change: image_changed truthy             :347 */
#define EGR_F_MEMORY_HIGH     (1u << 2)  /* metric: memory & anomalous & current > 90      :360 */
#define EGR_F_HPA_AT_MAX      (1u << 3)  /* metric: hpa & max & current == 1               :365 */
#define EGR_F_LATENCY_HIGH    (1u << 4)  /* metric: latency & current > 1                  :368 */
#define EGR_F_NODE_ISSUE      (1u << 5)  /* kubernetes_node: Ready.status != "True"        :375 */
#define EGR_F_NOT_READY       (1u << 6)  /* pod: Ready cond != "True" and phase Running    :335 */
#define EGR_F_READINESS_FAIL  (1u << 7)  /* ... and reason == "ContainersNotReady"        :337 */
#define EGR_F_ERR_FLOAT       (1u << 8)  /* row_err holds a non-integral value              */
#define EGR_NO_NODE 0xFFFFFFFFu

/* condition type codes (rules_engine.py:403-434) */
enum egr_cond {
  EGR_C_WAITING_REASON = 0, EGR_C_TERMINATED_REASON = 1, EGR_C_RECENT_DEPLOY = 2,
  EGR_C_NO_RECENT_DEPLOY = 3, EGR_C_MEMORY_USAGE_HIGH = 4, EGR_C_HPA_AT_MAX = 5,
  EGR_C_LATENCY_HIGH = 6, EGR_C_LOG_PATTERN = 7, EGR_C_NODE_UNHEALTHY = 8,
  EGR_C_MULTIPLE_PODS_SAME_NODE = 9, EGR_C_POD_NOT_READY = 10, EGR_C_READINESS_PROBE_FAILING = 11,
  EGR_C_NETWORK_ERRORS_HIGH = 12, EGR_C_UNSUPPORTED = -1
};

#define EGR_MAX_RULES 32
#define EGR_MAX_CONDS 4

typedef struct egr_rule {
  int32_t n_conds;                        /* 0 => never matches (rules_engine.py:390) */
  int32_t cond_type[EGR_MAX_CONDS];       /* enum egr_cond */
  uint32_t cond_mask[EGR_MAX_CONDS];      /* vocab bits for set-intersection conditions */
  double cond_param[EGR_MAX_CONDS];       /* threshold for types 9 and 12 */
  double cond_strength[EGR_MAX_CONDS];    /* fixed per type, rules_engine.py:404-433 */
  double confidence_base;                 /* rules_engine.py:26 etc. */
  double category_weight;                 /* hypothesis_ranker.py:28-40 (1.0 if absent) */
} egr_rule;

typedef struct egr_rule_table {
  int32_t n_rules;                        /* <= EGR_MAX_RULES, evaluation order = list order */
  uint32_t network_vocab_bit;             /* vocab bit of the literal "network" (:431) */
  double unknown_confidence;              /* 0.3 (rules_engine.py:465) */
  double unknown_category_weight;         /* weight of "unknown" (0.5) */
  egr_rule rules[EGR_MAX_RULES];
} egr_rule_table;

/* Per-incident outputs; R = table->n_rules, slot R = the "unknown" hypothesis.
 *   n_hyp[i]                 number of hypotheses (>= 1)
 *   mask[i]                  bit r = rule r matched
 *   order_conf[i*(R+1)+p]    slot index at position p in generate_hypotheses order (:228)
 *   order_rank[i*(R+1)+p]    slot index at position p after HypothesisRanker.rank (:67)
 *   confidence / final_score / strength [i*(R+1)+slot]  (float64, bit-exact with Python;
 *                            every slot is written: 0 for rules that did not match)       */
typedef struct egr_rules_out {
  uint32_t* mask;
  uint8_t* n_hyp;
  uint8_t* order_conf;
  uint8_t* order_rank;
  double* confidence;
  double* final_score;
  double* strength;
} egr_rules_out;

int egr_rules_eval(const egr_rule_table* table, const uint32_t* row_flags, const uint32_t* row_vocab,
                   const uint32_t* row_node, const double* row_err, const int64_t* seg_off,
                   int32_t n_incidents, const egr_rules_out* out, void* stream);

/* egr_rules_eval with its staging in the same call (the drop-in's low-latency launches,
 * egraph/batcher.py): [0, in_bytes) of the pinned host_in buffer is copied to dev_buf, the
 * kernel runs on the device copy -- off[12] = byte offsets, identical in both buffers, of
 * row_flags, row_vocab, row_node, row_err, seg_off, mask, n_hyp, order_conf, order_rank,
 * confidence, final_score, strength -- and [out_lo, out_hi) is copied back into host_out.
 * Asynchronous on `stream` (record an event to wait).                                      */
int egr_rules_eval_staged(const egr_rule_table* table, const void* host_in, void* dev_buf,
                          void* host_out, const int64_t* off, int64_t in_bytes, int64_t out_lo,
                          int64_t out_hi, int32_t n_incidents, void* stream);

/* egr_rules_eval for ONE incident of at most 128 rows whose row columns are HOST arrays: the
 * rows are copied into the kernel's argument block (no DMA copy, no PCIe reads by the kernel);
 * the outputs (one incident: mask[1], n_hyp[1], S-slot arrays) go to `out`, typically mapped
 * host memory (egr_host_alloc).  The drop-in's single generate_hypotheses calls.          */
int egr_rules_eval_small(const egr_rule_table* table, const uint32_t* row_flags,
                         const uint32_t* row_vocab, const uint32_t* row_node, const double* row_err,
                         int32_t n_rows, const egr_rules_out* out, void* stream);

/* The single-incident rules server: egr_rules_eval_small's job without a kernel launch per
 * call.  A one-wave kernel stays resident while calls keep coming, polling a mailbox in
 * mapped coherent host memory; post() writes one incident's encoded rows (at most 1024, host
 * arrays) and returns at once; poll() returns 1 once the incident's outputs are ready and
 * copies them into the caller's arrays (mask[1], n_hyp[1], S = n_rules + 1 slots each, the
 * layout of egr_rules_eval's outputs), 0 while pending -- and starts the wave again when it
 * has left (it leaves after ~2 ms without a request, ~2 s in all, or at free(); a
 * device-wide synchronize waits for it meanwhile).  One
 * incident in flight per server; post() refuses (EGR_ESTATE) while one is pending.  Same
 * outputs as egr_rules_eval, bit for bit (the same per-incident device code).  The drop-in's
 * idle generate_hypotheses calls (activities.py:124-170, one incident per activity).
 * Contract: a handle is single-caller -- post() and poll() from one thread at a time (its
 * sequence number is a plain counter).  The wave clears its `alive` word as it leaves with no
 * handshake: a post() or poll() that races that exit can queue one redundant wave behind the
 * leaving one (it idles ~2 ms and leaves) -- a wasted launch, never a wrong or lost answer,
 * since every wave starts from the last acknowledged request.  A request that is never
 * acknowledged (a wave that faulted) leaves post() refusing with EGR_ESTATE: the caller bounds
 * its wait on poll() and replaces the handle (egraph/batcher.py: _ServerWait, 5 s). */
typedef struct egr_rules_server egr_rules_server;
int egr_rules_server_create(const egr_rule_table* table, int32_t device, egr_rules_server** out);
int egr_rules_server_post(egr_rules_server* s, const uint32_t* row_flags, const uint32_t* row_vocab,
                          const uint32_t* row_node, const double* row_err, int32_t n_rows);
int egr_rules_server_poll(egr_rules_server* s, uint32_t* mask, uint8_t* n_hyp, uint8_t* order_conf,
                          uint8_t* order_rank, double* confidence, double* final_score,
                          double* strength);
void egr_rules_server_free(egr_rules_server* s);

/* Ranker (A6) over arbitrary hypothesis lists.  List j owns entries [list_off[j], list_off[j+1]).
 *   score = confidence * cat_weight; if support > 0: *= 1 + min(support,5)*0.05;
 *   *= 1 + strength*0.2; final = round(score, 4); stable sort descending.
 * out_order[list_off[j]+p] = index (within list j) of the entry ranked p+1.                */
int egr_rank(const double* confidence, const double* cat_weight, const double* support,
             const double* strength, const int64_t* list_off, int32_t n_lists,
             double* out_final, int32_t* out_order, void* stream);

/* Python-exact round(x, ndigits) for ndigits in [0, 15] (host; used by the CPU test suite to
 * pin the device implementation, which is the same source). */
double egr_py_round(double x, int32_t ndigits);

/* ------------------------------------------------------------------------------------------
 * Evidence graph (A7): host-side MERGE semantics of GraphService (neo4j.py:95-167).
 * Strings are passed as one byte blob plus n+1 int64 offsets (UTF-8, not NUL-terminated).
 * ---------------------------------------------------------------------------------------- */
typedef struct egr_graph egr_graph;

int egr_graph_create(egr_graph** out);
void egr_graph_free(egr_graph* g);
/* MERGE (n:label {id}) per item, in order.  out_vertex[i] (optional) = vertex index. */
int egr_graph_merge_nodes(egr_graph* g, const char* id_blob, const int64_t* id_off,
                          const char* label_blob, const int64_t* label_off, int64_t n,
                          int32_t* out_vertex);
/* MATCH (s {id}) MATCH (t {id}) MERGE (s)-[:type]->(t) per item, in order.  Label-less match:
 * every vertex carrying the id takes part; a missing endpoint drops the item silently.
 * *out_new (optional) = number of edges actually created.                                 */
int egr_graph_merge_edges(egr_graph* g, const char* src_blob, const int64_t* src_off,
                          const char* dst_blob, const int64_t* dst_off, const char* type_blob,
                          const int64_t* type_off, int64_t n, int64_t* out_new);
int64_t egr_graph_num_vertices(const egr_graph* g);
int64_t egr_graph_num_edges(const egr_graph* g);
int32_t egr_graph_num_labels(const egr_graph* g);
int32_t egr_graph_num_rel_types(const egr_graph* g);
/* name of label / relationship-type `i`; returns length, copies up to cap bytes */
int64_t egr_graph_label_name(const egr_graph* g, int32_t i, char* buf, int64_t cap);
int64_t egr_graph_rel_type_name(const egr_graph* g, int32_t i, char* buf, int64_t cap);
int64_t egr_graph_vertex_id(const egr_graph* g, int64_t v, char* buf, int64_t cap);
/* first vertex (lowest index) whose id equals each query id, -1 if none */
int egr_graph_lookup(const egr_graph* g, const char* blob, const int64_t* off, int64_t n,
                     int32_t* out_vertex);
/* MATCH (n:label {id: $id}) for n ids: the vertex carrying each id under its label (labels as a
 * blob + offsets, one per id), -1 if none (neo4j.py:169-202's incident MATCH, the GraphService
 * incident lookups; replaces a host dict mirror of every (label, id) pair). */
int egr_graph_lookup_labeled(const egr_graph* g, const char* blob, const int64_t* off, int64_t n,
                             const char* label_blob, const int64_t* label_off, int32_t* out_vertex);
/* egr_graph_lookup of ONE id given as bytes (len bytes, not NUL-terminated): the first vertex
 * carrying it, -1 if none (or bad arguments).  Read-only: safe from several threads at once
 * while no merge runs (the native seed attachment calls it from its worker threads; the
 * reference resolves these ids with Cypher MATCH ... {id: $id}, src/database/neo4j.py:145-167). */
int32_t egr_graph_find(const egr_graph* g, const char* id, int64_t len);
/* vertex labels [V] and edge list (src, dst, type) [E] in creation order */
int egr_graph_export(const egr_graph* g, uint8_t* vertex_label, int32_t* edge_src,
                     int32_t* edge_dst, uint8_t* edge_type);
/* Host copy of the symmetric typed CSR the snapshot uploads:
 * row v lists (u, meta = type<<1 | dir) for every edge touching v, sorted by (u, type, dir);
 * dir 0: edge u->v, dir 1: edge v->u.  val[e] = weight[type*2+dir] / deg(u) (fp32).
 * Sizes: row_ptr [V+1], col/meta/val [2E].  weights: [n_types*2], n_types may be smaller
 * than the graph's type count (missing types weigh 1.0).                                    */
int egr_graph_csr(const egr_graph* g, const float* weights, int32_t n_types, uint32_t* row_ptr,
                  uint32_t* col, uint8_t* meta, float* val);

/* ------------------------------------------------------------------------------------------
 * Snapshot: the CSR + node tables resident in HBM on one device.
 * ---------------------------------------------------------------------------------------- */
typedef struct egr_snapshot egr_snapshot;

int egr_snapshot_create(const egr_graph* g, const float* weights, int32_t n_types, int32_t device,
                        egr_snapshot** out);
void egr_snapshot_free(egr_snapshot* s);
int egr_snapshot_info(const egr_snapshot* s, int64_t* n_vertices, int64_t* n_entries);

/* ------------------------------------------------------------------------------------------
 * Plan: per-batch workspace for B incident columns on a snapshot (all device memory is
 * allocated here, none in the launch functions, so a step can be captured into a hipGraph).
 *   scores: fp32, tiled [B/TW][V][TW] with TW = 128 (B >= 128), 64, 16 or 4
 *           ($EGRAPH_TILE_WIDTH caps TW).
 *   reach : u64 bitsets, bit b%64 of word b/64 of vertex v = v within `hops` of the
 *           incident vertex of column b (undirected, all types: apoc.path.subgraphAll);
 *           held row-major (one vertex's words contiguous), exported as [ceil(B/64)][V].
 * n_cols <= EGR_MAX_COLS.
 * ---------------------------------------------------------------------------------------- */
typedef struct egr_plan egr_plan;
#define EGR_MAX_COLS 8192

int egr_plan_create(const egr_snapshot* s, int32_t n_cols, int64_t max_seeds, int32_t k,
                    egr_plan** out);
void egr_plan_free(egr_plan* p);
int egr_plan_tile_width(const egr_plan* p);
/* the vertex count of the plan's snapshot and the plan's column count: the shape of the dense
 * score array egr_plan_read_scores writes ([V][n_cols]) and of the reach bits egr_plan_read_reach
 * writes ([ceil(n_cols/64)][V]); callers size their outputs by it */
int egr_plan_shape(const egr_plan* p, int64_t* n_vertices, int32_t* n_cols);
/* Seeds s0[v, b] = max over triples (seed_vertex, seed_col, seed_val) (device arrays). */
int egr_plan_set_seeds(egr_plan* p, const uint32_t* seed_vertex, const uint32_t* seed_col,
                       const float* seed_val, int64_t n_seeds, void* stream);
/* Incident vertex per column (device array [n_cols]; EGR_NO_NODE = empty column).          */
int egr_plan_set_sources(egr_plan* p, const uint32_t* source_vertex, void* stream);
/* One propagation hop: s^{h+1}_v = s0_v + sum_{(u,t,d) in row v} val * s^h_u.               */
int egr_plan_hop(egr_plan* p, void* stream);
/* One reachability hop over the undirected graph.                                          */
int egr_plan_reach_hop(egr_plan* p, void* stream);
/* One hop of both recurrences (egr_plan_hop then egr_plan_reach_hop).                       */
int egr_plan_step(egr_plan* p, void* stream);
/* The last hop: egr_plan_step plus the top-k candidate lists (reached vertices whose label
 * is not exclude_label, per column, in vertex order), so egr_plan_topk with the same
 * exclude_label reads only the candidates instead of rescanning every score.  (Plans whose
 * worst-case lists, V*n_cols*4 B, exceed 16 GiB skip the lists and top-k rescans.)          */
int egr_plan_final_step(egr_plan* p, int32_t exclude_label, void* stream);
/* The candidate lists of egr_plan_final_step alone, from the current reach sets (for callers
 * that run the hops themselves).                                                            */
int egr_plan_candidates(egr_plan* p, int32_t exclude_label, void* stream);
/* Per column: top-k vertices by final score (desc), vertex id asc on ties, over the reach
 * set excluding vertices whose label is `exclude_label` (-1: none).  Outputs [n_cols*k];
 * unused slots hold EGR_NO_NODE / -inf.                                                     */
int egr_plan_topk(egr_plan* p, int32_t exclude_label, uint32_t* out_ids, float* out_scores,
                  void* stream);
/* Whole pass: seeds/sources must be set; runs `hops` of both recurrences then top-k.       */
int egr_plan_run(egr_plan* p, int32_t hops, int32_t exclude_label, uint32_t* out_ids,
                 float* out_scores, void* stream);
/* Copies (device->device) of the current state, for inspection and tests.
 * scores out: row-major [V][n_cols]; reach out: [ceil(n_cols/64)][V].                       */
int egr_plan_read_scores(const egr_plan* p, float* out, void* stream);
int egr_plan_read_reach(const egr_plan* p, uint64_t* out, void* stream);

/* Stand-alone top-k over explicit dense arrays (csrc/topk.hip; torch.ops.egraph.topk).
 * scores row-major [V][n_cols] fp32, reach [ceil(n_cols/64)][V] u64 bits (the layouts of
 * egr_plan_read_scores / egr_plan_read_reach, V = the snapshot's vertex count); per column
 * the k best reached vertices whose label != exclude_label (-1: none excluded), score
 * descending, vertex id ascending; out [n_cols*k], EGR_NO_NODE / -inf padded.  The engines'
 * own top-k (egr_plan_topk, egr_frontier_run) produce the same lists from their state.      */
int egr_topk(const egr_snapshot* s, const float* scores, const uint64_t* reach, int32_t n_cols,
             int32_t k, int32_t exclude_label, uint32_t* out_ids, float* out_scores, void* stream);
/* Induced subgraph of one column's reach set (get_incident_graph "relationships",
 * neo4j.py:193-200): every edge whose both endpoints are in the set, as (src, dst, type).
 * Writes min(total, cap) edges in unspecified order and the total to *out_n.  Synchronous
 * (waits for `stream`); not a hot-path call.                                               */
int egr_plan_induced_edges(const egr_plan* p, int32_t col, uint32_t* out_src, uint32_t* out_dst,
                           uint8_t* out_type, int64_t cap, int64_t* out_n, void* stream);

/* ------------------------------------------------------------------------------------------
 * Partitioned graphs (egraph/shard.py).  A rank's snapshot is built from its
 * local CSR: owned vertices first (their full rows, entries remapped to local ids, CSR order
 * kept so every row's fmaf chain is the unpartitioned one), then halo vertices (empty rows).
 * Per hop the owners' fresh rows of the exported vertices are packed, exchanged (RCCL
 * all-gather, done by the caller) and unpacked into the halo rows.
 *   egr_snapshot_from_csr : host arrays row_ptr [V+1], col/meta/val [row_ptr[V]], vlabel [V].
 *   egr_plan_set_owned    : rows [0, n_owned) are the only top-k candidates, and the hop /
 *                           reach sweeps cover only them (halo rows [n_owned, V) hold what
 *                           the exchange unpacks; their values are not computed here).
 *   egr_plan_pack_*       : out[i] = row rows[i] of the current scores ([n][Bpad] fp32, column
 *                           b at b) / reach ([n][ceil(n_cols/64)] u64).
 *   egr_plan_unpack_*     : row rows[i] = in[src[i]] (same layouts).
 * ---------------------------------------------------------------------------------------- */
int egr_snapshot_from_csr(const uint32_t* row_ptr, const uint32_t* col, const uint8_t* meta,
                          const float* val, const uint8_t* vlabel, int64_t n_vertices,
                          int32_t device, egr_snapshot** out);
int egr_plan_set_owned(egr_plan* p, int64_t n_owned);
int egr_plan_pack_scores(const egr_plan* p, const uint32_t* rows, int64_t n, float* out, void* stream);
int egr_plan_unpack_scores(egr_plan* p, const uint32_t* rows, const uint32_t* src, int64_t n,
                           const float* in, void* stream);
int egr_plan_pack_reach(const egr_plan* p, const uint32_t* rows, int64_t n, uint64_t* out, void* stream);
int egr_plan_unpack_reach(egr_plan* p, const uint32_t* rows, const uint32_t* src, int64_t n,
                          const uint64_t* in, void* stream);

/* Sparse halo exchange (the production form of the pack / unpack above): only the NON-ZERO
 * entries of the boundary rows cross the link.  what: 0 = scores (after a hop), 1 = reach
 * words.  pack: rows[0, n) grouped by destination rank, seg[P + 1] (host) their segment
 * starts; writes each peer's entries contiguously into `out` (device, int64 words: scores one
 * word per entry = (row-in-segment * width + column) << 32 | value bits, reach two words =
 * index, word; width = padded columns resp. reach words per row) and the entry count per
 * peer into counts[P] (host; the call synchronises its stream to learn them).  unpack: zeroes
 * the received halo rows (recv_vertex[n_rows]: the local vertex of each received row, rows
 * grouped by sender) and scatters n_entries entries (device; sender s owns entries
 * [eseg[s], eseg[s+1]) and its rows start at recv row rbase[s], both device arrays).
 * Bit-identical to the dense exchange.  At most EGR_SX_MAX_PEERS ranks.                     */
#define EGR_SX_MAX_PEERS 64
int egr_plan_pack_sparse(egr_plan* p, int32_t what, const uint32_t* rows, int64_t n,
                         const int64_t* seg, int32_t P, int64_t* out, int64_t cap,
                         int64_t* counts, void* stream);
int egr_plan_unpack_sparse(egr_plan* p, int32_t what, const uint32_t* recv_vertex, int64_t n_rows,
                           const int64_t* in, int64_t n_entries, const int64_t* eseg,
                           const int64_t* rbase, int32_t P, void* stream);
/* The same exchange with FIXED-CAPACITY peer slots and no host synchronisation (a halo exchange
 * per hop then never waits for the host: ONE all-to-all with equal splits).  A slot is
 * 1 + peer_cap * words_per_entry int64 words: a header word holding the sender's entry count
 * for that peer, then the entries.  pack_cap: seg_dev[P + 1] on the device; a count pass, a scan
 * and an emit pass write peer q's header and entries to out[q * slot ...) in (row, column) order
 * (the counts also to counts_dev[q] when it is not NULL), and *overflow_dev (device u32) gets 1
 * when a peer has more than peer_cap entries (the excess is dropped: the caller re-runs the pass
 * with larger slots) or 2 when a row's emitted entries disagree with its count pass.
 * unpack_cap: sender s's entries are the first min(header, peer_cap) of its slot of `in`; a
 * header past peer_cap (the sender overflowed) sets *overflow_dev when it is not NULL; zero +
 * scatter as egr_plan_unpack_sparse.  Both are enqueued on `stream` only. */
int egr_plan_pack_sparse_cap(egr_plan* p, int32_t what, const uint32_t* rows, int64_t n,
                             const int64_t* seg_dev, int32_t P, int64_t* out, int64_t peer_cap,
                             int64_t* counts_dev, uint32_t* overflow_dev, void* stream);
int egr_plan_unpack_sparse_cap(egr_plan* p, int32_t what, const uint32_t* recv_vertex, int64_t n_rows,
                               const int64_t* in, int64_t peer_cap, uint32_t* overflow_dev,
                               const int64_t* rbase, int32_t P, void* stream);
/* One whole halo exchange over an RCCL communicator, for callers that are not torch (SURVEY.md
 * §8b's egr_halo_allgather; egraph/shard.py's TorchComm path issues the same three steps): the
 * pack above into send_slots (P slots of 1 + peer_cap * (what ? 2 : 1) int64 words, device), ONE
 * ncclAllToAll of the slots over xGMI into recv_slots, the unpack above -- enqueued on `stream`,
 * no host synchronisation.  rccl_comm: an ncclComm_t of exactly P ranks (this rank's), e.g. from
 * ncclCommInitRank; send_rows / send_seg_dev / recv_vertex / recv_base_dev as the pack / unpack
 * above (egraph.shard.LocalGraph holds them).  *overflow_dev != 0 afterwards: a slot overflowed,
 * re-run the pass with a larger peer_cap.  Replaces the cross-partition part of the single-host
 * apoc.path.subgraphAll traversal (neo4j.py:169-202) for graphs split over GPUs. */
int egr_plan_halo_exchange(egr_plan* p, int32_t what, const uint32_t* send_rows, int64_t n_send,
                           const int64_t* send_seg_dev, int32_t P, int64_t peer_cap,
                           int64_t* send_slots, int64_t* recv_slots, const uint32_t* recv_vertex,
                           int64_t n_recv, const int64_t* recv_base_dev, uint32_t* overflow_dev,
                           void* rccl_comm, void* stream);

/* ------------------------------------------------------------------------------------------
 * Frontier engine: the same A8 + A9 + top-k results as a plan's egr_plan_run, computed per
 * incident column over only the vertices the column needs (one workgroup per column, its state
 * in LDS).  Scores, reach sets and top-k are bit-identical to the dense plan's.
 * Replaces, like the plan, apoc.path.subgraphAll (neo4j.py:169-202) plus the build-defined
 * propagation / top-k.
 *   egr_frontier_create : pool_entries = capacity of the member pool that keeps every
 *                         column's (vertex, score, depth) for the read functions; 0 picks
 *                         n_cols*4096 + 4V; -1 = no pool (top-k only: the narrow-table kernel,
 *                         whose last pull computes the candidates only; the read functions
 *                         return EGR_ESTATE).  Columns that do not fit a table or the pool are
 *                         still ranked.
 *   egr_frontier_run    : one pass; sources [n_cols] device; outputs [n_cols*k] as
 *                         egr_plan_topk (EGR_NO_NODE / -inf in unused slots).
 *   egr_frontier_stats  : synchronous; out[9] of the last run = CSR entries gathered by
 *                         pulls (col + val read), CSR entries read by expansions (col only),
 *                         rows walked (row_ptr pairs), members, columns handed on by an LDS
 *                         kernel (the narrow one and, with the retry on, the wide one), pool
 *                         entries used, valid seed entries, columns finished in a
 *                         continuation region, columns ranked by the global-memory variant.
 *   egr_frontier_read_* : dense copies like egr_plan_read_* (scores [V][n_cols] row-major,
 *                         reach [ceil(n_cols/64)][V]); EGR_ESTATE-free but a column whose
 *                         members did not fit the pool reads as all zero.
 *   egr_frontier_members: one column's members (unordered); depth = hops from the incident
 *                         vertex + 1, 0 = not reached.  Synchronous.
 * ---------------------------------------------------------------------------------------- */
typedef struct egr_frontier egr_frontier;

/* Top-k-only frontiers (pool_entries = -1, the narrow-table kernel): give the columns that
 * overflow the narrow LDS table (more than 1152 members) a second chance in the wide LDS table
 * (4608 members) before the global-memory variant, on a persistent grid of
 * `blocks` workgroups (0 = off, the default; graphs whose 3-hop neighbourhoods are small never
 * overflow and skip the launch).  Takes effect from the next run (capture it into a graph
 * after setting it).                                                                       */
int egr_frontier_set_retry(egr_frontier* f, int32_t blocks);
/* With the retry on and the narrow table first: a column that overflows the narrow table
 * continues in its own workgroup, in one of `regions` global-memory table regions (8192 slots,
 * 6144 members each; claimed one per overflowing column per run, cleared by the workgroup
 * after use), instead of waiting for the wide retry grid that runs after the narrow one --
 * the costliest columns start first, so they finish while the grid runs.  What overflows a
 * region, or finds none left, goes to the global-memory variant.  0 = off (the default).
 * Same results either way; EGR_EINVAL outside 0..4096; synchronises the device when it
 * allocates (about 128 KB per region).                                                     */
int egr_frontier_set_continuation(egr_frontier* f, int32_t regions);
/* Top-k-only frontiers with the retry on: the first table every column tries, for graphs where
 * most columns overflow the narrow one (the narrow attempt would be wasted work).  `on` = 0: the
 * narrow table; 1: EVERY column straight to the wide grid; 2: a 2.8k-slot mid table first (four
 * workgroups per CU), its overflowing columns through the wide grid (the dense C4).  Same
 * results in every mode; EGR_EINVAL outside 0..2; takes effect from the next egr_frontier_run. */
int egr_frontier_set_wide_first(egr_frontier* f, int32_t on);

int egr_frontier_create(const egr_snapshot* s, int32_t n_cols, int64_t max_seeds, int32_t k,
                        int64_t pool_entries, egr_frontier** out);
void egr_frontier_free(egr_frontier* f);
int egr_frontier_set_seeds(egr_frontier* f, const uint32_t* seed_vertex, const uint32_t* seed_col,
                           const float* seed_val, int64_t n_seeds, void* stream);
int egr_frontier_run(egr_frontier* f, const uint32_t* source_vertex, int32_t hops,
                     int32_t exclude_label, uint32_t* out_ids, float* out_scores, void* stream);
/* One pass over seeds already grouped by column (no sort, no set_seeds): column b's seeds are
 * entries [seed_ptr[b], seed_ptr[b+1]) of seed_vertex / seed_val (device; seed_ptr [n_cols+1]
 * u32, clamped to n_seeds; n_seeds <= the frontier's max_seeds; duplicates max-combined,
 * out-of-range vertices dropped).  Same results as egr_frontier_set_seeds + egr_frontier_run
 * with the same triples.  order [n_cols] (device): the order the columns start in, a
 * permutation of 0..n_cols-1 (entries >= n_cols are skipped); NULL = costliest first, computed
 * on the device in the same stream (cost = the column's seeds' 1 + degree, bucketed on a log
 * scale, as set_seeds orders them) -- longest-processing-time first; the pointers are read by
 * this call's kernels only (stream order). */
int egr_frontier_run_grouped(egr_frontier* f, const uint32_t* seed_ptr, const uint32_t* seed_vertex,
                             const float* seed_val, int64_t n_seeds, const uint32_t* order,
                             const uint32_t* source_vertex,
                             int32_t hops, int32_t exclude_label, uint32_t* out_ids,
                             float* out_scores, void* stream);
/* the columns and k a frontier was created with (callers size their output buffers by it) */
int egr_frontier_shape(const egr_frontier* f, int32_t* n_cols, int32_t* k);
int egr_frontier_stats(const egr_frontier* f, int64_t* out9, void* stream);
int egr_frontier_read_scores(const egr_frontier* f, float* out, void* stream);
/* Diagnostics: with $EGRAPH_FRONTIER_PROFILE set when the frontier was created, each column's
 * workgroup stamps s_memrealtime (100 MHz) at its phase boundaries: per column and slot, the
 * stamp after the barrier then each wave's stamp before it.  Copies [n_cols][slots][1+waves]
 * (0 = unused) into out (cap entries) and returns the int64 count per column (0: off).    */
int egr_frontier_phase_times(const egr_frontier* f, int64_t* out, int64_t cap, void* stream);
int egr_frontier_read_reach(const egr_frontier* f, uint64_t* out, void* stream);
int egr_frontier_members(const egr_frontier* f, int32_t col, uint32_t* out_vertex,
                         float* out_score, uint8_t* out_depth, int64_t cap, int64_t* out_n,
                         void* stream);

/* ---- Incremental snapshot update + download (csrc/update.hip) -----------------------------
 * egr_snapshot_update   append n_new vertices (labels new_vlabel) and n_edges NEW edges
 *                       (edge_src / edge_dst / edge_type; ids in the grown numbering) to a
 *                       device snapshot: the result equals egr_snapshot_create on the grown
 *                       graph (same row order, same val = w / deg with the new degrees).  All
 *                       delta arrays are DEVICE pointers; weights as egr_snapshot_create (host).
 *                       The edges must be absent from the snapshot and distinct -- the host
 *                       MERGE (egr_graph_merge_edges) guarantees it; a violation or an
 *                       out-of-range id returns EGR_EINVAL with the snapshot unchanged.
 *                       Synchronous on `stream`, and it first drains the whole device: the
 *                       merge writes into the previous version's arrays, which kernels
 *                       enqueued earlier on other streams may still read.  Plans created before an update return
 *                       EGR_ESTATE afterwards; a frontier keeps working while the snapshot
 *                       stays within the vertex headroom it was sized with (V + V/4 + 4096).
 *                       Replaces the per-item MERGE round trips of neo4j.py:95-167 for the
 *                       alert storm's per-tick deltas (BASELINE config C5).
 * egr_snapshot_download copy the CSR and labels to host buffers (NULL = skip): row_ptr [V+1],
 *                       col / meta / val [n_entries], vlabel [V].  Synchronous.
 * egr_snapshot_version  number of updates applied.
 * egr_graph_export_edges  edges [first, first + n) of the host graph in creation order (the
 *                       delta a MERGE batch appended).
 * ---------------------------------------------------------------------------------------- */
int egr_snapshot_update(egr_snapshot* s, const uint8_t* new_vlabel, int64_t n_new,
                        const uint32_t* edge_src, const uint32_t* edge_dst, const uint8_t* edge_type,
                        int64_t n_edges, const float* weights, int32_t n_types, void* stream);
int egr_snapshot_download(const egr_snapshot* s, uint32_t* row_ptr, uint32_t* col, uint8_t* meta,
                          float* val, uint8_t* vlabel);
int64_t egr_snapshot_version(const egr_snapshot* s);
/* The frontier engine's locality order of a CSR (host only; csrc/layout.hip):
 * out_order[i] = the vertex the snapshot's frontier layout places at internal position i.  Every
 * snapshot lays its frontier arrays out in this order at creation ($EGRAPH_FRONTIER_LAYOUT=0:
 * off); the frontier's inputs and outputs stay in original ids, and every result is unchanged
 * (rows keep their entry order).  No reference counterpart: a storage layout of the graph the
 * Cypher reads of neo4j.py:169-202 run against. */
int egr_locality_order(const uint32_t* row_ptr, const uint32_t* col, int64_t n_vertices,
                       uint32_t* out_order);
/* multi-source BFS: out_dist[v] (device, V bytes) = undirected hops from the nearest of the n
 * source vertices (device u32; ids >= V ignored), 0xFF beyond `hops`.  The alert storm marks
 * the incidents an update can affect with it. */
int egr_snapshot_within(const egr_snapshot* s, const uint32_t* sources, int64_t n, int32_t hops,
                        uint8_t* out_dist, void* stream);
/* One typed hop of a Cypher path pattern over the device snapshot: for query vertex i
 * (device u32 vertices[i]; ids >= V give 0), its neighbours u over the relationships of type
 * `rel_type` in direction `dir` -- 1: (vertices[i])-[:type]->(u), 0: (vertices[i])<-[:type]-(u)
 * -- whose label is `label` (-1: any), in CSR order, written to out_vertices[out_off[i] ..]
 * (device) with their count in out_counts[i].  out_vertices = NULL: counts only (out_off
 * unused), so a caller sizes the segments with one call and emits with a second.  Replaces the typed MATCH steps of GraphService.find_related_changes,
 * find_affected_by_node and get_service_dependencies (src/database/neo4j.py:205-279), which
 * egraph_dropin.graph_service chains from it. */
int egr_snapshot_typed_neighbors(const egr_snapshot* s, const uint32_t* vertices, int64_t n,
                                 int32_t rel_type, int32_t dir, int32_t label,
                                 const int64_t* out_off, uint32_t* out_vertices,
                                 uint32_t* out_counts, void* stream);
/* vertex count a frontier was sized for (it runs while the snapshot stays within it) */
int64_t egr_frontier_max_vertices(const egr_frontier* f);
int egr_graph_export_edges(const egr_graph* g, int64_t first, int64_t n, int32_t* edge_src,
                           int32_t* edge_dst, uint8_t* edge_type);
/* MERGE edges given by vertex INDEX (a restore from a snapshot file, egraph/snapfile.py: the
 * edge list in creation order reproduces the graph exactly; the label-less id MATCH of
 * egr_graph_merge_edges would fan out over vertices sharing an id).  type_idx indexes the
 * n_types names in type_blob/type_off.  out_new = edges created. */
int egr_graph_add_edges_indexed(egr_graph* g, const int32_t* src, const int32_t* dst,
                                const char* type_blob, const int64_t* type_off, int32_t n_types,
                                const int32_t* type_idx, int64_t n, int64_t* out_new);

/* ---- Alert-storm front end: fingerprints + TTL dedup table (csrc/alerts.hip) ---------------
 * egr_fingerprint   replaces AlertNormalizer._generate_fingerprint
 *                   (src/services/ingestion/normalizer.py:208-218) for a batch: key i is
 *                   blob[offsets[i] .. offsets[i+1]) (device arrays; the caller formats
 *                   f"{source}:{alertname}:{namespace}:{service}"), out16[i] = first 16 bytes
 *                   of its SHA-256, out_hex (optional, n*32 chars, no NULs) = the reference's
 *                   hexdigest()[:32].
 * egr_dedup_*       replace AlertDeduplicator (src/services/ingestion/deduplicator.py:41-140,
 *                   Redis with EX) on device: a key is live while now_ms < expiry.
 *   _ingest         the webhook loop (src/services/ingestion/main.py:141-170 with the
 *                   registration in create_incident, :392) for a batch in order: an alert whose
 *                   fingerprint is live is a duplicate of that incident (out_dup 1); the first
 *                   alert of a non-live fingerprint opens incident first_id + (its rank among
 *                   the batch's new incidents), registered with expiry now+ttl (out_dup 0);
 *                   later alerts of that fingerprint in the batch are its duplicates.
 *                   out_counts (device, 2 u32) = {alerts dropped because the table is full
 *                   (they fail open: not duplicates, incident EGR_NO_NODE), new incidents}.
 *   _lookup         check_duplicate (:41-71) for a batch.
 *   _register       register_fingerprint (:73-104): SET EX for a batch (last write of a
 *                   repeated key wins); out_full (device u32) = keys dropped (table full).
 *   _remove         remove_fingerprint (:106-118).
 *   _extend         extend_fingerprint (:120-140): new expiry for live keys only; out_ok
 *                   (optional) = was live.
 *   _stats          out3 = {slots holding a key, live keys, slots}.  Synchronous.
 *   _compact        rebuild with the live keys only, sized for max(capacity, live).  Synchronous.
 * ---------------------------------------------------------------------------------------- */
typedef struct egr_dedup egr_dedup;

int egr_fingerprint(const uint8_t* blob, const int64_t* offsets, int64_t n, uint8_t* out16,
                    char* out_hex, void* stream);
int egr_dedup_create(int32_t device, int64_t capacity, egr_dedup** out);
void egr_dedup_free(egr_dedup* d);
int egr_dedup_ingest(egr_dedup* d, const uint8_t* fp16, int64_t n, int64_t now_ms, int64_t ttl_ms,
                     uint32_t first_id, uint8_t* out_dup, uint32_t* out_incident,
                     uint32_t* out_counts, void* stream);
int egr_dedup_lookup(const egr_dedup* d, const uint8_t* fp16, int64_t n, int64_t now_ms,
                     uint8_t* out_dup, uint32_t* out_incident, void* stream);
int egr_dedup_register(egr_dedup* d, const uint8_t* fp16, int64_t n, int64_t now_ms, int64_t ttl_ms,
                       const uint32_t* incident, uint32_t* out_full, void* stream);
int egr_dedup_remove(egr_dedup* d, const uint8_t* fp16, int64_t n, void* stream);
int egr_dedup_extend(egr_dedup* d, const uint8_t* fp16, int64_t n, int64_t now_ms, int64_t ttl_ms,
                     uint8_t* out_ok, void* stream);
int egr_dedup_stats(const egr_dedup* d, int64_t now_ms, int64_t* out3);
int egr_dedup_compact(egr_dedup* d, int64_t now_ms, int64_t capacity);

#ifdef __cplusplus
}
#endif
#endif /* EGRAPH_H_ */
