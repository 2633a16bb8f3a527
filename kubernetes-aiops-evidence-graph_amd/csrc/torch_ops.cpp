// PyTorch-ROCm custom-op registration of the hot path (torch.ops.egraph.*).
//
// A thin layer over the SAME C-ABI the Python service classes bind with ctypes (include/egraph.h,
// libegraph.so): every op validates its tensors, takes torch's current HIP stream on the
// tensors' device, and calls the egr_* entry point.  There is no second implementation here and
// no CPU kernel: a call with CPU tensors fails in the dispatcher (no CPU registration).
//
//   egraph::rules_eval      <- RulesEngine.generate_hypotheses + HypothesisRanker.rank
//                              (reference rules_engine.py:199-478, hypothesis_ranker.py:13-80)
//   egraph::frontier_run    <- the graph stage of one incident batch: k-hop reach
//                              (neo4j.py:169-202 subgraphAll) + propagation + top-k
//   egraph::propagate       <- dense typed k-hop propagation (egr_plan_*), scores [V][B]
//   egraph::reach           <- dense k-hop reach bitsets (apoc.path.subgraphAll node sets)
//   egraph::topk            <- per-incident top-k over explicit score / reach arrays (egr_topk)
// Engine state (snapshot, plan, frontier workspaces) lives in libegraph objects; the ops take
// their handles as int64 (the Python wrappers in egraph/ops.py pass them).
#include <ATen/ATen.h>
#include <c10/hip/HIPStream.h>
#include <torch/library.h>

#include <string>
#include <tuple>

#include "egraph.h"

namespace {

void check_rc(int rc, const char* what) {
  if (rc == EGR_OK) return;
  const char* msg = egr_last_error();
  TORCH_CHECK_VALUE(rc != EGR_EINVAL, what, ": ", msg ? msg : "invalid argument");
  TORCH_CHECK(false, what, ": ", msg ? msg : "device error", " (status ", rc, ")");
}

void* cur_stream(const at::Tensor& t) {
  return (void*)c10::hip::getCurrentHIPStream(t.device().index()).stream();
}

void need(const at::Tensor& t, at::ScalarType st, const char* name) {
  TORCH_CHECK_VALUE(t.is_cuda(), name, " must be a device (HIP) tensor");
  TORCH_CHECK_VALUE(t.scalar_type() == st, name, " has dtype ", t.scalar_type(), ", need ", st);
  TORCH_CHECK_VALUE(t.is_contiguous(), name, " must be contiguous");
}

// the engine's own sizes: every op checks the caller's arguments against them, because the C
// calls read and write by the engine's sizes (a mismatch would be an out-of-bounds access)
void check_frontier_shape(const egr_frontier* f, int64_t n_cols, int64_t k) {
  int32_t B = 0, K = 0;
  check_rc(egr_frontier_shape(f, &B, &K), "egraph::frontier_run (shape)");
  TORCH_CHECK_VALUE(n_cols == B && k == K, "egraph::frontier_run: the frontier was created for ",
                    B, " columns and k = ", K, ", got n_cols = ", n_cols, ", k = ", k);
}

void check_plan_shape(const egr_plan* p, int64_t n_vertices, int64_t n_cols, const char* what) {
  int64_t V = 0;
  int32_t B = 0;
  check_rc(egr_plan_shape(p, &V, &B), what);
  TORCH_CHECK_VALUE(n_vertices == V && (n_cols < 0 || n_cols == B), what, ": the plan is for ", V,
                    " vertices and ", B, " columns, got n_vertices = ", n_vertices,
                    n_cols >= 0 ? ", n_cols = " : "", n_cols >= 0 ? std::to_string(n_cols) : "");
}

template <class T>
T* handle(int64_t h, const char* name) {
  TORCH_CHECK_VALUE(h != 0, name, " handle is null");
  return reinterpret_cast<T*>(static_cast<uintptr_t>(h));
}

// rules: rule_table is a CPU uint8 tensor holding one egr_rule_table (egraph.catalog lowers the
// reference's DIAGNOSIS_RULES into it)
std::tuple<at::Tensor, at::Tensor, at::Tensor, at::Tensor, at::Tensor, at::Tensor, at::Tensor>
rules_eval(const at::Tensor& flags, const at::Tensor& vocab, const at::Tensor& node,
           const at::Tensor& err, const at::Tensor& seg_off, const at::Tensor& rule_table) {
  need(flags, at::kInt, "row_flags");
  need(vocab, at::kInt, "row_vocab");
  need(node, at::kInt, "row_node");
  need(err, at::kDouble, "row_err");
  need(seg_off, at::kLong, "seg_off");
  TORCH_CHECK_VALUE(!rule_table.is_cuda() && rule_table.scalar_type() == at::kByte &&
                        rule_table.is_contiguous() &&
                        rule_table.numel() == (int64_t)sizeof(egr_rule_table),
                    "rule_table must be a contiguous CPU uint8 tensor of sizeof(egr_rule_table)");
  const int64_t rows = flags.numel();
  TORCH_CHECK_VALUE(vocab.numel() == rows && node.numel() == rows && err.numel() == rows,
                    "row columns differ in length");
  TORCH_CHECK_VALUE(seg_off.numel() >= 1, "seg_off needs n_incidents + 1 entries");
  const int64_t B = seg_off.numel() - 1;
  const auto* table = reinterpret_cast<const egr_rule_table*>(rule_table.data_ptr<uint8_t>());
  const int64_t S = (int64_t)table->n_rules + 1;
  auto o8 = flags.options().dtype(at::kByte);
  auto of = flags.options().dtype(at::kDouble);
  at::Tensor mask = at::empty({B}, flags.options());
  at::Tensor n_hyp = at::empty({B}, o8);
  at::Tensor order_conf = at::empty({B, S}, o8);
  at::Tensor order_rank = at::empty({B, S}, o8);
  at::Tensor confidence = at::zeros({B, S}, of);
  at::Tensor final_score = at::zeros({B, S}, of);
  at::Tensor strength = at::zeros({B, S}, of);
  if (B > 0) {
    egr_rules_out out{reinterpret_cast<uint32_t*>(mask.data_ptr<int32_t>()), n_hyp.data_ptr<uint8_t>(),
                      order_conf.data_ptr<uint8_t>(), order_rank.data_ptr<uint8_t>(),
                      confidence.data_ptr<double>(), final_score.data_ptr<double>(),
                      strength.data_ptr<double>()};
    check_rc(egr_rules_eval(table, reinterpret_cast<const uint32_t*>(flags.data_ptr<int32_t>()),
                            reinterpret_cast<const uint32_t*>(vocab.data_ptr<int32_t>()),
                            reinterpret_cast<const uint32_t*>(node.data_ptr<int32_t>()),
                            err.data_ptr<double>(), seg_off.data_ptr<int64_t>(), (int32_t)B, &out,
                            cur_stream(flags)),
             "egraph::rules_eval");
  }
  return {mask, n_hyp, order_conf, order_rank, confidence, final_score, strength};
}

// the frontier engine: seeds (vertex, column, value) triples + one source vertex per column
std::tuple<at::Tensor, at::Tensor> frontier_run(int64_t frontier, const at::Tensor& seed_vertex,
                                                const at::Tensor& seed_col, const at::Tensor& seed_val,
                                                const at::Tensor& sources, int64_t n_cols, int64_t k,
                                                int64_t hops, int64_t exclude_label) {
  auto* f = handle<egr_frontier>(frontier, "frontier");
  need(seed_vertex, at::kInt, "seed_vertex");
  need(seed_col, at::kInt, "seed_col");
  need(seed_val, at::kFloat, "seed_val");
  need(sources, at::kInt, "sources");
  const int64_t n = seed_vertex.numel();
  TORCH_CHECK_VALUE(seed_col.numel() == n && seed_val.numel() == n, "seed arrays differ in length");
  TORCH_CHECK_VALUE(sources.numel() == n_cols, "need one source vertex per column");
  check_frontier_shape(f, n_cols, k);
  void* st = cur_stream(sources);
  at::Tensor ids = at::empty({n_cols, k}, sources.options());
  at::Tensor scores = at::empty({n_cols, k}, seed_val.options());
  check_rc(egr_frontier_set_seeds(f, reinterpret_cast<const uint32_t*>(seed_vertex.data_ptr<int32_t>()),
                                  reinterpret_cast<const uint32_t*>(seed_col.data_ptr<int32_t>()),
                                  seed_val.data_ptr<float>(), n, st),
           "egraph::frontier_run (seeds)");
  check_rc(egr_frontier_run(f, reinterpret_cast<const uint32_t*>(sources.data_ptr<int32_t>()),
                            (int32_t)hops, (int32_t)exclude_label,
                            reinterpret_cast<uint32_t*>(ids.data_ptr<int32_t>()),
                            scores.data_ptr<float>(), st),
           "egraph::frontier_run");
  return {ids, scores};
}

// dense propagation: scores [V][B] after `hops` hops from the seeds
at::Tensor propagate(int64_t plan, const at::Tensor& seed_vertex, const at::Tensor& seed_col,
                     const at::Tensor& seed_val, int64_t n_vertices, int64_t n_cols, int64_t hops) {
  auto* p = handle<egr_plan>(plan, "plan");
  need(seed_vertex, at::kInt, "seed_vertex");
  need(seed_col, at::kInt, "seed_col");
  need(seed_val, at::kFloat, "seed_val");
  const int64_t n = seed_vertex.numel();
  TORCH_CHECK_VALUE(seed_col.numel() == n && seed_val.numel() == n, "seed arrays differ in length");
  TORCH_CHECK_VALUE(hops >= 1, "hops must be >= 1");
  check_plan_shape(p, n_vertices, n_cols, "egraph::propagate");
  void* st = cur_stream(seed_val);
  check_rc(egr_plan_set_seeds(p, reinterpret_cast<const uint32_t*>(seed_vertex.data_ptr<int32_t>()),
                              reinterpret_cast<const uint32_t*>(seed_col.data_ptr<int32_t>()),
                              seed_val.data_ptr<float>(), n, st),
           "egraph::propagate (seeds)");
  for (int64_t h = 0; h < hops; ++h) check_rc(egr_plan_hop(p, st), "egraph::propagate (hop)");
  at::Tensor out = at::empty({n_vertices, n_cols}, seed_val.options());
  check_rc(egr_plan_read_scores(p, out.data_ptr<float>(), st), "egraph::propagate (read)");
  return out;
}

// dense reach: bits [ceil(B/64)][V] of the vertices within `hops` undirected hops
at::Tensor reach(int64_t plan, const at::Tensor& sources, int64_t n_vertices, int64_t hops) {
  auto* p = handle<egr_plan>(plan, "plan");
  need(sources, at::kInt, "sources");
  TORCH_CHECK_VALUE(hops >= 0, "hops must be >= 0");
  check_plan_shape(p, n_vertices, sources.numel(), "egraph::reach");
  void* st = cur_stream(sources);
  check_rc(egr_plan_set_sources(p, reinterpret_cast<const uint32_t*>(sources.data_ptr<int32_t>()), st),
           "egraph::reach (sources)");
  for (int64_t h = 0; h < hops; ++h) check_rc(egr_plan_reach_hop(p, st), "egraph::reach (hop)");
  const int64_t W = (sources.numel() + 63) / 64;
  at::Tensor out = at::empty({W, n_vertices}, sources.options().dtype(at::kLong));
  check_rc(egr_plan_read_reach(p, reinterpret_cast<uint64_t*>(out.data_ptr<int64_t>()), st),
           "egraph::reach (read)");
  return out;
}

std::tuple<at::Tensor, at::Tensor> topk(int64_t snapshot, const at::Tensor& scores,
                                        const at::Tensor& reach_bits, int64_t k,
                                        int64_t exclude_label) {
  auto* s = handle<const egr_snapshot>(snapshot, "snapshot");
  need(scores, at::kFloat, "scores");
  need(reach_bits, at::kLong, "reach_bits");
  TORCH_CHECK_VALUE(scores.dim() == 2 && reach_bits.dim() == 2, "scores [V, B], reach_bits [W, V]");
  const int64_t B = scores.size(1);
  TORCH_CHECK_VALUE(reach_bits.size(0) == (B + 63) / 64 && reach_bits.size(1) == scores.size(0),
                    "reach_bits must be [ceil(B/64), V] for scores [V, B]");
  int64_t V = 0, nnz = 0;
  check_rc(egr_snapshot_info(s, &V, &nnz), "egraph::topk (shape)");
  TORCH_CHECK_VALUE(scores.size(0) == V, "egraph::topk: scores has ", scores.size(0),
                    " rows, the snapshot ", V, " vertices");
  TORCH_CHECK_VALUE(k >= 1 && k <= 16, "egraph::topk: need 1 <= k <= 16");
  at::Tensor ids = at::empty({B, k}, scores.options().dtype(at::kInt));
  at::Tensor out = at::empty({B, k}, scores.options());
  check_rc(egr_topk(s, scores.data_ptr<float>(),
                    reinterpret_cast<const uint64_t*>(reach_bits.data_ptr<int64_t>()), (int32_t)B,
                    (int32_t)k, (int32_t)exclude_label,
                    reinterpret_cast<uint32_t*>(ids.data_ptr<int32_t>()), out.data_ptr<float>(),
                    cur_stream(scores)),
           "egraph::topk");
  return {ids, out};
}

}  // namespace

TORCH_LIBRARY(egraph, m) {
  m.def("rules_eval(Tensor row_flags, Tensor row_vocab, Tensor row_node, Tensor row_err, "
        "Tensor seg_off, Tensor rule_table) -> (Tensor mask, Tensor n_hyp, Tensor order_conf, "
        "Tensor order_rank, Tensor confidence, Tensor final_score, Tensor strength)");
  m.def("frontier_run(int frontier, Tensor seed_vertex, Tensor seed_col, Tensor seed_val, "
        "Tensor sources, int n_cols, int k, int hops, int exclude_label) -> (Tensor ids, Tensor scores)");
  m.def("propagate(int plan, Tensor seed_vertex, Tensor seed_col, Tensor seed_val, int n_vertices, "
        "int n_cols, int hops) -> Tensor");
  m.def("reach(int plan, Tensor sources, int n_vertices, int hops) -> Tensor");
  m.def("topk(int snapshot, Tensor scores, Tensor reach_bits, int k, int exclude_label) "
        "-> (Tensor ids, Tensor scores)");
}

TORCH_LIBRARY_IMPL(egraph, CUDA, m) {
  m.impl("rules_eval", &rules_eval);
  m.impl("frontier_run", &frontier_run);
  m.impl("propagate", &propagate);
  m.impl("reach", &reach);
  m.impl("topk", &topk);
}
