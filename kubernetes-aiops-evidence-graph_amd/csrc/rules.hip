// Rules (A1-A6): batched deterministic diagnosis over encoded evidence rows, fused with the
// hypothesis ranker, plus the stand-alone ranker kernel.
//
// One 64-lane wavefront per incident segment:
//   * coalesced sweep of the segment's rows (20 B/row: flags, vocab, node key, error count),
//     wave-level OR / SUM reductions = RulesEngine._extract_signals (rules_engine.py:264-376);
//     the first 128 rows are loaded in one round trip;
//   * pods_by_node: max rows per node key (:323-330) by counting in a per-wave LDS hash table
//     (the max of the counts the rows' atomic adds return); segments with more node rows than
//     the table holds fall back to an exact pairwise count;
//   * lane r evaluates rule r's conditions (:378-441).  A rule emits only when ALL its
//     conditions hold, so its strength, confidence (:443-455) and ranker score
//     (hypothesis_ranker.py:44-63) are constants of the rule table: the host computes them in
//     float64 with Python-exact rounding into the compiled table (RulesDev), uploaded once per
//     distinct table, and the kernel does no floating-point arithmetic;
//   * both stable orders (by confidence, :228; then by final_score, hypothesis_ranker.py:67)
//     by counting, with the unknown fallback (:230-231, :457-478).
// The per-incident working set is a few KB, so the kernel is latency- not bandwidth-bound for
// realistic batches; its HBM cost is one read of the rows.
#include <cstring>
#include <mutex>
#include <string>
#include <tuple>
#include <vector>

#include "egr_internal.h"

namespace {

constexpr int kWave = 64;
constexpr int kWavesPerBlock = 4;

__device__ __forceinline__ uint32_t wave_or(uint32_t x) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) x |= __shfl_xor(x, o, kWave);
  return x;
}

__device__ __forceinline__ int wave_sum_i(int x) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o, kWave);
  return x;
}

__device__ __forceinline__ int wave_max_i(int x) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) x = max(x, __shfl_xor(x, o, kWave));
  return x;
}

// exact for integral values whose partial sums stay below 2^53 (the encoder guarantees it)
__device__ __forceinline__ double wave_sum_d(double x) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o, kWave);
  return x;
}

// The rule table as the kernel reads it: compiled on the host from egr_rule_table (conditions
// plus the constants of a matched rule: its strength, confidence (:443-455) and ranker score
// (hypothesis_ranker.py:44-63), computed in float64 with Python-exact rounding) and uploaded
// ONCE per distinct table into device memory (rules_table_dev below).  The kernel then gets one
// pointer instead of a 4.6-KB by-value argument block, and lane r reads rule r with a few
// 16-B loads of L2-resident data.
struct RuleDev {
  int32_t n_conds;
  int32_t cond_type[EGR_MAX_CONDS];
  uint32_t cond_mask[EGR_MAX_CONDS];
  double cond_param[EGR_MAX_CONDS];
  double conf, fin, str;
};
struct RulesDev {
  int32_t n_rules;
  uint32_t network_vocab_bit;
  double unknown_confidence, unknown_fin;
  RuleDev rules[EGR_MAX_RULES];
};

constexpr int kNodeSlots = 256;                 // per-wave pods_by_node hash table
constexpr uint32_t kNodeEmpty = 0xFFFFFFFFu;    // (EGR_NO_NODE rows are never inserted)

struct Signals {
  uint32_t flags;    // OR of EGR_F_* over the segment
  uint32_t vocab;    // OR of vocabulary bits (waiting / terminated reasons, log patterns)
  int n_node_rows;   // rows counted into pods_by_node
  int max_per_node;  // max(pods_by_node.values())
  double errors;     // signals["error_count"]
};

__device__ bool condition_holds(int type, uint32_t mask, double param, const Signals& s,
                                uint32_t network_bit) {
  switch (type) {
    case EGR_C_WAITING_REASON:
    case EGR_C_TERMINATED_REASON:
    case EGR_C_LOG_PATTERN:
      return (s.vocab & mask) != 0u;
    case EGR_C_RECENT_DEPLOY: return (s.flags & EGR_F_RECENT_DEPLOY) != 0u;
    case EGR_C_NO_RECENT_DEPLOY: return (s.flags & EGR_F_RECENT_DEPLOY) == 0u;
    case EGR_C_MEMORY_USAGE_HIGH: return (s.flags & EGR_F_MEMORY_HIGH) != 0u;
    case EGR_C_HPA_AT_MAX: return (s.flags & EGR_F_HPA_AT_MAX) != 0u;
    case EGR_C_LATENCY_HIGH: return (s.flags & EGR_F_LATENCY_HIGH) != 0u;
    case EGR_C_NODE_UNHEALTHY: return (s.flags & EGR_F_NODE_ISSUE) != 0u;
    case EGR_C_MULTIPLE_PODS_SAME_NODE:
      return s.n_node_rows > 0 && (double)s.max_per_node >= param;
    case EGR_C_POD_NOT_READY: return (s.flags & EGR_F_NOT_READY) != 0u;
    case EGR_C_READINESS_PROBE_FAILING: return (s.flags & EGR_F_READINESS_FAIL) != 0u;
    case EGR_C_NETWORK_ERRORS_HIGH:
      return s.errors >= param && network_bit < 32u && ((s.vocab >> network_bit) & 1u);
    default: return false;  // unknown condition types never match (:436-441)
  }
}

// One incident (rows [beg, end) of the row arrays) on one wave; hk / hc = the wave's LDS hash.
__device__ __forceinline__ void rules_incident(
    const RulesDev* __restrict__ D, const uint32_t* __restrict__ row_flags,
    const uint32_t* __restrict__ row_vocab, const uint32_t* __restrict__ row_node,
    const double* __restrict__ row_err, int64_t beg, int64_t end, int inc,
    const egr_rules_out& out, uint32_t* hk, uint32_t* hc) {
  const int lane = threadIdx.x & (kWave - 1);
  // lane r's rule, loaded up front (independent of the rows: its latency overlaps theirs)
  const int R = D->n_rules;
  const uint32_t network_bit = D->network_vocab_bit;
  const RuleDev* rule = &D->rules[lane < EGR_MAX_RULES ? lane : 0];
  const int nc = lane < R ? rule->n_conds : 0;

  // ---- signal extraction: one coalesced sweep (the first two row blocks in one round trip) --
  uint32_t f_or = 0, v_or = 0;
  double esum = 0.0;
  int n_node = 0;
  uint32_t k0 = EGR_NO_NODE, k1 = EGR_NO_NODE;   // this lane's node keys of rows 0..127
  {
    const int64_t r0 = beg + lane, r1 = beg + kWave + lane;
    const bool a0 = r0 < end, a1 = r1 < end;
    const uint32_t f0 = a0 ? row_flags[r0] : 0u, f1 = a1 ? row_flags[r1] : 0u;
    const uint32_t v0 = a0 ? row_vocab[r0] : 0u, v1 = a1 ? row_vocab[r1] : 0u;
    const double e0 = a0 ? row_err[r0] : 0.0, e1 = a1 ? row_err[r1] : 0.0;
    k0 = a0 ? row_node[r0] : EGR_NO_NODE;
    k1 = a1 ? row_node[r1] : EGR_NO_NODE;
    f_or = f0 | f1;
    v_or = v0 | v1;
    esum = e0 + e1;
    n_node = (k0 != EGR_NO_NODE) + (k1 != EGR_NO_NODE);
  }
  for (int64_t r = beg + 2 * kWave + lane; r < end; r += kWave) {
    f_or |= row_flags[r];
    v_or |= row_vocab[r];
    esum += row_err[r];
    n_node += row_node[r] != EGR_NO_NODE;
  }
  Signals s;
  s.flags = wave_or(f_or);
  s.vocab = wave_or(v_or);
  s.n_node_rows = wave_sum_i(n_node);
  if (s.flags & EGR_F_ERR_FLOAT) {
    // non-integral counts: replay Python's left-to-right accumulation exactly (:354)
    double acc = 0.0;
    if (lane == 0)
      for (int64_t r = beg; r < end; ++r) acc = acc + row_err[r];
    s.errors = __shfl(acc, 0, kWave);
  } else {
    s.errors = wave_sum_d(esum);
  }

  // ---- pods_by_node: max rows per node key ------------------------------------------------
  s.max_per_node = s.n_node_rows > 0 ? 1 : 0;
  if (s.n_node_rows >= 2 && s.n_node_rows <= kNodeSlots / 2 && end - beg <= 2 * kWave) {
    // LDS hash count (load <= 1/2): the count a row's add returns + 1 is the number of rows
    // of its node so far, so the max over all rows is max(pods_by_node.values())
#pragma unroll
    for (int j = 0; j < kNodeSlots / kWave; ++j) {
      hk[lane + j * kWave] = kNodeEmpty;
      hc[lane + j * kWave] = 0u;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    int best = 0;
    const uint32_t keys[2] = {k0, k1};
#pragma unroll
    for (int x = 0; x < 2; ++x) {
      const uint32_t k = keys[x];
      if (k == EGR_NO_NODE) continue;
      uint32_t h = (k * 0x9E3779B1u) >> 24;        // 8 bits: kNodeSlots = 256
      for (;;) {
        const uint32_t old = atomicCAS(&hk[h], kNodeEmpty, k);
        if (old == kNodeEmpty || old == k) {
          best = max(best, (int)atomicAdd(&hc[h], 1u) + 1);
          break;
        }
        h = (h + 1) & (kNodeSlots - 1);
      }
    }
    s.max_per_node = wave_max_i(best);
  } else if (s.n_node_rows >= 2) {
    int best = 0;
    for (int64_t ib = beg; ib < end; ib += kWave) {
      const int64_t i = ib + lane;
      const uint32_t ki = i < end ? row_node[i] : EGR_NO_NODE;
      int c = 0;
      for (int64_t jb = beg; jb < end; jb += kWave) {
        const int64_t j = jb + lane;
        const uint32_t kj = j < end ? row_node[j] : EGR_NO_NODE;
        const int lim = (int)min<int64_t>(kWave, end - jb);
        for (int p = 0; p < lim; ++p) c += __shfl(kj, p, kWave) == ki;
      }
      if (ki != EGR_NO_NODE) best = max(best, c);
    }
    s.max_per_node = wave_max_i(best);
  }

  // ---- rule r on lane r -----------------------------------------------------------------
  bool matched = false;
  double conf = 0.0, fin = 0.0, stren = 0.0;
  if (lane < R) {
    int mc = 0;
    for (int c = 0; c < nc && c < EGR_MAX_CONDS; ++c)
      mc += condition_holds(rule->cond_type[c], rule->cond_mask[c], rule->cond_param[c], s,
                            network_bit);
    matched = nc > 0 && mc == nc;
    if (matched) {                 // all conditions held: the rule's constants
      conf = rule->conf;
      fin = rule->fin;
      stren = rule->str;
    }
  }
  const uint64_t mm = __ballot(matched);
  const int nh = __popcll(mm);

  // stable positions: by confidence desc (ties: rule order), then by final_score desc (ties:
  // confidence order) -- exactly list.sort(reverse=True) applied twice
  int pc = 0;
  for (int j = 0; j < R; ++j) {
    const double cj = __shfl(conf, j, kWave);
    if ((mm >> j) & 1ull) pc += (cj > conf) || (cj == conf && j < lane);
  }
  int pr = 0;
  for (int j = 0; j < R; ++j) {
    const double fj = __shfl(fin, j, kWave);
    const int pcj = __shfl(pc, j, kWave);
    if ((mm >> j) & 1ull) pr += (fj > fin) || (fj == fin && pcj < pc);
  }

  // lane p owns output position p: find the rule that landed there (one writer per byte)
  const int S = R + 1;
  const int64_t base = (int64_t)inc * S;
  uint32_t at_c = 0xFFu, at_r = 0xFFu;
  for (int j = 0; j < R; ++j) {
    const int pcj = __shfl(pc, j, kWave);
    const int prj = __shfl(pr, j, kWave);
    if ((mm >> j) & 1ull) {
      if (pcj == lane) at_c = (uint32_t)j;
      if (prj == lane) at_r = (uint32_t)j;
    }
  }
  if (nh == 0 && lane == 0) at_c = at_r = (uint32_t)R;
  if (lane < S) {
    out.order_conf[base + lane] = (uint8_t)at_c;
    out.order_rank[base + lane] = (uint8_t)at_r;
  }
  // every slot is written (0 for a rule that did not match; slot R = unknown, set only when
  // nothing matched), so the outputs need no clearing before a launch
  if (lane < S) {
    const bool unk = lane == R && nh == 0;
    out.confidence[base + lane] = unk ? D->unknown_confidence : conf;
    out.final_score[base + lane] = unk ? D->unknown_fin : fin;
    out.strength[base + lane] = stren;
  }
  if (lane == 0) {
    out.mask[inc] = (uint32_t)mm;
    out.n_hyp[inc] = (uint8_t)(nh > 0 ? nh : 1);
  }
}

__global__ __launch_bounds__(256) void rules_eval_kernel(
    const RulesDev* __restrict__ D, const uint32_t* __restrict__ row_flags,
    const uint32_t* __restrict__ row_vocab, const uint32_t* __restrict__ row_node,
    const double* __restrict__ row_err, const int64_t* __restrict__ seg_off, int n_incidents,
    egr_rules_out out) {
  __shared__ uint32_t node_key[kWavesPerBlock][kNodeSlots];
  __shared__ uint32_t node_cnt[kWavesPerBlock][kNodeSlots];
  const int wv = threadIdx.x >> 6;
  const int inc = blockIdx.x * kWavesPerBlock + wv;
  if (inc >= n_incidents) return;  // wave-uniform; no block barrier below
  rules_incident(D, row_flags, row_vocab, row_node, row_err, seg_off[inc], seg_off[inc + 1], inc,
                 out, node_key[wv], node_cnt[wv]);
}

// One small incident whose rows travel IN THE KERNEL ARGUMENTS (the drop-in's single calls:
// no host-to-device copy, and no row read over PCIe from mapped host memory -- the argument
// block is in device memory when the kernel starts).  One wave.
constexpr int kSmallRows = 128;
struct SmallRows {
  const RulesDev* D;
  egr_rules_out out;
  int32_t n_rows;
  uint32_t flags[kSmallRows], vocab[kSmallRows], node[kSmallRows];
  double err[kSmallRows];
};

__global__ __launch_bounds__(64) void rules_small_kernel(const SmallRows a) {
  __shared__ uint32_t node_key[kNodeSlots];
  __shared__ uint32_t node_cnt[kNodeSlots];
  rules_incident(a.D, a.flags, a.vocab, a.node, a.err, 0, a.n_rows, 0, a.out, node_key, node_cnt);
}

// Stand-alone ranker: one wave per hypothesis list, stable descending order by counting.
// ---- the single-incident rules server (egr_rules_server_*) --------------------------------
// A one-wave kernel that stays resident while single generate_hypotheses calls keep coming:
// the host writes an incident's encoded rows into a mailbox in fine-grained (coherent) mapped
// host memory and bumps `req`; the wave, polling `req` across PCIe, evaluates the incident
// (rules_incident, the batched kernel's own per-incident code) straight into the mailbox's
// output block and publishes `ack` = req with a system-scope release.  A call then costs the
// PCIe round trips (~a few us) instead of a kernel launch and its event (~20-25 us, with a
// launch-queue tail the host enqueue itself shows: profiles/r05_dropin_latency_*.txt).
// Exit conditions every run reaches: the host's `stop`, SRV_IDLE_POLLS polls without a request
// (~2 ms: a device-wide synchronize waits for the resident wave, so it does not linger) or
// SRV_MAX_POLLS polls in all (~2 s); the wave then clears `alive`, and the host launches it
// again on the next call that finds it gone.
constexpr int kSrvRows = 1024;      // (activity incidents are ~100 rows; the C3 generator's up to ~300)
struct alignas(64) SrvMailbox {
  uint64_t req;                 // host: sequence number of the posted incident (written last)
  uint64_t ack;                 // device: the last sequence number evaluated (outputs ready)
  uint32_t stop;                // host: leave now
  uint32_t alive;               // host sets 1 before a launch; the wave clears it as it leaves
  int32_t n_rows;
  uint32_t pad;
  uint32_t flags[kSrvRows], vocab[kSrvRows], node[kSrvRows];
  double err[kSrvRows];
  // outputs of the incident (S = n_rules + 1 <= EGR_MAX_RULES + 1 slots)
  uint32_t mask;
  uint8_t n_hyp;
  uint8_t order_conf[EGR_MAX_RULES + 1], order_rank[EGR_MAX_RULES + 1];
  double confidence[EGR_MAX_RULES + 1], final_score[EGR_MAX_RULES + 1], strength[EGR_MAX_RULES + 1];
};
constexpr uint64_t SRV_IDLE_POLLS = 1000;
constexpr uint64_t SRV_MAX_POLLS = 1000000;

__global__ __launch_bounds__(64) void rules_server_kernel(const RulesDev* __restrict__ D,
                                                          SrvMailbox* mb) {
  __shared__ uint32_t node_key[kNodeSlots];
  __shared__ uint32_t node_cnt[kNodeSlots];
  const int lane = threadIdx.x;
  uint64_t last = __hip_atomic_load(&mb->ack, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
  uint64_t idle = 0;
  for (uint64_t it = 0; it < SRV_MAX_POLLS; ++it) {
    const uint64_t req = __hip_atomic_load(&mb->req, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
    if (__hip_atomic_load(&mb->stop, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)) break;
    if (req != last) {
      const int n = min(max(mb->n_rows, 0), kSrvRows);
      const egr_rules_out out{&mb->mask, &mb->n_hyp, mb->order_conf, mb->order_rank,
                              mb->confidence, mb->final_score, mb->strength};
      rules_incident(D, mb->flags, mb->vocab, mb->node, mb->err, 0, n, 0, out, node_key, node_cnt);
      __atomic_thread_fence(__ATOMIC_RELEASE);    // (the outputs before the ack, system-wide)
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
      if (lane == 0) __hip_atomic_store(&mb->ack, req, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
      last = req;
      idle = 0;
    } else if (++idle >= SRV_IDLE_POLLS) {
      break;
    } else {
      __builtin_amdgcn_s_sleep(8);
    }
  }
  if (lane == 0) __hip_atomic_store(&mb->alive, 0u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

__global__ __launch_bounds__(256) void rank_kernel(
    const double* __restrict__ conf, const double* __restrict__ catw,
    const double* __restrict__ support, const double* __restrict__ strength,
    const int64_t* __restrict__ list_off, int n_lists, double* __restrict__ out_final,
    int32_t* __restrict__ out_order) {
  const int lane = threadIdx.x & (kWave - 1);
  const int li = blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6);
  if (li >= n_lists) return;
  const int64_t beg = list_off[li], end = list_off[li + 1];
  for (int64_t ib = beg; ib < end; ib += kWave) {
    const int64_t i = ib + lane;
    const double fi =
        i < end ? egr::ranker_final_score(conf[i], catw[i], support[i], strength[i]) : 0.0;
    int pos = 0;
    for (int64_t jb = beg; jb < end; jb += kWave) {
      const int64_t j = jb + lane;
      const double fj_own =
          j < end ? egr::ranker_final_score(conf[j], catw[j], support[j], strength[j]) : 0.0;
      const int lim = (int)min<int64_t>(kWave, end - jb);
      for (int p = 0; p < lim; ++p) {
        const double fj = __shfl(fj_own, p, kWave);
        const int64_t jj = jb + p;
        pos += (fj > fi) || (fj == fi && jj < i);
      }
    }
    if (i < end) {
      out_final[i] = fi;
      out_order[beg + pos] = (int32_t)(i - beg);
    }
  }
}

}  // namespace

// The compiled table of `table` in device memory: compiled on the host (cheap) and looked up
// by content; a table seen for the first time on this device is uploaded once (synchronous
// copy into a new buffer -- never overwritten, so launches in flight keep their table valid).
// A first upload inside a HIP-graph capture is refused: run the table once uncaptured.
static int rules_table_dev(const egr_rule_table& table, hipStream_t stream, const RulesDev** out) {
  RulesDev h;
  std::memset(&h, 0, sizeof h);
  h.n_rules = table.n_rules;
  h.network_vocab_bit = table.network_vocab_bit;
  h.unknown_confidence = table.unknown_confidence;
  h.unknown_fin = egr::ranker_final_score(table.unknown_confidence, table.unknown_category_weight,
                                          0.0, 0.0);
  for (int r = 0; r < table.n_rules; ++r) {
    const egr_rule& rule = table.rules[r];
    RuleDev& d = h.rules[r];
    const int nc = rule.n_conds;
    d.n_conds = nc;
    for (int c = 0; c < EGR_MAX_CONDS; ++c) {
      d.cond_type[c] = rule.cond_type[c];
      d.cond_mask[c] = rule.cond_mask[c];
      d.cond_param[c] = rule.cond_param[c];
    }
    if (nc <= 0) continue;
    // a rule emits only when ALL its conditions hold: strength = the mean of the condition
    // strengths, then the confidence and the ranker's score of that strength
    double ssum = 0.0;
    for (int c = 0; c < nc; ++c) ssum = ssum + rule.cond_strength[c];
    d.str = ssum / (double)(nc > 1 ? nc : 1);
    d.conf = egr::rule_confidence(rule.confidence_base, nc, d.str);
    d.fin = egr::ranker_final_score(d.conf, rule.category_weight, (double)nc, d.str);
  }
  hipDevice_t dev = 0;                           // the stream's device (null stream: current)
  EGR_HIP(hipStreamGetDevice(stream, &dev));
  static std::mutex mu;
  static std::vector<std::tuple<hipDevice_t, std::vector<uint8_t>, RulesDev*>> cache;
  const uint8_t* hb = reinterpret_cast<const uint8_t*>(&h);
  std::lock_guard<std::mutex> lock(mu);
  for (auto& [d, bytes, ptr] : cache)
    if (d == dev && std::memcmp(bytes.data(), hb, sizeof h) == 0) {
      *out = ptr;
      return EGR_OK;
    }
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  EGR_HIP(hipStreamIsCapturing(stream, &cs));
  if (cs != hipStreamCaptureStatusNone)
    return egr::fail(EGR_EINVAL, "egr_rules_eval: a rule table's first launch on a device "
                                 "cannot be captured (launch it once uncaptured)");
  if (cache.size() >= 256)
    return egr::fail(EGR_EINVAL, "egr_rules_eval: more than 256 distinct rule tables");
  RulesDev* ptr = nullptr;
  EGR_HIP(hipMalloc(&ptr, sizeof h));
  EGR_HIP(hipMemcpy(ptr, &h, sizeof h, hipMemcpyHostToDevice));
  cache.emplace_back(dev, std::vector<uint8_t>(hb, hb + sizeof h), ptr);
  *out = ptr;
  return EGR_OK;
}

extern "C" int egr_rules_eval(const egr_rule_table* table, const uint32_t* row_flags,
                              const uint32_t* row_vocab, const uint32_t* row_node,
                              const double* row_err, const int64_t* seg_off, int32_t n_incidents,
                              const egr_rules_out* out, void* stream) {
  if (!table || !out || !seg_off || n_incidents < 0)
    return egr::fail(EGR_EINVAL, "egr_rules_eval: NULL argument");
  if (table->n_rules < 0 || table->n_rules > EGR_MAX_RULES)
    return egr::fail(EGR_EINVAL, "egr_rules_eval: n_rules out of range");
  for (int r = 0; r < table->n_rules; ++r)
    if (table->rules[r].n_conds < 0 || table->rules[r].n_conds > EGR_MAX_CONDS)
      return egr::fail(EGR_EINVAL, "egr_rules_eval: n_conds out of range");
  if (!out->mask || !out->n_hyp || !out->order_conf || !out->order_rank || !out->confidence ||
      !out->final_score || !out->strength)
    return egr::fail(EGR_EINVAL, "egr_rules_eval: NULL output");
  if (n_incidents == 0) return EGR_OK;
  const RulesDev* D = nullptr;
  const int rc = rules_table_dev(*table, (hipStream_t)stream, &D);
  if (rc != EGR_OK) return rc;
  const dim3 grid((n_incidents + kWavesPerBlock - 1) / kWavesPerBlock);
  hipLaunchKernelGGL(rules_eval_kernel, grid, dim3(256), 0, (hipStream_t)stream, D, row_flags,
                     row_vocab, row_node, row_err, seg_off, n_incidents, *out);
  EGR_CHECK_LAUNCH();
  return EGR_OK;
}

// One call for the drop-in's single / coalesced launches: inputs staged in ONE host buffer
// (pinned) go up in one copy, the kernel runs on the device copy, the outputs come back in one
// copy -- three stream operations, one host call.  off[12] = byte offsets (in both buffers) of
// flags, vocab, node, err, seg_off, mask, n_hyp, order_conf, order_rank, confidence,
// final_score, strength; [0, in_bytes) is copied up and [out_lo, out_hi) copied back.
extern "C" int egr_rules_eval_staged(const egr_rule_table* table, const void* host_in,
                                     void* dev_buf, void* host_out, const int64_t* off,
                                     int64_t in_bytes, int64_t out_lo, int64_t out_hi,
                                     int32_t n_incidents, void* stream) {
  if (!table || !host_in || !dev_buf || !host_out || !off || in_bytes < 0 || out_lo < in_bytes ||
      out_hi < out_lo || n_incidents < 0)
    return egr::fail(EGR_EINVAL, "egr_rules_eval_staged: bad arguments");
  hipStream_t st = (hipStream_t)stream;
  uint8_t* d = static_cast<uint8_t*>(dev_buf);
  if (in_bytes) EGR_HIP(hipMemcpyAsync(d, host_in, (size_t)in_bytes, hipMemcpyHostToDevice, st));
  const egr_rules_out out{reinterpret_cast<uint32_t*>(d + off[5]), d + off[6], d + off[7], d + off[8],
                          reinterpret_cast<double*>(d + off[9]), reinterpret_cast<double*>(d + off[10]),
                          reinterpret_cast<double*>(d + off[11])};
  const int rc = egr_rules_eval(table, reinterpret_cast<const uint32_t*>(d + off[0]),
                                reinterpret_cast<const uint32_t*>(d + off[1]),
                                reinterpret_cast<const uint32_t*>(d + off[2]),
                                reinterpret_cast<const double*>(d + off[3]),
                                reinterpret_cast<const int64_t*>(d + off[4]), n_incidents, &out, stream);
  if (rc != EGR_OK) return rc;
  if (out_hi > out_lo)
    EGR_HIP(hipMemcpyAsync(static_cast<uint8_t*>(host_out) + out_lo, d + out_lo,
                           (size_t)(out_hi - out_lo), hipMemcpyDeviceToHost, st));
  return EGR_OK;
}

extern "C" int egr_rules_eval_small(const egr_rule_table* table, const uint32_t* row_flags,
                                    const uint32_t* row_vocab, const uint32_t* row_node,
                                    const double* row_err, int32_t n_rows,
                                    const egr_rules_out* out, void* stream) {
  if (!table || !out || n_rows < 0 || n_rows > kSmallRows ||
      (n_rows > 0 && (!row_flags || !row_vocab || !row_node || !row_err)))
    return egr::fail(EGR_EINVAL, "egr_rules_eval_small: bad arguments (at most 128 rows)");
  if (!out->mask || !out->n_hyp || !out->order_conf || !out->order_rank || !out->confidence ||
      !out->final_score || !out->strength)
    return egr::fail(EGR_EINVAL, "egr_rules_eval_small: NULL output");
  if (table->n_rules < 0 || table->n_rules > EGR_MAX_RULES)
    return egr::fail(EGR_EINVAL, "egr_rules_eval_small: n_rules out of range");
  const RulesDev* D = nullptr;
  const int rc = rules_table_dev(*table, (hipStream_t)stream, &D);
  if (rc != EGR_OK) return rc;
  SmallRows a;
  a.D = D;
  a.out = *out;
  a.n_rows = n_rows;
  if (n_rows > 0) {
    std::memcpy(a.flags, row_flags, sizeof(uint32_t) * n_rows);
    std::memcpy(a.vocab, row_vocab, sizeof(uint32_t) * n_rows);
    std::memcpy(a.node, row_node, sizeof(uint32_t) * n_rows);
    std::memcpy(a.err, row_err, sizeof(double) * n_rows);
  }
  hipLaunchKernelGGL(rules_small_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, a);
  EGR_CHECK_LAUNCH();
  return EGR_OK;
}

struct egr_rules_server {
  int device = 0;
  const RulesDev* D = nullptr;
  SrvMailbox* h = nullptr;      // host view of the mailbox (mapped, coherent)
  SrvMailbox* d = nullptr;      // the device's address of the same bytes
  hipStream_t st = nullptr;     // the server wave's own stream
  int S = 0;
  uint64_t seq = 0;             // last posted sequence number
  bool launched = false;
};

static int srv_launch(egr_rules_server* s) {
  __atomic_store_n(&s->h->alive, 1u, __ATOMIC_RELEASE);
  hipLaunchKernelGGL(rules_server_kernel, dim3(1), dim3(64), 0, s->st, s->D, s->d);
  EGR_CHECK_LAUNCH();
  s->launched = true;
  return EGR_OK;
}

extern "C" int egr_rules_server_create(const egr_rule_table* table, int32_t device,
                                       egr_rules_server** out) {
  if (!table || !out || table->n_rules < 0 || table->n_rules > EGR_MAX_RULES)
    return egr::fail(EGR_EINVAL, "egr_rules_server_create: bad arguments");
  for (int r = 0; r < table->n_rules; ++r)
    if (table->rules[r].n_conds < 0 || table->rules[r].n_conds > EGR_MAX_CONDS)
      return egr::fail(EGR_EINVAL, "egr_rules_server_create: n_conds out of range");
  *out = nullptr;
  egr::DeviceGuard guard(device);
  auto* s = new egr_rules_server();
  s->device = device;
  s->S = table->n_rules + 1;
  hipError_t e = hipStreamCreateWithFlags(&s->st, hipStreamNonBlocking);
  void* h = nullptr;
  if (e == hipSuccess) e = hipHostMalloc(&h, sizeof(SrvMailbox), hipHostMallocMapped | hipHostMallocCoherent);
  if (e == hipSuccess) {
    s->h = static_cast<SrvMailbox*>(h);
    std::memset(s->h, 0, sizeof(SrvMailbox));
    void* d = nullptr;
    e = hipHostGetDevicePointer(&d, h, 0);
    s->d = static_cast<SrvMailbox*>(d);
  }
  int rc = e == hipSuccess ? EGR_OK : egr::fail(EGR_EDEVICE, std::string("egr_rules_server_create: ") +
                                                             hipGetErrorString(e));
  if (rc == EGR_OK) rc = rules_table_dev(*table, s->st, &s->D);
  if (rc != EGR_OK) {
    egr_rules_server_free(s);
    return rc;
  }
  *out = s;
  return EGR_OK;
}

extern "C" int egr_rules_server_post(egr_rules_server* s, const uint32_t* row_flags,
                                     const uint32_t* row_vocab, const uint32_t* row_node,
                                     const double* row_err, int32_t n_rows) {
  if (!s || n_rows < 0 || n_rows > kSrvRows ||
      (n_rows > 0 && (!row_flags || !row_vocab || !row_node || !row_err)))
    return egr::fail(EGR_EINVAL, "egr_rules_server_post: bad arguments (at most 1024 rows)");
  SrvMailbox* m = s->h;
  if (__atomic_load_n(&m->ack, __ATOMIC_ACQUIRE) != s->seq)
    return egr::fail(EGR_ESTATE, "egr_rules_server_post: the previous incident is still pending");
  if (n_rows > 0) {
    std::memcpy(m->flags, row_flags, sizeof(uint32_t) * n_rows);
    std::memcpy(m->vocab, row_vocab, sizeof(uint32_t) * n_rows);
    std::memcpy(m->node, row_node, sizeof(uint32_t) * n_rows);
    std::memcpy(m->err, row_err, sizeof(double) * n_rows);
  }
  m->n_rows = n_rows;
  __atomic_store_n(&m->req, ++s->seq, __ATOMIC_RELEASE);     // (the rows before the request)
  if (!__atomic_load_n(&m->alive, __ATOMIC_ACQUIRE)) {
    egr::DeviceGuard guard(s->device);
    return srv_launch(s);
  }
  return EGR_OK;
}

extern "C" int egr_rules_server_poll(egr_rules_server* s, uint32_t* mask, uint8_t* n_hyp,
                                     uint8_t* order_conf, uint8_t* order_rank, double* confidence,
                                     double* final_score, double* strength) {
  if (!s || !mask || !n_hyp || !order_conf || !order_rank || !confidence || !final_score || !strength)
    return egr::fail(EGR_EINVAL, "egr_rules_server_poll: bad arguments");
  SrvMailbox* m = s->h;
  if (__atomic_load_n(&m->ack, __ATOMIC_ACQUIRE) != s->seq) {
    // the wave left (idle or lifetime bound) before it saw this request: start another one,
    // which picks the pending request up (it starts from the last acknowledged number)
    if (!__atomic_load_n(&m->alive, __ATOMIC_ACQUIRE)) {
      egr::DeviceGuard guard(s->device);
      const int rc = srv_launch(s);
      if (rc != EGR_OK) return rc;
    }
    return 0;
  }
  const int S = s->S;
  *mask = m->mask;
  *n_hyp = m->n_hyp;
  std::memcpy(order_conf, m->order_conf, S);
  std::memcpy(order_rank, m->order_rank, S);
  std::memcpy(confidence, m->confidence, sizeof(double) * S);
  std::memcpy(final_score, m->final_score, sizeof(double) * S);
  std::memcpy(strength, m->strength, sizeof(double) * S);
  return 1;
}

extern "C" void egr_rules_server_free(egr_rules_server* s) {
  if (!s) return;
  egr::DeviceGuard guard(s->device);
  if (s->h) {
    __atomic_store_n(&s->h->stop, 1u, __ATOMIC_RELEASE);
    if (s->launched && s->st) (void)hipStreamSynchronize(s->st);   // (the wave leaves at its next poll)
    (void)hipHostFree(s->h);
  }
  if (s->st) (void)hipStreamDestroy(s->st);
  delete s;
}

extern "C" int egr_rank(const double* confidence, const double* cat_weight, const double* support,
                        const double* strength, const int64_t* list_off, int32_t n_lists,
                        double* out_final, int32_t* out_order, void* stream) {
  if (!list_off || n_lists < 0) return egr::fail(EGR_EINVAL, "egr_rank: bad arguments");
  if (n_lists == 0) return EGR_OK;
  const dim3 grid((n_lists + kWavesPerBlock - 1) / kWavesPerBlock);
  hipLaunchKernelGGL(rank_kernel, grid, dim3(256), 0, (hipStream_t)stream, confidence,
                     cat_weight, support, strength, list_off, n_lists, out_final, out_order);
  EGR_CHECK_LAUNCH();
  return EGR_OK;
}
