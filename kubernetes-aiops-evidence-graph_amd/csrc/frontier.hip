// Frontier engine: the whole graph stage of one incident column -- apoc-style k-hop reach
// (A8, src/database/neo4j.py:169-202), typed k-hop propagation (A9) and the
// per-incident top-k -- in ONE workgroup, with the incident's state in an LDS hash table.
//
// Why: a column's scores are non-zero only within `hops` hops of its seeds.  On the 100k-pod
// graph that is ~1.9k of 229k vertices after 3 hops (0.8 %), so the dense [V x B] sweep of
// propagate.hip spends >99 % of its HBM bytes on exact zeros.  Here a workgroup keeps only the
// touched vertices: key = vertex id, s = current score, fl = reach depth + 1 (0 = not reached).
//
// Exactness (bit-identical to the dense plan and to oracle/egraph_oracle.c): for every member
// v the pull  s'[v] = sum_{e in row v, CSR order} fmaf(val_e, s[col_e], acc)  then  s'[v] + s0[v]
// is the dense recurrence with the terms of non-members skipped; a non-member's dense value is
// exactly +0 and fmaf(w, +0, acc) == acc for finite w and acc != -0 (acc starts at +0 and can
// never become -0 under round-to-nearest), so skipping them changes no bit.  Members are
// (seeds) U (N(u) for every member u with s[u] != 0) U (reach set), which contains every
// vertex whose dense value can be non-zero.
//
// Work layout: a hop is two phases over the member list, GROW (the reach level and the
// expansion of the non-zero members insert their neighbours) and PULL (the members an
// expansion touched recompute their score).  A wave takes 64 members at a time: a row of up to
// the geometry's light limit (12 / 16 entries) is one lane's, which loads and probes its first
// entries at once and runs the in-order fmaf chain in registers, the rest of every row (its
// tail) spread over the wave one entry per lane with the chain continued from the wave's LDS
// pair scratch; a longer (hub) row is taken by the whole wave, 64 entries per round, its chain
// run over its non-zero terms only.  Top-k packs (score, vertex) into one u64 key: each wave
// extracts its k best with DPP wave-max rounds, wave 0 merges the lists.
//
// Capacity: three LDS geometries of the kernels (frontier_body.h).  The narrow one (pruned
// top-k runs: ~0.6k members per column on C3) holds 1536 slots and one score buffer in 22 KB,
// 4-wave workgroups, seven per CU; the mid one (C4-sized columns, ~1.4k members) 2816 slots in
// 39 KB, four per CU; the wide one (member-pool runs, every member's score exact, and the
// retry of what overflows the others) 6144 slots in 80 KB, 8-wave workgroups, two per CU.  A
// column with more members than the table's limit is flagged and redone by the next table, and
// last by the global-memory variant of the same code (a table of >= 2V slots per resident
// workgroup, never overflows), launched unconditionally (it drains an empty work list at once).
// A narrow-table overflow (pruned C3: 0.56 % of the columns, 1.2-1.6k members) continues in its
// own workgroup instead, in a global-memory region (egr_frontier_set_continuation): those columns
// start early, costliest first, and finish while the grid runs -- the serial wide-retry grid
// after it was 6.6 % of the launch (C3 -3 % per step, profiles/r05_ab_continuation.txt).
//
// (Round 3 measured a two-phase alternative for top-k runs -- discover the column's member set
// and its member-restricted local CSR first, then propagate in LDS only -- at 0.14-0.16 ms per
// C3 step against 0.065 for this kernel: its discovery walks cost as much as the pulls they
// replace, and hub members serialise the LDS hops; profiles/r03_ab_local_kernel.txt.)
#include <algorithm>
#include <type_traits>
#include <vector>

#include "graph_dev.h"

// Per-phase wall-clock stamps ($EGRAPH_FRONTIER_PROFILE, scripts/frontier_profile.py) exist only
// in a profiling build (-DEGR_FR_PROFILE=1, scripts/build_variant.sh): the shipped kernels carry
// no timing state in their registers.
#ifndef EGR_FR_PROFILE
#define EGR_FR_PROFILE 0
#endif
#define FR_PROF_ON(A) (EGR_FR_PROFILE && (A).prof != nullptr)

using egr::DeviceGuard;
using egr::dalloc;
using egr::dfree;

namespace {

constexpr uint32_t EMPTY = 0xFFFFFFFFu;
constexpr uint32_t NO_NODE = EGR_NO_NODE;
constexpr int KMAXF = 16;
constexpr uint8_t FL_DEPTH = 0x3F;          // fl: depth + 1 in the low bits
constexpr uint8_t FL_SEED = 0x40;           // the member is one of the column's seeds
constexpr uint8_t FL_CLAIM = 0x80;          // a seed entry already represents this vertex
constexpr uint8_t NEED_EXCL = 0x80;         // need: a candidate carrying the excluded label
constexpr uint8_t NEED_REC = 0x04;          // need: the member's row slots are recorded (FR_REC)
constexpr int MAX_HOPS = 60;
constexpr int PROF_SLOTS = 40;
// a continuation region (egr_frontier_set_continuation): 8192 slots (2048 four-slot buckets),
// members up to 6144 (load 0.75) -- more than the wide LDS table's 4608, so what the wide retry
// used to take fits.  Keys, scores, flags, need bits, then the member list and pull results.
constexpr uint32_t CONT_CAP = 8192, CONT_LIMIT = 6144;
constexpr size_t CONT_REGION_BYTES = 10 * (size_t)CONT_CAP + 8 * (size_t)CONT_LIMIT;

struct FArgs {
  const uint32_t* row_ptr;
  const uint2* cv;             // (col, val bits) per CSR entry
  const uint8_t* vlabel;
  // the snapshot's locality layout (layout.hip): row_ptr / cv / vlabel are in its internal ids;
  // inputs are mapped in through perm, outputs and tie-breaks use iperm (nullptr: identity)
  const uint32_t* perm;
  const uint32_t* iperm;
  uint32_t V;
  int B, hops, k, exclude;
  int prune;                   // no member pool: the last hop pulls the candidates only
  const uint32_t* seed_ptr;    // [B+1] per column
  const uint32_t* seed_vert;   // grouped by column, any order, duplicates allowed
  const float* seed_val;       // (duplicates are max-combined in the kernel, as fmaxf)
  uint32_t n_seeds;            // entries in seed_vert / seed_val (seed_ptr is clamped to it)
  uint2* seed_rep;             // per seed entry: (slot, s0 bits) of a vertex's representative
  const uint32_t* sources;     // [B] incident vertex per column (EGR_NO_NODE: none)
  const uint32_t* order;       // [B] launch order: workgroup i runs column order[i] (costly first)
  uint32_t* seed_cnt;          // [2B] set_seeds' counters / costs, zeroed per column once
                               // consumed (nullptr: grouped seeds, nothing to zero)
  uint32_t* out_ids;           // [B*k]
  float* out_scores;
  // member pool: every column's (vertex, score, depth+1) after the last hop
  uint32_t* pool_v;
  float* pool_s;
  uint8_t* pool_d;
  unsigned long long pool_cap;
  unsigned long long* pool_ctr;
  unsigned long long* mem_off;  // [B]
  uint32_t* mem_cnt;            // [B], EGR_NO_NODE = not kept (pool full)
  // overflow work list
  uint32_t* ovf_list;           // where an LDS kernel hands on its overflowing columns
  uint32_t* ovf_n;
  uint32_t* ovf_next;           // the global-memory variant's work counter (over ovf_list)
  uint32_t* retry_next;         // the wide retry's work counter (over retry_list)
  uint32_t ovf_cap;             // ovf_list entries; further overflowing columns go to spill_*
  uint32_t* spill_list;
  uint32_t* spill_n;
  const uint32_t* retry_list;   // the retry kernel's input list and count (drained through
  const uint32_t* retry_n;      // the retry_next work counter)
  float* lsnew;                 // [B][LLIMIT] pull results by member index
  // global tables (one per resident workgroup of the fallback kernel)
  uint32_t* gkeys;              // [nbig][gcap]
  float* gs;                    // [nbig][gcap]
  uint8_t* gfl;                 // [nbig][gcap]
  uint8_t* gneed;               // [nbig][gcap]
  uint32_t* gmlist;             // [nbig][V]
  float* gsnew;                 // [nbig][V]
  uint32_t gcap;
  unsigned long long* prof;     // [B][PROF_SLOTS] wall-clock stamps per phase, or nullptr
  // [0] CSR entries gathered by pulls (col + val), [1] entries read by expansions (col),
  // [2] rows walked (row_ptr pairs), [3] members, [4] columns that overflowed an LDS table,
  // [5] columns finished in a continuation region
  unsigned long long* stats;
  // overflow continuation (egr_frontier_set_continuation): cont_n global-memory table regions
  // of CONT_REGION_BYTES from cont_base, claimed through *cont_ctr (zeroed with the run's
  // counters)
  unsigned long long* cont_ctr;
  uint32_t cont_n;
  uint8_t* cont_base;
  uint32_t* ghist;              // the grouped cost histogram: zeroed by the run's last kernel
  uint16_t* rec;                // [B][REC_STRIDE] row slot records of the narrow table (FR_REC;
                                // nullptr: off)
};

struct alignas(8) Pair2 { uint32_t c0, v0, c1, v1; };   // two CSR entries, 8-B aligned
struct alignas(4) RowPair { uint32_t e0, e1; };           // row_ptr[v], row_ptr[v + 1]

// The kernels' table geometries (frontier_body.h): the wide table keeps every member of a
// column (member-pool runs: exact scores for every member, ~1.9k per column on C3; the retry of
// what overflows a smaller table), 80 KB with a 2^15-bit filter so two fit a CU, and since
// round 4 the narrow / mid tables' light-row treatment (LDS hub chains, tails after 8 entries,
// limit 16: C4 -1.6 %, profiles/r04_ab_wide_tails.txt); the narrow one serves the pruned top-k
// runs (~0.6k members per column on C3), whose 22 KB of LDS and 72 VGPRs fit seven 4-wave
// workgroups per CU instead of two 8-wave ones.
namespace fr_wide {
#define FR_FT 512
#define FR_LCAP 6144
#define FR_LLIMIT 4608
#define FR_BLOOM_LOG 15
#define FR_WAVES_PER_EU 4
#define FR_KERNELS 7
#define FR_LMAX 16
#define FR_FIND_SELECT 1
#define FR_HEAD 8
#include "frontier_body.h"
#undef FR_FT
#undef FR_LCAP
#undef FR_LLIMIT
#undef FR_BLOOM_LOG
#undef FR_WAVES_PER_EU
#undef FR_LMAX
#undef FR_FIND_SELECT
#undef FR_HEAD
#undef FR_KERNELS
}  // namespace fr_wide

namespace fr_narrow {
// hub-row chains through LDS, one lane (+4 % at three batches in flight,
// profiles/r02_ab_hubchain.txt); one LDS score buffer (pull results by member index in HBM and
// a copy phase) and a 2^14-bit filter: 22 KB and 72 VGPRs (3 spilled in the plain kernel, 18
// in the continuation instantiation <true> the headline runs), seven workgroups per
// CU (-1.7 % against six at 24 KB with a 2^15-bit filter, profiles/r04_ab_one_buffer.txt).  Round 2's two slot-indexed buffers
// (no copy phase, +2.5 % at five per CU, profiles/r02_ab_frontier_session3.txt) lost to the
// sixth workgroup once the light-row tails cut the registers: C3 -4.5 %
// (profiles/r04_ab_one_buffer.txt; round 3 measured six per CU neutral at 94 VGPRs).
#define FR_FT 256
#define FR_LCAP 1536
#define FR_LLIMIT 1152
#define FR_BLOOM_LOG 14
#define FR_WAVES_PER_EU 7
#define FR_KERNELS 1
#define FR_LMAX 12
#define FR_FIND_SELECT 0
#define FR_HEAD 4
// row slot records (frontier_body.h, FR_REC): measured and off -- with mixed walks a wave still
// runs the probe code for its unrecorded rows, VALU fell 6.4 % and the launch 0.3 %, behind the
// plain kernel's registers (profiles/r06_ab_row_records.txt); -DEGR_FR_NARROW_REC=1 builds it
#ifndef EGR_FR_NARROW_REC
#define EGR_FR_NARROW_REC 0
#endif
#define FR_REC EGR_FR_NARROW_REC
#include "frontier_body.h"
#undef FR_FT
#undef FR_LCAP
#undef FR_LLIMIT
#undef FR_BLOOM_LOG
#undef FR_WAVES_PER_EU
#undef FR_LMAX
#undef FR_FIND_SELECT
#undef FR_HEAD
#undef FR_KERNELS
}  // namespace fr_narrow

// A 2.8k-slot table at 256 threads for graphs whose columns mostly overflow the narrow table
// but fit 2.1k members (the dense C4: ~1.4k, 92 % of its columns): the first attempt of a
// mid-first frontier (egr_frontier_set_wide_first(f, 2)), whose overflowing columns take the
// wide retry.  One LDS score buffer (pull results by member index in HBM and a copy phase, like
// the wide table): 39 KB, four workgroups per CU -- with the second buffer it was 50 KB and three,
// 16 % slower on C4 (profiles/r04_ab_mid_one_buffer.txt); C4 -2.4 % per step against
// wide-first at its start (profiles/r04_ab_mid_first.txt).
namespace fr_mid {
#define FR_FT 256
#define FR_LCAP 2816
#define FR_LLIMIT 2112
#define FR_BLOOM_LOG 15
#define FR_WAVES_PER_EU 4
#define FR_KERNELS 1
#define FR_LMAX 16
#define FR_FIND_SELECT 1
#define FR_HEAD 8
#include "frontier_body.h"
#undef FR_FT
#undef FR_LCAP
#undef FR_LLIMIT
#undef FR_BLOOM_LOG
#undef FR_WAVES_PER_EU
#undef FR_LMAX
#undef FR_FIND_SELECT
#undef FR_HEAD
#undef FR_KERNELS
}  // namespace fr_mid

// The overflow fallback's launch geometry: one wave per workgroup.  Its grid is launched after
// every narrow run and nearly always finds no overflowing column; a one-wave workgroup is
// dispatched as soon as a single SIMD has room, instead of waiting behind the other batch in
// flight for a CU to drain (scripts/ab_global.sh).  Only frontier_global_kernel is launched
// from this instantiation.
namespace fr_fallback {
#define FR_FT 64
#define FR_LCAP 256
#define FR_LLIMIT 192
#define FR_BLOOM_LOG 10
#define FR_WAVES_PER_EU 4
#define FR_KERNELS 4
#define FR_LMAX 12
#define FR_FIND_SELECT 0
#define FR_HEAD 0
#include "frontier_body.h"
#undef FR_FT
#undef FR_LCAP
#undef FR_LLIMIT
#undef FR_BLOOM_LOG
#undef FR_WAVES_PER_EU
#undef FR_LMAX
#undef FR_FIND_SELECT
#undef FR_HEAD
#undef FR_KERNELS
}  // namespace fr_fallback

// members -> dense row-major scores [V][B] / reach bits [W][V] (inspection and tests)
__global__ void scatter_scores_kernel(const uint32_t* __restrict__ pool_v,
                                      const float* __restrict__ pool_s,
                                      const unsigned long long* __restrict__ mem_off,
                                      const uint32_t* __restrict__ mem_cnt, int B,
                                      float* __restrict__ out) {
  const int b = blockIdx.x;
  const uint32_t n = mem_cnt[b];
  if (n == NO_NODE) return;
  const unsigned long long o = mem_off[b];
  for (uint32_t i = threadIdx.x; i < n; i += blockDim.x)
    out[(size_t)pool_v[o + i] * B + b] = pool_s[o + i];
}

__global__ void scatter_reach_kernel(const uint32_t* __restrict__ pool_v,
                                     const uint8_t* __restrict__ pool_d,
                                     const unsigned long long* __restrict__ mem_off,
                                     const uint32_t* __restrict__ mem_cnt, uint32_t V,
                                     unsigned long long* __restrict__ out) {
  const int b = blockIdx.x;
  const uint32_t n = mem_cnt[b];
  if (n == NO_NODE) return;
  const unsigned long long o = mem_off[b];
  for (uint32_t i = threadIdx.x; i < n; i += blockDim.x)
    if (pool_d[o + i]) atomicOr(&out[(size_t)(b >> 6) * V + pool_v[o + i]], 1ull << (b & 63));
}

// seeds grouped by column without a sort: count, one-block scan, scatter.  Seeds usually arrive
// grouped by column, so a wave's lanes form runs of equal columns: one atomic per run (the run's
// first lane adds the run length; the others take their rank in the run).
struct SeedRun {
  bool ok;
  uint32_t col, leader, rank, len;
};

__device__ __forceinline__ SeedRun seed_run(const uint32_t* __restrict__ sv,
                                            const uint32_t* __restrict__ sc, int64_t n, uint32_t V,
                                            int B) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int lane = threadIdx.x & 63;
  SeedRun r;
  r.ok = i < n && sv[i] < V && sc[i] < (uint32_t)B;
  r.col = r.ok ? sc[i] : 0xFFFFFFFFu;
  const uint32_t prev = __shfl_up(r.col, 1, 64);
  const bool start = r.ok && (lane == 0 || prev != r.col);
  const uint64_t starts = __ballot(start);
  const uint64_t below = starts & ((2ull << lane) - 1ull);          // starts at lanes <= lane
  r.leader = below ? 63u - (uint32_t)__clzll((long long)below) : 0u;
  r.rank = (uint32_t)lane - r.leader;
  const uint64_t above = starts & ~((2ull << lane) - 1ull);          // starts at lanes > lane
  const uint32_t next = above ? (uint32_t)__ffsll((long long)above) - 1u : 64u;
  // a run ends at the next start or at the first invalid lane
  const uint64_t okm = __ballot(r.ok);
  const uint64_t bad_above = ~okm & ~((2ull << lane) - 1ull);
  const uint32_t nbad = bad_above ? (uint32_t)__ffsll((long long)bad_above) - 1u : 64u;
  r.len = min(next, nbad) - r.leader;
  return r;
}

// A run's pool / stats counters and overflow-list heads cleared in one launch (one graph node
// instead of two fill nodes in a captured replay: each node costs its own dispatch gap).
__global__ __launch_bounds__(64) void clear_counters_kernel(unsigned long long* ctr, uint32_t* ovf) {
  const int tid = threadIdx.x;
  if (tid < 8) ctr[tid] = 0;
  if (tid < 4) ovf[tid] = 0;
}

// cnt[c] += seeds of column c; cost[c] += 1 + degree of each seed vertex (a cheap predictor of
// the column's frontier work, for longest-first launch order).  Both are wave-aggregated: one
// atomic per run of equal columns (a segmented sum over an inclusive wave scan).
__global__ void seed_count_kernel(const uint32_t* __restrict__ sv, const uint32_t* __restrict__ sc,
                                  int64_t n, uint32_t V, int B, const uint32_t* __restrict__ row_ptr,
                                  uint32_t* cnt, uint32_t* cost) {
  const SeedRun r = seed_run(sv, sc, n, V, B);
  const int lane = threadIdx.x & 63;
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t d = 0;
  if (r.ok) {
    const uint32_t v = sv[i];
    d = 1u + row_ptr[v + 1] - row_ptr[v];
  }
  uint32_t incl = d;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const uint32_t x = __shfl_up(incl, off, 64);
    if (lane >= off) incl += x;
  }
  const int last = (int)(r.leader + r.len) - 1;
  const uint32_t hi = __shfl(incl, r.ok ? last : lane, 64);
  const uint32_t lo = __shfl(incl, r.ok && r.leader > 0 ? (int)r.leader - 1 : lane, 64);
  if (r.ok && r.rank == 0) {
    atomicAdd(&cnt[r.col], r.len);
    atomicAdd(&cost[r.col], hi - (r.leader > 0 ? lo : 0u));
  }
}

// ptr[0..B] = exclusive scan of cnt; cnt becomes the scatter cursor (= ptr[c]); order = the
// columns by descending cost bucket (a log-scale counting sort: longest-processing-time-first
// launch order, so the costly columns do not start in the last round); the next run's counters
// and overflow lists are zeroed.  One block of SCAN_T threads, each owning a contiguous run of
// columns.  SCAN_T is 256 (one wave per SIMD), not 1024: the block is launched while the other
// batches in flight hold the CUs, and a small block is dispatched as soon as one workgroup of
// theirs finishes (profiles/r01_ab_scan_t.txt).
constexpr int COST_BUCKETS = 64;
constexpr int SCAN_T = 256;

__device__ __forceinline__ int cost_bucket(uint32_t cost) {
  const int lg = (int)(__log2f((float)cost + 1.0f) * 3.0f);
  return COST_BUCKETS - 1 - min(COST_BUCKETS - 1, lg);
}

__global__ __launch_bounds__(SCAN_T) void seed_scan_kernel(uint32_t* cnt, int B, uint32_t* ptr,
                                                         const uint32_t* __restrict__ cost,
                                                         uint32_t* order, unsigned long long* ctr,
                                                         uint32_t* ovf) {
  __shared__ uint32_t part[SCAN_T];
  __shared__ uint32_t hist[COST_BUCKETS];
  const int tid = threadIdx.x;
  const int per = (B + SCAN_T - 1) / SCAN_T;
  const int c0 = min(B, tid * per), c1 = min(B, c0 + per);
  uint32_t sum = 0;
  for (int c = c0; c < c1; ++c) sum += cnt[c];
  part[tid] = sum;
  if (tid < COST_BUCKETS) hist[tid] = 0;
  __syncthreads();
  for (int off = 1; off < SCAN_T; off <<= 1) {   // Hillis-Steele inclusive scan of the run sums
    const uint32_t x = tid >= off ? part[tid - off] : 0u;
    __syncthreads();
    part[tid] += x;
    __syncthreads();
  }
  uint32_t run = tid ? part[tid - 1] : 0u;
  for (int c = c0; c < c1; ++c) {
    const uint32_t x = cnt[c];
    ptr[c] = run;
    cnt[c] = run;
    run += x;
  }
  if (tid == SCAN_T - 1) ptr[B] = part[SCAN_T - 1];
  if (tid < 8) ctr[tid] = 0;      // the next run's pool / stats counters and overflow lists
  if (tid < 4) ovf[tid] = 0;
  for (int c = c0; c < c1; ++c) atomicAdd(&hist[cost_bucket(cost[c])], 1u);
  __syncthreads();
  if (tid == 0) {
    uint32_t acc = 0;
    for (int j = 0; j < COST_BUCKETS; ++j) {
      const uint32_t x = hist[j];
      hist[j] = acc;
      acc += x;
    }
  }
  __syncthreads();
  for (int c = c0; c < c1; ++c) order[atomicAdd(&hist[cost_bucket(cost[c])], 1u)] = (uint32_t)c;
}

// Grouped runs without a caller order (egr_frontier_run_grouped with order = NULL): the columns
// costliest-first by the log-scale cost bucket of seed_scan_kernel, where the cost of column c is
// the sum over its seeds of 1 + the seed vertex's degree (the predictor set_seeds sorts by;
// original ids, canonical row_ptr).  Order within a bucket is arbitrary -- results do not depend
// on the order.  Two many-block kernels (one block with a serial histogram was 128 us at 40k
// columns): the first computes 64 columns per block (16 lanes per column: C3's ~74 seeds per
// column are ~5 rounds of two dependent loads, not ~19 at 4 lanes -- 12.6 us per 20k-column
// launch), ranks them inside the block with LDS atomics and claims each bucket's block total
// with ONE global atomic on the histogram `ghist` (zero at its start: the previous run's last
// kernel cleared it;
// 64 columns per block keep those atomics few); the second scans the 64-bucket histogram in one
// wave per block and scatters each column to its slot.
constexpr int COST_LANES = 16, COST_T = 64 * COST_LANES;
__global__ __launch_bounds__(COST_T) void grouped_cost_kernel(const uint32_t* __restrict__ seed_ptr,
                                                          const uint32_t* __restrict__ seed_v,
                                                          uint32_t n_seeds, int B,
                                                          const uint32_t* __restrict__ row_ptr,
                                                          uint32_t V, uint32_t* __restrict__ gbk,
                                                          uint32_t* __restrict__ gpos,
                                                          uint32_t* __restrict__ ghist) {
  __shared__ uint32_t hist[COST_BUCKETS];
  __shared__ uint32_t base[COST_BUCKETS];
  const int tid = threadIdx.x, q = tid & (COST_LANES - 1);
  const int c = (int)(blockIdx.x * 64 + tid / COST_LANES);
  if (tid < COST_BUCKETS) hist[tid] = 0;
  uint32_t sum = 0;
  if (c < B) {
    const uint32_t s0 = min(seed_ptr[c], n_seeds), s1 = max(s0, min(seed_ptr[c + 1], n_seeds));
    for (uint32_t i = s0 + q; i < s1; i += COST_LANES) {
      const uint32_t v = seed_v[i];
      if (v < V) sum += 1u + row_ptr[v + 1] - row_ptr[v];
    }
  }
#pragma unroll
  for (int o = 1; o < COST_LANES; o <<= 1) sum += __shfl_xor(sum, o, 64);
  __syncthreads();
  const int bk = cost_bucket(sum);
  uint32_t lpos = 0;
  if (c < B && q == 0) lpos = atomicAdd(&hist[bk], 1u);
  __syncthreads();
  if (tid < COST_BUCKETS) base[tid] = hist[tid] ? atomicAdd(&ghist[tid], hist[tid]) : 0u;
  __syncthreads();
  if (c < B && q == 0) {
    gbk[c] = (uint32_t)bk;
    gpos[c] = base[bk] + lpos;
  }
}

// (It also clears the run's counters -- block 0, ahead of the frontier kernel that counts into
// them -- so a grouped run launches no clear_counters_kernel of its own; the histogram is
// zeroed again by the run's last kernel, frontier_global_kernel, for the next run; a run that
// returned before enqueueing that kernel leaves egr_frontier::ghist_dirty set and the next
// grouped run clears the histogram first.  A position past B cannot occur then; it is dropped
// rather than written out of bounds.)
__global__ __launch_bounds__(256) void cost_order_kernel(const uint32_t* __restrict__ gbk,
                                                        const uint32_t* __restrict__ gpos,
                                                        const uint32_t* __restrict__ ghist, int B,
                                                        uint32_t* __restrict__ order,
                                                        unsigned long long* ctr, uint32_t* ovf) {
  __shared__ uint32_t pre[COST_BUCKETS];
  const int tid = threadIdx.x;
  if (blockIdx.x == 0) {
    if (tid < 8) ctr[tid] = 0;
    if (tid < 4) ovf[tid] = 0;
  }
  if (tid < COST_BUCKETS) {                      // exclusive scan of the histogram, one wave
    const uint32_t x = ghist[tid];
    uint32_t inc = x;
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t y = __shfl_up(inc, o, 64);
      if (tid >= o) inc += y;
    }
    pre[tid] = inc - x;
  }
  __syncthreads();
  const int c = (int)(blockIdx.x * 256 + tid);
  if (c < B) {
    const uint32_t pos = pre[gbk[c]] + gpos[c];
    if (pos < (uint32_t)B) order[pos] = (uint32_t)c;
  }
}

__global__ void seed_scatter_kernel(const uint32_t* __restrict__ sv, const uint32_t* __restrict__ sc,
                                    const float* __restrict__ sval, int64_t n, uint32_t V, int B,
                                    uint32_t* cursor, uint32_t* out_v, float* out_s) {
  const SeedRun r = seed_run(sv, sc, n, V, B);
  uint32_t base = 0;
  if (r.ok && r.rank == 0) base = atomicAdd(&cursor[r.col], r.len);
  base = __shfl(base, (int)r.leader, 64);
  if (!r.ok) return;
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  out_v[base + r.rank] = sv[i];
  out_s[base + r.rank] = sval[i];
}

}  // namespace

struct egr_frontier {
  const egr_snapshot* s = nullptr;
  bool big_geom = false;          // global variant in 512-thread workgroups (egr_frontier_set_retry)
  int first = 0;                  // narrow frontier whose columns mostly overflow: 1 = straight to
                                  // the wide retry grid over every column, 2 = the mid table first
                                  // (egr_frontier_set_wide_first)
  uint32_t* all_n = nullptr;      // device word = B (the wide-first grid's list length)
  int32_t retry_blocks = -1;      // wide-table second chance for narrow overflows: grid size
                                  // (0 = off; -1 = unset: $EGRAPH_FRONTIER_WIDE_RETRY decides)
  int64_t vmax = 0;               // vertex count the V-sized buffers were sized for (headroom
                                  // for incremental snapshot updates)
  int B = 0, k = 0, nbig = 0;
  bool narrow = false;            // no member pool: the narrow-table kernels (fr_narrow)
  int64_t max_seeds = 0;
  uint32_t gcap = 0;
  int64_t n_seeds = 0;
  uint32_t* seed_ptr = nullptr;   // [B+1] exclusive scan of seed_cnt
  uint32_t* seed_cnt = nullptr;   // [2B]: per-column counts, then scatter cursors; costs
  uint32_t* order = nullptr;      // [B] launch order of the columns (set_seeds: costly first)
  uint32_t* gcost = nullptr;      // [2B + 64] grouped runs' device launch order: column cost
                                  // buckets [B], ranks within the bucket [B], bucket histogram
  uint32_t* gorder = nullptr;     // [B] the grouped runs' device-computed launch order (its own
                                  // buffer: set_seeds' order stays for the next egr_frontier_run)
  uint32_t* ident = nullptr;      // [B] 0..B-1 (grouped runs: column order)
  uint32_t* seed_v = nullptr;     // [max_seeds] grouped by column
  float* seed_s = nullptr;
  uint2* seed_rep = nullptr;
  uint32_t* pool_v = nullptr;
  float* pool_s = nullptr;
  uint8_t* pool_d = nullptr;
  unsigned long long pool_cap = 0;
  unsigned long long* ctr = nullptr;   // [0] pool, [1..5] stats
  unsigned long long* mem_off = nullptr;
  uint32_t* mem_cnt = nullptr;
  // [0] n, [1] next of the list the global-memory variant drains, [2] n, [3] (unused) of the
  // narrow kernel's list the wide retry drains, [4..4+B) and [4+B..4+2B) the two lists
  uint32_t* ovf = nullptr;
  uint32_t* gkeys = nullptr;
  float* gs = nullptr;
  float* gsnew = nullptr;
  float* lsnew = nullptr;
  unsigned long long* prof = nullptr;   // [B][PROF_SLOTS] when $EGRAPH_FRONTIER_PROFILE is set
  uint8_t* gfl = nullptr;
  uint8_t* gneed = nullptr;
  uint32_t* gmlist = nullptr;
  bool seeds_set = false;
  bool ran = false;
  bool cnt_clean = true;          // seed_cnt is zero in stream order (the run's kernel zeroes it)
  bool ctr_clean = false;         // ctr / ovf zeroed by the last set_seeds, no run since
  // test hooks, read once at creation ($EGRAPH_FRONTIER_NO_PRUNE, _GLOBAL_ONLY, _WIDE_RETRY,
  // _CONT_DRY: see frontier_run_impl) -- a run pays no environment scans
  bool env_no_prune = false, env_global_only = false, env_wide_retry = false, env_cont_dry = false;
  // $EGRAPH_FRONTIER_MID_CONT=1: the mid table's overflows continue in regions too (off by
  // default: at C4 its 1,559 overflowing columns per 20-batch launch take 30 % longer that way
  // than through the serial wide retry, profiles/r06_ab_c4_mid_continuation.txt)
  bool env_mid_cont = false;
  // a grouped run's cost histogram may hold counts: set when grouped_cost_kernel is enqueued,
  // cleared once the run's last kernel (which zeroes the histogram) is enqueued -- a run that
  // returns between the two (a failed launch) leaves it set, and the next grouped run clears the
  // histogram first instead of ordering its columns by stale counts
  bool ghist_dirty = false;
  int64_t last_n_seeds = -1;      // seed entries of the last grouped run (-1: the last run was
                                  // a set_seeds run; its valid count is seed_ptr[B])
  // overflow continuation regions (egr_frontier_set_continuation; cont_n = 0: off)
  uint32_t cont_n = 0;
  uint8_t* cont_base = nullptr;
  // the narrow table's row slot records ([B][fr_narrow::REC_STRIDE] u16; nullptr: off, e.g. a
  // member-pool frontier or $EGRAPH_FRONTIER_NO_REC)
  uint16_t* rec = nullptr;
};



// default persistent grid of the wide-table second chance ($EGRAPH_FRONTIER_WIDE_RETRY, or
// egr_frontier_set_retry): two 78-KB workgroups per CU on 256 CUs
constexpr int RETRY_BLOCKS = 512;
// global-memory variant workgroups once the retry is on (one 2V-slot HBM table each)
constexpr int GLOBAL_BLOCKS_BIG = 128;

// stamps per profiling slot: the post-barrier stamp + one per wave of the kernel's workgroup
static int prof_w(const egr_frontier* f) { return f->narrow ? fr_narrow::PROF_W : fr_wide::PROF_W; }

extern "C" {

int egr_frontier_create(const egr_snapshot* s, int32_t n_cols, int64_t max_seeds, int32_t k,
                        int64_t pool_entries, egr_frontier** out) {
  if (!s || !out || n_cols <= 0 || n_cols > (1 << 20) || max_seeds < 0 || k < 1 || k > KMAXF ||
      pool_entries < -1)
    return egr::fail(EGR_EINVAL,
                     "egr_frontier_create: bad arguments (need 0 < n_cols <= 2^20, 1 <= k <= 16)");
  *out = nullptr;
  DeviceGuard guard(s->device);
  auto* f = new egr_frontier();
  f->s = s;
  f->B = n_cols;
  f->k = k;
  f->max_seeds = max_seeds;
  f->env_no_prune = getenv("EGRAPH_FRONTIER_NO_PRUNE") != nullptr;
  f->env_global_only = getenv("EGRAPH_FRONTIER_GLOBAL_ONLY") != nullptr;
  f->env_wide_retry = getenv("EGRAPH_FRONTIER_WIDE_RETRY") != nullptr;
  f->env_cont_dry = getenv("EGRAPH_FRONTIER_CONT_DRY") != nullptr;
  f->env_mid_cont = getenv("EGRAPH_FRONTIER_MID_CONT") != nullptr;
  // sized with headroom so the snapshot can grow by incremental updates (egr_snapshot_update)
  const int64_t vmax = std::min<int64_t>(s->V + s->V / 4 + 4096, (int64_t)EGR_NO_NODE - 1);
  f->vmax = vmax;
  const uint32_t V = (uint32_t)vmax;
  // top-k-only frontiers run pruned (egr_frontier_run): their columns fit the narrow table
  f->narrow = pool_entries < 0;
  const uint32_t lcap = f->narrow ? fr_narrow::LCAP : fr_wide::LCAP;
  // pull results by member index: the narrow kernel and the wide retry index the same buffer
  const uint32_t llimit = std::max(fr_narrow::LLIMIT, fr_wide::LLIMIT);
  static_assert(fr_mid::LLIMIT <= std::max(fr_narrow::LLIMIT, fr_wide::LLIMIT),
                "the mid kernel's pull results by member index fit lsnew's column stride");
  // fallback table: 2 x nextpow2(V) slots, never more than half full
  size_t gcap = 2 * lcap;
  while (gcap < 2ull * V) gcap *= 2;
  f->gcap = (uint32_t)gcap;
  f->nbig = std::min(n_cols, 32);
  f->pool_cap = pool_entries < 0 ? 0ull   // top-k only: no member pool
              : pool_entries > 0 ? (unsigned long long)pool_entries
                                 : (unsigned long long)n_cols * 4096ull + 4ull * V;
  int rc = EGR_OK;
  const size_t ms = (size_t)std::max<int64_t>(max_seeds, 1);
  if ((rc = dalloc(&f->seed_ptr, (size_t)n_cols + 1)) || (rc = dalloc(&f->seed_cnt, 2 * (size_t)n_cols)) ||
      (rc = dalloc(&f->order, (size_t)n_cols)) || (rc = dalloc(&f->ident, (size_t)n_cols)) ||
      (rc = dalloc(&f->gcost, 2 * (size_t)n_cols + 64)) || (rc = dalloc(&f->gorder, (size_t)n_cols)) ||
      (rc = dalloc(&f->seed_v, ms)) || (rc = dalloc(&f->seed_s, ms)) ||
      (rc = dalloc(&f->seed_rep, ms)) ||
      (rc = dalloc(&f->pool_v, f->pool_cap)) || (rc = dalloc(&f->pool_s, f->pool_cap)) ||
      (rc = dalloc(&f->pool_d, f->pool_cap)) || (rc = dalloc(&f->ctr, 8)) ||
      (rc = dalloc(&f->mem_off, (size_t)n_cols)) || (rc = dalloc(&f->mem_cnt, (size_t)n_cols)) ||
      (rc = dalloc(&f->ovf, 2 * (size_t)n_cols + 4)) || (rc = dalloc(&f->all_n, 1)) ||
      (rc = dalloc(&f->gkeys, gcap * f->nbig)) || (rc = dalloc(&f->gs, gcap * f->nbig)) ||
      (rc = dalloc(&f->gfl, gcap * f->nbig)) || (rc = dalloc(&f->gneed, gcap * f->nbig)) ||
      (rc = dalloc(&f->gsnew, (size_t)V * f->nbig)) || (rc = dalloc(&f->gmlist, (size_t)V * f->nbig)) ||
      (rc = dalloc(&f->lsnew, (size_t)n_cols * llimit))) {
    egr_frontier_free(f);
    return rc;
  }
  if (fr_narrow::REC && f->narrow && !getenv("EGRAPH_FRONTIER_NO_REC") &&
      (rc = dalloc(&f->rec, (size_t)n_cols * fr_narrow::REC_STRIDE))) {
    egr_frontier_free(f);
    return rc;
  }
  if (EGR_FR_PROFILE && getenv("EGRAPH_FRONTIER_PROFILE") &&
      (rc = dalloc(&f->prof, (size_t)n_cols * PROF_SLOTS * prof_w(f)))) {
    egr_frontier_free(f);
    return rc;
  }
  if (hipMemset(f->gkeys, 0xFF, gcap * f->nbig * 4) != hipSuccess ||
      hipMemset(f->gs, 0, gcap * f->nbig * 4) != hipSuccess ||
      hipMemset(f->gfl, 0, gcap * f->nbig) != hipSuccess ||
      hipMemset(f->gneed, 0, gcap * f->nbig) != hipSuccess ||
      hipMemset(f->mem_cnt, 0xFF, (size_t)n_cols * 4) != hipSuccess ||
      hipMemset(f->seed_cnt, 0, (size_t)n_cols * 8) != hipSuccess ||
      hipMemset(f->ctr, 0, 8 * 8) != hipSuccess ||
      hipMemset(f->gcost, 0, (2 * (size_t)n_cols + 64) * 4) != hipSuccess) {
    egr_frontier_free(f);
    return egr::fail(EGR_EDEVICE, "egr_frontier_create: table init failed");
  }
  {
    std::vector<uint32_t> id((size_t)n_cols);
    for (int i = 0; i < n_cols; ++i) id[i] = (uint32_t)i;
    const uint32_t nb = (uint32_t)n_cols;
    if (hipMemcpy(f->ident, id.data(), (size_t)n_cols * 4, hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(f->order, id.data(), (size_t)n_cols * 4, hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(f->all_n, &nb, 4, hipMemcpyHostToDevice) != hipSuccess) {
      egr_frontier_free(f);
      return egr::fail(EGR_EDEVICE, "egr_frontier_create: order init failed");
    }
  }
  *out = f;
  return EGR_OK;
}

void egr_frontier_free(egr_frontier* f) {
  if (!f) return;
  DeviceGuard guard(f->s->device);
  dfree(f->seed_ptr);
  dfree(f->seed_cnt);
  dfree(f->order);
  dfree(f->gorder);
  dfree(f->gcost);
  dfree(f->ident);
  dfree(f->seed_v);
  dfree(f->seed_s);
  dfree(f->seed_rep);
  dfree(f->pool_v);
  dfree(f->pool_s);
  dfree(f->pool_d);
  dfree(f->ctr);
  dfree(f->mem_off);
  dfree(f->mem_cnt);
  dfree(f->ovf);
  dfree(f->all_n);
  dfree(f->gkeys);
  dfree(f->gs);
  dfree(f->gsnew);
  dfree(f->lsnew);
  dfree(f->prof);
  dfree(f->gfl);
  dfree(f->gneed);
  dfree(f->gmlist);
  dfree(f->cont_base);
  dfree(f->rec);
  delete f;
}

static int frontier_outgrown(const egr_frontier* f, const char* what) {
  return egr::fail(EGR_ESTATE, std::string(what) + ": the snapshot grew past the " +
                   std::to_string(f->vmax) + " vertices this frontier was sized for; create a new one");
}

int64_t egr_frontier_max_vertices(const egr_frontier* f) { return f ? f->vmax : -1; }

int egr_frontier_shape(const egr_frontier* f, int32_t* n_cols, int32_t* k) {
  if (!f) return egr::fail(EGR_EINVAL, "egr_frontier_shape: NULL frontier");
  if (n_cols) *n_cols = f->B;
  if (k) *k = f->k;
  return EGR_OK;
}

int egr_frontier_set_seeds(egr_frontier* f, const uint32_t* seed_vertex, const uint32_t* seed_col,
                           const float* seed_val, int64_t n_seeds, void* stream) {
  if (!f || n_seeds < 0 || n_seeds > f->max_seeds ||
      (n_seeds > 0 && (!seed_vertex || !seed_col || !seed_val)))
    return egr::fail(EGR_EINVAL,
                     "egr_frontier_set_seeds: bad arguments (n_seeds above capacity?)");
  if (f->s->V > f->vmax) return frontier_outgrown(f, "egr_frontier_set_seeds");
  DeviceGuard guard(f->s->device);
  const uint32_t V = (uint32_t)f->s->V;
  hipStream_t st = (hipStream_t)stream;
  // counting sort by column: count, one-block exclusive scan, scatter (order within a column
  // is arbitrary; the kernel max-combines duplicates).  Invalid triples are dropped.
  if (!f->cnt_clean) EGR_HIP(hipMemsetAsync(f->seed_cnt, 0, (size_t)f->B * 8, st));
  const unsigned g = (unsigned)((std::max<int64_t>(n_seeds, 1) + 255) / 256);
  if (n_seeds > 0) {
    hipLaunchKernelGGL(seed_count_kernel, dim3(g), dim3(256), 0, st, seed_vertex, seed_col,
                       n_seeds, V, f->B, f->s->row_ptr, f->seed_cnt, f->seed_cnt + f->B);
    EGR_CHECK_LAUNCH();
  }
  hipLaunchKernelGGL(seed_scan_kernel, dim3(1), dim3(SCAN_T), 0, st, f->seed_cnt, f->B, f->seed_ptr,
                     f->seed_cnt + f->B, f->order, f->ctr, f->ovf);
  EGR_CHECK_LAUNCH();
  if (n_seeds > 0) {
    hipLaunchKernelGGL(seed_scatter_kernel, dim3(g), dim3(256), 0, st, seed_vertex, seed_col,
                       seed_val, n_seeds, V, f->B, f->seed_cnt, f->seed_v, f->seed_s);
    EGR_CHECK_LAUNCH();
  }
  f->n_seeds = n_seeds;
  f->seeds_set = true;
  f->cnt_clean = false;
  f->ctr_clean = true;
  return EGR_OK;
}

// One run over seeds grouped by column (seed_ptr [B+1] into seed_v / seed_s, n_seeds entries).
// `sorted` = the seeds came from egr_frontier_set_seeds: its launch order (costly columns first)
// is used, its counters are consumed (zeroed) by the narrow kernel, and its scan zeroed the
// run's counters.
static int frontier_run_impl(egr_frontier* f, const uint32_t* seed_ptr, const uint32_t* seed_v,
                             const float* seed_s, int64_t n_seeds, bool sorted, const uint32_t* order, const uint32_t* source_vertex,
                             int32_t hops, int32_t exclude_label, uint32_t* out_ids,
                             float* out_scores, hipStream_t st) {
  const egr_snapshot* s = f->s;
  // (a grouped run with its order computed on the device clears its counters in
  // cost_order_kernel: one launch fewer)
  if (!(sorted && f->ctr_clean) && !(!sorted && !order)) {
    hipLaunchKernelGGL(clear_counters_kernel, dim3(1), dim3(64), 0, st, f->ctr, f->ovf);
    EGR_CHECK_LAUNCH();
  }
  FArgs a{};
  const FrLayoutView lay = layout_view(s);
  a.row_ptr = lay.row_ptr;
  a.cv = lay.cv;
  a.vlabel = lay.vlabel;
  a.perm = lay.perm;
  a.iperm = lay.iperm;
  a.V = (uint32_t)s->V;
  a.B = f->B;
  a.hops = hops;
  a.k = f->k;
  a.exclude = exclude_label;
  // ($EGRAPH_FRONTIER_NO_PRUNE: every member exact in a top-k run too -- a test hook)
  a.prune = (f->pool_cap == 0 && !f->env_no_prune) ? 1 : 0;
  a.seed_ptr = seed_ptr;
  a.seed_vert = seed_v;
  a.seed_val = seed_s;
  a.n_seeds = (uint32_t)n_seeds;
  a.seed_rep = f->seed_rep;
  a.sources = source_vertex;
  if (!sorted && !order) {
    // grouped seeds without a caller order: costliest-first on the device (two small kernels
    // ahead of the frontier launch, in the same stream -- and in a captured replay)
    uint32_t* gbk = f->gcost;
    uint32_t* gpos = f->gcost + f->B;
    uint32_t* ghist = f->gcost + 2 * (size_t)f->B;
    if (f->ghist_dirty) EGR_HIP(hipMemsetAsync(ghist, 0, COST_BUCKETS * sizeof(uint32_t), st));
    f->ghist_dirty = true;
    hipLaunchKernelGGL(grouped_cost_kernel, dim3((unsigned)((f->B + 63) / 64)), dim3(COST_T), 0, st,
                       seed_ptr, seed_v, (uint32_t)n_seeds, f->B, s->row_ptr, (uint32_t)s->V, gbk,
                       gpos, ghist);
    hipLaunchKernelGGL(cost_order_kernel, dim3((unsigned)((f->B + 255) / 256)), dim3(256), 0, st,
                       gbk, gpos, ghist, f->B, f->gorder, f->ctr, f->ovf);
    EGR_CHECK_LAUNCH();
  }
  a.order = sorted ? f->order : order ? order : f->gorder;
  a.seed_cnt = sorted ? f->seed_cnt : nullptr;
  a.out_ids = out_ids;
  a.out_scores = out_scores;
  a.pool_v = f->pool_v;
  a.pool_s = f->pool_s;
  a.pool_d = f->pool_d;
  a.pool_cap = f->pool_cap;
  a.pool_ctr = f->ctr;
  a.mem_off = f->mem_off;
  a.mem_cnt = f->mem_cnt;
  a.ovf_n = f->ovf;
  a.ovf_next = f->ovf + 1;
  a.retry_next = f->ovf + 3;
  a.ovf_list = f->ovf + 4;
  a.ovf_cap = (uint32_t)f->B;
  a.spill_list = a.ovf_list;
  a.spill_n = a.ovf_n;
  a.retry_n = f->ovf + 2;
  a.retry_list = f->ovf + 4 + f->B;
  a.gkeys = f->gkeys;
  a.gs = f->gs;
  a.gsnew = f->gsnew;
  a.gfl = f->gfl;
  a.gneed = f->gneed;
  a.gmlist = f->gmlist;
  a.gcap = f->gcap;
  a.lsnew = f->lsnew;
  a.rec = f->rec;
  a.prof = f->prof;
  if (f->prof) EGR_HIP(hipMemsetAsync(f->prof, 0, (size_t)f->B * PROF_SLOTS * prof_w(f) * 8, st));
  a.stats = f->ctr + 1;
  a.ghist = f->gcost + 2 * (size_t)f->B;
  bool skipped_lds = false;       // no LDS kernel ran: the set_seeds counters were not consumed
  if (f->env_global_only) {
    // (a test hook: every column through the global-memory variant, as if every LDS kernel had
    // handed it on)
    a.ovf_list = const_cast<uint32_t*>(a.order);
    a.ovf_n = f->all_n;
    skipped_lds = true;
  } else if (f->narrow) {
    // narrow: its overflowing columns go to the global-memory variant -- or, with the wide
    // retry on (egr_frontier_set_retry / $EGRAPH_FRONTIER_WIDE_RETRY), to a persistent grid of
    // the wide LDS table first, which hands on only what overflows 4608 members.  Off by
    // default: pruned C2 / C3 columns never overflow, and the retry's 78-KB workgroups would
    // wait for LDS held by the other batches in flight (~30 us per run in rocprof,
    // profiles/r01_kernel_stats_v9.csv).  Graphs whose 3-hop neighbourhoods are larger (the
    // dense C4) turn it on after a run reports overflowing columns (egraph.graph.Frontier.adapt).
    FArgs an = a;
    an.ovf_n = f->ovf + 2;
    an.ovf_list = f->ovf + 4 + f->B;
    const int32_t rb = f->retry_blocks >= 0 ? f->retry_blocks
                       : f->env_wide_retry ? RETRY_BLOCKS : 0;
    an.ovf_cap = rb > 0 ? (uint32_t)f->B : 0u;     // every overflowing column gets the retry
    a.prof = nullptr;   // the wide kernels' stamp layout differs: only the narrow pass is profiled
    if (f->first == 2 && rb > 0) {
      // mid-first: every column in the 2.8k-slot table; what overflows it takes the wide retry
      // -- or, with $EGRAPH_FRONTIER_MID_CONT, continues in its own workgroup in a global-memory
      // region (as the narrow table's do), the retry taking what finds no region
      FArgs am = an;
      if (f->cont_n > 0 && f->env_mid_cont) {
        am.cont_ctr = f->ctr + 7;
        am.cont_n = f->env_cont_dry ? 0u : f->cont_n;
        am.cont_base = f->cont_base;
        hipLaunchKernelGGL(fr_mid::frontier_lds_kernel<true>, dim3(f->B), dim3(fr_mid::FT), 0, st, am);
      } else {
        hipLaunchKernelGGL(fr_mid::frontier_lds_kernel<false>, dim3(f->B), dim3(fr_mid::FT), 0, st, am);
      }
      EGR_CHECK_LAUNCH();
      hipLaunchKernelGGL(fr_wide::frontier_lds_retry_kernel, dim3(std::min(rb, f->B)),
                         dim3(fr_wide::FT), 0, st, a);
      EGR_CHECK_LAUNCH();
    } else if (f->first == 1 && rb > 0) {
      // most columns overflow the narrow table: every column goes straight to the wide grid,
      // in launch order (the narrow kernel, which also zeroes the seed counters, is skipped)
      FArgs aw = a;
      aw.retry_list = a.order;
      aw.retry_n = f->all_n;
      hipLaunchKernelGGL(fr_wide::frontier_lds_retry_kernel, dim3(std::min(rb, f->B)),
                         dim3(fr_wide::FT), 0, st, aw);
      EGR_CHECK_LAUNCH();
      skipped_lds = true;
    } else if (rb > 0 && f->cont_n > 0) {
      // continuation: an overflowing column finishes in its own workgroup, in a global-memory
      // region, while the grid runs (no serial retry after it); what overflows a region too, or
      // finds none left, goes straight to the global-memory variant's list
      FArgs ac = an;
      ac.ovf_n = a.ovf_n;
      ac.ovf_list = a.ovf_list;
      ac.ovf_cap = a.ovf_cap;
      ac.cont_ctr = f->ctr + 7;
      // ($EGRAPH_FRONTIER_CONT_DRY: the continuation kernel with no region -- a test hook that
      // prices its code against the plain kernel's)
      ac.cont_n = f->env_cont_dry ? 0u : f->cont_n;
      ac.cont_base = f->cont_base;
      hipLaunchKernelGGL(fr_narrow::frontier_lds_kernel<true>, dim3(f->B), dim3(fr_narrow::FT), 0, st, ac);
      EGR_CHECK_LAUNCH();
    } else {
      hipLaunchKernelGGL(fr_narrow::frontier_lds_kernel<false>, dim3(f->B), dim3(fr_narrow::FT), 0, st, an);
      EGR_CHECK_LAUNCH();
      if (rb > 0) {
        hipLaunchKernelGGL(fr_wide::frontier_lds_retry_kernel, dim3(std::min(rb, f->B)),
                           dim3(fr_wide::FT), 0, st, a);
        EGR_CHECK_LAUNCH();
      }
    }
  } else {
    hipLaunchKernelGGL(fr_wide::frontier_lds_kernel<false>, dim3(f->B), dim3(fr_wide::FT), 0, st, a);
    EGR_CHECK_LAUNCH();
  }
  // the overflow fallback: one-wave workgroups (they are dispatched as soon as one SIMD has
  // room, profiles/r01_ab_fallback_geom.txt), or 512-thread ones once the retry is on
  if (f->big_geom)
    hipLaunchKernelGGL(fr_wide::frontier_global_kernel, dim3(f->nbig), dim3(fr_wide::FT), 0, st, a);
  else
    hipLaunchKernelGGL(fr_fallback::frontier_global_kernel, dim3(f->nbig), dim3(fr_fallback::FT), 0, st, a);
  EGR_CHECK_LAUNCH();
  f->ghist_dirty = false;         // (the kernel just enqueued zeroes the histogram)
  f->ran = true;
  f->ctr_clean = false;
  // the narrow / wide LDS kernels zero each column's set_seeds counters as they consume them;
  // a run that skipped them leaves the counters for the next set_seeds to clear
  if (sorted) f->cnt_clean = !skipped_lds;
  return EGR_OK;
}

int egr_frontier_run(egr_frontier* f, const uint32_t* source_vertex, int32_t hops,
                     int32_t exclude_label, uint32_t* out_ids, float* out_scores, void* stream) {
  if (!f || !source_vertex || !out_ids || !out_scores || hops < 1 || hops > MAX_HOPS)
    return egr::fail(EGR_EINVAL, "egr_frontier_run: bad arguments (need 1 <= hops <= 60)");
  if (!f->seeds_set) return egr::fail(EGR_ESTATE, "egr_frontier_run: seeds not set");
  if (f->s->V > f->vmax) return frontier_outgrown(f, "egr_frontier_run");
  DeviceGuard guard(f->s->device);
  const int rc = frontier_run_impl(f, f->seed_ptr, f->seed_v, f->seed_s, f->n_seeds, true, nullptr, source_vertex, hops,
                                   exclude_label, out_ids, out_scores, (hipStream_t)stream);
  if (rc == EGR_OK) f->last_n_seeds = -1;
  return rc;
}

int egr_frontier_run_grouped(egr_frontier* f, const uint32_t* seed_ptr, const uint32_t* seed_vertex,
                             const float* seed_val, int64_t n_seeds, const uint32_t* order,
                             const uint32_t* source_vertex,
                             int32_t hops, int32_t exclude_label, uint32_t* out_ids,
                             float* out_scores, void* stream) {
  if (!f || !seed_ptr || !source_vertex || !out_ids || !out_scores || hops < 1 || hops > MAX_HOPS ||
      n_seeds < 0 || n_seeds > f->max_seeds || n_seeds > (int64_t)0xFFFFFFFFu ||
      (n_seeds > 0 && (!seed_vertex || !seed_val)))
    return egr::fail(EGR_EINVAL, "egr_frontier_run_grouped: bad arguments (need 1 <= hops <= 60, "
                                 "n_seeds <= the frontier's max_seeds)");
  if (f->s->V > f->vmax) return frontier_outgrown(f, "egr_frontier_run_grouped");
  DeviceGuard guard(f->s->device);
  const int rc = frontier_run_impl(f, seed_ptr, seed_vertex, seed_val, n_seeds, false, order, source_vertex, hops,
                                   exclude_label, out_ids, out_scores, (hipStream_t)stream);
  if (rc == EGR_OK) f->last_n_seeds = n_seeds;
  return rc;
}

int egr_frontier_set_wide_first(egr_frontier* f, int32_t on) {
  if (!f || on < 0 || on > 2) return egr::fail(EGR_EINVAL, "egr_frontier_set_wide_first: bad arguments");
  f->first = on;
  return EGR_OK;
}

int egr_frontier_set_retry(egr_frontier* f, int32_t blocks) {
  if (!f || blocks < 0) return egr::fail(EGR_EINVAL, "egr_frontier_set_retry: bad arguments");
  f->retry_blocks = blocks;
  // graphs that need the retry also send more columns past the wide table: the global-memory
  // variant then gets up to GLOBAL_BLOCKS_BIG workgroups (one HBM table each) in 256-thread
  // workgroups instead of 32 one-wave ones
  const int want = blocks > 0 ? std::min(f->B, GLOBAL_BLOCKS_BIG) : f->nbig;
  if (want > f->nbig) {
    DeviceGuard guard(f->s->device);
    EGR_HIP(hipDeviceSynchronize());            // runs in flight still use the old tables
    const size_t gcap = f->gcap, V = (size_t)f->vmax;
    dfree(f->gkeys);
    dfree(f->gs);
    dfree(f->gfl);
    dfree(f->gneed);
    dfree(f->gsnew);
    dfree(f->gmlist);
    f->nbig = want;
    int rc;
    if ((rc = dalloc(&f->gkeys, gcap * want)) || (rc = dalloc(&f->gs, gcap * want)) ||
        (rc = dalloc(&f->gfl, gcap * want)) || (rc = dalloc(&f->gneed, gcap * want)) ||
        (rc = dalloc(&f->gsnew, V * want)) || (rc = dalloc(&f->gmlist, V * want))) {
      f->nbig = 0;
      return rc;
    }
    if (hipMemset(f->gkeys, 0xFF, gcap * want * 4) != hipSuccess ||
        hipMemset(f->gs, 0, gcap * want * 4) != hipSuccess ||
        hipMemset(f->gfl, 0, gcap * want) != hipSuccess ||
        hipMemset(f->gneed, 0, gcap * want) != hipSuccess)
      return egr::fail(EGR_EDEVICE, "egr_frontier_set_retry: table init failed");
    f->big_geom = true;
  }
  return EGR_OK;
}

int egr_frontier_set_continuation(egr_frontier* f, int32_t regions) {
  if (!f || regions < 0 || regions > 4096)
    return egr::fail(EGR_EINVAL, "egr_frontier_set_continuation: bad arguments (0..4096 regions)");
  if ((uint32_t)regions > f->cont_n) {
    DeviceGuard guard(f->s->device);
    EGR_HIP(hipDeviceSynchronize());            // runs in flight still use the old regions
    dfree(f->cont_base);
    f->cont_base = nullptr;
    f->cont_n = 0;
    const size_t n = (size_t)regions;
    int rc;
    if ((rc = dalloc(&f->cont_base, n * CONT_REGION_BYTES))) return rc;
    // every region: keys EMPTY, scores / flags / need zero (a used region is left so again)
    if (hipMemset(f->cont_base, 0, n * CONT_REGION_BYTES) != hipSuccess)
      return egr::fail(EGR_EDEVICE, "egr_frontier_set_continuation: region init failed");
    for (size_t r = 0; r < n; ++r)
      if (hipMemset(f->cont_base + r * CONT_REGION_BYTES, 0xFF, 4 * (size_t)CONT_CAP) != hipSuccess)
        return egr::fail(EGR_EDEVICE, "egr_frontier_set_continuation: region init failed");
  }
  f->cont_n = (uint32_t)regions;
  return EGR_OK;
}

int egr_frontier_stats(const egr_frontier* f, int64_t* out8, void* stream) {
  // out8 holds 9 values (egraph.h: out9)
  if (!f || !out8) return egr::fail(EGR_EINVAL, "egr_frontier_stats: NULL argument");
  if (!f->ran) return egr::fail(EGR_ESTATE, "egr_frontier_stats: not run yet");
  DeviceGuard guard(f->s->device);
  unsigned long long h[7];
  uint32_t nu = 0, ng = 0;
  EGR_HIP(hipMemcpyAsync(h, f->ctr, sizeof(h), hipMemcpyDeviceToHost, (hipStream_t)stream));
  if (f->last_n_seeds < 0)       // a set_seeds run: the valid entries its scan counted
    EGR_HIP(hipMemcpyAsync(&nu, f->seed_ptr + f->B, 4, hipMemcpyDeviceToHost, (hipStream_t)stream));
  EGR_HIP(hipMemcpyAsync(&ng, f->ovf, 4, hipMemcpyDeviceToHost, (hipStream_t)stream));
  EGR_HIP(hipStreamSynchronize((hipStream_t)stream));
  out8[8] = (int64_t)ng;     // columns the global-memory variant ranked
  for (int i = 0; i < 5; ++i) out8[i] = (int64_t)h[i + 1];
  out8[5] = (int64_t)h[0];
  out8[6] = f->last_n_seeds < 0 ? (int64_t)nu : f->last_n_seeds;
  out8[7] = (int64_t)h[6];   // columns finished in a continuation region
  return EGR_OK;
}

int egr_frontier_phase_times(const egr_frontier* f, int64_t* out, int64_t cap, void* stream) {
  if (!f || (cap > 0 && !out) || cap < 0)
    return egr::fail(EGR_EINVAL, "egr_frontier_phase_times: bad arguments");
  if (!f->prof) return 0;
  DeviceGuard guard(f->s->device);
  const int64_t n = std::min<int64_t>(cap, (int64_t)f->B * PROF_SLOTS * prof_w(f));
  if (n > 0) {
    EGR_HIP(hipMemcpyAsync(out, f->prof, n * 8, hipMemcpyDeviceToHost, (hipStream_t)stream));
    EGR_HIP(hipStreamSynchronize((hipStream_t)stream));
  }
  return PROF_SLOTS * prof_w(f);
}

int egr_frontier_read_scores(const egr_frontier* f, float* out, void* stream) {
  if (!f || !out) return egr::fail(EGR_EINVAL, "egr_frontier_read_scores: NULL argument");
  if (!f->ran) return egr::fail(EGR_ESTATE, "egr_frontier_read_scores: not run yet");
  if (!f->pool_cap) return egr::fail(EGR_ESTATE, "egr_frontier_read_scores: frontier created without a member pool");
  DeviceGuard guard(f->s->device);
  hipStream_t st = (hipStream_t)stream;
  EGR_HIP(hipMemsetAsync(out, 0, (size_t)f->s->V * f->B * 4, st));
  hipLaunchKernelGGL(scatter_scores_kernel, dim3(f->B), dim3(256), 0, st, f->pool_v, f->pool_s,
                     f->mem_off, f->mem_cnt, f->B, out);
  EGR_CHECK_LAUNCH();
  return EGR_OK;
}

int egr_frontier_read_reach(const egr_frontier* f, uint64_t* out, void* stream) {
  if (!f || !out) return egr::fail(EGR_EINVAL, "egr_frontier_read_reach: NULL argument");
  if (!f->ran) return egr::fail(EGR_ESTATE, "egr_frontier_read_reach: not run yet");
  if (!f->pool_cap) return egr::fail(EGR_ESTATE, "egr_frontier_read_reach: frontier created without a member pool");
  DeviceGuard guard(f->s->device);
  hipStream_t st = (hipStream_t)stream;
  EGR_HIP(hipMemsetAsync(out, 0, (size_t)((f->B + 63) / 64) * f->s->V * 8, st));
  hipLaunchKernelGGL(scatter_reach_kernel, dim3(f->B), dim3(256), 0, st, f->pool_v, f->pool_d,
                     f->mem_off, f->mem_cnt, (uint32_t)f->s->V,
                     reinterpret_cast<unsigned long long*>(out));
  EGR_CHECK_LAUNCH();
  return EGR_OK;
}

int egr_frontier_members(const egr_frontier* f, int32_t col, uint32_t* out_vertex,
                         float* out_score, uint8_t* out_depth, int64_t cap, int64_t* out_n,
                         void* stream) {
  if (!f || !out_n || col < 0 || col >= f->B || cap < 0)
    return egr::fail(EGR_EINVAL, "egr_frontier_members: bad arguments");
  if (!f->ran) return egr::fail(EGR_ESTATE, "egr_frontier_members: not run yet");
  if (!f->pool_cap) return egr::fail(EGR_ESTATE, "egr_frontier_members: frontier created without a member pool");
  DeviceGuard guard(f->s->device);
  hipStream_t st = (hipStream_t)stream;
  unsigned long long off = 0;
  uint32_t n = 0;
  EGR_HIP(hipMemcpyAsync(&off, f->mem_off + col, 8, hipMemcpyDeviceToHost, st));
  EGR_HIP(hipMemcpyAsync(&n, f->mem_cnt + col, 4, hipMemcpyDeviceToHost, st));
  EGR_HIP(hipStreamSynchronize(st));
  if (n == NO_NODE) return egr::fail(EGR_ESTATE, "egr_frontier_members: member pool was full");
  *out_n = n;
  const size_t m = std::min<int64_t>(cap, n);
  if (m && out_vertex) EGR_HIP(hipMemcpyAsync(out_vertex, f->pool_v + off, m * 4, hipMemcpyDefault, st));
  if (m && out_score) EGR_HIP(hipMemcpyAsync(out_score, f->pool_s + off, m * 4, hipMemcpyDefault, st));
  if (m && out_depth) EGR_HIP(hipMemcpyAsync(out_depth, f->pool_d + off, m, hipMemcpyDefault, st));
  EGR_HIP(hipStreamSynchronize(st));
  return EGR_OK;
}

}  // extern "C"
