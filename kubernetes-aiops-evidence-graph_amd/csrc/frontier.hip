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
// expansion touched recompute their score).  A wave takes 64 members at a time: a row of <= 16
// entries is one lane's, which loads and probes all its entries at once and runs the in-order
// fmaf chain in registers; a longer (hub) row is taken by the whole wave, 64 entries per round,
// with the chain run over v_readlane operands.  Top-k packs (score, vertex) into one u64 key:
// each wave extracts its k best with DPP wave-max rounds, wave 0 merges the lists.
//
// Capacity: the LDS table holds 6144 slots (keys, scores, depths, member list: ~70 KB, two
// workgroups per CU); a column with more than 4608 members is flagged and redone by the
// global-memory variant of the same code (a table of >= 2V slots per resident workgroup, never
// overflows), launched unconditionally right after (it drains an empty work list at once).
#include <algorithm>
#include <type_traits>
#include <vector>

#include "graph_dev.h"

using egr::DeviceGuard;
using egr::dalloc;
using egr::dfree;

namespace {

constexpr uint32_t EMPTY = 0xFFFFFFFFu;
constexpr uint32_t NO_NODE = EGR_NO_NODE;
constexpr int FT = 512;                     // threads per workgroup (8 waves)
constexpr int NWAVES = FT / 64;
// Table geometry (override all four together for A/B builds; scripts/ab_lib.sh).  Members per
// column on C3 / C4 reach 3711 / 3824 at most (scripts/frontier_members.py).
#ifndef EGR_FR_LCAP
#define EGR_FR_LCAP 6144
#define EGR_FR_LLIMIT 4608
#define EGR_FR_BLOOM_LOG 16
#define EGR_FR_WAVES_PER_EU 4
#endif
constexpr uint32_t LCAP = EGR_FR_LCAP;      // LDS table slots
constexpr uint32_t LLIMIT = EGR_FR_LLIMIT;  // members before a column overflows (load 0.75)
constexpr int LPPT = LCAP / FT;             // slots cleared per thread
constexpr int LMAX = 16;                    // rows up to this many entries run one lane per row
constexpr int LB = 4;                       // keys probed together per lane
constexpr int BLOOM_LOG = EGR_FR_BLOOM_LOG;
constexpr uint32_t BLOOM_WORDS = (1u << BLOOM_LOG) / 32;  // 64 Kbit filter: rejects absent keys in one read
constexpr int MPT = (LLIMIT + FT - 1) / FT; // members per thread (top-k candidate registers)
constexpr int KMAXF = 16;
constexpr uint8_t FL_DEPTH = 0x3F;          // fl: depth + 1 in the low bits
constexpr uint8_t FL_SEED = 0x40;           // the member is one of the column's seeds
constexpr uint8_t FL_CLAIM = 0x80;          // a seed entry already represents this vertex
constexpr int MAX_HOPS = 60;
constexpr int PROF_SLOTS = 32;
constexpr int PROF_W = NWAVES + 1;          // per slot: post-barrier stamp + each wave's finish


struct FArgs {
  const uint32_t* row_ptr;
  const uint2* cv;             // (col, val bits) per CSR entry
  const uint8_t* vlabel;
  uint32_t V;
  int B, hops, k, exclude;
  int prune;                   // no member pool: the last hop pulls the candidates only
  const uint32_t* seed_ptr;    // [B+1] per column
  const uint32_t* seed_vert;   // grouped by column, any order, duplicates allowed
  const float* seed_val;       // (duplicates are max-combined in the kernel, as fmaxf)
  uint2* seed_rep;             // per seed entry: (slot, s0 bits) of a vertex's representative
  const uint32_t* sources;     // [B] incident vertex per column (EGR_NO_NODE: none)
  const uint32_t* order;       // [B] launch order: workgroup i runs column order[i] (costly first)
  uint32_t* seed_cnt;          // [2B] seed counters / costs, zeroed per column once consumed
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
  uint32_t* ovf_list;
  uint32_t* ovf_n;
  uint32_t* ovf_next;
  float* lsnew;                 // [B][LLIMIT] pull results of the LDS variant (by member index)
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
  // [2] rows walked (row_ptr pairs), [3] members, [4] columns that overflowed
  unsigned long long* stats;
};

// The table of one column.  keys/s/fl are indexed by slot; mlist lists the member slots in
// insertion order (u16 in LDS, u32 in the global variant) and snew the pull results by member
// index.
template <bool GT>
struct Tab {
  using MT = typename std::conditional<GT, uint32_t, uint16_t>::type;
  uint32_t* keys;
  float* s;
  uint8_t* fl;
  uint8_t* need;    // touched by an expansion this hop: pulled
  MT* mlist;
  float* snew;
  uint32_t cap, limit;
  uint32_t* count;  // LDS
  uint32_t* ovf;    // LDS
  uint32_t* bloom;  // LDS variant: BLOOM_BITS-bit membership filter (nullptr: none)
};

// Buckets of 4 slots (one 16-B read), probed linearly.  A bucket fills from its first slot: an
// insert CASes the lowest empty slot it sees and moves on only when that slot is taken, so a
// bucket with an empty slot ends every probe sequence that passes through it.
// Hashes use only full-rate 24-bit multiplies (a 32-bit v_mul_lo / v_mul_hi is quarter rate,
// and every probed key pays for its hashes): the id is folded to 24 bits, multiplied by an odd
// 24-bit constant, and 16 mixed bits are range-reduced to [0, nb) by a second 24-bit multiply.
__device__ __forceinline__ uint32_t mix24(uint32_t v, uint32_t c) {
  return __umul24((v ^ (v >> 24)) & 0xFFFFFFu, c);
}

__device__ __forceinline__ uint32_t hbucket(uint32_t v, uint32_t nb) {
  return __umul24((mix24(v, 0x9E3779u) >> 8) & 0xFFFFu, nb) >> 16;
}

__device__ __forceinline__ uint4 read_bucket(const uint32_t* keys, uint32_t bk) {
  return reinterpret_cast<const uint4*>(keys)[bk];
}

// outcome of one bucket read for key v: slot (>= 0), -1 = absent, -2 = continue probing
__device__ __forceinline__ int bucket_match(const uint4& kk, uint32_t v, uint32_t bk) {
  if (kk.x == v) return (int)(4 * bk);
  if (kk.y == v) return (int)(4 * bk + 1);
  if (kk.z == v) return (int)(4 * bk + 2);
  if (kk.w == v) return (int)(4 * bk + 3);
  if (kk.w == EMPTY) return -1;            // slots fill in order: an empty last slot ends it
  return -2;
}

__device__ __forceinline__ uint32_t bloom_hash(uint32_t v) {   // BLOOM_LOG bits
  return (mix24(v, 0xB5297Au | 1u) >> 8) & ((1u << BLOOM_LOG) - 1u);
}

// slot of v, inserting it if absent (-1: table full)
template <bool GT>
__device__ __forceinline__ int tab_insert(const Tab<GT>& t, uint32_t v) {
  const uint32_t nb = t.cap / 4;
  uint32_t bk = hbucket(v, nb);
  for (uint32_t n = 0; n < nb; ++n) {
    uint4 kk = read_bucket(t.keys, bk);
    uint32_t ks[4] = {kk.x, kk.y, kk.z, kk.w};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if (ks[j] == v) return (int)(4 * bk + j);
      if (ks[j] == EMPTY) {
        const uint32_t p = 4 * bk + j;
        const uint32_t old = atomicCAS(&t.keys[p], EMPTY, v);
        if (old == EMPTY) {
          if constexpr (!GT) {
            const uint32_t h = bloom_hash(v);
            atomicOr(&t.bloom[h >> 5], 1u << (h & 31u));
          }
          const uint32_t c = atomicAdd(t.count, 1u);
          if (c < t.limit) t.mlist[c] = (typename Tab<GT>::MT)p;
          else *t.ovf = 1u;
          return (int)p;
        }
        if (old == v) return (int)p;
        // taken by another key: look at the next slot
      }
    }
    bk = bk + 1 == nb ? 0 : bk + 1;
  }
  *t.ovf = 1u;
  return -1;
}

// slot of v or -1 (only called while no insertion is in flight)
template <bool GT>
__device__ __forceinline__ int tab_find(const Tab<GT>& t, uint32_t v) {
  if constexpr (!GT) {
    const uint32_t h = bloom_hash(v);
    if (!((t.bloom[h >> 5] >> (h & 31u)) & 1u)) return -1;
  }
  const uint32_t nb = t.cap / 4;
  uint32_t bk = hbucket(v, nb);
  for (uint32_t n = 0; n < nb; ++n) {
    const int r = bucket_match(read_bucket(t.keys, bk), v, bk);
    if (r != -2) return r;
    bk = bk + 1 == nb ? 0 : bk + 1;
  }
  return -1;
}

struct Work {
  uint32_t pull = 0, expand = 0, rows = 0;
};

// a top-k candidate's depth: reached within `hops` of the incident vertex (fl = depth + 1)
__device__ __forceinline__ bool cand_depth(uint8_t f, int hops) {
  const uint32_t d = f & FL_DEPTH;
  return d != 0 && d <= (uint32_t)(hops + 1);
}

// diagnostics: per-wave sums of sub-step times (profiling builds of a phase only)
struct Ticker {
  bool on = false;
  uint64_t t0 = 0;
  uint64_t sub[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  __device__ __forceinline__ void tick(int k) {
    if (on) {
      asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
      const uint64_t t1 = wall_clock64();
      sub[k] += t1 - t0;
      t0 = t1;
    }
  }
};


// Lockstep probe of NQ keys (the first nq valid): every round reads one bucket for every key
// still unresolved, so a lane's NQ probe sequences share round trips.
template <bool GT, int NQ>
__device__ __forceinline__ void find_batch(const Tab<GT>& t, const uint32_t (&key)[NQ], uint32_t nq,
                                           int (&q)[NQ]) {
  const uint32_t nb = t.cap / 4;
  uint32_t bk[NQ];
  uint32_t pend = 0;
#pragma unroll
  for (int x = 0; x < NQ; ++x) {
    bk[x] = hbucket(key[x], nb);
    q[x] = -1;
    if ((uint32_t)x < nq) pend |= 1u << x;
  }
  if constexpr (!GT) {
    // the filter: a key whose bit is clear is not a member (most pulled neighbours are not)
    uint32_t bw[NQ];
#pragma unroll
    for (int x = 0; x < NQ; ++x)
      bw[x] = (pend & (1u << x)) ? t.bloom[bloom_hash(key[x]) >> 5] : ~0u;
#pragma unroll
    for (int x = 0; x < NQ; ++x)
      if (!((bw[x] >> (bloom_hash(key[x]) & 31u)) & 1u)) pend &= ~(1u << x);
  }
  for (uint32_t n = 0; n < nb && __any(pend != 0); ++n) {
    uint4 kk[NQ];
#pragma unroll
    for (int x = 0; x < NQ; ++x)
      if (pend & (1u << x)) kk[x] = read_bucket(t.keys, bk[x]);
#pragma unroll
    for (int x = 0; x < NQ; ++x) {
      if (pend & (1u << x)) {
        const int r = bucket_match(kk[x], key[x], bk[x]);
        if (r != -2) {
          q[x] = r;
          pend &= ~(1u << x);
        } else {
          bk[x] = bk[x] + 1 == nb ? 0 : bk[x] + 1;
        }
      }
    }
  }
}

// Row kinds of a phase: K_REACH = reach frontier (insert neighbours, give new ones the next
// depth), K_PULL = recompute the row's score, K_PROP = expansion for the next hop (insert
// neighbours and mark them `need` for it).
// K_NOINS (pruned runs, hop hops - 2): the expansion only marks members already present --
// every candidate exists by then, and the last pull reads nothing else.
constexpr uint32_t K_REACH = 1u, K_PULL = 2u, K_PROP = 4u, K_NOINS = 8u;
// Reach runs two walks ahead of the pulls: level 1 is the incident row (a pre-pass), walk h
// (SEEDS: h = -1) expands the members at depth h + 2 into level h + 3 (fl = depth + 1).
constexpr int REACH_AHEAD = 2;

enum Phase { SEEDS, PULL };

// `need` bits: bit (h & 1) marks the members pulled at hop h; set with a 32-bit LDS / global
// atomic OR because the other parity's bit of the same byte is read concurrently
template <bool GT>
__device__ __forceinline__ void set_need(const Tab<GT>& t, uint32_t q, uint32_t par) {
  atomicOr(reinterpret_cast<uint32_t*>(t.need) + (q >> 2), (1u << par) << ((q & 3u) * 8u));
}

// Insertion side of a row entry (after its probe): q = the slot if present, else insert.
template <bool GT>
__device__ __forceinline__ void grow_entry(const Tab<GT>& t, uint32_t key, int q, uint32_t kind,
                                           int h) {
  if (q < 0 && (kind & (K_NOINS | K_REACH)) == K_NOINS) return;
  const int qq = q >= 0 ? q : tab_insert<GT>(t, key);
  if (qq < 0) return;
  if (kind & K_REACH) {   // walk h builds reach level h + 1 + REACH_AHEAD (fl = depth + 1)
    const uint8_t fo = t.fl[qq];
    if ((fo & FL_DEPTH) == 0) t.fl[qq] = fo | (uint8_t)(h + 2 + REACH_AHEAD);   // all write this
  }
  if (kind & K_PROP) set_need<GT>(t, (uint32_t)qq, (uint32_t)(h + 1) & 1u);
}

// One row of dl <= LMAX entries, one lane per row: every entry is loaded in one round trip,
// probed LB keys at a time (lockstep), then the in-order fmaf chain runs in registers (K_PULL)
// and the absent neighbours are inserted (K_REACH / K_PROP).
template <bool GT>
__device__ __forceinline__ void light_row(const FArgs& A, const Tab<GT>& t, uint32_t e0, uint32_t dl,
                                          uint32_t kind, int h, float& acc, Ticker& tk) {
  uint32_t c[LMAX];
  float w[LMAX];
#pragma unroll
  for (int x = 0; x < LMAX; ++x) {
    uint2 ce = make_uint2(0u, 0u);
    if ((uint32_t)x < dl) ce = A.cv[e0 + x];
    c[x] = ce.x;
    w[x] = __uint_as_float(ce.y);
  }
  tk.tick(4);
#pragma unroll
  for (int sb = 0; sb < LMAX / LB; ++sb) {
    if (!__any(dl > (uint32_t)(sb * LB))) continue;   // (continue, not break: keeps it unrolled)
    const uint32_t nq = dl > (uint32_t)(sb * LB) ? min(dl - sb * LB, (uint32_t)LB) : 0u;
    uint32_t key[LB];
#pragma unroll
    for (int x = 0; x < LB; ++x) key[x] = c[sb * LB + x];
    int q[LB];
    find_batch<GT, LB>(t, key, nq, q);
    tk.tick(5);
    if (kind & K_PULL) {
      float xs[LB];
#pragma unroll
      for (int x = 0; x < LB; ++x) xs[x] = q[x] >= 0 ? t.s[q[x]] : 0.f;
#pragma unroll
      for (int x = 0; x < LB; ++x)
        if (q[x] >= 0) acc = fmaf(w[sb * LB + x], xs[x], acc);   // absent: skipped (exact)
    }
    tk.tick(6);
    if (kind & (K_REACH | K_PROP)) {
#pragma unroll
      for (int x = 0; x < LB; ++x)
        if ((uint32_t)x < nq) grow_entry<GT>(t, key[x], q[x], kind, h);
    }
    tk.tick(7);
  }
}

__device__ __forceinline__ float readlane_f(float x, int l) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(x), l));
}

// One pass over the members [0, n) present when it starts, a wave taking 64 at a time.
//   SEEDS (before hop 0, h = -1): the seeds insert their neighbours and mark them `need` for
//         hop 0; the incident vertex inserts its neighbours at depth 1.
//   PULL (hop h): a member pulled at h (`need` bit h & 1, or a seed) recomputes its score:
//         its sum over its row, CSR order, of val * s[neighbour] (non-members skipped: exact,
//         see the file comment) -> snew[member index]; unless h is the last hop it also
//         inserts its neighbours and marks them `need` for h + 1 (a superset of the expansion
//         of the non-zero members: harmless).  Members at reach depth h + 1 insert their
//         neighbours with depth h + 2 in the same walk (reach runs one walk ahead of the
//         pulls, so with A.prune the last pull skips every member outside the candidate set:
//         their final scores are never read).  Insertions during the pass are exact: a new
//         member's score is +0, so a pull that sees it or not reads the same term.
// Rows of <= LMAX entries run one lane per row (light_row); longer rows (hubs) run one at a
// time across the whole wave: 64 entries loaded and probed per round, the fmaf chain over the
// present entries in lane (= CSR) order with v_readlane operands (every lane computes the
// same chain; the owner keeps it).
template <bool GT, Phase PH>
__device__ __forceinline__ void row_phase(const FArgs& A, const Tab<GT>& t, uint32_t n, int h, Work& work,
                                          int b = -1) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  // diagnostics (profiling on, b >= 0): per-wave sums of sub-step times into slots 24..31
  Ticker tk;
  tk.on = A.prof && b >= 0;
  if (tk.on) tk.t0 = wall_clock64();
  const bool prop_next = h + 1 < A.hops;
  const uint32_t par = (uint32_t)h & 1u;
  // walk h (SEEDS: h = -1) expands the members at depth h + REACH_AHEAD into reach level
  // h + REACH_AHEAD + 1: every level <= hops exists before the walk of hop hops - 2 starts
  const uint32_t reach_fl = (uint32_t)(h + REACH_AHEAD + 1);   // fl of the expanded depth
  const bool reach_lvl = h + REACH_AHEAD + 1 <= A.hops;
  const bool prune_now = PH == PULL && A.prune && h == A.hops - 1;
  const uint32_t noins = (A.prune && h == A.hops - 2) ? K_NOINS : 0u;
  auto is_cand = [&](uint8_t f) { return cand_depth(f, A.hops); };
  // members are striped across the waves (i = wave + NWAVES * (lane + 64 k)): vertices inserted
  // together (e.g. the incident's Node hubs, all reached at one level) spread over all waves.
  // The next chunk's selection and row_ptr loads are issued before the current chunk is walked
  // (a member's kind cannot change during the pass: see the comment above).
  struct Chunk {
    uint32_t i, kind, e0, e1;
  };
  auto fetch = [&](uint32_t k0) {
    Chunk c{wave + NWAVES * (lane + 64u * k0), 0u, 0u, 0u};
    uint32_t v = 0;
    if (c.i < n) {
      const uint32_t p = t.mlist[c.i];
      v = t.keys[p];
      const uint8_t f = t.fl[p];
      if (reach_lvl && (f & FL_DEPTH) == reach_fl) c.kind |= K_REACH;
      if constexpr (PH == SEEDS) {
        if (f & FL_SEED) c.kind |= K_PROP | noins;
      } else {
        if ((((t.need[p] >> par) & 1u) || (f & FL_SEED)) && (!prune_now || is_cand(f)))
          c.kind |= K_PULL | (prop_next ? K_PROP | noins : 0u);
      }
    }
    if (c.kind) {
      c.e0 = A.row_ptr[v];
      c.e1 = A.row_ptr[v + 1];
    }
    return c;
  };
  const uint32_t nk = (n + FT - 1) / FT;
  Chunk nxt = nk ? fetch(0) : Chunk{0u, 0u, 0u, 0u};
  for (uint32_t k0 = 0; k0 < nk; ++k0) {
    const Chunk cur = nxt;
    if (k0 + 1 < nk) nxt = fetch(k0 + 1);
    const uint32_t i = cur.i, kind = cur.kind, e0 = cur.e0, deg = cur.e1 - cur.e0;
    if (kind) {
      ++work.rows;
      if (kind & K_PULL) work.pull += deg;
      else work.expand += deg;
    }
    tk.tick(0);
    const bool light = deg <= (uint32_t)LMAX;
    float acc = 0.f;
    light_row<GT>(A, t, e0, light ? deg : 0u, kind, h, acc, tk);
    tk.tick(1);
    uint64_t heavy = __ballot(!light);
    while (heavy) {
      const int m = __ffsll((long long)heavy) - 1;
      heavy &= heavy - 1;
      const uint32_t he0 = __builtin_amdgcn_readlane(e0, m);
      const uint32_t hdeg = __builtin_amdgcn_readlane(deg, m);
      const uint32_t hkind = __builtin_amdgcn_readlane(kind, m);
      float hacc = 0.f;
      for (uint32_t base = 0; base < hdeg; base += 64) {
        const uint32_t j = base + lane;
        const bool act = j < hdeg;
        const uint2 ce = act ? A.cv[he0 + j] : make_uint2(0u, 0u);
        const uint32_t u = ce.x;
        const int q = act ? tab_find<GT>(t, u) : -1;
        if (hkind & K_PULL) {
          const float w = __uint_as_float(ce.y);
          const float x = q >= 0 ? t.s[q] : 0.f;
          // the chain runs over the present entries only, in lane (= CSR) order
          for (uint64_t fm = __ballot(q >= 0); fm; fm &= fm - 1) {
            const int y = __ffsll((long long)fm) - 1;
            hacc = fmaf(readlane_f(w, y), readlane_f(x, y), hacc);
          }
        }
        if ((hkind & (K_REACH | K_PROP)) && act) grow_entry<GT>(t, u, q, hkind, h);
      }
      if (lane == m) acc = hacc;
    }
    tk.tick(2);
    if constexpr (PH == PULL) {
      if (kind & K_PULL) t.snew[i] = acc;
    }
    tk.tick(3);
  }
  if (tk.on && lane == 0)
    for (int k = 0; k < 8; ++k)
      A.prof[((size_t)b * PROF_SLOTS + 24 + k) * PROF_W + 1 + wave] = tk.sub[k];
}

// ---- top-k keys: (score desc, vertex asc) as one u64, larger = better, 0 = none -----------
__device__ __forceinline__ uint64_t topk_key(float s, uint32_t v) {
  const uint32_t f = __float_as_uint(s);
  const uint32_t o = (f & 0x80000000u) ? ~f : (f | 0x80000000u);
  return ((uint64_t)o << 32) | (uint32_t)~v;
}

__device__ __forceinline__ void topk_unkey(uint64_t k, float& s, uint32_t& v) {
  if (k == 0) {
    s = -INFINITY;
    v = NO_NODE;
    return;
  }
  const uint32_t o = (uint32_t)(k >> 32);
  s = __uint_as_float((o & 0x80000000u) ? (o & 0x7FFFFFFFu) : ~o);
  v = ~(uint32_t)k;
}

// wave-wide max of a u32 with DPP row ops (quad perms, half / full row mirror, row broadcasts
// 15 and 31), result from lane 63; every lane gets it
__device__ __forceinline__ uint32_t wave_max_u32(uint32_t x) {
  x = max(x, (uint32_t)__builtin_amdgcn_update_dpp((int)x, (int)x, 0xB1, 0xF, 0xF, false));
  x = max(x, (uint32_t)__builtin_amdgcn_update_dpp((int)x, (int)x, 0x4E, 0xF, 0xF, false));
  x = max(x, (uint32_t)__builtin_amdgcn_update_dpp((int)x, (int)x, 0x141, 0xF, 0xF, false));
  x = max(x, (uint32_t)__builtin_amdgcn_update_dpp((int)x, (int)x, 0x140, 0xF, 0xF, false));
  x = max(x, (uint32_t)__builtin_amdgcn_update_dpp((int)x, (int)x, 0x142, 0xA, 0xF, false));
  x = max(x, (uint32_t)__builtin_amdgcn_update_dpp((int)x, (int)x, 0x143, 0xC, 0xF, false));
  return (uint32_t)__builtin_amdgcn_readlane((int)x, 63);
}

// wave-wide max of a u64 key: the max high word, then the max low word among its holders
__device__ __forceinline__ uint64_t wave_max_u64(uint64_t k) {
  const uint32_t hi = (uint32_t)(k >> 32);
  const uint32_t mh = wave_max_u32(hi);
  const uint32_t ml = wave_max_u32(hi == mh ? (uint32_t)k : 0u);
  return ((uint64_t)mh << 32) | ml;
}

struct Shared {
  uint32_t count, ovf, item;
  unsigned long long base;
  uint64_t top[NWAVES][KMAXF];
  uint32_t w_pull, w_expand, w_rows;
};

// candidate key of member slot p: reached within `hops`, not carrying the excluded label
template <bool GT>
__device__ __forceinline__ uint64_t cand_key(const FArgs& A, const Tab<GT>& t, uint32_t p,
                                             uint8_t maxd) {
  const uint8_t f = t.fl[p] & FL_DEPTH;
  if (f < 1 || f > maxd) return 0;
  const uint32_t v = t.keys[p];
  if (A.exclude >= 0 && A.vlabel[v] == (uint8_t)A.exclude) return 0;
  return topk_key(t.s[p], v);
}

// This thread's best candidate key strictly below `bound` (global variant: rescans).
template <bool GT>
__device__ __forceinline__ uint64_t rescan_best(const FArgs& A, const Tab<GT>& t, uint32_t n,
                                                uint8_t maxd, uint64_t bound) {
  uint64_t b = 0;
  for (uint32_t i = threadIdx.x; i < n; i += FT) {
    const uint64_t kk = cand_key<GT>(A, t, t.mlist[i], maxd);
    if (kk < bound && kk > b) b = kk;
  }
  return b;
}

// Per-wave top-k into sh.top[wave][0..k) (k wave-wide max rounds, no block barrier).
template <bool GT>
__device__ __forceinline__ void wave_topk(const FArgs& A, const Tab<GT>& t, Shared& sh, uint32_t n,
                                          uint8_t maxd) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if constexpr (!GT) {
    uint64_t kk[MPT];
#pragma unroll
    for (int j = 0; j < MPT; ++j) {
      const uint32_t i = threadIdx.x + j * FT;
      kk[j] = i < n ? cand_key<GT>(A, t, t.mlist[i], maxd) : 0ull;
    }
    auto best = [&]() {
      uint64_t b = 0;
#pragma unroll
      for (int j = 0; j < MPT; ++j) b = kk[j] > b ? kk[j] : b;
      return b;
    };
    uint64_t lb = best();
    for (int q = 0; q < A.k; ++q) {
      const uint64_t wb = wave_max_u64(lb);
      if (lane == 0) sh.top[wave][q] = wb;
      if (wb == 0) {                         // uniform: no candidate left in this wave
        for (int r = q + 1 + lane; r < A.k; r += 64) sh.top[wave][r] = 0;
        break;
      }
      if (lb == wb) {
#pragma unroll
        for (int j = 0; j < MPT; ++j)
          if (kk[j] == wb) kk[j] = 0;
        lb = best();
      }
    }
  } else {
    uint64_t lb = rescan_best<GT>(A, t, n, maxd, ~0ull);
    for (int q = 0; q < A.k; ++q) {
      const uint64_t wb = wave_max_u64(lb);
      if (lane == 0) sh.top[wave][q] = wb;
      if (wb == 0) {
        for (int r = q + 1 + lane; r < A.k; r += 64) sh.top[wave][r] = 0;
        break;
      }
      if (lb == wb) lb = rescan_best<GT>(A, t, n, maxd, wb);
    }
  }
}

// One column end to end.  Returns false (uniformly) if the table overflowed.
template <bool GT>
__device__ __forceinline__ bool run_column(const FArgs& A, const Tab<GT>& t, Shared& sh, int b) {
  const uint32_t tid = threadIdx.x;
  const int hops = A.hops;
  Work work;
  // phase-boundary timestamps (s_memrealtime, 100 MHz), thread 0, when profiling is on
  // (each wave's lane 0 also stamps its own finish before the barrier: wstamp)
  int slot = 0;
  auto stamp = [&]() {
    if (A.prof && tid == 0 && slot < PROF_SLOTS)
      A.prof[((size_t)b * PROF_SLOTS + slot) * PROF_W] = wall_clock64();
    ++slot;
  };
  auto wstamp = [&]() {
    if (A.prof && (tid & 63) == 0 && slot < PROF_SLOTS)
      A.prof[((size_t)b * PROF_SLOTS + slot) * PROF_W + 1 + (tid >> 6)] = wall_clock64();
  };
  stamp();
  // seeds: insert (s = -inf), max-combine duplicates (fmaxf, like the dense plan's seed prep),
  // then one entry per vertex claims it and records (slot, s0) for the per-hop seed add
  const uint32_t sb = A.seed_ptr[b], se = A.seed_ptr[b + 1];
  for (uint32_t i = sb + tid; i < se; i += FT) {
    const int q = tab_insert<GT>(t, A.seed_vert[i]);
    if (q >= 0) {
      t.s[q] = -INFINITY;               // every writer writes the same
      t.fl[q] = FL_SEED;
    }
  }
  __syncthreads();
  for (uint32_t i = sb + tid; i < se; i += FT) {
    const int q = tab_find<GT>(t, A.seed_vert[i]);
    if (q < 0) continue;
    unsigned int* sp = reinterpret_cast<unsigned int*>(&t.s[q]);
    unsigned int old = *sp;
    for (;;) {
      const float m = fmaxf(__uint_as_float(old), A.seed_val[i]);
      if (__float_as_uint(m) == old) break;
      const unsigned int got = atomicCAS(sp, old, __float_as_uint(m));
      if (got == old) break;
      old = got;
    }
  }
  __syncthreads();
  for (uint32_t i = sb + tid; i < se; i += FT) {
    const int q = tab_find<GT>(t, A.seed_vert[i]);
    uint2 r = make_uint2(NO_NODE, 0u);
    if (q >= 0) {
      const uint32_t sh8 = ((uint32_t)q & 3u) * 8u;
      const uint32_t old = atomicOr(reinterpret_cast<uint32_t*>(t.fl) + ((uint32_t)q >> 2),
                                    (uint32_t)FL_CLAIM << sh8);
      if (!((old >> sh8) & FL_CLAIM)) r = make_uint2((uint32_t)q, __float_as_uint(t.s[q]));
    }
    A.seed_rep[i] = r;
  }
  __syncthreads();
  if (tid == 0) {
    const uint32_t src = A.sources[b];
    if (src < A.V) {
      const int q = tab_insert<GT>(t, src);
      if (q >= 0) t.fl[q] |= 1;
    }
  }
  __syncthreads();
  // reach level 1 (REACH_AHEAD pre-pass): the incident vertex's row, spread over the workgroup
  if (A.hops >= 1 && A.sources[b] < A.V) {
    const uint32_t src = A.sources[b];
    const uint32_t e0 = A.row_ptr[src], e1 = A.row_ptr[src + 1];
    if (tid == 0) {
      ++work.rows;
      work.expand += e1 - e0;
    }
    for (uint32_t e = e0 + tid; e < e1; e += FT) {
      const int q = tab_insert<GT>(t, A.cv[e].x);
      if (q >= 0 && (t.fl[q] & FL_DEPTH) == 0) t.fl[q] |= 2;   // every writer writes this
    }
  }
  wstamp();
  __syncthreads();
  stamp();
  if (sh.ovf) return false;
  // the seeds' neighbours are the members pulled at hop 0
  row_phase<GT, SEEDS>(A, t, sh.count, -1, work, -1);
  wstamp();
  __syncthreads();
  stamp();
  if (sh.ovf) return false;
  for (int h = 0; h < hops; ++h) {
    // pull hop h (+ the expansion for hop h + 1 and reach level h + 2, in the same walk)
    const uint32_t n0 = sh.count;
    row_phase<GT, PULL>(A, t, n0, h, work, h == hops - 1 ? b : -1);
    wstamp();
    __syncthreads();
    stamp();
    if (sh.ovf) return false;
    // members not pulled at h have no non-zero neighbour and are no seed: exactly +0
    // (pruned last pull: a non-candidate was not pulled and keeps +0; nothing reads it)
    const uint32_t n = sh.count, bit = 1u << ((uint32_t)h & 1u);
    const bool prune_now = A.prune && h == hops - 1;
    for (uint32_t i = tid; i < n; i += FT) {
      const uint32_t p = t.mlist[i];
      const uint8_t nd = t.need[p], f = t.fl[p];
      const bool pulled = i < n0 && ((nd & bit) || (f & FL_SEED)) &&
                          (!prune_now || cand_depth(f, hops));
      t.s[p] = pulled ? t.snew[i] : 0.f;
      if (nd & bit) t.need[p] = nd & ~bit;
    }
    __syncthreads();
    for (uint32_t i = sb + tid; i < se; i += FT) {
      const uint2 r = A.seed_rep[i];
      if (r.x != NO_NODE) t.s[r.x] = t.s[r.x] + __uint_as_float(r.y);
    }
    __syncthreads();
    stamp();
  }
  const uint32_t n = sh.count;
  // top-k over the reach set: each wave its own k best, then wave 0 merges the NWAVES lists
  const int lane = tid & 63, wave = tid >> 6;
  wave_topk<GT>(A, t, sh, n, (uint8_t)(hops + 1));
  wstamp();
  __syncthreads();
  if (wave == 0) {
    uint64_t c[2];
#pragma unroll
    for (int y = 0; y < 2; ++y) {
      const int cc = lane + 64 * y, w = cc / KMAXF, r = cc % KMAXF;
      c[y] = (w < NWAVES && r < A.k) ? sh.top[w][r] : 0ull;
    }
    for (int q = 0; q < A.k; ++q) {
      const uint64_t mine = c[0] > c[1] ? c[0] : c[1];
      const uint64_t wb = wave_max_u64(mine);
      if (lane == 0) {
        float sc;
        uint32_t v;
        topk_unkey(wb, sc, v);
        A.out_ids[(size_t)b * A.k + q] = v;
        A.out_scores[(size_t)b * A.k + q] = sc;
      }
      if (wb != 0) {
        if (c[0] == wb) c[0] = 0;
        if (c[1] == wb) c[1] = 0;
      }
    }
  }
  stamp();
  // members -> pool (coalesced by member index)
  if (tid == 0) sh.base = A.pool_cap ? atomicAdd(A.pool_ctr, (unsigned long long)n) : 0ull;
  {   // work counters: one LDS atomic per wave
    uint32_t wp = work.pull, we = work.expand, wr = work.rows;
    for (int o = 32; o > 0; o >>= 1) {
      wp += __shfl_xor(wp, o);
      we += __shfl_xor(we, o);
      wr += __shfl_xor(wr, o);
    }
    if (lane == 0) {
      atomicAdd(&sh.w_pull, wp);
      atomicAdd(&sh.w_expand, we);
      atomicAdd(&sh.w_rows, wr);
    }
  }
  __syncthreads();
  const unsigned long long base = sh.base;
  const bool keep = A.pool_cap && base + n <= A.pool_cap;
  if (keep) {
    for (uint32_t i = tid; i < n; i += FT) {
      const uint32_t p = t.mlist[i];
      A.pool_v[base + i] = t.keys[p];
      A.pool_s[base + i] = t.s[p];
      A.pool_d[base + i] = t.fl[p] & FL_DEPTH;
    }
  }
  if (tid == 0) {
    A.mem_off[b] = base;
    A.mem_cnt[b] = keep ? n : NO_NODE;
    atomicAdd(&A.stats[0], (unsigned long long)sh.w_pull);
    atomicAdd(&A.stats[1], (unsigned long long)sh.w_expand);
    atomicAdd(&A.stats[2], (unsigned long long)sh.w_rows);
    atomicAdd(&A.stats[3], (unsigned long long)n);
  }
  stamp();
  return true;
}

__global__ __launch_bounds__(FT) __attribute__((amdgpu_waves_per_eu(EGR_FR_WAVES_PER_EU)))
void frontier_lds_kernel(const FArgs A) {
  __shared__ uint32_t keys[LCAP];
  __shared__ float s[LCAP];
  __shared__ uint32_t flw[LCAP / 4];
  __shared__ uint32_t needw[LCAP / 4];
  __shared__ uint16_t mlist[LLIMIT];
  __shared__ uint32_t bloom[BLOOM_WORDS];
  __shared__ Shared sh;
  const uint32_t tid = threadIdx.x;
  const int b = (int)A.order[blockIdx.x];
  if (tid == 0) {               // the seed counters are consumed: leave them zero for the next set
    A.seed_cnt[b] = 0;
    A.seed_cnt[A.B + b] = 0;
  }
  for (uint32_t i = tid; i < BLOOM_WORDS; i += FT) bloom[i] = 0;
#pragma unroll
  for (int i = 0; i < LPPT; ++i) {
    keys[tid + i * FT] = EMPTY;
    s[tid + i * FT] = 0.f;
  }
  for (uint32_t i = tid; i < LCAP / 4; i += FT) flw[i] = 0;
  for (uint32_t i = tid; i < LCAP / 4; i += FT) needw[i] = 0;
  if (tid == 0) {
    sh.count = 0;
    sh.ovf = 0;
    sh.w_pull = sh.w_expand = sh.w_rows = 0;
  }
  __syncthreads();
  Tab<false> t{keys, s, reinterpret_cast<uint8_t*>(flw), reinterpret_cast<uint8_t*>(needw), mlist, A.lsnew + (size_t)b * LLIMIT, LCAP, LLIMIT, &sh.count,
               &sh.ovf, bloom};
  if (!run_column<false>(A, t, sh, b) && tid == 0) {
    A.ovf_list[atomicAdd(A.ovf_n, 1u)] = (uint32_t)b;
    atomicAdd(&A.stats[4], 1ull);
  }
}

// Persistent fallback: each workgroup owns one global table and drains the overflow list.
__global__ __launch_bounds__(FT, 2) void frontier_global_kernel(const FArgs A) {
  __shared__ Shared sh;
  const uint32_t tid = threadIdx.x;
  const size_t cap = A.gcap;
  Tab<true> t{A.gkeys + blockIdx.x * cap, A.gs + blockIdx.x * cap, A.gfl + blockIdx.x * cap,
              A.gneed + blockIdx.x * cap, A.gmlist + (size_t)blockIdx.x * A.V,
              A.gsnew + (size_t)blockIdx.x * A.V, (uint32_t)cap, A.V, &sh.count, &sh.ovf, nullptr};
  const uint32_t n_items = *A.ovf_n;
  for (;;) {
    if (tid == 0) {
      sh.item = atomicAdd(A.ovf_next, 1u);
      sh.count = 0;
      sh.ovf = 0;
      sh.w_pull = sh.w_expand = sh.w_rows = 0;
    }
    __syncthreads();
    const uint32_t item = sh.item;
    if (item >= n_items) break;
    const int b = (int)A.ovf_list[item];
    if (!run_column<true>(A, t, sh, b)) {   // cannot happen: members <= V
      for (int q = tid; q < A.k; q += FT) {
        A.out_ids[(size_t)b * A.k + q] = NO_NODE;
        A.out_scores[(size_t)b * A.k + q] = -INFINITY;
      }
      if (tid == 0) A.mem_cnt[b] = NO_NODE;
    }
    __syncthreads();
    // reset the slots this column used (the table starts clean: memset at creation)
    const uint32_t n = min(sh.count, A.V);
    for (uint32_t i = tid; i < n; i += FT) {
      const uint32_t p = t.mlist[i];
      t.keys[p] = EMPTY;
      t.s[p] = 0.f;
      t.fl[p] = 0;
      t.need[p] = 0;
    }
    __syncthreads();
  }
}

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
// launch order, so the costly columns do not start in the last round).  One block of 1024
// threads, each owning a contiguous run of columns.
constexpr int COST_BUCKETS = 64;

__device__ __forceinline__ int cost_bucket(uint32_t cost) {
  const int lg = (int)(__log2f((float)cost + 1.0f) * 3.0f);
  return COST_BUCKETS - 1 - min(COST_BUCKETS - 1, lg);
}

__global__ __launch_bounds__(1024) void seed_scan_kernel(uint32_t* cnt, int B, uint32_t* ptr,
                                                         const uint32_t* __restrict__ cost,
                                                         uint32_t* order, unsigned long long* ctr,
                                                         uint32_t* ovf) {
  __shared__ uint32_t part[1024];
  __shared__ uint32_t hist[COST_BUCKETS];
  const int tid = threadIdx.x;
  const int per = (B + 1023) / 1024;
  const int c0 = min(B, tid * per), c1 = min(B, c0 + per);
  uint32_t sum = 0;
  for (int c = c0; c < c1; ++c) sum += cnt[c];
  part[tid] = sum;
  __syncthreads();
  for (int off = 1; off < 1024; off <<= 1) {   // Hillis-Steele inclusive scan of the run sums
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
  if (tid == 1023) ptr[B] = part[1023];
  if (tid < 6) ctr[tid] = 0;      // the next run's pool / stats counters and overflow list
  if (tid < 2) ovf[tid] = 0;
  // launch order
  if (tid < COST_BUCKETS) hist[tid] = 0;
  __syncthreads();
  for (int c = c0; c < c1; ++c) atomicAdd(&hist[cost_bucket(cost[c])], 1u);
  __syncthreads();
  if (tid == 0) {
    uint32_t acc = 0;
    for (int i = 0; i < COST_BUCKETS; ++i) {
      const uint32_t x = hist[i];
      hist[i] = acc;
      acc += x;
    }
  }
  __syncthreads();
  for (int c = c0; c < c1; ++c) order[atomicAdd(&hist[cost_bucket(cost[c])], 1u)] = (uint32_t)c;
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
  int64_t vmax = 0;               // vertex count the V-sized buffers were sized for (headroom
                                  // for incremental snapshot updates)
  int B = 0, k = 0, nbig = 0;
  int64_t max_seeds = 0;
  uint32_t gcap = 0;
  int64_t n_seeds = 0;
  uint32_t* seed_ptr = nullptr;   // [B+1] exclusive scan of seed_cnt
  uint32_t* seed_cnt = nullptr;   // [2B]: per-column counts, then scatter cursors; then costs
  uint32_t* order = nullptr;      // [B] launch order of the columns
  uint32_t* ident = nullptr;      // [B] 0..B-1 ($EGRAPH_FRONTIER_NO_ORDER: launch in column order)
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
  uint32_t* ovf = nullptr;             // [0] n, [1] next, [2..] list (B)
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
};

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
  // sized with headroom so the snapshot can grow by incremental updates (egr_snapshot_update)
  const int64_t vmax = std::min<int64_t>(s->V + s->V / 4 + 4096, (int64_t)EGR_NO_NODE - 1);
  f->vmax = vmax;
  const uint32_t V = (uint32_t)vmax;
  // fallback table: 2 x nextpow2(V) slots, never more than half full
  size_t gcap = 2 * LCAP;
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
      (rc = dalloc(&f->seed_v, ms)) || (rc = dalloc(&f->seed_s, ms)) ||
      (rc = dalloc(&f->seed_rep, ms)) ||
      (rc = dalloc(&f->pool_v, f->pool_cap)) || (rc = dalloc(&f->pool_s, f->pool_cap)) ||
      (rc = dalloc(&f->pool_d, f->pool_cap)) || (rc = dalloc(&f->ctr, 6)) ||
      (rc = dalloc(&f->mem_off, (size_t)n_cols)) || (rc = dalloc(&f->mem_cnt, (size_t)n_cols)) ||
      (rc = dalloc(&f->ovf, (size_t)n_cols + 2)) ||
      (rc = dalloc(&f->gkeys, gcap * f->nbig)) || (rc = dalloc(&f->gs, gcap * f->nbig)) ||
      (rc = dalloc(&f->gfl, gcap * f->nbig)) || (rc = dalloc(&f->gneed, gcap * f->nbig)) || (rc = dalloc(&f->gsnew, (size_t)V * f->nbig)) ||
      (rc = dalloc(&f->gmlist, (size_t)V * f->nbig)) ||
      (rc = dalloc(&f->lsnew, (size_t)n_cols * LLIMIT))) {
    egr_frontier_free(f);
    return rc;
  }
  if (getenv("EGRAPH_FRONTIER_PROFILE") &&
      (rc = dalloc(&f->prof, (size_t)n_cols * PROF_SLOTS * PROF_W))) {
    egr_frontier_free(f);
    return rc;
  }
  if (hipMemset(f->gkeys, 0xFF, gcap * f->nbig * 4) != hipSuccess ||
      hipMemset(f->gs, 0, gcap * f->nbig * 4) != hipSuccess ||
      hipMemset(f->gfl, 0, gcap * f->nbig) != hipSuccess ||
      hipMemset(f->gneed, 0, gcap * f->nbig) != hipSuccess ||
      hipMemset(f->mem_cnt, 0xFF, (size_t)n_cols * 4) != hipSuccess ||
      hipMemset(f->seed_cnt, 0, (size_t)n_cols * 8) != hipSuccess ||
      hipMemset(f->ctr, 0, 6 * 8) != hipSuccess) {
    egr_frontier_free(f);
    return egr::fail(EGR_EDEVICE, "egr_frontier_create: table init failed");
  }
  {
    std::vector<uint32_t> id((size_t)n_cols);
    for (int i = 0; i < n_cols; ++i) id[i] = (uint32_t)i;
    if (hipMemcpy(f->ident, id.data(), (size_t)n_cols * 4, hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(f->order, id.data(), (size_t)n_cols * 4, hipMemcpyHostToDevice) != hipSuccess) {
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
  dfree(f->gkeys);
  dfree(f->gs);
  dfree(f->gsnew);
  dfree(f->lsnew);
  dfree(f->prof);
  dfree(f->gfl);
  dfree(f->gneed);
  dfree(f->gmlist);
  delete f;
}


static int frontier_outgrown(const egr_frontier* f, const char* what) {
  return egr::fail(EGR_ESTATE, std::string(what) + ": the snapshot grew past the " +
                   std::to_string(f->vmax) + " vertices this frontier was sized for; create a new one");
}

int64_t egr_frontier_max_vertices(const egr_frontier* f) { return f ? f->vmax : -1; }

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
  hipLaunchKernelGGL(seed_scan_kernel, dim3(1), dim3(1024), 0, st, f->seed_cnt, f->B, f->seed_ptr,
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

int egr_frontier_run(egr_frontier* f, const uint32_t* source_vertex, int32_t hops,
                     int32_t exclude_label, uint32_t* out_ids, float* out_scores, void* stream) {
  if (!f || !source_vertex || !out_ids || !out_scores || hops < 1 || hops > MAX_HOPS)
    return egr::fail(EGR_EINVAL, "egr_frontier_run: bad arguments (need 1 <= hops <= 60)");
  if (!f->seeds_set) return egr::fail(EGR_ESTATE, "egr_frontier_run: seeds not set");
  if (f->s->V > f->vmax) return frontier_outgrown(f, "egr_frontier_run");
  DeviceGuard guard(f->s->device);
  hipStream_t st = (hipStream_t)stream;
  const egr_snapshot* s = f->s;
  if (!f->ctr_clean) {
    EGR_HIP(hipMemsetAsync(f->ctr, 0, 6 * 8, st));
    EGR_HIP(hipMemsetAsync(f->ovf, 0, 2 * 4, st));
  }
  FArgs a;
  a.row_ptr = s->row_ptr;
  a.cv = s->cv;
  a.vlabel = s->vlabel;
  a.V = (uint32_t)s->V;
  a.B = f->B;
  a.hops = hops;
  a.k = f->k;
  a.exclude = exclude_label;
  a.prune = (f->pool_cap == 0 && !getenv("EGRAPH_FRONTIER_NO_PRUNE")) ? 1 : 0;
  a.seed_ptr = f->seed_ptr;
  a.seed_vert = f->seed_v;
  a.seed_val = f->seed_s;
  a.seed_rep = f->seed_rep;
  a.sources = source_vertex;
  a.order = getenv("EGRAPH_FRONTIER_NO_ORDER") ? f->ident : f->order;
  a.seed_cnt = f->seed_cnt;
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
  a.ovf_list = f->ovf + 2;
  a.gkeys = f->gkeys;
  a.gs = f->gs;
  a.gsnew = f->gsnew;
  a.gfl = f->gfl;
  a.gneed = f->gneed;
  a.gmlist = f->gmlist;
  a.gcap = f->gcap;
  a.lsnew = f->lsnew;
  a.prof = f->prof;
  if (f->prof) EGR_HIP(hipMemsetAsync(f->prof, 0, (size_t)f->B * PROF_SLOTS * PROF_W * 8, st));
  a.stats = f->ctr + 1;
  hipLaunchKernelGGL(frontier_lds_kernel, dim3(f->B), dim3(FT), 0, st, a);
  EGR_CHECK_LAUNCH();
  hipLaunchKernelGGL(frontier_global_kernel, dim3(f->nbig), dim3(FT), 0, st, a);
  EGR_CHECK_LAUNCH();
  f->ran = true;
  f->ctr_clean = false;
  f->cnt_clean = true;
  return EGR_OK;
}

int egr_frontier_stats(const egr_frontier* f, int64_t* out8, void* stream) {
  if (!f || !out8) return egr::fail(EGR_EINVAL, "egr_frontier_stats: NULL argument");
  if (!f->ran) return egr::fail(EGR_ESTATE, "egr_frontier_stats: not run yet");
  DeviceGuard guard(f->s->device);
  unsigned long long h[6];
  uint32_t nu = 0;
  EGR_HIP(hipMemcpyAsync(h, f->ctr, sizeof(h), hipMemcpyDeviceToHost, (hipStream_t)stream));
  EGR_HIP(hipMemcpyAsync(&nu, f->seed_ptr + f->B, 4, hipMemcpyDeviceToHost, (hipStream_t)stream));
  EGR_HIP(hipStreamSynchronize((hipStream_t)stream));
  for (int i = 0; i < 5; ++i) out8[i] = (int64_t)h[i + 1];
  out8[5] = (int64_t)h[0];
  out8[6] = (int64_t)nu;
  out8[7] = 0;
  return EGR_OK;
}

int egr_frontier_phase_times(const egr_frontier* f, int64_t* out, int64_t cap, void* stream) {
  if (!f || (cap > 0 && !out) || cap < 0)
    return egr::fail(EGR_EINVAL, "egr_frontier_phase_times: bad arguments");
  if (!f->prof) return 0;
  DeviceGuard guard(f->s->device);
  const int64_t n = std::min<int64_t>(cap, (int64_t)f->B * PROF_SLOTS * PROF_W);
  if (n > 0) {
    EGR_HIP(hipMemcpyAsync(out, f->prof, n * 8, hipMemcpyDeviceToHost, (hipStream_t)stream));
    EGR_HIP(hipStreamSynchronize((hipStream_t)stream));
  }
  return PROF_SLOTS * PROF_W;
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
