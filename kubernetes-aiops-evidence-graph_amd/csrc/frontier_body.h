// Frontier engine kernels for ONE table geometry; included by csrc/frontier.hip once per
// geometry, each time inside its own namespace (no include guard, no includes: by design).
// FR_KERNELS selects the kernels the geometry emits (below).

// Geometry of this instantiation (set by the includer, csrc/frontier.hip):
//   FR_FT threads per workgroup, FR_LCAP LDS table slots, FR_LLIMIT members before a column
//   overflows to the global-memory variant, FR_BLOOM_LOG filter bits (log2), FR_WAVES_PER_EU,
//   FR_LMAX (light-row limit), FR_FIND_SELECT (1: branch-free probe rounds, see find_batch),
//   FR_HEAD (light-row entries probed in the row's lane; the rest of the row is spread over the
//   wave, see light_row; 0: all in-lane).  Every combination instantiated by frontier.hip is a
//   shipped path.  Pull results go by member index to HBM (lsnew) and a copy phase moves them
//   into the one LDS score buffer after each walk (round 2's second slot-indexed buffer, with
//   no copy phase, lost to the extra workgroup per CU its LDS paid for:
//   profiles/r04_ab_one_buffer.txt; git history holds that variant, and the v_readlane hub
//   chains, r02_ab_hubchain.txt).
constexpr int FT = FR_FT;                   // threads per workgroup
constexpr int NWAVES = FT / 64;
constexpr uint32_t LCAP = FR_LCAP;          // LDS table slots
constexpr uint32_t LLIMIT = FR_LLIMIT;      // members before a column overflows (load 0.75)
constexpr int LPPT = LCAP / FT;             // slots cleared per thread
// rows of up to LMAX = FR_LMAX entries run one lane per row (longer ones across the wave, one
// 64-entry segment per round); per geometry: C3's rows are <= 12 but for its Node hubs (12
// measured best against 8 and 16 there, profiles/r02_ab_frontier_session3.txt), C4's telemetry
// links put 29 % of its entries in rows of 13..16 (profiles/r04_ab_lmax.txt)
constexpr int LMAX = FR_LMAX;
static_assert(LMAX % 4 == 0 && LMAX <= 32, "light rows: whole probe batches of LB = 4");
constexpr int LB = 4;                       // keys probed together per lane
constexpr int BLOOM_LOG = FR_BLOOM_LOG;
constexpr uint32_t BLOOM_WORDS = (1u << BLOOM_LOG) / 32;  // rejects absent keys in one read
constexpr int MPT = (LLIMIT + FT - 1) / FT; // members per thread (top-k candidate registers)
constexpr int PROF_W = NWAVES + 1;          // per slot: post-barrier stamp + each wave's finish
static_assert(LCAP % FT == 0 && LLIMIT <= LCAP && NWAVES <= 8, "frontier geometry");
constexpr int CHAIN_W = 64;                 // hub-chain / tail pair scratch per wave
// Row slot records (FR_REC, round 6): a light row's neighbour slots, once resolved by the hash
// probe (and the inserts of the walk that resolved them), are stored in the column's record
// region -- LMAX u16 per member index, 0xFFFF = absent -- and every later walk of the row reads
// them instead of probing again.  A slot never moves, so a recorded slot stays valid; an absent
// entry is recorded only by a walk after which nothing is inserted any more (see rec_walk in
// row_phase), so it stays absent.  Rows longer than LMAX (hubs) are probed in every walk.
#ifndef FR_REC
#define FR_REC 0
#endif
constexpr bool REC = FR_REC != 0;
constexpr size_t REC_STRIDE = (size_t)LLIMIT * LMAX;   // u16 per column
constexpr uint16_t REC_ABSENT = 0xFFFFu;


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
  float2* chain;    // LDS: per-wave hub-chain / tail pair scratch [NWAVES][64]
  uint16_t* rec;    // the column's row slot records [LLIMIT][LMAX] (nullptr: off; LDS tables only)

  __device__ __forceinline__ uint32_t key(uint32_t p) const { return keys[p]; }
  __device__ __forceinline__ float& sc(uint32_t p) const { return s[p]; }
  // the keys of bucket bk's 4 slots (one 16-B read)
  __device__ __forceinline__ uint4 bucket(uint32_t bk) const {
    return reinterpret_cast<const uint4*>(keys)[bk];
  }
};

// Buckets of 4 slots (one 16-B read), probed linearly.  A bucket fills from its first slot: an
// insert CASes the lowest empty slot it sees and moves on only when that slot is taken, so a
// bucket with an empty slot ends every probe sequence that passes through it.
// Hashes use only full-rate 24-bit multiplies (a 32-bit v_mul_lo / v_mul_hi is quarter rate,
// and every probed key pays for its hashes): the id is folded to 24 bits, multiplied by an odd
// 24-bit constant, and 16 mixed bits are range-reduced to [0, nb) by a second 24-bit multiply.
__device__ __forceinline__ uint32_t mix24(uint32_t v, uint32_t c) {
  return (uint32_t)__umul24((v ^ (v >> 24)) & 0xFFFFFFu, c);
}

// (HIP's __umul24 returns a signed int: the product is taken as unsigned before the shift, or a
// table of more than 2^15 buckets would get negative -- out of range -- start buckets.  Tables
// of more than 2^16 buckets, the global-memory variant's on large graphs, reduce a full 32-bit
// hash with __umulhi instead.)
__device__ __forceinline__ uint32_t hbucket(uint32_t v, uint32_t nb) {
  const uint32_t h = mix24(v, 0x9E3779u);
  if (nb > 65536u) return __umulhi(h, nb);
  return (uint32_t)__umul24((h >> 8) & 0xFFFFu, nb) >> 16;
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

// slot of v, inserting it if absent (-1: table full, or an LDS table that has overflowed)
template <bool GT>
__device__ __forceinline__ int tab_insert(const Tab<GT>& t, uint32_t v) {
  const uint32_t nb = GT ? t.cap / 4 : LCAP / 4;   // LDS: a compile-time bucket count
  uint32_t bk = hbucket(v, nb);
  for (uint32_t n = 0; n < nb; ++n) {
    // An LDS table past its member limit hands its column on (the result is discarded), so an
    // insert that has to probe past its first bucket stops there -- a table filled to the last
    // slot would make every insert of a new key scan all its buckets (the dense C4 spent ~4 ms
    // per launch there before this exit).  Checked only past the first bucket: the common
    // insert pays nothing.
    if constexpr (!GT) {
      if (n > 0 && *t.ovf) return -1;
    }
    uint4 kk = t.bucket(bk);
    uint32_t ks[4] = {kk.x, kk.y, kk.z, kk.w};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if (ks[j] == v) return (int)(4 * bk + j);
      if (ks[j] == EMPTY) {
        const uint32_t p = 4 * bk + j;
        const uint32_t old = atomicCAS(t.keys + p, EMPTY, v);
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
  const uint32_t nb = GT ? t.cap / 4 : LCAP / 4;   // LDS: a compile-time bucket count
  uint32_t bk = hbucket(v, nb);
  for (uint32_t n = 0; n < nb; ++n) {
    const int r = bucket_match(t.bucket(bk), v, bk);
    if (r != -2) return r;
    bk = bk + 1 == nb ? 0 : bk + 1;
  }
  return -1;
}

// The column's work counters (egr_frontier_stats: CSR entries pulled / expanded, rows walked)
// live in LDS (Shared::w_pull, w_expand, w_rows): a row walk adds one wave's sums per chunk from
// one lane.  Kept per lane in registers they were live across every walk of the column and, at
// the narrow table's 72 VGPRs, spilled to scratch and reloaded in every chunk.
struct Work {
  uint32_t* ctr;    // LDS: pull, expand, rows
};

// a top-k candidate's depth: reached within `hops` of the incident vertex (fl = depth + 1)
__device__ __forceinline__ bool cand_depth(uint8_t f, int hops) {
  const uint32_t d = f & FL_DEPTH;
  return d != 0 && d <= (uint32_t)(hops + 1);
}

// diagnostics: per-wave sums of sub-step times (profiling builds, -DEGR_FR_PROFILE=1, of a
// phase only).  In the shipped build it holds nothing: its twelve 64-bit sums were live across
// the whole row walk and cost ~24 scalar registers whether or not a run was profiled.
#if EGR_FR_PROFILE
struct Ticker {
  bool on = false;
  uint64_t t0 = 0;
  uint64_t sub[12] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
  __device__ __forceinline__ void tick(int k) {
    if (on) {
      asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
      const uint64_t t1 = wall_clock64();
      sub[k] += t1 - t0;
      t0 = t1;
    }
  }
};
#else
struct Ticker {
  static constexpr bool on = false;
  __device__ __forceinline__ void tick(int) {}
};
#endif


// Lockstep probe of NQ keys (the first nq valid): every round reads one bucket for every key
// still unresolved, so a lane's NQ probe sequences share round trips.
// (EGR_FR_LIGHT_BLOOM=0, an A/B build: the branchy light-row probe skips the membership filter
// and goes straight to the buckets.)
#ifndef EGR_FR_LIGHT_BLOOM
#define EGR_FR_LIGHT_BLOOM 1
#endif
#if FR_FIND_SELECT
template <bool GT, int NQ>
__device__ __forceinline__ void find_batch(const Tab<GT>& t, const uint32_t (&key)[NQ], uint32_t nq,
                                           int (&q)[NQ]) {
  // Branch-free per key: every key reads its filter word and, while any lane still probes, its
  // bucket (a resolved or unused key re-reads one in range, its result unused); the matches,
  // slots and the next bucket are selects, not branches -- a wave no longer steps through the
  // exec-mask bookkeeping of NQ divergent ifs per round
  const uint32_t nb = GT ? t.cap / 4 : LCAP / 4;   // LDS: a compile-time bucket count
  uint32_t bk[NQ];
  bool pend[NQ];
#pragma unroll
  for (int x = 0; x < NQ; ++x) {
    bk[x] = hbucket(key[x], nb);
    q[x] = -1;
    pend[x] = (uint32_t)x < nq;
  }
  if constexpr (!GT) {
    // the filter: a key whose bit is clear is not a member
    uint32_t bw[NQ];
#pragma unroll
    for (int x = 0; x < NQ; ++x) bw[x] = t.bloom[bloom_hash(key[x]) >> 5];
#pragma unroll
    for (int x = 0; x < NQ; ++x) pend[x] = pend[x] && ((bw[x] >> (bloom_hash(key[x]) & 31u)) & 1u);
  }
  for (uint32_t n = 0; n < nb; ++n) {
    bool anyp = false;
#pragma unroll
    for (int x = 0; x < NQ; ++x) anyp = anyp || pend[x];
    if (!__any(anyp)) break;
    uint4 kk[NQ];
#pragma unroll
    for (int x = 0; x < NQ; ++x) kk[x] = t.bucket(bk[x]);
#pragma unroll
    for (int x = 0; x < NQ; ++x) {
      const uint32_t v = key[x];
      const bool m0 = kk[x].x == v, m1 = kk[x].y == v, m2 = kk[x].z == v, m3 = kk[x].w == v;
      const bool hit = m0 || m1 || m2 || m3;
      const uint32_t sl = m0 ? 0u : m1 ? 1u : m2 ? 2u : 3u;
      // slots fill in order: an empty last slot ends the probe sequence
      const bool stop = hit || kk[x].w == EMPTY;
      q[x] = (pend[x] && hit) ? (int)(4 * bk[x] + sl) : q[x];
      const bool go = pend[x] && !stop;
      const uint32_t nx = bk[x] + 1 == nb ? 0u : bk[x] + 1;
      bk[x] = go ? nx : bk[x];
      pend[x] = go;
    }
  }
}
#else
// (branchy: only the keys still probing read -- C3's short rows leave most of a lane's keys
// unused, and the select form measured +0.4 % there, profiles/r04_ab_branch_free_probe.txt)
template <bool GT, int NQ>
__device__ __forceinline__ void find_batch(const Tab<GT>& t, const uint32_t (&key)[NQ], uint32_t nq,
                                           int (&q)[NQ]) {
  const uint32_t nb = GT ? t.cap / 4 : LCAP / 4;   // LDS: a compile-time bucket count
  uint32_t bk[NQ];
  uint32_t pend = 0;
#pragma unroll
  for (int x = 0; x < NQ; ++x) {
    bk[x] = hbucket(key[x], nb);
    q[x] = -1;
    if ((uint32_t)x < nq) pend |= 1u << x;
  }
  if constexpr (!GT && EGR_FR_LIGHT_BLOOM) {
    // the filter: a key whose bit is clear is not a member
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
      if (pend & (1u << x)) kk[x] = t.bucket(bk[x]);
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
#endif

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

// K_REC: the row's slots are recorded (read them, no probe); K_MKREC: record them in this walk
constexpr uint32_t K_REC = 16u, K_MKREC = 32u;

// Insertion side of a row entry (after its probe): q = the slot if present, else insert.
// Returns the entry's slot after it (-1: absent and not inserted, or the table overflowed).
template <bool GT>
__device__ __forceinline__ int grow_entry(const Tab<GT>& t, uint32_t key, int q, uint32_t kind,
                                          int h) {
  if (q < 0 && (kind & (K_NOINS | K_REACH)) == K_NOINS) return -1;
  const int qq = q >= 0 ? q : tab_insert<GT>(t, key);
  if (qq < 0) return -1;
  if (kind & K_REACH) {   // walk h builds reach level h + 1 + REACH_AHEAD (fl = depth + 1)
    const uint8_t fo = t.fl[qq];
    if ((fo & FL_DEPTH) == 0) t.fl[qq] = fo | (uint8_t)(h + 2 + REACH_AHEAD);   // all write this
  }
  if (kind & K_PROP) set_need<GT>(t, (uint32_t)qq, (uint32_t)(h + 1) & 1u);
  return qq;
}

__device__ __forceinline__ int rec_slot(uint32_t w, int hi) {   // u16 hi of a packed word
  const uint32_t s = hi ? (w >> 16) : (w & 0xFFFFu);
  return s == REC_ABSENT ? -1 : (int)s;
}

// Inclusive sum over the wave's 64 lanes (every lane active): DPP row shifts inside each row of
// 16 lanes, then the row broadcasts of lanes 15 and 31.
__device__ __forceinline__ uint32_t wave_incl_sum(uint32_t x) {
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xF, 0xF, true);    // row_shr:1
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xF, 0xF, true);    // row_shr:2
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xF, 0xF, true);    // row_shr:4
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xF, 0xF, true);    // row_shr:8
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xA, 0xF, false);   // row_bcast:15
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xC, 0xF, false);   // row_bcast:31
  return x;
}

__device__ __forceinline__ void wave_sync_lds() {
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
}

// One row of dl <= LMAX entries, one lane per row.  Its first NH entries (FR_HEAD; all LMAX
// when FR_HEAD is 0) are loaded in one round trip, probed LB keys at a time (lockstep), then
// the in-order fmaf chain runs in registers (K_PULL) and the absent neighbours are inserted
// (K_REACH / K_PROP).  With FR_HEAD, the rest of every row (its tail, entries NH..dl-1) is
// spread over the wave's lanes 64 entries a round, one entry per lane -- a wave's rows are
// mostly short (C3: 78 % of <= 4 entries), so probing LMAX keys per lane left most lanes idle
// in the later probe batches: each tail lane loads its entry, probes it, inserts it, and writes
// (w, x) (w = 0 if absent or not pulled) to the wave's pair scratch, from which the row's lane
// continues its chain in CSR order.
template <bool GT>
__device__ __forceinline__ void light_row(const FArgs& A, const Tab<GT>& t, uint32_t e0, uint32_t dl,
                                          uint32_t kind, int h, float& acc, Ticker& tk, uint32_t mi) {
  constexpr int NH = FR_HEAD ? FR_HEAD : LMAX;
  static_assert(NH % LB == 0 && NH <= LMAX && LMAX - NH <= 16, "light-row head");
  constexpr bool RC = REC && !GT;
  const uint32_t dh = min(dl, (uint32_t)NH);
  const bool hr = RC && (kind & K_REC) && dh != 0;     // slots recorded: no probe
  const bool mr = RC && (kind & K_MKREC) && dh != 0;   // record them in this walk
  uint16_t* const rr = RC ? t.rec + (size_t)mi * LMAX : nullptr;
  uint32_t c[NH];
  float w[NH];
  // two entries per 16-B load (8-B aligned: gfx950 global loads need only dword alignment);
  // the second entry of an odd row's last pair lies past the row -- read (the CSR arrays carry
  // two entries of padding) but never used: the probes and the chain stop at dl
#pragma unroll
  for (int x = 0; x < NH; x += 2) {
    Pair2 ce = {0u, 0u, 0u, 0u};
    if ((uint32_t)x < dh) ce = *reinterpret_cast<const Pair2*>(A.cv + e0 + x);
    c[x] = ce.c0;
    w[x] = __uint_as_float(ce.v0);
    c[x + 1] = ce.c1;
    w[x + 1] = __uint_as_float(ce.v1);
  }
  // the head's recorded slots: LB u16 per 8-B word pair (record rows are LMAX * 2 B, 8-B aligned)
  uint2 rw[NH / LB];
#pragma unroll
  for (int sb = 0; sb < NH / LB; ++sb) {
    rw[sb] = make_uint2(0xFFFFFFFFu, 0xFFFFFFFFu);
    if (hr && (uint32_t)(sb * LB) < dh) rw[sb] = *reinterpret_cast<const uint2*>(rr + sb * LB);
  }
  tk.tick(4);
#pragma unroll
  for (int sb = 0; sb < NH / LB; ++sb) {
    if (!__any(dh > (uint32_t)(sb * LB))) continue;   // (continue, not break: keeps it unrolled)
    const uint32_t nq = dh > (uint32_t)(sb * LB) ? min(dh - sb * LB, (uint32_t)LB) : 0u;
    uint32_t key[LB];
#pragma unroll
    for (int x = 0; x < LB; ++x) key[x] = c[sb * LB + x];
    int q[LB];
    if (!RC || __any(!hr && nq != 0u)) {
      find_batch<GT, LB>(t, key, hr ? 0u : nq, q);
    } else {
#pragma unroll
      for (int x = 0; x < LB; ++x) q[x] = -1;
    }
    if (hr) {
#pragma unroll
      for (int x = 0; x < LB; ++x) q[x] = rec_slot(x < 2 ? rw[sb].x : rw[sb].y, x & 1);
    }
    tk.tick(5);
    if (kind & K_PULL) {
      float xs[LB];
#pragma unroll
#if FR_FIND_SELECT
      for (int x = 0; x < LB; ++x) xs[x] = t.s[q[x] >= 0 ? q[x] : 0];   // (slot 0: unused)
#pragma unroll
      for (int x = 0; x < LB; ++x)   // absent: skipped (exact)
        acc = q[x] >= 0 ? fmaf(w[sb * LB + x], xs[x], acc) : acc;
#else
      for (int x = 0; x < LB; ++x) xs[x] = q[x] >= 0 ? t.s[q[x]] : 0.f;
#pragma unroll
      for (int x = 0; x < LB; ++x)
        if (q[x] >= 0) acc = fmaf(w[sb * LB + x], xs[x], acc);   // absent: skipped (exact)
#endif
    }
    tk.tick(6);
    int rq[LB];
#pragma unroll
    for (int x = 0; x < LB; ++x) rq[x] = q[x];
    if (kind & (K_REACH | K_PROP)) {
#pragma unroll
      for (int x = 0; x < LB; ++x)
        if ((uint32_t)x < nq) rq[x] = grow_entry<GT>(t, key[x], q[x], kind, h);
    }
    if (mr && nq != 0u) {   // the batch's slots after its inserts (-1 -> REC_ABSENT)
      const uint32_t u0 = (uint32_t)rq[0] & 0xFFFFu, u1 = (uint32_t)rq[1] & 0xFFFFu;
      const uint32_t u2 = (uint32_t)rq[2] & 0xFFFFu, u3 = (uint32_t)rq[3] & 0xFFFFu;
      *reinterpret_cast<uint2*>(rr + sb * LB) = make_uint2(u0 | (u1 << 16), u2 | (u3 << 16));
    }
    tk.tick(7);
  }
#if FR_HEAD
  const uint32_t tl = dl - dh;                    // this row's tail
  if (!__any(tl != 0u)) return;                   // (wave-uniform)
  const int lane = threadIdx.x & 63;
  const uint32_t incl = wave_incl_sum(tl);
  const uint32_t off = incl - tl;                 // the tail's first position
  const uint32_t R = __builtin_amdgcn_readlane(incl, 63);
  float2* const pr = t.chain + (threadIdx.x >> 6) * CHAIN_W;   // the wave's pair scratch
  uint8_t* const mk = reinterpret_cast<uint8_t*>(pr);          // (owner marks, read first)
  for (uint32_t r0 = 0; r0 < R; r0 += 64) {
    // the owner lane of every position of this round's window [r0, r0 + 64)
    for (uint32_t y = 0; y < (uint32_t)(LMAX - NH) && __any(y < tl); ++y) {
      const int p = (int)(off + y) - (int)r0;
      if (y < tl && p >= 0 && p < 64) mk[p] = (uint8_t)lane;
    }
    wave_sync_lds();
    const uint32_t pos = r0 + lane;
    const bool valid = pos < R;
    const int o = valid ? (int)mk[lane] : lane;
    wave_sync_lds();                              // (the marks are read before the pairs land)
    const uint32_t oe0 = (uint32_t)__shfl((int)e0, o, 64);
    const uint32_t ooff = (uint32_t)__shfl((int)off, o, 64);
    const uint32_t okind = (uint32_t)__shfl((int)kind, o, 64);
    const uint2 ce = valid ? A.cv[oe0 + NH + (pos - ooff)] : make_uint2(0u, 0u);
    const uint32_t key1[1] = {ce.x};
    int q1[1];
    // a recorded row's tail entry: its slot from the owner's record (owner member index by
    // shuffle), no probe
    uint16_t* trec = nullptr;
    bool thr = false;
    uint32_t tslot = REC_ABSENT;
    if constexpr (RC) {
      const uint32_t omi = (uint32_t)__shfl((int)mi, o, 64);
      trec = t.rec + (size_t)omi * LMAX + NH + (pos - ooff);
      thr = valid && (okind & K_REC);
      if (thr) tslot = *trec;
    }
    if (!RC || __any(valid && !thr)) {
      find_batch<GT, 1>(t, key1, (valid && !thr) ? 1u : 0u, q1);
    } else {
      q1[0] = -1;
    }
    if (thr) q1[0] = tslot == REC_ABSENT ? -1 : (int)tslot;
    tk.tick(5);
    const bool term = q1[0] >= 0 && (okind & K_PULL);
    const float x = term ? t.sc((uint32_t)q1[0]) : 0.f;
    pr[lane] = make_float2(term ? __uint_as_float(ce.y) : 0.f, x);
    int tq = q1[0];
    if (valid && (okind & (K_REACH | K_PROP))) tq = grow_entry<GT>(t, ce.x, q1[0], okind, h);
    if constexpr (RC) {
      if (valid && (okind & K_MKREC)) *trec = tq < 0 ? REC_ABSENT : (uint16_t)tq;
    }
    tk.tick(7);
    wave_sync_lds();
    // each row's lane continues its chain over its positions in this window, in CSR order
    // (an absent or unpulled term is (+0, +0): fmaf leaves acc unchanged, acc != -0)
    const int a0 = max((int)off - (int)r0, 0);
    const int a1 = min((int)(off + tl) - (int)r0, 64);
    // (two pairs a step, the wave leaving as soon as no lane has more: most tails are one to
    // four entries, and holding all LMAX - NH pairs at once was the walk's register peak)
    const bool pulls = (kind & K_PULL) && a0 < a1;
#pragma unroll
    for (int y = 0; y < LMAX - NH; y += 2) {
      if (!__any(pulls && a0 + y < a1)) break;
      const float2 p0 = pr[min(a0 + y, 63)], p1 = pr[min(a0 + y + 1, 63)];
      if (pulls) {
        acc = a0 + y < a1 ? fmaf(p0.x, p0.y, acc) : acc;
        acc = a0 + y + 1 < a1 ? fmaf(p1.x, p1.y, acc) : acc;
      }
    }
    tk.tick(6);
    wave_sync_lds();                              // (read before the next round's marks)
  }
#endif
}

__device__ __forceinline__ float readlane_f(float x, int l) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(x), l));
}

// The in-order fmaf chain of one hub-row segment: lane j holds entry j's (w, x).  Only the
// non-zero terms run: an absent neighbour (x = +0) or a member whose score is +0 gives
// fmaf(w, +0, acc) == acc for finite w and acc != -0 (acc starts at +0 and no fmaf of finite
// operands turns it into -0), so the chain over the non-zero entries, in lane (= CSR) order,
// equals the chain over every entry.  Hub rows are mostly non-members: the chain shrinks to the
// few members' terms.  The non-zero pairs are compacted into the wave's LDS scratch (mbcnt rank)
// and lane m runs the chain from 16-B LDS reads (one lane, 4-cycle dependent fmas); the result
// is in lane m.
__device__ __forceinline__ void hub_chain(float w, float x, bool present, int m, float& hacc,
                                          float2* chain) {
  const bool nz = present && x != 0.f;
  const uint64_t mk = __ballot(nz);
  if (mk == 0) return;                      // (wave-uniform)
  const int lane = threadIdx.x & 63;
  const uint32_t r = __builtin_amdgcn_mbcnt_hi((uint32_t)(mk >> 32),
                                               __builtin_amdgcn_mbcnt_lo((uint32_t)mk, 0u));
  const int n = __popcll(mk);
  if (nz) chain[r] = make_float2(w, x);
  if (lane == 0 && (n & 1)) chain[n] = make_float2(0.f, 0.f);   // pads the last 16-B read
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  if (lane == m) {
    const float4* c4 = reinterpret_cast<const float4*>(chain);
    const int n2 = (n + 1) / 2;
    float a = hacc;
    for (int y0 = 0; y0 < n2; y0 += 4) {
      float4 p[4];
#pragma unroll
      for (int y = 0; y < 4; ++y) p[y] = c4[y0 + y];
#pragma unroll
      for (int y = 0; y < 4; ++y) {
        if (y0 + y < n2) {
          a = fmaf(p[y].x, p[y].y, a);
          a = fmaf(p[y].z, p[y].w, a);
        }
      }
    }
    hacc = a;
  }
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
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
                                          int b) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  // diagnostics (profiling on, b >= 0): per-wave sums of sub-step times into slots 24..31
  Ticker tk;
#if EGR_FR_PROFILE
  tk.on = FR_PROF_ON(A) && b >= 0;
  if (tk.on) tk.t0 = wall_clock64();
#endif
  const bool prop_next = h + 1 < A.hops;
  const uint32_t par = (uint32_t)h & 1u;
  // walk h (SEEDS: h = -1) expands the members at depth h + REACH_AHEAD into reach level
  // h + REACH_AHEAD + 1: every level <= hops exists before the walk of hop hops - 2 starts
  const uint32_t reach_fl = (uint32_t)(h + REACH_AHEAD + 1);   // fl of the expanded depth
  const bool reach_lvl = h + REACH_AHEAD + 1 <= A.hops;
  const bool prune_now = PH == PULL && A.prune && h == A.hops - 1;
  const uint32_t noins = (A.prune && h == A.hops - 2) ? K_NOINS : 0u;
  float2* const chain = t.chain ? t.chain + wave * CHAIN_W : nullptr;
  auto is_cand = [&](uint8_t f) { return cand_depth(f, A.hops); };
  // Work split.  A walk is cut into chunks of FT members, striped over the waves: wave w walks
  // chunks k = 0, 1, ... holding members w + NWAVES * (lane + 64 k), so vertices inserted
  // together (e.g. the incident's Node hubs, all reached at one level) spread over different
  // waves.  The next chunk's selection and row_ptr loads are issued before the current chunk is
  // walked (a member's kind cannot change during the pass: see the comment above).
  struct Chunk {
    uint32_t i, kind, e0, e1;
  };
  const uint32_t nch = (n + FT - 1) / FT;
  auto member_of = [&](uint32_t c) { return wave + NWAVES * (lane + 64u * c); };
  // Row slot records (REC): a walk with a later walk records the light rows it walks for the
  // first time.  Every such walk either inserts every absent entry of the rows it walks (reach
  // rows, and expansions without K_NOINS: the record holds a slot for each entry), or is the
  // pruned walk of hop hops - 2 (K_NOINS), after which nothing is inserted any more (its last
  // walk pulls only, and reach level hops + 1 is never built): an absent entry it records stays
  // absent.  The member's NEED_REC bit says the record exists (set here, read by the next walks'
  // fetch; a hub row's bit is ignored -- hubs are never recorded).
  const bool rec_walk = REC && !GT && t.rec != nullptr && h + 1 < A.hops;
  auto fetch = [&](uint32_t c) {
    Chunk ch{member_of(c), 0u, 0u, 0u};
    uint32_t v = 0;
    if (c < nch && ch.i < n) {
      uint32_t p = t.mlist[ch.i];
      v = t.key(p);
      const uint8_t f = t.fl[p];
      if (reach_lvl && (f & FL_DEPTH) == reach_fl) ch.kind |= K_REACH;
      uint32_t nd = 0;
      if constexpr (PH == SEEDS) {
        if (f & FL_SEED) ch.kind |= K_PROP | noins;
      } else {
        nd = t.need[p];
        if ((((nd >> par) & 1u) || (f & FL_SEED)) && (!prune_now || is_cand(f)))
          ch.kind |= K_PULL | (prop_next ? K_PROP | noins : 0u);
      }
      if constexpr (REC && !GT) {
        if (ch.kind && t.rec) {
          if (nd & NEED_REC) {
            ch.kind |= K_REC;
          } else if (rec_walk) {
            ch.kind |= K_MKREC;
            atomicOr(reinterpret_cast<uint32_t*>(t.need) + (p >> 2),
                     (uint32_t)NEED_REC << ((p & 3u) * 8u));
          }
        }
      }
    }
    if (ch.kind) {
      const RowPair rp = *reinterpret_cast<const RowPair*>(A.row_ptr + v);   // one 8-B load
      ch.e0 = rp.e0;
      ch.e1 = rp.e1;
    }
    return ch;
  };
  Chunk nxt = fetch(0);
  for (uint32_t c_cur = 0; c_cur < nch; ++c_cur) {
    if constexpr (!GT) {
      if (*t.ovf) break;        // overflowed LDS table: the column is redone elsewhere
    }
    const Chunk cur = nxt;
    nxt = fetch(c_cur + 1);
    const uint32_t i = cur.i, kind = cur.kind, e0 = cur.e0, deg = cur.e1 - cur.e0;
    {   // the chunk's work counters: wave sums, one lane adds them (all 64 lanes active here)
      const uint32_t sp = wave_incl_sum((kind & K_PULL) ? deg : 0u);
      const uint32_t se = wave_incl_sum((kind && !(kind & K_PULL)) ? deg : 0u);
      const uint64_t rows = __ballot(kind != 0u);
      if (lane == 63) {
        atomicAdd(work.ctr, sp);
        atomicAdd(work.ctr + 1, se);
        atomicAdd(work.ctr + 2, (uint32_t)__popcll(rows));
      }
    }
    tk.tick(0);
    const bool light = deg <= (uint32_t)LMAX;
    float acc = 0.f;
    light_row<GT>(A, t, e0, light ? deg : 0u, kind, h, acc, tk, i);
    tk.tick(1);
    // hub rows, one 64-entry segment at a time across the wave; the next segment's entries (of
    // this hub, or the first of the next one) are loaded before the current one is probed
    uint64_t heavy = __ballot(!light);
    if (heavy) {
      int m = __ffsll((long long)heavy) - 1;
      heavy &= heavy - 1;
      uint32_t he0 = __builtin_amdgcn_readlane(e0, m);
      uint32_t hdeg = __builtin_amdgcn_readlane(deg, m);
      uint32_t hkind = __builtin_amdgcn_readlane(kind, m);
      uint32_t base = 0;
      uint2 ce = lane < (int)hdeg ? A.cv[he0 + lane] : make_uint2(0u, 0u);
      float hacc = 0.f;
      for (;;) {
        int m2 = m;
        uint32_t he02 = he0, hdeg2 = hdeg, hkind2 = hkind, base2 = base + 64;
        bool more = true;
        if (base2 >= hdeg) {
          if (heavy) {
            m2 = __ffsll((long long)heavy) - 1;
            heavy &= heavy - 1;
            he02 = __builtin_amdgcn_readlane(e0, m2);
            hdeg2 = __builtin_amdgcn_readlane(deg, m2);
            hkind2 = __builtin_amdgcn_readlane(kind, m2);
            base2 = 0;
          } else {
            more = false;
          }
        }
        const uint32_t j2 = base2 + lane;
        const uint2 cn = (more && j2 < hdeg2) ? A.cv[he02 + j2] : make_uint2(0u, 0u);
        const uint32_t j = base + lane;
        const bool act = j < hdeg;
        const uint32_t u = ce.x;
        tk.tick(8);
        const int q = act ? tab_find<GT>(t, u) : -1;
        tk.tick(9);
        if (hkind & K_PULL) {
          const float w = __uint_as_float(ce.y);
          const float x = q >= 0 ? t.sc(q) : 0.f;
          hub_chain(w, x, q >= 0, m, hacc, chain);
        }
        tk.tick(10);
        if ((hkind & (K_REACH | K_PROP)) && act) grow_entry<GT>(t, u, q, hkind, h);
        tk.tick(11);
        if (base2 == 0 || !more) {          // the hub's last segment
          if (lane == m) acc = hacc;
          hacc = 0.f;
        }
        if (!more) break;
        ce = cn;
        m = m2;
        he0 = he02;
        hdeg = hdeg2;
        hkind = hkind2;
        base = base2;
      }
    }
    tk.tick(2);
    if constexpr (PH == PULL) {
      if (kind & K_PULL) t.snew[i] = acc;
    }
    tk.tick(3);
#ifdef EGR_FR_VALU_PAD
    {   // perturbation builds only (scripts/build_variant.sh): EGR_FR_VALU_PAD extra VALU
        // instructions per chunk that change no result -- what a VALU instruction costs the
        // launch (profiles/r06_ab_valu_perturbation.txt)
      uint32_t z = (uint32_t)lane;
#pragma unroll
      for (int k = 0; k < EGR_FR_VALU_PAD; ++k) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(z) : "v"(lane));
      asm volatile("" ::"v"(z));
    }
#endif
  }
#if EGR_FR_PROFILE
  if (tk.on && lane == 0)
    for (int k = 0; k < 12; ++k)
      A.prof[((size_t)b * PROF_SLOTS + 24 + k) * PROF_W + 1 + wave] = tk.sub[k];
#endif
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

// wave-wide max of a u64 key: the max high word, then the max low word among its holders (a
// second reduction only when several lanes hold that high word: scores are mostly distinct)
__device__ __forceinline__ uint64_t wave_max_u64(uint64_t k) {
  const uint32_t hi = (uint32_t)(k >> 32);
  const uint32_t mh = wave_max_u32(hi);
  const uint64_t holders = __ballot(hi == mh);
  const uint32_t ml = (holders & (holders - 1))
                          ? wave_max_u32(hi == mh ? (uint32_t)k : 0u)
                          : (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)k, __ffsll((long long)holders) - 1);
  return ((uint64_t)mh << 32) | ml;
}

struct Shared {
  uint32_t count, ovf, item;
  float2 chain[NWAVES][CHAIN_W];   // hub-row chain / light-row tail pairs, one row per wave
#define SH_CHAIN (&sh.chain[0][0])
  unsigned long long base;
  uint64_t top[NWAVES][KMAXF];
  uint32_t w_pull, w_expand, w_rows;   // (contiguous: Work::ctr)
};

// candidate key of member slot p: reached within `hops`, not carrying the excluded label
template <bool GT>
__device__ __forceinline__ uint64_t cand_key(const FArgs& A, const Tab<GT>& t, uint32_t p,
                                             uint8_t maxd) {
  if (p >= t.cap) return 0;
  const uint8_t f = t.fl[p] & FL_DEPTH;
  if (f < 1 || f > maxd) return 0;
  const uint32_t v = t.key(p);
  if (v >= A.V) return 0;
  if (A.exclude >= 0 && (t.need[p] & NEED_EXCL)) return 0;   // marked after the last pull
  // (ties break by the ORIGINAL vertex id, which the key also carries out to the caller)
  return topk_key(t.sc(p), A.iperm ? A.iperm[v] : v);
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
                                          uint8_t maxd, int b = -1) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if constexpr (!GT) {
    // diagnostics (profiling on): per-wave time of the candidate loads and of the k rounds
    const bool prof = FR_PROF_ON(A) && b >= 0;
    const uint64_t tp0 = prof ? wall_clock64() : 0;
    uint64_t kk[MPT];
#pragma unroll
    for (int j = 0; j < MPT; ++j) {
      const uint32_t i = threadIdx.x + j * FT;
      kk[j] = i < n ? cand_key<GT>(A, t, t.mlist[i], maxd) : 0ull;
    }
    // descending odd-even transposition sort of the lane's keys (MPT passes): the round's
    // winner lane then only shifts its registers (profiles/r02_ab_topk_sort.txt)
    static_assert(MPT <= 9, "sorted candidate registers");
#pragma unroll
    for (int pass = 0; pass < MPT; ++pass)
#pragma unroll
      for (int j = pass & 1; j + 1 < MPT; j += 2) {
        const uint64_t x = kk[j], y = kk[j + 1];
        const bool sw = y > x;
        kk[j] = sw ? y : x;
        kk[j + 1] = sw ? x : y;
      }
    uint64_t lb = kk[0];
    uint64_t tp1 = 0;
    if (prof) {
      asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
      tp1 = wall_clock64();
    }
    // one round: the wave's next best key into sh.top[wave][q]; stop once the wave has no
    // candidate left (the rest of its list zero-filled)
    for (int q = 0; q < A.k; ++q) {
      const uint64_t wb = wave_max_u64(lb);
      if (lane == 0) sh.top[wave][q] = wb;
      if (wb == 0) {                         // uniform: no candidate left in this wave
        for (int r = q + 1 + lane; r < A.k; r += 64) sh.top[wave][r] = 0;
        break;
      }
      if (lb == wb) {                        // keys are distinct: one lane, its head taken
#pragma unroll
        for (int j = 0; j + 1 < MPT; ++j) kk[j] = kk[j + 1];
        kk[MPT - 1] = 0;
        lb = kk[0];
      }
    }
    if (prof && lane == 0) {
      const uint64_t tp2 = wall_clock64();
      A.prof[((size_t)b * PROF_SLOTS + 36) * PROF_W + 1 + wave] = tp1 - tp0;
      A.prof[((size_t)b * PROF_SLOTS + 37) * PROF_W + 1 + wave] = tp2 - tp1;
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

// Phase boundary: a barrier, then the member count and overflow flag every thread sees, then a
// second barrier.  Reading them after a single barrier races with the next phase's inserts by
// faster waves: a late wave could see an overflow the others missed and leave alone, and the
// rest would walk a member list longer than the table's limit.
__device__ __forceinline__ bool phase_sync(Shared& sh, uint32_t& cnt) {
  __syncthreads();
  cnt = sh.count;
  const bool ovf = sh.ovf != 0;
  __syncthreads();
  return ovf;
}

// The end of a column after its last pull: top-k over the reach set, the member pool, the
// work counters.  `slot` continues run_column's profiling stamps.
template <bool GT>
__device__ __forceinline__ bool finish_column(const FArgs& A, const Tab<GT>& t, Shared& sh, int b,
                                              uint32_t cnt, const Work& work, int slot) {
  const uint32_t tid = threadIdx.x;
  const int hops = A.hops;
  auto stamp = [&]() {
    if (FR_PROF_ON(A) && tid == 0 && slot < PROF_SLOTS)
      A.prof[((size_t)b * PROF_SLOTS + slot) * PROF_W] = wall_clock64();
    ++slot;
  };
  auto wstamp = [&]() {
    if (FR_PROF_ON(A) && (tid & 63) == 0 && slot < PROF_SLOTS)
      A.prof[((size_t)b * PROF_SLOTS + slot) * PROF_W + 1 + (tid >> 6)] = wall_clock64();
  };
  const uint32_t n = cnt;
  // top-k over the reach set: each wave its own k best, then wave 0 merges the NWAVES lists
  const int lane = tid & 63, wave = tid >> 6;
  wave_topk<GT>(A, t, sh, n, (uint8_t)(hops + 1), b);
  wstamp();
  __syncthreads();
  if (wave == 0) {
    // merge by rank: each of the NWAVES * k candidates counts the candidates above it (keys
    // are distinct: a member is in one wave's list) and lands at its rank; the slots past the
    // number of candidates get EGR_NO_NODE / -inf
    uint64_t c[2];
    uint32_t nnz = 0;
#pragma unroll
    for (int y = 0; y < 2; ++y) {
      const int cc = lane + 64 * y, w = cc / KMAXF, r = cc % KMAXF;
      c[y] = (w < NWAVES && r < A.k) ? sh.top[w][r] : 0ull;
      nnz += (uint32_t)__popcll(__ballot(c[y] != 0));
    }
    uint32_t rank[2] = {0u, 0u};
    for (int w = 0; w < NWAVES; ++w)
      for (int r = 0; r < A.k; ++r) {
        const uint64_t o = sh.top[w][r];
        rank[0] += o > c[0];
        rank[1] += o > c[1];
      }
#pragma unroll
    for (int y = 0; y < 2; ++y) {
      if (c[y] != 0 && rank[y] < (uint32_t)A.k) {
        float sc;
        uint32_t v;
        topk_unkey(c[y], sc, v);
        A.out_ids[(size_t)b * A.k + rank[y]] = v;
        A.out_scores[(size_t)b * A.k + rank[y]] = sc;
      }
    }
    for (uint32_t q = nnz + lane; q < (uint32_t)A.k; q += 64) {
      A.out_ids[(size_t)b * A.k + q] = NO_NODE;
      A.out_scores[(size_t)b * A.k + q] = -INFINITY;
    }
  }
  stamp();
  // members -> pool (coalesced by member index)
  if (tid == 0) sh.base = A.pool_cap ? atomicAdd(A.pool_ctr, (unsigned long long)n) : 0ull;
  (void)work;      // (the work counters are in sh.w_*, complete after the last walk's barrier)
  __syncthreads();
  const unsigned long long base = sh.base;
  const bool keep = A.pool_cap && base + n <= A.pool_cap;
  if (keep) {
    for (uint32_t i = tid; i < n; i += FT) {
      const uint32_t p = t.mlist[i];
      A.pool_v[base + i] = A.iperm ? A.iperm[t.key(p)] : t.key(p);
      A.pool_s[base + i] = t.sc(p);
      A.pool_d[base + i] = t.fl[p] & FL_DEPTH;
    }
  }
  if (FR_PROF_ON(A) && tid == 0) A.prof[((size_t)b * PROF_SLOTS + 20) * PROF_W] = n;   // members
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

// One column end to end.  Returns false (uniformly) if the table overflowed.
template <bool GT>
__device__ __forceinline__ bool run_column(const FArgs& A, const Tab<GT>& t, Shared& sh, int b) {
  const uint32_t tid = threadIdx.x;
  const int hops = A.hops;
  Work work{&sh.w_pull};
  // phase-boundary timestamps (s_memrealtime, 100 MHz), thread 0, when profiling is on
  // (each wave's lane 0 also stamps its own finish before the barrier: wstamp)
  int slot = 0;
  auto stamp = [&]() {
    if (FR_PROF_ON(A) && tid == 0 && slot < PROF_SLOTS)
      A.prof[((size_t)b * PROF_SLOTS + slot) * PROF_W] = wall_clock64();
    ++slot;
  };
  auto wstamp = [&]() {
    if (FR_PROF_ON(A) && (tid & 63) == 0 && slot < PROF_SLOTS)
      A.prof[((size_t)b * PROF_SLOTS + slot) * PROF_W + 1 + (tid >> 6)] = wall_clock64();
  };
  stamp();
  // The incident vertex and its row (reach level 1) are loaded first: their latency hides
  // behind the seed passes.
  // inputs name original vertex ids: mapped to the layout's (perm; identity without a layout)
  auto inmap = [&](uint32_t v) { return (A.perm && v < A.V) ? A.perm[v] : v; };
  const uint32_t src = inmap(A.sources[b]);
  const bool src_ok = A.hops >= 1 && src < A.V;
  const uint32_t ie0 = src_ok ? A.row_ptr[src] : 0u, ie1 = src_ok ? A.row_ptr[src + 1] : 0u;
  const uint32_t ic0 = ie0 + tid < ie1 ? A.cv[ie0 + tid].x : 0u;   // first stripe of the row
  // Seeds, two passes.  Pass 1 inserts every seed vertex and max-combines duplicate entries
  // with one atomicMax on the order-preserving u32 image of the value (ord(): the cleared
  // slot's 0 lies below every float's image, -inf included) -- fmaxf, like the dense plan's
  // seed prep.  Pass 2: one entry per vertex claims it, turns the slot back into the float and
  // records (slot, s0) for the per-hop seed add; thread 0 also inserts the incident vertex.
  // (offsets clamped to the entries given: egr_frontier_run_grouped takes them from the caller)
  const uint32_t sb = min(A.seed_ptr[b], A.n_seeds);
  const uint32_t se = max(sb, min(A.seed_ptr[b + 1], A.n_seeds));
  auto ord = [](float f) {
    const uint32_t u = __float_as_uint(f);
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
  };
  auto unord = [](uint32_t o) {
    return __uint_as_float((o & 0x80000000u) ? (o & 0x7FFFFFFFu) : ~o);
  };
  const uint32_t i0 = sb + tid;
  const uint32_t v0 = i0 < se ? inmap(A.seed_vert[i0]) : 0u;   // the first stripe stays in registers
  const float x0 = i0 < se ? A.seed_val[i0] : 0.f;
  for (uint32_t i = i0; i < se; i += FT) {
    const uint32_t v = i == i0 ? v0 : inmap(A.seed_vert[i]);
    const float x = i == i0 ? x0 : A.seed_val[i];
    if (v >= A.V) continue;          // (grouped seeds: out-of-range vertices are dropped)
    const int q = tab_insert<GT>(t, v);
    if (q >= 0) {
      atomicMax(reinterpret_cast<unsigned int*>(&t.s[q]), ord(x));
      atomicOr(reinterpret_cast<uint32_t*>(t.fl) + ((uint32_t)q >> 2),
               (uint32_t)FL_SEED << (((uint32_t)q & 3u) * 8u));
    }
  }
  __syncthreads();
  for (uint32_t i = i0; i < se; i += FT) {
    const int q = tab_find<GT>(t, i == i0 ? v0 : inmap(A.seed_vert[i]));
    uint2 r = make_uint2(NO_NODE, 0u);
    if (q >= 0) {
      const uint32_t sh8 = ((uint32_t)q & 3u) * 8u;
      const uint32_t old = atomicOr(reinterpret_cast<uint32_t*>(t.fl) + ((uint32_t)q >> 2),
                                    (uint32_t)FL_CLAIM << sh8);
      if (!((old >> sh8) & FL_CLAIM)) {        // the claimer alone touches the value now
        const float s0 = unord(*reinterpret_cast<unsigned int*>(&t.s[q]));
        t.sc(q) = s0;
        r = make_uint2((uint32_t)q, __float_as_uint(s0));
      }
    }
    A.seed_rep[i] = r;
  }
  if (tid == 0 && src_ok) {       // (a find of a seed is unaffected by concurrent inserts)
    const int q = tab_insert<GT>(t, src);
    if (q >= 0)
      atomicOr(reinterpret_cast<uint32_t*>(t.fl) + ((uint32_t)q >> 2), 1u << (((uint32_t)q & 3u) * 8u));
  }
  __syncthreads();
  // reach level 1 (REACH_AHEAD pre-pass): the incident vertex's row, spread over the workgroup
  if (src_ok) {
    if (tid == 0) {
      atomicAdd(&sh.w_rows, 1u);
      atomicAdd(&sh.w_expand, ie1 - ie0);
    }
    for (uint32_t e = ie0 + tid; e < ie1; e += FT) {
      const int q = tab_insert<GT>(t, e == ie0 + tid ? ic0 : A.cv[e].x);
      if (q >= 0 && (t.fl[q] & FL_DEPTH) == 0) t.fl[q] |= 2;   // every writer writes this
    }
  }
  wstamp();
  uint32_t cnt;
  bool ovf = phase_sync(sh, cnt);
  stamp();
  if (ovf) return false;
  // the seeds' neighbours are the members pulled at hop 0
  row_phase<GT, SEEDS>(A, t, cnt, -1, work, -1);
  wstamp();
  ovf = phase_sync(sh, cnt);
  stamp();
  if (ovf) return false;
  for (int h = 0; h < hops; ++h) {
    // pull hop h (+ the expansion for hop h + 1 and reach level h + 3, in the same walk)
    const uint32_t n0 = cnt;
    row_phase<GT, PULL>(A, t, n0, h, work, h == hops - 1 ? b : -1);
    wstamp();
    ovf = phase_sync(sh, cnt);
    stamp();
    if (ovf) return false;
    // members not pulled at h have no non-zero neighbour and are no seed: exactly +0
    // (pruned last pull: a non-candidate was not pulled and keeps +0; nothing reads it)
    const uint32_t n = cnt, bit = 1u << ((uint32_t)h & 1u);
    const bool last = h == hops - 1;
    const bool prune_now = A.prune && last;
    // after the last pull, a candidate carrying the excluded label is marked NEED_EXCL for
    // top-k; its label load is issued beside the member's pull-result load
    const bool mark_excl = last && A.exclude >= 0;
    // this thread's first seed entry: its load is issued beside the copy's loads
    const uint32_t ir = sb + tid;
    const uint2 r0 = ir < se ? A.seed_rep[ir] : make_uint2(NO_NODE, 0u);
    auto copy_one = [&](uint32_t i, uint32_t p, uint8_t nd, uint8_t f, float sn, uint8_t lab) {
      const bool pulled = i < n0 && ((nd & bit) || (f & FL_SEED)) &&
                          (!prune_now || cand_depth(f, hops));
      t.sc(p) = pulled ? sn : 0.f;
      uint8_t nn = nd & ~bit;
      if (mark_excl && cand_depth(f, hops) && lab == (uint8_t)A.exclude) nn |= NEED_EXCL;
      if (nn != nd) t.need[p] = nn;
    };
      for (uint32_t i = tid; i < n; i += FT) {
        const uint32_t p = t.mlist[i];
        if (p >= t.cap) continue;
        const uint8_t f = t.fl[p];
        const uint8_t lab = (mark_excl && cand_depth(f, hops)) ? A.vlabel[t.key(p)] : 0xFF;
        copy_one(i, p, t.need[p], f, i < n0 ? t.snew[i] : 0.f, lab);
    }
    __syncthreads();
    if (r0.x != NO_NODE) t.sc(r0.x) = t.sc(r0.x) + __uint_as_float(r0.y);
    for (uint32_t i = ir + FT; i < se; i += FT) {
      const uint2 r = A.seed_rep[i];
      if (r.x != NO_NODE) t.sc(r.x) = t.sc(r.x) + __uint_as_float(r.y);
    }
    __syncthreads();
    stamp();
  }
  return finish_column<GT>(A, t, sh, b, cnt, work, slot);
}

// The LDS table of one workgroup (static shared memory of the kernel that declares it).
struct LdsTab {
  uint32_t keys[LCAP];
  float s[LCAP];
  uint32_t flw[LCAP / 4];
  uint32_t needw[LCAP / 4];
  uint16_t mlist[LLIMIT];
  uint32_t bloom[BLOOM_WORDS];
};

// The rest of a column that overflowed the LDS table, in the same workgroup: run again from its
// seeds in a global-memory table region of its own (A.cont_*: 2k-slot-bucket tables, claimed one
// per column and run from a counter zeroed with the run's counters -- a region is used by one
// workgroup per run, so no other XCD's L2 holds a stale line of it), then the region's every
// slot cleared for the next run.  The overflowing columns start early (costliest first), so
// finishing them here, while the grid runs, leaves no serial retry tail after it.  False (the
// caller hands the column on) when the regions are used up or the column overflows this table too.
// (Inlined: a noinline call measured +37 % on the whole kernel, profiles/r05_ab_continuation.txt.)
template <bool CONT>
__device__ __forceinline__ bool continue_column(const FArgs& A, int b, Shared& sh) {
  if constexpr (!CONT) {
    return false;
  } else {
    const uint32_t tid = threadIdx.x;
    __syncthreads();                         // (every wave is past the LDS attempt's sh reads)
    if (tid == 0) {
      sh.item = atomicAdd(A.cont_ctr, 1u);
      sh.count = 0;
      sh.ovf = 0;
      sh.w_pull = sh.w_expand = sh.w_rows = 0;
    }
    __syncthreads();
    const uint32_t r = sh.item;
    if (r >= A.cont_n) return false;
    // (profiling builds: slot 38 keeps the column's first stamp -- run_column restamps the
    // phases from slot 0 -- and slot 39 the continuation's start and end)
    const size_t pb = (size_t)b * PROF_SLOTS * PROF_W;
    if (FR_PROF_ON(A) && tid == 0) {
      A.prof[pb + 38 * PROF_W] = A.prof[pb];
      A.prof[pb + 39 * PROF_W] = wall_clock64();
    }
    // one allocation, region r at cont_base + r * CONT_REGION_BYTES, its arrays at fixed offsets
    // (one base register pair for all six: the continuation adds no live pointers of its own
    // to the kernel, whose register budget its LDS path shares)
    uint8_t* rb = A.cont_base + (size_t)r * CONT_REGION_BYTES;
    constexpr uint32_t cap = CONT_CAP;
    Tab<true> g{reinterpret_cast<uint32_t*>(rb), reinterpret_cast<float*>(rb + 4 * cap), rb + 8 * cap,
                rb + 9 * cap, reinterpret_cast<uint32_t*>(rb + 10 * cap),
                reinterpret_cast<float*>(rb + 10 * cap + 4 * CONT_LIMIT), cap, CONT_LIMIT, &sh.count,
                &sh.ovf, nullptr, SH_CHAIN};
    const bool ok = run_column<true>(A, g, sh, b);
    if (ok && tid == 0) atomicAdd(&A.stats[5], 1ull);
    if (FR_PROF_ON(A) && tid == 0) A.prof[pb + 39 * PROF_W + 1] = wall_clock64();
    __syncthreads();
    // every slot back to empty (an overflowed column may have inserted past its member list)
    for (uint32_t i = tid; i < cap; i += FT) {
      g.keys[i] = EMPTY;
      g.s[i] = 0.f;
      g.fl[i] = 0;
      g.need[i] = 0;
    }
    return ok;
  }
}

// One column in the LDS table: clear, run, and on overflow either continue it in a global
// region (CONT) or hand it on (A.ovf_list).  `row`: the row of A.lsnew that holds the column's
// pull results by member index.  (The row pointer is formed here, not by the caller: a pointer
// argument stays live through the column and costs the narrow kernel 20 B of scratch.)
template <bool CONT>
__device__ __forceinline__ void lds_column(const FArgs& A, int b, LdsTab& L, Shared& sh, uint32_t row) {
  const uint32_t tid = threadIdx.x;
  for (uint32_t i = tid; i < BLOOM_WORDS; i += FT) L.bloom[i] = 0;
#pragma unroll
  for (int i = 0; i < LPPT; ++i) {
    L.keys[tid + i * FT] = EMPTY;
    L.s[tid + i * FT] = 0.f;
  }
  for (uint32_t i = tid; i < LCAP / 4; i += FT) L.flw[i] = 0;
  for (uint32_t i = tid; i < LCAP / 4; i += FT) L.needw[i] = 0;
  if (tid == 0) {
    sh.count = 0;
    sh.ovf = 0;
    sh.w_pull = sh.w_expand = sh.w_rows = 0;
  }
  __syncthreads();
  Tab<false> t{L.keys, L.s, reinterpret_cast<uint8_t*>(L.flw), reinterpret_cast<uint8_t*>(L.needw),
               L.mlist, A.lsnew + (size_t)row * LLIMIT, LCAP, LLIMIT, &sh.count, &sh.ovf, L.bloom, SH_CHAIN,
               (REC && A.rec) ? A.rec + (size_t)row * REC_STRIDE : nullptr};
  if (run_column<false>(A, t, sh, b)) return;
  if (tid == 0) atomicAdd(&A.stats[4], 1ull);
  if (continue_column<CONT>(A, b, sh)) return;
  if (tid == 0) {
    const uint32_t i = atomicAdd(A.ovf_n, 1u);
    if (i < A.ovf_cap) A.ovf_list[i] = (uint32_t)b;
    else A.spill_list[atomicAdd(A.spill_n, 1u)] = (uint32_t)b;
  }
}

// The kernels this geometry launches (FR_KERNELS: 1 = frontier_lds_kernel, 2 =
// frontier_lds_retry_kernel, 4 = frontier_global_kernel).
#if FR_KERNELS & 1
// One workgroup per column, in launch order (A.order).  CONT: an overflowing column continues in
// a global-memory region (continue_column; a separate instantiation, so the plain kernel carries
// none of that code).
template <bool CONT>
__global__ __launch_bounds__(FT) __attribute__((amdgpu_waves_per_eu(FR_WAVES_PER_EU)))
void frontier_lds_kernel(const FArgs A) {
  __shared__ LdsTab L;
  __shared__ Shared sh;
  const int b = (int)A.order[blockIdx.x];
  if (b < 0 || b >= A.B) return;          // (a caller's order that is no permutation)
  if (threadIdx.x == 0 && A.seed_cnt) {   // the sort's seed counters are consumed: leave them
    A.seed_cnt[b] = 0;                      // zero for the next set_seeds
    A.seed_cnt[A.B + b] = 0;
  }
  lds_column<CONT>(A, b, L, sh, (uint32_t)b);
}
#endif

#if FR_KERNELS & 2
// Second chance: a persistent grid over the columns another geometry's LDS kernel handed on
// (A.retry_list, *A.retry_n entries), drained through a work queue; those that overflow this
// table too go on to the global-memory variant.  Every block leaves once the list is drained
// (an empty list: at once).
__global__ __launch_bounds__(FT) __attribute__((amdgpu_waves_per_eu(FR_WAVES_PER_EU)))
void frontier_lds_retry_kernel(const FArgs A) {
  __shared__ LdsTab L;
  __shared__ Shared sh;
  const uint32_t n = *A.retry_n;
  // a work queue (*A.retry_next, zeroed with the run's counters): a block takes the next entry
  // when it is free, so ~3 columns per block of uneven cost do not leave a fourth static round
  // to a few blocks
  for (;;) {
    if (threadIdx.x == 0) sh.item = atomicAdd(A.retry_next, 1u);
    __syncthreads();
    const uint32_t i = sh.item;
    if (i >= n) break;
    const uint32_t b = A.retry_list[i];
    lds_column<false>(A, (int)b, L, sh, b);
    __syncthreads();              // the next column clears the table this one used
  }
}
#endif

#if FR_KERNELS & 4
// Persistent fallback: each workgroup owns one global table and drains the overflow list.
__global__ __launch_bounds__(FT, 2) void frontier_global_kernel(const FArgs A) {
  __shared__ Shared sh;
  const uint32_t tid = threadIdx.x;
  // (every run ends with this kernel: it leaves the grouped cost histogram zero for the next)
  if (A.ghist && blockIdx.x == 0 && tid < 64) A.ghist[tid] = 0;
  const size_t cap = A.gcap;
  Tab<true> t{A.gkeys + blockIdx.x * cap, A.gs + blockIdx.x * cap, A.gfl + blockIdx.x * cap,
              A.gneed + blockIdx.x * cap, A.gmlist + (size_t)blockIdx.x * A.V,
              A.gsnew + (size_t)blockIdx.x * A.V, (uint32_t)cap, A.V, &sh.count, &sh.ovf, nullptr,
              SH_CHAIN};
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
      if (p >= cap) continue;
      t.keys[p] = EMPTY;
      t.sc(p) = 0.f;
      t.fl[p] = 0;
      t.need[p] = 0;
    }
    __syncthreads();
  }
}
#endif
#undef SH_CHAIN
#undef FR_REC
