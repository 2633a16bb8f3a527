// The local-subgraph frontier kernel: every top-k-only ("pruned") incident column in ONE
// workgroup, in two phases, with a persistent grid pulling columns from a device work counter.
// Included by csrc/frontier.hip (after frontier_common.h), inside namespace fr_local.
//
// Which vertices matter.  For column b with seeds S, incident vertex src and H
// hops, the dense recurrence s^{h+1} = s0 + A s^h (fmaf chain over each row in CSR order, then
// + s0) can be non-zero at hop h only within h hops of S, and top-k reads s^H on the candidate
// set C = the vertices within H hops of src.  So the column needs exactly
//   B2 = the vertices within H-1 hops of S   (every s^h, h < H, that can be non-zero)
//   C  = the vertices within H   hops of src (the candidates)
// and, per member v of M = B2 u C, the entries of v's row whose target is in B2 -- an entry to a
// vertex outside B2 multiplies an exact +0 at every hop < H, and fmaf(w, +0, acc) == acc for
// acc != -0 (acc starts at +0 and never becomes -0), so dropping it changes no bit.
// On C3 that is 600 members and 1.2k local entries per column (p99 860 / 1.75k), against 5.4k
// CSR entries the per-hop frontier walks pulled (scripts/column_shape.py).
//
// Phase A (discover), in LDS, a hash table keyed by vertex id:
//   walk 0   insert the seeds (seed distance 0) and src (reach depth 0); max-combine the seed
//            values per vertex;
//   walk k   (k = 1..H) expand the vertices first reached at level k-1 -- by reach while
//            k <= H, by seed distance while k <= H-1 -- inserting their neighbours; a vertex
//            whose level is first set in walk k is queued for walk k+1 (per-walk slot lists);
//   walk L   read the row of every member once, resolve each entry's target to its member
//            index (bloom filter, then 16-B bucket reads; no inserts run any more), keep the
//            entries into B2: the member-restricted local CSR, in CSR order per row.
// Phase B (propagate), LDS only: H hops of the recurrence over the local CSR by member index
//   (two score buffers; the last hop computes the candidates only), then top-k over C minus
//   the excluded label, ties by vertex id.  No hash probe, no atomic, no global load.
//
// Capacity: 1152 members, 128 distinct seed vertices, rows of up to 255 kept entries and
// ECAP + ESPILL local entries (the first ECAP in LDS, the rest in a per-workgroup global
// buffer).  A column past any of these is handed on (A.ovf_list) to the wide / global-memory
// kernels of frontier_body.h, which compute the same bits.
//
// LDS: 32 KB per workgroup (5 per CU, 20 waves): phase A's table and phase B's score buffers
// share one region.

constexpr int FT = 256;
constexpr int NWAVES = FT / 64;
constexpr uint32_t LCAP = 1536;            // table slots (4-slot buckets; load <= 0.75)
constexpr uint32_t LLIMIT = 1152;          // members
constexpr int BLOOM_LOG = 14;              // membership filter bits (log2)
constexpr uint32_t BLOOM_WORDS = (1u << BLOOM_LOG) / 32;
constexpr uint32_t SCAP = 128;             // members [0, SCAP) may carry a seed value
constexpr uint32_t WLCAP = 512;            // a walk list past this: the walk scans every member
constexpr uint32_t ESPILL = 4096;          // local entries past ECAP, per workgroup, in HBM
constexpr int LMAX = 12;                   // rows of up to LMAX entries run one lane per row
constexpr int LB = 4;                      // keys probed together per lane
constexpr int MAXH = 14;                   // levels are 4-bit (depth + 1)
constexpr int MPT = (LLIMIT + FT - 1) / FT;
constexpr int PROF_W = NWAVES + 1;
constexpr uint32_t CAND = 0x8000u;         // loff: the member is a top-k candidate
constexpr int WAVES_PER_EU = 5;
constexpr uint32_t LDS_BUDGET = 163840 / WAVES_PER_EU;   // 5 workgroups per CU

struct PhaseA {                // discovery: the hash table, by slot, and the member list
  uint32_t keys[LCAP];
  uint16_t mem[LCAP];          // slot -> member index
  uint8_t fl[LCAP];            // reach depth + 1 (bits 0-3) | seed distance + 1 (bits 4-7)
  uint32_t bloom[BLOOM_WORDS];
  uint16_t mlist[LLIMIT];      // member index -> slot
  uint16_t wl[2][WLCAP];       // slots to expand in the next walk (by walk parity)
};
struct PhaseB {                // propagation, by member index
  float s[2][LLIMIT];
  uint32_t vid[LLIMIT];
};
union Region {
  PhaseA a;
  PhaseB b;
};
struct Scalars {
  uint64_t top[NWAVES][KMAXF];
  uint32_t count, ecnt, ovf, item, n0;
  uint32_t nwl[2];
};
constexpr size_t FIXED = sizeof(Region) + LLIMIT * 3 + SCAP * 4 + sizeof(Scalars);
constexpr uint32_t ECAP = (uint32_t)(((LDS_BUDGET - FIXED) / 6) & ~7ull);   // LDS local entries
static_assert(ECAP + ESPILL < 32768, "loff keeps a 15-bit entry offset");

struct Lds {
  Region u;
  uint16_t loff[LLIMIT];       // local row start | CAND
  uint8_t llen[LLIMIT];        // local row length
  uint32_t s0[SCAP];           // seed values by member index (order-preserving images first)
  uint16_t eidx[ECAP];         // local entries: target member index, weight
  float ew[ECAP];
  Scalars sc;
};
static_assert(sizeof(Lds) <= LDS_BUDGET, "local frontier LDS budget");

__device__ __forceinline__ uint32_t vload(const uint32_t& x) {
  return __atomic_load_n(&x, __ATOMIC_RELAXED);
}

__device__ __forceinline__ uint32_t bloom_hash(uint32_t v) { return bloom_hash_bits(v, BLOOM_LOG); }

// slot of v, inserting it if absent (-1: table full, or the column has overflowed)
__device__ __forceinline__ int ins(Lds& L, uint32_t v) {
  constexpr uint32_t nb = LCAP / 4;
  PhaseA& a = L.u.a;
  uint32_t bk = hbucket(v, nb);
  for (uint32_t n = 0; n < nb; ++n) {
    // an overflowed column is discarded: stop at once instead of scanning a full table
    if (n > 0 && vload(L.sc.ovf)) return -1;
    const uint4 kk = reinterpret_cast<const uint4*>(a.keys)[bk];
    const uint32_t ks[4] = {kk.x, kk.y, kk.z, kk.w};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if (ks[j] == v) return (int)(4 * bk + j);
      if (ks[j] == EMPTY) {
        const uint32_t p = 4 * bk + j;
        const uint32_t old = atomicCAS(&a.keys[p], EMPTY, v);
        if (old == EMPTY) {
          const uint32_t h = bloom_hash(v);
          atomicOr(&a.bloom[h >> 5], 1u << (h & 31u));
          const uint32_t c = atomicAdd(&L.sc.count, 1u);
          if (c < LLIMIT) {
            a.mlist[c] = (uint16_t)p;
            a.mem[p] = (uint16_t)c;
          } else {
            L.sc.ovf = 1u;
          }
          return (int)p;
        }
        if (old == v) return (int)p;
      }
    }
    bk = bk + 1 == nb ? 0 : bk + 1;
  }
  L.sc.ovf = 1u;
  return -1;
}

// Lockstep probe of NQ keys (the first nq valid): the filter first, then one bucket read per
// round for every key still unresolved.  q = slot or -1.  (Exact when no insert runs
// concurrently; during a walk that inserts, a miss is re-checked by ins().)
template <int NQ>
__device__ __forceinline__ void find_batch(const Lds& L, const uint32_t (&key)[NQ], uint32_t nq,
                                           int (&q)[NQ]) {
  constexpr uint32_t nb = LCAP / 4;
  const PhaseA& a = L.u.a;
  uint32_t bk[NQ], pend = 0;
#pragma unroll
  for (int x = 0; x < NQ; ++x) {
    q[x] = -1;
    bk[x] = hbucket(key[x], nb);
    if ((uint32_t)x < nq) pend |= 1u << x;
  }
  uint32_t bw[NQ];
#pragma unroll
  for (int x = 0; x < NQ; ++x) bw[x] = (pend & (1u << x)) ? a.bloom[bloom_hash(key[x]) >> 5] : ~0u;
#pragma unroll
  for (int x = 0; x < NQ; ++x)
    if (!((bw[x] >> (bloom_hash(key[x]) & 31u)) & 1u)) pend &= ~(1u << x);
  for (uint32_t n = 0; n < nb && __any(pend != 0); ++n) {
    uint4 kk[NQ];
#pragma unroll
    for (int x = 0; x < NQ; ++x)
      if (pend & (1u << x)) kk[x] = reinterpret_cast<const uint4*>(a.keys)[bk[x]];
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

// Set the level nibble (shift 0: reach, 4: seeds) of slot q to val if it is unset; true if
// this call set it.  Every writer of a nibble within one walk writes the same value.
__device__ __forceinline__ bool set_level(Lds& L, uint32_t q, uint32_t shift, uint32_t val) {
  uint8_t* fl = L.u.a.fl;
  if ((fl[q] >> shift) & 0xFu) return false;
  const uint32_t sh = (q & 3u) * 8u + shift;
  const uint32_t old = atomicOr(reinterpret_cast<uint32_t*>(fl) + (q >> 2), val << sh);
  return ((old >> sh) & 0xFu) == 0u;
}

__device__ __forceinline__ void wl_push(Lds& L, int list, uint32_t q) {
  const uint32_t j = atomicAdd(&L.sc.nwl[list], 1u);
  if (j < WLCAP) L.u.a.wl[list][j] = (uint16_t)q;
}

// One neighbour u of a row expanded in walk k (er: by reach, es: by seed distance); q = its
// slot if a probe found it
__device__ __forceinline__ void expand_entry(Lds& L, uint32_t u, int q, bool er, bool es, int k,
                                             int H) {
  if (q < 0) q = ins(L, u);
  if (q < 0) return;
  bool push = false;
  if (er && set_level(L, (uint32_t)q, 0, (uint32_t)k + 1) && k + 1 <= H) push = true;
  if (es && set_level(L, (uint32_t)q, 4, (uint32_t)k + 1) && k + 1 <= H - 1) push = true;
  if (push) wl_push(L, (k + 1) & 1, (uint32_t)q);
}

struct Counters {
  uint32_t pull = 0, expand = 0, rows = 0, members = 0;
};

// Phase boundary: a barrier, then the member count and the overflow flag every thread sees
// (and the walk list just consumed emptied), then a second barrier -- reading them after one
// barrier would race with the next phase's inserts and pushes by faster waves.
__device__ __forceinline__ bool phase_sync(Lds& L, uint32_t& cnt, int reset_list) {
  __syncthreads();
  cnt = L.sc.count;
  const bool ovf = L.sc.ovf != 0;
  if (reset_list >= 0 && threadIdx.x == 0) L.sc.nwl[reset_list] = 0;
  __syncthreads();
  return ovf;
}

// Expansion walk k over its list (or, when the list overflowed, over every member)
__device__ __forceinline__ void expand_walk(const FArgs& A, Lds& L, int k, int H, uint32_t n, Counters& ct) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const uint32_t nl_raw = L.sc.nwl[k & 1];
  const bool scan = nl_raw > WLCAP;
  const uint32_t nl = scan ? n : nl_raw;
  const uint32_t nch = (nl + FT - 1) / FT;
  for (uint32_t c = 0; c < nch; ++c) {
    if (vload(L.sc.ovf)) break;
    const uint32_t j = wave + NWAVES * (lane + 64u * c);
    bool er = false, es = false;
    uint32_t e0 = 0, deg = 0;
    if (j < nl) {
      const uint32_t p = scan ? L.u.a.mlist[j] : L.u.a.wl[k & 1][j];
      const uint32_t f = L.u.a.fl[p];
      er = (f & 0xFu) == (uint32_t)k && k <= H;
      es = (f >> 4) == (uint32_t)k && k <= H - 1;
      if (er || es) {
        const RowPair rp = *reinterpret_cast<const RowPair*>(A.row_ptr + L.u.a.keys[p]);
        e0 = rp.e0;
        deg = rp.e1 - rp.e0;
        ++ct.rows;
        ct.expand += deg;
      }
    }
    const bool light = (er || es) && deg <= (uint32_t)LMAX;
    // light rows: every entry in one round trip, probed LB at a time, absent ones inserted
    uint32_t col[LMAX];
#pragma unroll
    for (int x = 0; x < LMAX; x += 2) {
      Pair2 ce = {0u, 0u, 0u, 0u};
      if (light && (uint32_t)x < deg) ce = *reinterpret_cast<const Pair2*>(A.cv + e0 + x);
      col[x] = ce.c0;
      col[x + 1] = ce.c1;
    }
    // (one entry per iteration, the row's registers shifted down: a single copy of the insert
    // path in the code -- expansion rows are few, ~85 per C3 column)
    const uint32_t ld = light ? deg : 0u;
#pragma unroll 1
    for (uint32_t x = 0; __any(ld > x); ++x) {
      const uint32_t u = col[0];
#pragma unroll
      for (int y = 0; y + 1 < LMAX; ++y) col[y] = col[y + 1];
      uint32_t key[1] = {u};
      int q[1];
      find_batch<1>(L, key, ld > x ? 1u : 0u, q);
      if (ld > x) expand_entry(L, u, q[0], er, es, k, H);
    }
    // hub rows: one at a time across the wave, 64 entries per round
    uint64_t heavy = __ballot((er || es) && deg > (uint32_t)LMAX);
    while (heavy) {
      const int m = __ffsll((long long)heavy) - 1;
      heavy &= heavy - 1;
      const uint32_t he0 = __builtin_amdgcn_readlane(e0, m);
      const uint32_t hdeg = __builtin_amdgcn_readlane(deg, m);
      const bool her = __builtin_amdgcn_readlane((int)er, m) != 0;
      const bool hes = __builtin_amdgcn_readlane((int)es, m) != 0;
      for (uint32_t base = 0; base < hdeg; base += 64) {
        const uint32_t jj = base + lane;
        const bool act = jj < hdeg;
        const uint32_t u = act ? A.cv[he0 + jj].x : 0u;
        uint32_t key[1] = {u};
        int q[1];
        find_batch<1>(L, key, act ? 1u : 0u, q);
        if (act) expand_entry(L, u, q[0], her, hes, k, H);
      }
    }
  }
}

// The local CSR: every member's row once, its entries into B2 kept (target member index,
// weight) in CSR order.  Also marks the candidates (reach depth <= H, label not excluded).
__device__ __forceinline__ void local_walk(const FArgs& A, Lds& L, int H, uint32_t n, Counters& ct,
                           uint2* spill) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const uint32_t nch = (n + FT - 1) / FT;
  struct Mem {
    uint32_t i, e0, deg;
    bool ok, cand;
  };
  auto fetch = [&](uint32_t c) {
    Mem m{wave + NWAVES * (lane + 64u * c), 0u, 0u, false, false};
    if (c < nch && m.i < n) {
      m.ok = true;
      const uint32_t p = L.u.a.mlist[m.i];
      const uint32_t v = L.u.a.keys[p];
      const uint32_t rd = L.u.a.fl[p] & 0xFu;
      m.cand = rd >= 1 && rd <= (uint32_t)H + 1;
      const RowPair rp = *reinterpret_cast<const RowPair*>(A.row_ptr + v);
      if (m.cand && A.exclude >= 0) m.cand = (int)A.vlabel[v] != A.exclude;
      m.e0 = rp.e0;
      m.deg = rp.e1 - rp.e0;
    }
    return m;
  };
  auto put = [&](uint32_t e, uint32_t idx, float w) {
    if (e < ECAP) {
      L.eidx[e] = (uint16_t)idx;
      L.ew[e] = w;
    } else if (e < ECAP + ESPILL) {
      spill[e - ECAP] = make_uint2(idx, __float_as_uint(w));
    }
  };
  Mem nxt = fetch(0);
  for (uint32_t c = 0; c < nch; ++c) {
    const Mem cur = nxt;
    nxt = fetch(c + 1);
    if (cur.ok) {
      ++ct.rows;
      ct.pull += cur.deg;
    }
    const bool light = cur.ok && cur.deg <= (uint32_t)LMAX;
    uint32_t col[LMAX];
    float w[LMAX];
#pragma unroll
    for (int x = 0; x < LMAX; x += 2) {
      Pair2 ce = {0u, 0u, 0u, 0u};
      if (light && (uint32_t)x < cur.deg) ce = *reinterpret_cast<const Pair2*>(A.cv + cur.e0 + x);
      col[x] = ce.c0;
      w[x] = __uint_as_float(ce.v0);
      col[x + 1] = ce.c1;
      w[x + 1] = __uint_as_float(ce.v1);
    }
    uint32_t kmask = 0;
    uint16_t kix[LMAX];
#pragma unroll
    for (int sb = 0; sb < LMAX / LB; ++sb) {
      const uint32_t ld = light ? cur.deg : 0u;
      if (!__any(ld > (uint32_t)(sb * LB))) continue;
      const uint32_t nq = ld > (uint32_t)(sb * LB) ? min(ld - sb * LB, (uint32_t)LB) : 0u;
      uint32_t key[LB];
#pragma unroll
      for (int x = 0; x < LB; ++x) key[x] = col[sb * LB + x];
      int q[LB];
      find_batch<LB>(L, key, nq, q);
#pragma unroll
      for (int x = 0; x < LB; ++x) {
        kix[sb * LB + x] = 0;
        if (q[x] >= 0 && (L.u.a.fl[q[x]] >> 4) != 0u) {
          kmask |= 1u << (sb * LB + x);
          kix[sb * LB + x] = L.u.a.mem[q[x]];
        }
      }
    }
    // light rows: one allocation per wave (exclusive scan of the kept counts)
    uint32_t tot;
    const uint32_t mine = wave_excl_scan((uint32_t)__popc(kmask), tot);
    uint32_t o = 0;
    if (tot) {
      if (lane == 0) o = atomicAdd(&L.sc.ecnt, tot);
      o = (uint32_t)__builtin_amdgcn_readfirstlane((int)o);
    }
    if (light) {
      const uint32_t r0 = o + mine;
#pragma unroll
      for (int x = 0; x < LMAX; ++x)
        if (kmask & (1u << x)) put(r0 + (uint32_t)__popc(kmask & ((1u << x) - 1u)), kix[x], w[x]);
      L.loff[cur.i] = (uint16_t)(min(r0, 0x7FFFu) | (cur.cand ? CAND : 0u));
      L.llen[cur.i] = (uint8_t)__popc(kmask);
    }
    // hub rows: one at a time across the wave; space for the whole row is taken up front,
    // the kept entries are compacted in CSR (= lane) order
    uint64_t heavy = __ballot(cur.ok && cur.deg > (uint32_t)LMAX);
    while (heavy) {
      const int m = __ffsll((long long)heavy) - 1;
      heavy &= heavy - 1;
      const uint32_t he0 = __builtin_amdgcn_readlane(cur.e0, m);
      const uint32_t hdeg = __builtin_amdgcn_readlane(cur.deg, m);
      uint32_t ho = 0;
      if (lane == 0) ho = atomicAdd(&L.sc.ecnt, hdeg);
      ho = (uint32_t)__builtin_amdgcn_readfirstlane((int)ho);
      uint32_t kept = 0;
      for (uint32_t base = 0; base < hdeg; base += 64) {
        const uint32_t jj = base + lane;
        const bool act = jj < hdeg;
        const uint2 ce = act ? A.cv[he0 + jj] : make_uint2(0u, 0u);
        uint32_t key[1] = {ce.x};
        int q[1];
        find_batch<1>(L, key, act ? 1u : 0u, q);
        const bool keep = q[0] >= 0 && (L.u.a.fl[q[0]] >> 4) != 0u;
        const uint64_t bal = __ballot(keep);
        if (keep) {
          const uint32_t r = __builtin_amdgcn_mbcnt_hi((uint32_t)(bal >> 32),
                                                       __builtin_amdgcn_mbcnt_lo((uint32_t)bal, 0u));
          put(ho + kept + r, L.u.a.mem[q[0]], __uint_as_float(ce.y));
        }
        kept += (uint32_t)__popcll(bal);
      }
      if (lane == m) {
        L.loff[cur.i] = (uint16_t)(min(ho, 0x7FFFu) | (cur.cand ? CAND : 0u));
        L.llen[cur.i] = (uint8_t)min(kept, 255u);
        if (kept > 255u) L.sc.ovf = 1u;       // a row longer than llen holds: hand the column on
      }
    }
  }
}

__device__ __forceinline__ void entry(const Lds& L, const uint2* spill, uint32_t e, uint32_t& idx,
                                      float& w) {
  if (e < ECAP) {
    idx = L.eidx[e];
    w = L.ew[e];
  } else {
    const uint2 x = spill[e - ECAP];
    idx = x.x;
    w = __uint_as_float(x.y);
  }
}

// Phase B: H hops over the local CSR, then top-k.  s^0 = the seed values (members [0, n0)).
__device__ __forceinline__ void propagate_topk(const FArgs& A, Lds& L, int b, int H, uint32_t n, uint32_t n0,
                               const uint2* spill) {
  const uint32_t tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const float* s0 = reinterpret_cast<const float*>(L.s0);
  for (int h = 0; h < H; ++h) {
    const float* cur = L.u.b.s[h & 1];
    float* nxt = L.u.b.s[(h + 1) & 1];
    const bool last = h == H - 1;
#pragma unroll
    for (int j = 0; j < MPT; ++j) {
      const uint32_t i = tid + j * FT;
      if (i >= n) break;
      const uint32_t o16 = L.loff[i];
      if (last && !(o16 & CAND)) continue;           // pruned: never read
      const uint32_t o = o16 & 0x7FFFu, end = o + L.llen[i];
      float acc = 0.f;
      uint32_t e = o;
      for (; e + 4 <= end; e += 4) {                 // four entries' loads in flight
        uint32_t ix[4];
        float w[4], x[4];
#pragma unroll
        for (int y = 0; y < 4; ++y) entry(L, spill, e + y, ix[y], w[y]);
#pragma unroll
        for (int y = 0; y < 4; ++y) x[y] = cur[ix[y]];
#pragma unroll
        for (int y = 0; y < 4; ++y) acc = fmaf(w[y], x[y], acc);
      }
      for (; e < end; ++e) {
        uint32_t ix;
        float w;
        entry(L, spill, e, ix, w);
        acc = fmaf(w, cur[ix], acc);
      }
      // (+ s0 for the members that can carry a seed; a non-seed's s0 is +0 and acc + +0 == acc)
      nxt[i] = i < n0 ? acc + s0[i] : acc;
    }
    __syncthreads();
    if (A.prof && tid == 0) A.prof[((size_t)b * PROF_SLOTS + 3 + H + h) * PROF_W] = wall_clock64();
  }
  const float* fin = L.u.b.s[H & 1];
  uint64_t kk[MPT];
#pragma unroll
  for (int j = 0; j < MPT; ++j) {
    const uint32_t i = tid + j * FT;
    kk[j] = (i < n && (L.loff[i] & CAND)) ? topk_key(fin[i], L.u.b.vid[i]) : 0ull;
  }
  wave_topk_sorted<MPT>(kk, A.k, L.sc.top[wave]);
  __syncthreads();
  if (wave == 0) merge_topk<NWAVES>(L.sc.top, A.k, b, A.out_ids, A.out_scores);
  (void)lane;
}

// One column end to end; false (uniformly) when it has to be handed on.
__device__ __forceinline__ bool column(const FArgs& A, Lds& L, int b, Counters& ct, uint2* spill) {
  const uint32_t tid = threadIdx.x;
  const int H = A.hops;
  auto stamp = [&](int slot) {
    if (A.prof && tid == 0) A.prof[((size_t)b * PROF_SLOTS + slot) * PROF_W] = wall_clock64();
  };
  stamp(0);
  // walk 0: clear, then the seeds and the incident vertex
  PhaseA& a = L.u.a;
#pragma unroll
  for (uint32_t i = tid; i < LCAP; i += FT) a.keys[i] = EMPTY;
  for (uint32_t i = tid; i < LCAP / 4; i += FT) reinterpret_cast<uint32_t*>(a.fl)[i] = 0u;
  for (uint32_t i = tid; i < BLOOM_WORDS; i += FT) a.bloom[i] = 0u;
  if (tid < SCAP) L.s0[tid] = 0u;
  if (tid == 0) {
    L.sc.count = 0;
    L.sc.ecnt = 0;
    L.sc.ovf = 0;
    L.sc.nwl[0] = L.sc.nwl[1] = 0;
  }
  const uint32_t src = A.sources[b];
  const bool src_ok = src < A.V;
  const uint32_t ns = A.n_seeds;
  const uint32_t sb = min(A.seed_ptr[b], ns), se = max(sb, min(A.seed_ptr[b + 1], ns));
  __syncthreads();
  if (H > MAXH) {
    if (tid == 0) L.sc.ovf = 1u;
  } else {
    for (uint32_t i = sb + tid; i < se; i += FT) {
      const uint32_t v = A.seed_vert[i];
      if (v >= A.V) continue;
      const int q = ins(L, v);
      if (q >= 0 && set_level(L, (uint32_t)q, 4, 1u) && 1 <= H - 1) wl_push(L, 1, (uint32_t)q);
    }
    if (tid == 0 && src_ok) {
      const int q = ins(L, src);
      if (q >= 0 && set_level(L, (uint32_t)q, 0, 1u)) wl_push(L, 1, (uint32_t)q);
    }
  }
  uint32_t n;
  if (phase_sync(L, n, -1) || n > SCAP) return false;
  // the seed values: max-combined on order-preserving u32 images (fmaxf, like the dense plan's
  // seed prep); a member without a seed keeps image 0 -> +0
  auto ord = [](float f) {
    const uint32_t u = __float_as_uint(f);
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
  };
  for (uint32_t i = sb + tid; i < se; i += FT) {
    const uint32_t v = A.seed_vert[i];
    if (v >= A.V) continue;
    uint32_t key[1] = {v};
    int q[1];
    find_batch<1>(L, key, 1u, q);
    if (q[0] >= 0) atomicMax(&L.s0[a.mem[q[0]]], ord(A.seed_val[i]));
  }
  __syncthreads();
  const uint32_t n0 = n;
  if (tid < n0) {
    const uint32_t o = L.s0[tid];
    L.s0[tid] = o == 0u ? 0u : ((o & 0x80000000u) ? (o & 0x7FFFFFFFu) : ~o);
  }
  stamp(1);
  // walks 1..H: expansions
  for (int k = 1; k <= H; ++k) {
    expand_walk(A, L, k, H, n, ct);
    if (phase_sync(L, n, k & 1)) return false;
    stamp(1 + k);
  }
  // walk L: the local CSR
  local_walk(A, L, H, n, ct, spill);
  uint32_t n2;
  if (phase_sync(L, n2, -1) || L.sc.ecnt > ECAP + ESPILL) return false;
  stamp(2 + H);
  ct.members += tid == 0 ? n : 0u;
  // phase B: member vertex ids and s^0 into the region the table used
  uint32_t vr[MPT];
#pragma unroll
  for (int j = 0; j < MPT; ++j) {
    const uint32_t i = tid + j * FT;
    vr[j] = i < n ? a.keys[a.mlist[i]] : 0u;
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < MPT; ++j) {
    const uint32_t i = tid + j * FT;
    if (i < n) {
      L.u.b.vid[i] = vr[j];
      L.u.b.s[0][i] = i < n0 ? reinterpret_cast<const float*>(L.s0)[i] : 0.f;
    }
  }
  __syncthreads();
  if (A.prof && tid == 0) {
    A.prof[((size_t)b * PROF_SLOTS + 30) * PROF_W] = L.sc.ecnt;
    A.prof[((size_t)b * PROF_SLOTS + 31) * PROF_W] = n;
  }
  propagate_topk(A, L, b, H, n, n0, spill);
  stamp(3 + 2 * H);
  return true;
}

__global__ __launch_bounds__(FT) __attribute__((amdgpu_waves_per_eu(WAVES_PER_EU)))
void frontier_local_kernel(const FArgs A) {
  __shared__ Lds L;
  uint2* const spill = A.lspill + (size_t)blockIdx.x * ESPILL;
  Counters ct;
  for (;;) {
    if (threadIdx.x == 0) L.sc.item = atomicAdd(A.qhead, 1u);
    __syncthreads();
    const uint32_t item = L.sc.item;
    if (item >= (uint32_t)A.B) break;
    const int b = (int)A.order[item];
    if (threadIdx.x == 0 && A.seed_cnt) {    // the sorting path's counters: consumed
      A.seed_cnt[b] = 0;
      A.seed_cnt[A.B + b] = 0;
    }
    if (!column(A, L, b, ct, spill) && threadIdx.x == 0) {
      const uint32_t i = atomicAdd(A.ovf_n, 1u);
      if (i < A.ovf_cap) A.ovf_list[i] = (uint32_t)b;
      else A.spill_list[atomicAdd(A.spill_n, 1u)] = (uint32_t)b;
      atomicAdd(&A.stats[4], 1ull);
    }
    __syncthreads();          // the next column clears what this one used
  }
  // work counters: one global atomic per wave and counter for the whole launch
  uint32_t c4[4] = {ct.pull, ct.expand, ct.rows, ct.members};
#pragma unroll
  for (int x = 0; x < 4; ++x)
    for (int o = 32; o > 0; o >>= 1) c4[x] += __shfl_xor(c4[x], o);
  if ((threadIdx.x & 63) == 0) {
#pragma unroll
    for (int x = 0; x < 4; ++x)
      if (c4[x]) atomicAdd(&A.stats[x], (unsigned long long)c4[x]);
  }
  // the last workgroup out resets the work counter for the next launch (stream order)
  if (threadIdx.x == 0 && atomicAdd(A.qdone, 1u) == gridDim.x - 1) {
    *A.qhead = 0u;
    *A.qdone = 0u;
  }
}
