// Geometry-independent pieces of the frontier engine (csrc/frontier.hip): the kernel argument
// block, the LDS / global hash-table hashing, top-k keys and the wave reductions.  Included once,
// inside frontier.hip's anonymous namespace, before the kernel bodies (frontier_local.h,
// frontier_body.h).
#pragma once

constexpr uint32_t EMPTY = 0xFFFFFFFFu;
constexpr uint32_t NO_NODE = EGR_NO_NODE;
constexpr int KMAXF = 16;                   // largest k
constexpr int MAX_HOPS = 60;
constexpr int PROF_SLOTS = 40;

struct alignas(8) Pair2 { uint32_t c0, v0, c1, v1; };   // two CSR entries, 8-B aligned
struct alignas(4) RowPair { uint32_t e0, e1; };           // row_ptr[v], row_ptr[v + 1]

struct FArgs {
  const uint32_t* row_ptr;
  const uint2* cv;             // (col, val bits) per CSR entry (two entries of padding past the end)
  const uint8_t* vlabel;
  uint32_t V;
  int B, hops, k, exclude;
  int prune;                   // no member pool: the last hop computes the candidates only
  const uint32_t* seed_ptr;    // [B+1] per column (clamped to n_seeds by the kernels)
  const uint32_t* seed_vert;   // grouped by column, any order, duplicates allowed
  const float* seed_val;       // (duplicates are max-combined in the kernel, as fmaxf)
  uint32_t n_seeds;
  uint2* seed_rep;             // per seed entry: (slot, s0 bits) of a vertex's representative
  const uint32_t* sources;     // [B] incident vertex per column (EGR_NO_NODE: none)
  const uint32_t* order;       // [B] launch order: work item i is column order[i]
  uint32_t* seed_cnt;          // [3B] seed counters of the sorting path, zeroed per column
                               // once consumed (nullptr: grouped seeds, nothing to zero)
  uint32_t* qhead;             // persistent grids: the work-item counter and the exit count
  uint32_t* qdone;             // (the last workgroup out resets both for the next launch)
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
  // overflow work lists
  uint32_t* ovf_list;           // where a kernel hands on its overflowing columns
  uint32_t* ovf_n;
  uint32_t* ovf_next;           // the global-memory variant's work counter (over ovf_list)
  uint32_t ovf_cap;             // ovf_list entries; further overflowing columns go to spill_*
  uint32_t* spill_list;
  uint32_t* spill_n;
  const uint32_t* retry_list;   // the wide retry's input list and count
  const uint32_t* retry_n;
  float* lsnew;                 // [B][LLIMIT] wide LDS table: pull results by member index
  uint2* lspill;                // local kernel: per-workgroup local-CSR entries past the LDS
  // global tables (one per resident workgroup of the fallback kernel)
  uint32_t* gkeys;              // [nbig][gcap]
  float* gs;                    // [nbig][gcap]
  uint8_t* gfl;                 // [nbig][gcap]
  uint8_t* gneed;               // [nbig][gcap]
  uint32_t* gmlist;             // [nbig][V]
  float* gsnew;                 // [nbig][V]
  uint32_t gcap;
  unsigned long long* prof;     // [B][PROF_SLOTS][PROF_W] wall-clock stamps per phase, or nullptr
  // [0] CSR entries gathered by pulls / local-CSR builds (col + val), [1] entries read by
  // expansions, [2] rows walked (row_ptr pairs), [3] members, [4] columns that overflowed,
  // [5] member keys outside the graph (a guard compiled in with -DEGR_FR_GUARDS; 0 otherwise)
  unsigned long long* stats;
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

__device__ __forceinline__ uint32_t bloom_hash_bits(uint32_t v, int log_bits) {
  return (mix24(v, 0xB5297Bu) >> 8) & ((1u << log_bits) - 1u);
}

__device__ __forceinline__ float readlane_f(float x, int l) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(x), l));
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

// exclusive prefix sum of x over the wave's lanes (and the wave total in every lane)
__device__ __forceinline__ uint32_t wave_excl_scan(uint32_t x, uint32_t& total) {
  const int lane = threadIdx.x & 63;
  uint32_t incl = x;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const uint32_t y = __shfl_up(incl, off, 64);
    if (lane >= off) incl += y;
  }
  total = (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
  return incl - x;
}

// Sorted per-lane candidate registers (descending) -> the wave's k best keys into out[0..k)
// (zero-filled past the wave's last candidate): k wave-wide max rounds, the winner lane shifts
// its registers.  Keys are distinct (a vertex is in one lane).
template <int MPT>
__device__ __forceinline__ void wave_topk_sorted(uint64_t (&kk)[MPT], int k, uint64_t* out) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int pass = 0; pass < MPT; ++pass)          // odd-even transposition sort, descending
#pragma unroll
    for (int j = pass & 1; j + 1 < MPT; j += 2) {
      const uint64_t x = kk[j], y = kk[j + 1];
      const bool sw = y > x;
      kk[j] = sw ? y : x;
      kk[j + 1] = sw ? x : y;
    }
  uint64_t lb = kk[0];
  for (int q = 0; q < k; ++q) {
    const uint64_t wb = wave_max_u64(lb);
    if (lane == 0) out[q] = wb;
    if (wb == 0) {                               // uniform: no candidate left in this wave
      for (int r = q + 1 + lane; r < k; r += 64) out[r] = 0;
      break;
    }
    if (lb == wb) {
#pragma unroll
      for (int j = 0; j + 1 < MPT; ++j) kk[j] = kk[j + 1];
      kk[MPT - 1] = 0;
      lb = kk[0];
    }
  }
}

// Wave 0 merges NW per-wave lists top[w][0..k) by rank (keys distinct; a list ends zero-filled)
// and writes column b's output row; slots past the candidates get EGR_NO_NODE / -inf.
template <int NW>
__device__ __forceinline__ void merge_topk(const uint64_t (*top)[KMAXF], int k, int b,
                                           uint32_t* out_ids, float* out_scores) {
  const int lane = threadIdx.x & 63;
  uint64_t c[2];
  uint32_t nnz = 0;
#pragma unroll
  for (int y = 0; y < 2; ++y) {
    const int cc = lane + 64 * y, w = cc / KMAXF, r = cc % KMAXF;
    c[y] = (w < NW && r < k) ? top[w][r] : 0ull;
    nnz += (uint32_t)__popcll(__ballot(c[y] != 0));
  }
  uint32_t rank[2] = {0u, 0u};
  for (int w = 0; w < NW; ++w)
    for (int r = 0; r < k; ++r) {
      const uint64_t o = top[w][r];
      rank[0] += o > c[0];
      rank[1] += o > c[1];
    }
#pragma unroll
  for (int y = 0; y < 2; ++y) {
    if (c[y] != 0 && rank[y] < (uint32_t)k) {
      float sc;
      uint32_t v;
      topk_unkey(c[y], sc, v);
      out_ids[(size_t)b * k + rank[y]] = v;
      out_scores[(size_t)b * k + rank[y]] = sc;
    }
  }
  for (uint32_t q = nnz + lane; q < (uint32_t)k; q += 64) {
    out_ids[(size_t)b * k + q] = NO_NODE;
    out_scores[(size_t)b * k + q] = -INFINITY;
  }
}
