// Alert-storm front end (BASELINE config C5): alert fingerprints and the
// TTL deduplication table, batched on the GPU.
//
// Reference:
//   src/services/ingestion/normalizer.py:208-218  AlertNormalizer._generate_fingerprint
//       key = f"{source}:{alertname}:{namespace}:{service}"; sha256(key).hexdigest()[:32]
//       -> the fingerprint is the first 16 bytes of the digest (32 lowercase hex chars).
//   src/services/ingestion/deduplicator.py:41-140  AlertDeduplicator (Redis, key
//       "aiops:fingerprint:<fp>" -> incident id, EX = FINGERPRINT_TTL = 4 h):
//       check_duplicate (:41-71) = GET, register_fingerprint (:73-104) = SET EX (overwrites),
//       remove_fingerprint (:106-118) = DEL, extend_fingerprint (:120-140) = EXPIRE if EXISTS.
//   src/services/ingestion/main.py:141-170 (webhook loop): per firing alert, in payload order:
//       normalize -> check_duplicate -> duplicate: skip; else create_incident, which registers
//       the fingerprint (:392) -- so a later alert of the same fingerprint in the SAME payload
//       is a duplicate of the incident the first one opened.
//
// Device layout.  Fingerprints are 16-byte digests (uint4).  The table is open addressing with
// linear probing over `cap` (power of two) slots, structure of arrays:
//   state u32 (0 empty, 1 being written, 2 published), key uint4, expiry i64 (ms; a key is
//   live while now < expiry -- Redis EX semantics), incident u32, claim u64.
// Slots are never freed in place (DEL / expiry leave the key with expiry 0, so probe chains stay
// intact); egr_dedup_compact rebuilds the table from the live entries.
#include <hipcub/hipcub.hpp>

#include "graph_dev.h"

namespace {

using egr::DeviceGuard;
using egr::dalloc;
using egr::dfree;

// ---------------------------------------------------------------------------------------------
// SHA-256 (FIPS 180-4), one thread per message.  Messages are short (alert keys, ~20-80 B);
// the block loop handles any length.
// ---------------------------------------------------------------------------------------------
__constant__ uint32_t K256[64] = {
    0x428a2f98u, 0x71374491u, 0xb5c0fbcfu, 0xe9b5dba5u, 0x3956c25bu, 0x59f111f1u, 0x923f82a4u,
    0xab1c5ed5u, 0xd807aa98u, 0x12835b01u, 0x243185beu, 0x550c7dc3u, 0x72be5d74u, 0x80deb1feu,
    0x9bdc06a7u, 0xc19bf174u, 0xe49b69c1u, 0xefbe4786u, 0x0fc19dc6u, 0x240ca1ccu, 0x2de92c6fu,
    0x4a7484aau, 0x5cb0a9dcu, 0x76f988dau, 0x983e5152u, 0xa831c66du, 0xb00327c8u, 0xbf597fc7u,
    0xc6e00bf3u, 0xd5a79147u, 0x06ca6351u, 0x14292967u, 0x27b70a85u, 0x2e1b2138u, 0x4d2c6dfcu,
    0x53380d13u, 0x650a7354u, 0x766a0abbu, 0x81c2c92eu, 0x92722c85u, 0xa2bfe8a1u, 0xa81a664bu,
    0xc24b8b70u, 0xc76c51a3u, 0xd192e819u, 0xd6990624u, 0xf40e3585u, 0x106aa070u, 0x19a4c116u,
    0x1e376c08u, 0x2748774cu, 0x34b0bcb5u, 0x391c0cb3u, 0x4ed8aa4au, 0x5b9cca4fu, 0x682e6ff3u,
    0x748f82eeu, 0x78a5636fu, 0x84c87814u, 0x8cc70208u, 0x90befffau, 0xa4506cebu, 0xbef9a3f7u,
    0xc67178f2u};

__device__ __forceinline__ uint32_t rotr(uint32_t x, int n) { return __builtin_rotateright32(x, n); }

__device__ __forceinline__ void sha256_block(uint32_t h[8], uint32_t w[16]) {
  uint32_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], hh = h[7];
#pragma unroll
  for (int t = 0; t < 64; ++t) {
    uint32_t wt;
    if (t < 16) {
      wt = w[t];
    } else {
      const uint32_t w15 = w[(t + 1) & 15], w2 = w[(t + 14) & 15];
      const uint32_t s0 = rotr(w15, 7) ^ rotr(w15, 18) ^ (w15 >> 3);
      const uint32_t s1 = rotr(w2, 17) ^ rotr(w2, 19) ^ (w2 >> 10);
      wt = w[t & 15] + s0 + w[(t + 9) & 15] + s1;
      w[t & 15] = wt;
    }
    const uint32_t S1 = rotr(e, 6) ^ rotr(e, 11) ^ rotr(e, 25);
    const uint32_t ch = (e & f) ^ (~e & g);
    const uint32_t t1 = hh + S1 + ch + K256[t] + wt;
    const uint32_t S0 = rotr(a, 2) ^ rotr(a, 13) ^ rotr(a, 22);
    const uint32_t maj = (a & b) ^ (a & c) ^ (b & c);
    const uint32_t t2 = S0 + maj;
    hh = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
  }
  h[0] += a; h[1] += b; h[2] += c; h[3] += d; h[4] += e; h[5] += f; h[6] += g; h[7] += hh;
}

__global__ void __launch_bounds__(256) fingerprint_kernel(const uint8_t* __restrict__ blob,
                                                          const int64_t* __restrict__ off,
                                                          int64_t n, uint4* __restrict__ out,
                                                          char* __restrict__ hex) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int64_t beg = off[i], len = off[i + 1] - beg;
  const uint8_t* m = blob + beg;
  uint32_t h[8] = {0x6a09e667u, 0xbb67ae85u, 0x3c6ef372u, 0xa54ff53au,
                   0x510e527fu, 0x9b05688cu, 0x1f83d9abu, 0x5be0cd19u};
  // padded length: len + 1 (0x80) + 8 (bit length), rounded up to 64
  const int64_t nblk = (len + 9 + 63) / 64;
  const uint64_t bits = (uint64_t)len * 8u;
  for (int64_t blk = 0; blk < nblk; ++blk) {
    uint32_t w[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      uint32_t word = 0;
#pragma unroll
      for (int b = 0; b < 4; ++b) {
        const int64_t p = blk * 64 + j * 4 + b;
        uint32_t byte;
        if (p < len) byte = m[p];
        else if (p == len) byte = 0x80u;
        else byte = 0u;
        word = word << 8 | byte;
      }
      w[j] = word;
    }
    if (blk == nblk - 1) {  // the last block ends with the big-endian bit length
      w[14] = (uint32_t)(bits >> 32);
      w[15] = (uint32_t)bits;
    }
    sha256_block(h, w);
  }
  // digest bytes 0..15 = big-endian h[0..3]; stored as raw bytes (uint4 of byte-swapped words)
  uint4 d;
  d.x = __builtin_bswap32(h[0]);
  d.y = __builtin_bswap32(h[1]);
  d.z = __builtin_bswap32(h[2]);
  d.w = __builtin_bswap32(h[3]);
  out[i] = d;
  if (hex) {
    const char* digits = "0123456789abcdef";
    char* o = hex + i * 32;
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int b = 0; b < 8; ++b) o[j * 8 + b] = digits[(h[j] >> (28 - 4 * b)) & 15u];
  }
}

// ---------------------------------------------------------------------------------------------
// Dedup table
// ---------------------------------------------------------------------------------------------
constexpr uint32_t ST_EMPTY = 0, ST_BUSY = 1, ST_READY = 2;

struct Table {
  uint32_t* state;
  uint4* key;
  int64_t* expiry;
  uint32_t* incident;
  unsigned long long* claim;
  uint32_t cap;   // power of two
};

__device__ __forceinline__ bool key_eq(uint4 a, uint4 b) {
  return a.x == b.x && a.y == b.y && a.z == b.z && a.w == b.w;
}

__device__ __forceinline__ uint32_t slot_of(uint4 k, uint32_t cap) {
  // the key is a SHA-256 prefix: its words are already uniform
  return (k.x ^ (k.y * 0x9E3779B1u)) & (cap - 1u);
}

// Find the slot holding `k`; insert it when `insert`.  Returns the slot, or 0xFFFFFFFF (absent /
// table full).  `*fresh` = the key was inserted by this call.  A claimer publishes (key, then
// state READY) in the same loop iteration, so lanes spinning on BUSY never wait on a lane of
// their own wave that has not run yet.
__device__ uint32_t find_slot(const Table& t, uint4 k, bool insert, bool* fresh) {
  uint32_t s = slot_of(k, t.cap);
  *fresh = false;
  for (uint32_t probes = 0; probes < t.cap;) {
    const uint32_t st = __hip_atomic_load(&t.state[s], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
    if (st == ST_READY) {
      if (key_eq(t.key[s], k)) return s;
      s = (s + 1) & (t.cap - 1u);
      ++probes;
      continue;
    }
    if (st == ST_BUSY) continue;  // being published: read again
    if (!insert) return 0xFFFFFFFFu;
    uint32_t expect = ST_EMPTY;
    if (__hip_atomic_compare_exchange_strong(&t.state[s], &expect, ST_BUSY, __ATOMIC_ACQ_REL,
                                             __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT)) {
      t.key[s] = k;
      t.expiry[s] = 0;
      t.incident[s] = EGR_NO_NODE;
      __hip_atomic_store(&t.state[s], ST_READY, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
      *fresh = true;
      return s;
    }
    // lost the race for this slot: look at it again
  }
  return 0xFFFFFFFFu;
}

// Ingest pass 1: find-or-insert every fingerprint, note whether its entry was live before this
// batch (expiry is only written in pass 2) and claim the slot for the batch's first alert of
// that fingerprint: claim = (~seq << 32 | i), atomicMin -- a newer batch (larger seq) always
// undercuts an older claim, and within the batch the smallest alert index wins.
__global__ void __launch_bounds__(256) ingest_probe_kernel(Table t, const uint4* __restrict__ fp,
                                                           int64_t n, int64_t now, uint32_t seq,
                                                           uint32_t* __restrict__ slot,
                                                           uint32_t* __restrict__ prior,
                                                           uint32_t* __restrict__ n_full) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  bool fresh;
  const uint32_t s = find_slot(t, fp[i], true, &fresh);
  slot[i] = s;
  if (s == 0xFFFFFFFFu) {
    atomicAdd(n_full, 1u);
    prior[i] = EGR_NO_NODE;
    return;
  }
  const bool live = !fresh && t.expiry[s] > now;
  prior[i] = live ? t.incident[s] : EGR_NO_NODE;
  if (!live)
    atomicMin(&t.claim[s], (unsigned long long)(~seq) << 32 | (unsigned long long)(uint32_t)i);
}

// pass 2: is_new[i] = 1 for the first alert of a non-live fingerprint
__global__ void __launch_bounds__(256) ingest_first_kernel(Table t, const uint32_t* __restrict__ slot,
                                                           const uint32_t* __restrict__ prior,
                                                           int64_t n, uint32_t* __restrict__ is_new) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t s = slot[i];
  is_new[i] = (s != 0xFFFFFFFFu && prior[i] == EGR_NO_NODE &&
               (uint32_t)(t.claim[s] & 0xFFFFFFFFull) == (uint32_t)i) ? 1u : 0u;
}

// pass 3 (after the exclusive scan of is_new into rank): register the new incidents and
// resolve every alert's incident
__global__ void __launch_bounds__(256) ingest_resolve_kernel(
    Table t, const uint32_t* __restrict__ slot, const uint32_t* __restrict__ prior,
    const uint32_t* __restrict__ is_new, const uint32_t* __restrict__ rank, int64_t n,
    int64_t expiry, uint32_t first_id, uint8_t* __restrict__ out_dup,
    uint32_t* __restrict__ out_incident, uint32_t* __restrict__ n_new) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t s = slot[i];
  if (i == n - 1) *n_new = rank[i] + is_new[i];
  if (s == 0xFFFFFFFFu) {          // table full: fail open like the reference (not a duplicate)
    out_dup[i] = 0;
    out_incident[i] = EGR_NO_NODE;
    return;
  }
  if (prior[i] != EGR_NO_NODE) {   // live before the batch
    out_dup[i] = 1;
    out_incident[i] = prior[i];
    return;
  }
  const uint32_t first = (uint32_t)(t.claim[s] & 0xFFFFFFFFull);
  const uint32_t id = first_id + rank[first];
  if (is_new[i]) {
    t.incident[s] = id;
    t.expiry[s] = expiry;
    out_dup[i] = 0;
  } else {
    out_dup[i] = 1;
  }
  out_incident[i] = id;
}

__global__ void __launch_bounds__(256) lookup_kernel(Table t, const uint4* __restrict__ fp, int64_t n,
                                                     int64_t now, uint8_t* __restrict__ out_dup,
                                                     uint32_t* __restrict__ out_incident) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  bool fresh;
  const uint32_t s = find_slot(t, fp[i], false, &fresh);
  const bool live = s != 0xFFFFFFFFu && t.expiry[s] > now;
  out_dup[i] = live ? 1 : 0;
  out_incident[i] = live ? t.incident[s] : EGR_NO_NODE;
}

// SET key value EX ttl for n keys (in order: the last write of a repeated key wins)
__global__ void __launch_bounds__(256) register_kernel(Table t, const uint4* __restrict__ fp, int64_t n,
                                                       uint32_t* __restrict__ slot,
                                                       uint32_t* __restrict__ n_full) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  bool fresh;
  const uint32_t s = find_slot(t, fp[i], true, &fresh);
  slot[i] = s;
  if (s == 0xFFFFFFFFu) atomicAdd(n_full, 1u);
}

// the winner of each slot = the largest index among the batch's keys that map to it
__global__ void __launch_bounds__(256) register_last_kernel(Table t, const uint32_t* __restrict__ slot,
                                                            int64_t n, uint32_t seq) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n || slot[i] == 0xFFFFFFFFu) return;
  // smallest claim = newest batch, largest index: (~seq << 32 | ~i)
  atomicMin(&t.claim[slot[i]], (unsigned long long)(~seq) << 32 | (unsigned long long)(~(uint32_t)i));
}

__global__ void __launch_bounds__(256) register_write_kernel(Table t, const uint32_t* __restrict__ slot,
                                                             int64_t n, int64_t expiry,
                                                             const uint32_t* __restrict__ incident) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n || slot[i] == 0xFFFFFFFFu) return;
  const uint32_t s = slot[i];
  if ((uint32_t)(t.claim[s] & 0xFFFFFFFFull) != ~(uint32_t)i) return;
  t.incident[s] = incident[i];
  t.expiry[s] = expiry;
}

// DEL (remove_fingerprint) and EXPIRE-if-EXISTS (extend_fingerprint)
__global__ void __launch_bounds__(256) remove_kernel(Table t, const uint4* __restrict__ fp, int64_t n) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  bool fresh;
  const uint32_t s = find_slot(t, fp[i], false, &fresh);
  if (s != 0xFFFFFFFFu) t.expiry[s] = 0;
}

__global__ void __launch_bounds__(256) extend_kernel(Table t, const uint4* __restrict__ fp, int64_t n,
                                                     int64_t now, int64_t expiry,
                                                     uint8_t* __restrict__ out_ok) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  bool fresh;
  const uint32_t s = find_slot(t, fp[i], false, &fresh);
  const bool live = s != 0xFFFFFFFFu && t.expiry[s] > now;
  // every key of the batch sets the same expiry: concurrent writes agree
  if (live) t.expiry[s] = expiry;
  if (out_ok) out_ok[i] = live ? 1 : 0;
}

// compaction: re-insert the live entries of `src` into the empty table `dst`
__global__ void __launch_bounds__(256) compact_kernel(Table src, Table dst, int64_t now,
                                                      uint32_t* __restrict__ n_live) {
  const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= src.cap) return;
  if (src.state[s] != ST_READY || src.expiry[s] <= now) return;
  bool fresh;
  const uint32_t d = find_slot(dst, src.key[s], true, &fresh);
  if (d == 0xFFFFFFFFu) return;  // cannot happen: dst has at least as many slots
  dst.expiry[d] = src.expiry[s];
  dst.incident[d] = src.incident[s];
  atomicAdd(n_live, 1u);
}

__global__ void __launch_bounds__(256) stats_kernel(Table t, int64_t now, unsigned long long* out) {
  const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= t.cap) return;
  const bool used = t.state[s] == ST_READY;
  const bool live = used && t.expiry[s] > now;
  if (used) atomicAdd(&out[0], 1ull);
  if (live) atomicAdd(&out[1], 1ull);
}

inline unsigned grid(int64_t n, int bs = 256) { return (unsigned)((n + bs - 1) / bs); }

}  // namespace

struct egr_dedup {
  int device = 0;
  Table t{};
  uint32_t seq = 0;
  // per-batch scratch (grown on demand)
  int64_t scratch_n = 0;
  uint32_t *slot = nullptr, *prior = nullptr, *is_new = nullptr, *rank = nullptr;
  uint32_t* ctr = nullptr;            // [0] table-full count, [1] new incidents, [2] live (compact)
  void* temp = nullptr;
  size_t temp_bytes = 0;
};

namespace {

int table_alloc(Table* t, uint32_t cap) {
  t->cap = cap;
  int rc = EGR_OK;
  if ((rc = dalloc(&t->state, cap)) || (rc = dalloc(&t->key, cap)) || (rc = dalloc(&t->expiry, cap)) ||
      (rc = dalloc(&t->incident, cap)) || (rc = dalloc(&t->claim, cap)))
    return rc;
  if (hipMemset(t->state, 0, (size_t)cap * 4) != hipSuccess ||
      hipMemset(t->expiry, 0, (size_t)cap * 8) != hipSuccess ||
      hipMemset(t->claim, 0xFF, (size_t)cap * 8) != hipSuccess)
    return egr::fail(EGR_EDEVICE, "dedup table init failed");
  return EGR_OK;
}

void table_free(Table* t) {
  dfree(t->state);
  dfree(t->key);
  dfree(t->expiry);
  dfree(t->incident);
  dfree(t->claim);
}

int ensure_scratch(egr_dedup* d, int64_t n) {
  if (n <= d->scratch_n) return EGR_OK;
  dfree(d->slot);
  dfree(d->prior);
  dfree(d->is_new);
  dfree(d->rank);
  dfree(d->temp);
  d->scratch_n = 0;
  int rc = EGR_OK;
  const int64_t m = std::max<int64_t>(n, 1024);
  if ((rc = dalloc(&d->slot, m)) || (rc = dalloc(&d->prior, m)) || (rc = dalloc(&d->is_new, m)) ||
      (rc = dalloc(&d->rank, m)))
    return rc;
  size_t tb = 0;
  if (hipcub::DeviceScan::ExclusiveSum(nullptr, tb, d->is_new, d->rank, (int)m) != hipSuccess)
    return egr::fail(EGR_EDEVICE, "dedup: scan sizing failed");
  if ((rc = dalloc((uint8_t**)&d->temp, tb))) return rc;
  d->temp_bytes = tb;
  d->scratch_n = m;
  return EGR_OK;
}

bool bad_batch(int64_t n) { return n < 0 || n > 0x7FFFFFFF; }

}  // namespace

extern "C" {

int egr_fingerprint(const uint8_t* blob, const int64_t* offsets, int64_t n, uint8_t* out16,
                    char* out_hex, void* stream) {
  if (n < 0 || (n > 0 && (!offsets || !out16))) return egr::fail(EGR_EINVAL, "egr_fingerprint: bad arguments");
  if (n == 0) return EGR_OK;
  hipLaunchKernelGGL(fingerprint_kernel, dim3(grid(n)), dim3(256), 0, (hipStream_t)stream, blob,
                     offsets, n, (uint4*)out16, out_hex);
  EGR_CHECK_LAUNCH();
  return EGR_OK;
}

int egr_dedup_create(int32_t device, int64_t capacity, egr_dedup** out) {
  if (!out || capacity < 1 || capacity > (1ll << 30))
    return egr::fail(EGR_EINVAL, "egr_dedup_create: bad arguments (1 <= capacity <= 2^30)");
  *out = nullptr;
  int ndev = 0;
  EGR_HIP(hipGetDeviceCount(&ndev));
  if (device < 0 || device >= ndev) return egr::fail(EGR_EINVAL, "egr_dedup_create: bad device");
  DeviceGuard guard(device);
  uint32_t cap = 64;
  while (cap < 2 * capacity) cap *= 2;   // at most half full at the requested capacity
  auto* d = new egr_dedup();
  d->device = device;
  int rc = EGR_OK;
  if ((rc = table_alloc(&d->t, cap)) || (rc = dalloc(&d->ctr, 4)) || (rc = ensure_scratch(d, 1024))) {
    egr_dedup_free(d);
    return rc;
  }
  *out = d;
  return EGR_OK;
}

void egr_dedup_free(egr_dedup* d) {
  if (!d) return;
  DeviceGuard guard(d->device);
  table_free(&d->t);
  dfree(d->slot);
  dfree(d->prior);
  dfree(d->is_new);
  dfree(d->rank);
  dfree(d->temp);
  dfree(d->ctr);
  delete d;
}

int egr_dedup_ingest(egr_dedup* d, const uint8_t* fp16, int64_t n, int64_t now_ms, int64_t ttl_ms,
                     uint32_t first_id, uint8_t* out_dup, uint32_t* out_incident,
                     uint32_t* out_counts, void* stream) {
  if (!d || bad_batch(n) || ttl_ms < 0 || (n > 0 && (!fp16 || !out_dup || !out_incident)) || !out_counts)
    return egr::fail(EGR_EINVAL, "egr_dedup_ingest: bad arguments");
  DeviceGuard guard(d->device);
  hipStream_t st = (hipStream_t)stream;
  EGR_HIP(hipMemsetAsync(out_counts, 0, 2 * 4, st));
  if (n == 0) return EGR_OK;
  EGR_TRY(ensure_scratch(d, n));
  const uint32_t seq = ++d->seq;
  const uint4* fp = (const uint4*)fp16;
  hipLaunchKernelGGL(ingest_probe_kernel, dim3(grid(n)), dim3(256), 0, st, d->t, fp, n, now_ms,
                     seq, d->slot, d->prior, out_counts);
  hipLaunchKernelGGL(ingest_first_kernel, dim3(grid(n)), dim3(256), 0, st, d->t, d->slot,
                     d->prior, n, d->is_new);
  size_t tb = d->temp_bytes;
  if (hipcub::DeviceScan::ExclusiveSum(d->temp, tb, d->is_new, d->rank, (int)n, st) != hipSuccess)
    return egr::fail(EGR_EDEVICE, "egr_dedup_ingest: scan failed");
  hipLaunchKernelGGL(ingest_resolve_kernel, dim3(grid(n)), dim3(256), 0, st, d->t, d->slot,
                     d->prior, d->is_new, d->rank, n, now_ms + ttl_ms, first_id, out_dup,
                     out_incident, out_counts + 1);
  EGR_CHECK_LAUNCH();
  return EGR_OK;
}

int egr_dedup_lookup(const egr_dedup* d, const uint8_t* fp16, int64_t n, int64_t now_ms,
                     uint8_t* out_dup, uint32_t* out_incident, void* stream) {
  if (!d || bad_batch(n) || (n > 0 && (!fp16 || !out_dup || !out_incident)))
    return egr::fail(EGR_EINVAL, "egr_dedup_lookup: bad arguments");
  if (n == 0) return EGR_OK;
  DeviceGuard guard(d->device);
  hipLaunchKernelGGL(lookup_kernel, dim3(grid(n)), dim3(256), 0, (hipStream_t)stream, d->t,
                     (const uint4*)fp16, n, now_ms, out_dup, out_incident);
  EGR_CHECK_LAUNCH();
  return EGR_OK;
}

int egr_dedup_register(egr_dedup* d, const uint8_t* fp16, int64_t n, int64_t now_ms, int64_t ttl_ms,
                       const uint32_t* incident, uint32_t* out_full, void* stream) {
  if (!d || bad_batch(n) || ttl_ms < 0 || (n > 0 && (!fp16 || !incident)) || !out_full)
    return egr::fail(EGR_EINVAL, "egr_dedup_register: bad arguments");
  DeviceGuard guard(d->device);
  hipStream_t st = (hipStream_t)stream;
  EGR_HIP(hipMemsetAsync(out_full, 0, 4, st));
  if (n == 0) return EGR_OK;
  EGR_TRY(ensure_scratch(d, n));
  const uint32_t seq = ++d->seq;
  hipLaunchKernelGGL(register_kernel, dim3(grid(n)), dim3(256), 0, st, d->t, (const uint4*)fp16, n,
                     d->slot, out_full);
  hipLaunchKernelGGL(register_last_kernel, dim3(grid(n)), dim3(256), 0, st, d->t, d->slot, n, seq);
  hipLaunchKernelGGL(register_write_kernel, dim3(grid(n)), dim3(256), 0, st, d->t, d->slot, n,
                     now_ms + ttl_ms, incident);
  EGR_CHECK_LAUNCH();
  return EGR_OK;
}

int egr_dedup_remove(egr_dedup* d, const uint8_t* fp16, int64_t n, void* stream) {
  if (!d || bad_batch(n) || (n > 0 && !fp16)) return egr::fail(EGR_EINVAL, "egr_dedup_remove: bad arguments");
  if (n == 0) return EGR_OK;
  DeviceGuard guard(d->device);
  hipLaunchKernelGGL(remove_kernel, dim3(grid(n)), dim3(256), 0, (hipStream_t)stream, d->t,
                     (const uint4*)fp16, n);
  EGR_CHECK_LAUNCH();
  return EGR_OK;
}

int egr_dedup_extend(egr_dedup* d, const uint8_t* fp16, int64_t n, int64_t now_ms, int64_t ttl_ms,
                     uint8_t* out_ok, void* stream) {
  if (!d || bad_batch(n) || ttl_ms < 0 || (n > 0 && !fp16))
    return egr::fail(EGR_EINVAL, "egr_dedup_extend: bad arguments");
  if (n == 0) return EGR_OK;
  DeviceGuard guard(d->device);
  hipLaunchKernelGGL(extend_kernel, dim3(grid(n)), dim3(256), 0, (hipStream_t)stream, d->t,
                     (const uint4*)fp16, n, now_ms, now_ms + ttl_ms, out_ok);
  EGR_CHECK_LAUNCH();
  return EGR_OK;
}

int egr_dedup_stats(const egr_dedup* d, int64_t now_ms, int64_t* out3) {
  if (!d || !out3) return egr::fail(EGR_EINVAL, "egr_dedup_stats: bad arguments");
  DeviceGuard guard(d->device);
  unsigned long long* dv = nullptr;
  EGR_TRY(dalloc(&dv, 2));
  unsigned long long hv[2] = {0, 0};
  hipError_t e = hipMemset(dv, 0, 16);
  if (e == hipSuccess) {
    hipLaunchKernelGGL(stats_kernel, dim3(grid(d->t.cap)), dim3(256), 0, nullptr, d->t, now_ms, dv);
    e = hipMemcpy(hv, dv, 16, hipMemcpyDeviceToHost);
  }
  dfree(dv);
  if (e != hipSuccess) return egr::fail(EGR_EDEVICE, std::string("egr_dedup_stats: ") + hipGetErrorString(e));
  out3[0] = (int64_t)hv[0];   // slots holding a key (live, expired or removed)
  out3[1] = (int64_t)hv[1];   // live keys
  out3[2] = (int64_t)d->t.cap;
  return EGR_OK;
}

int egr_dedup_compact(egr_dedup* d, int64_t now_ms, int64_t capacity) {
  if (!d || capacity < 0 || capacity > (1ll << 30)) return egr::fail(EGR_EINVAL, "egr_dedup_compact: bad arguments");
  DeviceGuard guard(d->device);
  int64_t st3[3];
  EGR_TRY(egr_dedup_stats(d, now_ms, st3));
  uint32_t cap = 64;
  const int64_t want = std::max<int64_t>(capacity, st3[1]);
  while (cap < 2 * want) cap *= 2;
  Table nt{};
  int rc = table_alloc(&nt, cap);
  if (rc) {
    table_free(&nt);
    return rc;
  }
  EGR_HIP(hipMemset(d->ctr, 0, 16));
  hipLaunchKernelGGL(compact_kernel, dim3(grid(d->t.cap)), dim3(256), 0, nullptr, d->t, nt, now_ms,
                     d->ctr + 2);
  hipError_t e = hipDeviceSynchronize();
  if (e != hipSuccess) {
    table_free(&nt);
    return egr::fail(EGR_EDEVICE, std::string("egr_dedup_compact: ") + hipGetErrorString(e));
  }
  table_free(&d->t);
  d->t = nt;
  return EGR_OK;
}

}  // extern "C"
