// Internal helpers shared by the HIP kernels and the host side of libegraph.so.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstring>
#include <string>

#include "egraph.h"

namespace egr {

// ---- error reporting (thread-local last error; see egr_last_error) ----------------------
void set_error(const std::string& msg);
int fail(int code, const std::string& msg);

#define EGR_HIP(call)                                                                   \
  do {                                                                                  \
    hipError_t e_ = (call);                                                             \
    if (e_ != hipSuccess)                                                               \
      return ::egr::fail(EGR_EDEVICE, std::string(#call) + ": " + hipGetErrorString(e_)); \
  } while (0)

#define EGR_CHECK_LAUNCH()                                                                  \
  do {                                                                                      \
    hipError_t e_ = hipGetLastError();                                                      \
    if (e_ != hipSuccess)                                                                   \
      return ::egr::fail(EGR_EDEVICE, std::string("kernel launch (" __FILE__ ":") +           \
                                          std::to_string(__LINE__) + "): " + hipGetErrorString(e_)); \
  } while (0)

// ---- the current device for a scope (host) ----------------------------------------------
struct DeviceGuard {
  int prev = -1;
  explicit DeviceGuard(int dev) {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    if (prev != dev) (void)hipSetDevice(dev);
  }
  ~DeviceGuard() {
    int cur;
    if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
  }
};

// ---- Python-exact float rounding -----------------------------------------------------------
// round(x, nd) in CPython (Objects/floatobject.c, double_round) is: take the exact binary value
// of x, round x*10^nd to an integer q half-to-even, return the double nearest to q/10^nd.
// Signs are symmetric, NaN/inf and integer-valued doubles come back unchanged.
// We do the same exactly with 128-bit integer arithmetic; the common case (q < 2^53) ends in
// one IEEE division of two exactly representable doubles, which is correctly rounded.

__host__ __device__ inline uint64_t pow10_u64(int nd) {
  uint64_t p = 1;
  for (int i = 0; i < nd; ++i) p *= 10u;
  return p;
}

__host__ __device__ inline int bitlen128(unsigned __int128 v) {
  int n = 0;
  while (v) { v >>= 1; ++n; }
  return n;
}

// floor(n / d) and n % d for n < 2^120, d < 2^50, by 14-bit long division (no __udivti3 on
// the device).
__host__ __device__ inline unsigned __int128 divmod_small(unsigned __int128 n, uint64_t d,
                                                          uint64_t* rem) {
  unsigned __int128 q = 0;
  uint64_t r = 0;
  for (int shift = 112; shift >= 0; shift -= 14) {
    uint64_t digit = (uint64_t)((n >> shift) & 0x3FFFu);
    uint64_t cur = (r << 14) | digit;  // r < d < 2^50 so cur < 2^64
    q = (q << 14) | (cur / d);
    r = cur % d;
  }
  *rem = r;
  return q;
}

// correctly rounded double of q / 10^nd
__host__ __device__ inline double div_pow10_rn(unsigned __int128 q, int nd) {
  const uint64_t p10 = pow10_u64(nd);
  if (q < ((unsigned __int128)1 << 53)) return (double)(uint64_t)q / (double)p10;
  // rare path (|x| * 10^nd >= 2^53): long division to >= 55 quotient bits, then round.
  int L = bitlen128(q);
  int lp = bitlen128(p10);
  int s = 57 - (L - lp);
  if (s < 0) s = 0;
  unsigned __int128 n = q << s;
  uint64_t rem = 0;
  unsigned __int128 Q = divmod_small(n, p10, &rem);
  int QL = bitlen128(Q);
  int drop = QL - 53;
  uint64_t mant;
  if (drop <= 0) {
    mant = (uint64_t)Q;  // cannot happen with s chosen above, kept for safety
    drop = 0;
  } else {
    unsigned __int128 low = Q & (((unsigned __int128)1 << drop) - 1);
    unsigned __int128 half = (unsigned __int128)1 << (drop - 1);
    mant = (uint64_t)(Q >> drop);
    bool sticky = rem != 0;
    if (low > half || (low == half && (sticky || (mant & 1u)))) ++mant;
    else if (low == half && !sticky && !(mant & 1u)) { /* tie to even: keep */ }
  }
  double r = (double)mant;  // mant <= 2^53 exactly representable
  int e2 = drop - s;
#ifdef __HIP_DEVICE_COMPILE__
  return ldexp(r, e2);
#else
  return __builtin_ldexp(r, e2);
#endif
}

__host__ __device__ inline double py_round(double x, int nd) {
  if (!(x == x)) return x;                     // NaN
  if (x == 0.0) return x;                      // keeps the sign of zero
  uint64_t bits;
  memcpy(&bits, &x, 8);
  const bool neg = bits >> 63;
  const int bexp = (int)((bits >> 52) & 0x7FF);
  if (bexp == 0x7FF) return x;                 // +-inf
  uint64_t m = bits & ((1ull << 52) - 1);
  int e;
  if (bexp == 0) {
    e = -1074;
  } else {
    m |= 1ull << 52;
    e = bexp - 1075;
  }
  if (e >= 0) return x;                        // integer-valued
  const int k = -e;                            // x = m / 2^k
  const unsigned __int128 P = (unsigned __int128)m * pow10_u64(nd);  // < 2^103 for nd <= 15
  unsigned __int128 q;
  if (k >= 110) {
    q = 0;                                     // P < 2^103 <= 2^(k-1): below one half
  } else {
    q = P >> k;
    const unsigned __int128 r = P & (((unsigned __int128)1 << k) - 1);
    const unsigned __int128 half = (unsigned __int128)1 << (k - 1);
    if (r > half || (r == half && (q & 1))) q += 1;
  }
  double res = q == 0 ? 0.0 : div_pow10_rn(q, nd);
  return neg ? -res : res;
}

// Python's min(a, b): returns a unless b < a (NaN-faithful, unlike fmin)
__host__ __device__ inline double py_min(double a, double b) { return (b < a) ? b : a; }

// ---- the confidence / ranker formulas, operation-for-operation -----------------------------
// rules_engine.py:443-455
__host__ __device__ inline double rule_confidence(double base, int match_count, double strength) {
  double c = base * 0.6 + strength * 0.4;
  if (match_count > 2) c = py_min(c * 1.1, 0.99);
  return py_round(c, 3);
}

// hypothesis_ranker.py:44-63 (support and strength already as doubles)
__host__ __device__ inline double ranker_final_score(double confidence, double cat_weight,
                                                     double support, double strength) {
  double score = confidence;
  score = score * cat_weight;
  if (support > 0) score = score * (1.0 + py_min(support, 5.0) * 0.05);
  score = score * (1.0 + strength * 0.2);
  return py_round(score, 4);
}

}  // namespace egr
