// A training step's random inputs in one launch: the router noise of both generator forwards (N(0, 1), the eps of
// the reparameterised router weights, t2i_moe_gan.py:302-333) and the mismatched-caption permutation (randperm of
// the batch, :1278).  Counter-based (splitmix64 of seed and element index), so a step's draws depend only on its
// seeds: bench.py refills its fixed input buffers with it before every (eager or replayed) step, where torch's
// normal_ / randperm took ~9 launches.
//
//  * normals: Box-Muller on pairs, u1 in (0, 1] and u2 in [0, 1) from 24-bit fields of one 64-bit hash;
//  * permutation: one block sorts B unique 64-bit keys (random high bits, the index in the low 12) with a bitonic
//    network in LDS; the sorted order is a uniformly random permutation (B <= 4096).
#include "mg_common.h"

namespace {

MG_DEV uint64_t splitmix(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

constexpr int RT = 256;      // threads per block
constexpr int PMAX = 4096;   // largest permutation

__global__ __launch_bounds__(RT) void k_step_inputs(float* __restrict__ a, int64_t na, float* __restrict__ b,
                                                    int64_t nb, int32_t* __restrict__ perm, int B, uint64_t seed_eps,
                                                    uint64_t seed_perm, int rand_blocks) {
  if ((int)blockIdx.x == rand_blocks) {  // the permutation block
    __shared__ uint64_t key[PMAX];
    int n = 1;
    while (n < B) n <<= 1;
    for (int i = threadIdx.x; i < n; i += RT)
      key[i] = i < B ? (splitmix(seed_perm ^ (0xA24BAED4963EE407ull * (uint64_t)(i + 1))) & ~0xFFFull) | (uint64_t)i
                     : ~0ull;
    __syncthreads();
    for (int k = 2; k <= n; k <<= 1)
      for (int j = k >> 1; j > 0; j >>= 1) {
        for (int i = threadIdx.x; i < n; i += RT) {
          const int ij = i ^ j;
          if (ij > i) {
            const uint64_t x = key[i], y = key[ij];
            const bool up = (i & k) == 0;
            if ((x > y) == up) {
              key[i] = y;
              key[ij] = x;
            }
          }
        }
        __syncthreads();
      }
    for (int i = threadIdx.x; i < B; i += RT) perm[i] = (int32_t)(key[i] & 0xFFFull);
    return;
  }
  const int64_t n = na + nb, pairs = (n + 1) / 2;
  for (int64_t q = (int64_t)blockIdx.x * RT + threadIdx.x; q < pairs; q += (int64_t)rand_blocks * RT) {
    const uint64_t h = splitmix(seed_eps + 0x9E3779B97F4A7C15ull * (uint64_t)q);
    const float u1 = (float)((h >> 40) + 1) * 5.9604644775390625e-8f;        // (0, 1]
    const float u2 = (float)((h >> 16) & 0xFFFFFFull) * 5.9604644775390625e-8f;  // [0, 1)
    const float r = sqrtf(-2.f * logf(u1));
    float s, c;
    sincosf(6.283185307179586f * u2, &s, &c);
    const int64_t i0 = 2 * q, i1 = i0 + 1;
    if (i0 < na) a[i0] = r * c; else b[i0 - na] = r * c;
    if (i1 < n) {
      if (i1 < na) a[i1] = r * s; else b[i1 - na] = r * s;
    }
  }
}

}  // namespace

extern "C" int mg_step_inputs(float* eps_a, int64_t na, float* eps_b, int64_t nb, int32_t* perm, int B,
                              uint64_t seed_eps, uint64_t seed_perm, void* stream) {
  MG_REQUIRE(na >= 0 && nb >= 0 && (na == 0 || eps_a) && (nb == 0 || eps_b), "bad noise buffers");
  MG_REQUIRE(B >= 0 && B <= PMAX && (B == 0 || perm), "B must be in [0, 4096]");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const int64_t pairs = (na + nb + 1) / 2;
  const int rand_blocks = (int)std::max<int64_t>(1, std::min<int64_t>(cdiv(pairs, RT), 1024));
  hipLaunchKernelGGL(k_step_inputs, dim3(rand_blocks + (B > 0 ? 1 : 0)), dim3(RT), 0, st, eps_a, na, eps_b, nb, perm,
                     B, seed_eps, seed_perm, rand_blocks);
  return mg_check_launch("mg_step_inputs");
}
