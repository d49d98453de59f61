// numpy_rng.cuh — the reference sampler's random streams on the device.
//
// The reference seeds numpy's global legacy RandomState per chain
// (np.random.seed(random_seed), Samplers.py:70; random_seed = chain index,
// Framework.py:1015/1020) and per MH iteration draws, in this order:
//   normal(0, 0.05) for each walking parameter        parameter.rwalk, Framework.py:119/122
//   one standard normal per walking lognorm prior       pdf() -> dist.rvs, Framework.py:103
//                                                        (scipy lognorm._rvs = exp(s * standard_normal))
//   rand()                                              the acceptance uniform, Samplers.py:127
// numpy's legacy generator (numpy/random/_mt19937, legacy-distributions.c) is MT19937
// (Matsumoto & Nishimura 1998) seeded by init_genrand, doubles from two 32-bit words
// ((a >> 5) * 2^26 + (b >> 6)) / 2^53, and normals from the polar Box–Muller method that
// returns f*x2 and keeps f*x1 for the next call.  This file restates those published
// algorithms, one chain per lane.  Only the final `log` of the polar method is a libm
// call; ocml and glibc agree to <= 1 ulp there, everything else is exact integer / IEEE
// arithmetic (checked against numpy itself in tests/).
//
// MT state layout: key [W][624] in HBM (a chain's words contiguous), pos/gauss/has_gauss
// [W].  A draw launch stages the keys of kNpChainsPerBlock chains through LDS, transposed
// to [624][chains] so a wave's lanes at the same word index hit distinct banks, draws there
// and writes them back: each 32-bit word costs LDS latency instead of a dependent global
// load chain (r04: 299 -> see profiles/NOTES.md per chunk of the notebook fit).  The twist is
// done lazily one word per draw (word i of generation g+1 needs words i, i+1 of generation g
// and word i+397 mod 624 of g or g+1 — exactly the values the block twist reads), so lanes
// whose polar rejections differ never diverge into a 624-word loop.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace oe {

constexpr int kMtN = 624, kMtM = 397;

struct NpState {
  uint32_t* key;       // [W][624]
  int32_t* pos;        // [W] index of the next word of the current generation to twist + emit
  double* gauss;       // [W] cached second normal
  int32_t* has_gauss;  // [W]
};

struct NpDrawArgs {
  int64_t W;
  int32_t it0, it1;      // iterations [it0, it1) of this chunk (1-based reference `it`)
  int32_t P;
  int32_t prior_draws;   // standard normals consumed after the proposal normals
  int32_t zero_static;   // write dz = 0 for static parameters (stream export)
  uint64_t walk_mask;
  double step_sd;
  NpState st;
  double* dz;            // [it1 - it0][P][W]
  double* u;             // [it1 - it0][W]
};

constexpr int kNpChainsPerBlock = 64;  // 64 x 624 words = 156 KiB of LDS: one wave per CU

// One chain's generator.  key[i * STRIDE] is word i (STRIDE = chains per block in LDS).
// `nxt` carries word i+1 of the old generation from one draw to the next: it is the next
// draw's word i and has not been overwritten in between (only word i is written per draw).
template <int STRIDE>
struct NpLane {
  uint32_t* key;
  int pos;
  double gauss;
  bool has_gauss;
  uint32_t cur;  // key[pos] (old generation)

  __device__ __forceinline__ void start() { cur = key[pos * STRIDE]; }
  __device__ __forceinline__ uint32_t next32() {
    const int i = pos;
    const int i1 = (i + 1 == kMtN) ? 0 : i + 1;
    const int im = (i + kMtM >= kMtN) ? i + kMtM - kMtN : i + kMtM;
    const uint32_t nxt = key[i1 * STRIDE];
    const uint32_t y = (cur & 0x80000000u) | (nxt & 0x7fffffffu);
    const uint32_t v = key[im * STRIDE] ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
    key[i * STRIDE] = v;
    pos = i1;
    cur = nxt;  // (at i = 623, word 0 is already the new generation's in both uses)
    uint32_t t = v;  // tempering
    t ^= t >> 11;
    t ^= (t << 7) & 0x9d2c5680u;
    t ^= (t << 15) & 0xefc60000u;
    t ^= t >> 18;
    return t;
  }
  // random_sample(): 53-bit double in [0, 1)
  __device__ __forceinline__ double next_double() {
    const uint32_t a = next32() >> 5, b = next32() >> 6;
    return ((double)a * 67108864.0 + (double)b) / 9007199254740992.0;
  }
  // standard_normal() of the legacy RandomState (polar method, one cached value)
  __device__ __forceinline__ double next_gauss() {
    if (has_gauss) {
      has_gauss = false;
      return gauss;
    }
    double x1, x2, r2;
    do {
      x1 = 2.0 * next_double() - 1.0;
      x2 = 2.0 * next_double() - 1.0;
      r2 = x1 * x1 + x2 * x2;
    } while (r2 >= 1.0 || r2 == 0.0);
    const double f = sqrt(-2.0 * log(r2) / r2);
    gauss = f * x1;
    has_gauss = true;
    return f * x2;
  }
};

// init_genrand(seed): key[0] = seed, key[i] = 1812433253 (key[i-1] ^ key[i-1] >> 30) + i
__device__ __forceinline__ void np_seed_lane(const NpState& st, int64_t w, uint32_t seed) {
  uint32_t* key = st.key + w * kMtN;
  uint32_t s = seed;
  for (int i = 0; i < kMtN; ++i) {
    key[i] = s;
    s = 1812433253u * (s ^ (s >> 30)) + (uint32_t)(i + 1);
  }
  st.pos[w] = 0;  // numpy's pos = 624: the first draw twists (lazily here)
  st.has_gauss[w] = 0;
  st.gauss[w] = 0.0;
}

// The draws of chains [blockIdx.x * CPB, + CPB) with their keys staged in LDS; blockDim.x
// == CPB.  Global <-> LDS copies are coalesced over the block's contiguous key region.
template <int CPB>
__device__ __forceinline__ void np_draw_block(const NpDrawArgs& d) {
  __shared__ uint32_t sk[kMtN * CPB];
  const int64_t W = d.W;
  const int64_t w0 = (int64_t)blockIdx.x * CPB;
  const int nw = (int)((W - w0 < CPB) ? W - w0 : CPB);
  uint32_t* gk = d.st.key + w0 * kMtN;
  for (int r = threadIdx.x; r < nw * kMtN; r += CPB) {
    const int c = r / kMtN, i = r - c * kMtN;
    sk[i * CPB + c] = gk[r];
  }
  __syncthreads();
  const int c = threadIdx.x;
  if (c < nw) {
    const int64_t w = w0 + c;
    NpLane<CPB> L{sk + c, d.st.pos[w], d.st.gauss[w], d.st.has_gauss[w] != 0, 0u};
    L.start();
    for (int it = d.it0; it < d.it1; ++it) {
      double* dz = d.dz + (int64_t)(it - d.it0) * d.P * W + w;
      for (int j = 0; j < d.P; ++j) {
        if ((d.walk_mask >> j) & 1ull) dz[(int64_t)j * W] = 0.0 + d.step_sd * L.next_gauss();  // loc + scale*gauss
        else if (d.zero_static) dz[(int64_t)j * W] = 0.0;
      }
      for (int k = 0; k < d.prior_draws; ++k) (void)L.next_gauss();
      d.u[(int64_t)(it - d.it0) * W + w] = L.next_double();
    }
    d.st.pos[w] = L.pos;
    d.st.gauss[w] = L.gauss;
    d.st.has_gauss[w] = L.has_gauss ? 1 : 0;
  }
  __syncthreads();
  for (int r = threadIdx.x; r < nw * kMtN; r += CPB) {
    const int c2 = r / kMtN, i = r - c2 * kMtN;
    gk[r] = sk[i * CPB + c2];
  }
}

}  // namespace oe
