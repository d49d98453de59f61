// pipe_bench.hip — producer/consumer store pipeline sweep (diagnostic tool).
// NC compute waves (one walker per lane, `work` dependent fma per state per step) write
// rows into an LDS ring; NS store waves drain it with 16-B (2 walkers/lane) or 8-B stores.
// Build: hipcc -O3 --offload-arch=gfx950 -o pipe_bench tools/pipe_bench.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1);} } while (0)
typedef unsigned int u4v __attribute__((ext_vector_type(4)));
typedef unsigned int u2v __attribute__((ext_vector_type(2)));

template <int NC, int NS, int H, bool WIDE>
__global__ void __launch_bounds__(64 * (NC + NS)) pipe(double* out, long W, int T, int work, double a) {
  constexpr int S = 4, WB = 64 * NC;
  __shared__ double ring[2][H][S][WB];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const long base = (long)blockIdx.x * WB;
  const int nph = (T + H - 1) / H;
  if (wave < NC) {
    const int b = wave * 64 + lane;
    double y[S];
    for (int s = 0; s < S; ++s) y[s] = 1.0 + 1e-3 * s + 1e-9 * (double)(base + b);
    for (int ph = 0; ph <= nph; ++ph) {
      if (ph < nph) {
        for (int r = ph * H; r < ph * H + H && r < T; ++r) {
          for (int k = 0; k < work; ++k)
#pragma unroll
            for (int s = 0; s < S; ++s) y[s] = fma(y[s], a, 1e-7);
#pragma unroll
          for (int s = 0; s < S; ++s) ring[ph & 1][r - ph * H][s][b] = y[s];
        }
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
    }
  } else {
    const int sw = wave - NC;
    constexpr int per = WB / NS;  // walkers per store wave
    const unsigned rowb = (unsigned)(S * W * 8);
    for (int ph = 0; ph <= nph; ++ph) {
      if (ph >= 1) {
        const int half = (ph - 1) & 1;
        for (int r = (ph - 1) * H; r < (ph - 1) * H + H && r < T; ++r) {
          auto rs = __builtin_amdgcn_make_buffer_rsrc((void*)(out + (long)r * S * W), 0, rowb, 0x00020000);
#pragma unroll
          for (int s = 0; s < S; ++s) {
            if (WIDE) {  // 2 walkers per lane, per/128 instructions
              for (int c = 0; c < per / 128; ++c) {
                const int b = sw * per + c * 128 + 2 * lane;
                u4v v = *reinterpret_cast<const u4v*>(&ring[half][r - (ph - 1) * H][s][b]);
                __builtin_amdgcn_raw_buffer_store_b128(v, rs, (unsigned)(base + b) * 8u, (unsigned)(s * W * 8), 2);
              }
            } else {
              for (int c = 0; c < per / 64; ++c) {
                const int b = sw * per + c * 64 + lane;
                u2v v = *reinterpret_cast<const u2v*>(&ring[half][r - (ph - 1) * H][s][b]);
                __builtin_amdgcn_raw_buffer_store_b64(v, rs, (unsigned)(base + b) * 8u, (unsigned)(s * W * 8), 2);
              }
            }
          }
        }
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
    }
  }
}

template <int NC, int NS, int H, bool WIDE>
void run(double* out, long W, int T, int work, double bytes) {
  dim3 g((unsigned)(W / (64 * NC))), b(64 * (NC + NS));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0)); CHECK(hipEventCreate(&e1));
  hipLaunchKernelGGL((pipe<NC, NS, H, WIDE>), g, b, 0, 0, out, W, T, work, 0.999999);
  CHECK(hipDeviceSynchronize());
  CHECK(hipEventRecord(e0));
  for (int r = 0; r < 10; ++r) hipLaunchKernelGGL((pipe<NC, NS, H, WIDE>), g, b, 0, 0, out, W, T, work, 0.999999);
  CHECK(hipEventRecord(e1)); CHECK(hipEventSynchronize(e1));
  float ms; CHECK(hipEventElapsedTime(&ms, e0, e1)); ms /= 10;
  printf("NC=%d NS=%d H=%2d %s work=%2d : %.3f ms %.2f TB/s\n", NC, NS, H, WIDE ? "16B" : " 8B", work, ms, bytes / (ms * 1e-3) / 1e12);
}

int main() {
  const long W = 65536; const int T = 1000;
  double* out; const double bytes = (double)T * 4 * W * 8;
  CHECK(hipMalloc(&out, (size_t)bytes));
  for (int work : {0, 14}) {
    run<4, 2, 2, true>(out, W, T, work, bytes);
    run<4, 2, 4, true>(out, W, T, work, bytes);
    run<4, 2, 8, true>(out, W, T, work, bytes);
    run<4, 1, 8, true>(out, W, T, work, bytes);
    run<4, 4, 8, true>(out, W, T, work, bytes);
    run<4, 4, 8, false>(out, W, T, work, bytes);
    run<2, 2, 8, true>(out, W, T, work, bytes);
    run<2, 1, 16, true>(out, W, T, work, bytes);
    run<8, 4, 4, true>(out, W, T, work, bytes);
  }
  return 0;
}
