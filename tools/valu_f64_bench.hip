// valu_f64_bench.hip — fp64 VALU issue rate and dependent latency on gfx950, measured
// in shader cycles (s_memtime) per wave, independent of the DVFS clock.
//
//   hipcc -O3 --offload-arch=gfx950 -o /tmp/valu_f64_bench tools/valu_f64_bench.hip
//   ./valu_f64_bench            (prints one JSON line per case)
//
// Each lane runs ITERS iterations of CH independent fp64 FMA chains (CH = 1 is a
// single dependent chain; CH = 8 gives eight independent FMAs per dependent step).
// Grids of 1, 2 and 4 waves per SIMD (256 CUs x 4 SIMDs, 256-thread blocks).
// Reported: cycles per FMA per wave (the wave's issue cost at that ILP and occupancy).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <algorithm>

constexpr int ITERS = 4096;

template <int CH>
__global__ void __launch_bounds__(256) k_fma(const double* in, double* out, unsigned long long* cyc) {
  const int gid = blockIdx.x * blockDim.x + threadIdx.x;
  double a[CH];
#pragma unroll
  for (int c = 0; c < CH; ++c) a[c] = in[(gid + c) & 1023];
  const double m = in[1024 + (gid & 7)], b = in[1032 + (gid & 7)];
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < ITERS; ++i) {
#pragma unroll
    for (int c = 0; c < CH; ++c) a[c] = fma(a[c], m, b);
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  double s = 0.0;
#pragma unroll
  for (int c = 0; c < CH; ++c) s += a[c];
  out[gid] = s;
  if ((threadIdx.x & 63) == 0) cyc[gid >> 6] = t1 - t0;
}

template <int CH>
void run(int waves_per_simd, const double* d_in, double* d_out, unsigned long long* d_cyc) {
  const int blocks = 256 * waves_per_simd;  // 256 CUs, 4 waves (one per SIMD) per block
  hipLaunchKernelGGL(k_fma<CH>, dim3(blocks), dim3(256), 0, 0, d_in, d_out, d_cyc);
  hipLaunchKernelGGL(k_fma<CH>, dim3(blocks), dim3(256), 0, 0, d_in, d_out, d_cyc);
  hipDeviceSynchronize();
  const int nw = blocks * 4;
  std::vector<unsigned long long> c(nw);
  hipMemcpy(c.data(), d_cyc, sizeof(unsigned long long) * nw, hipMemcpyDeviceToHost);
  std::sort(c.begin(), c.end());
  const double med = (double)c[nw / 2];
  printf("{\"chains\": %d, \"waves_per_simd\": %d, \"cycles_per_fma_per_wave\": %.3f, "
         "\"simd_cycles_per_fma\": %.3f}\n",
         CH, waves_per_simd, med / (ITERS * CH), med / (ITERS * CH) / waves_per_simd);
}

int main() {
  double *d_in, *d_out;
  unsigned long long* d_cyc;
  std::vector<double> h(2048);
  for (int i = 0; i < 2048; ++i) h[i] = 1.0 + 1e-9 * i;
  for (int i = 1024; i < 1040; ++i) h[i] = 0.999999;
  hipMalloc(&d_in, 2048 * sizeof(double));
  hipMalloc(&d_out, 256 * 4 * 256 * sizeof(double));
  hipMalloc(&d_cyc, 256 * 4 * 16 * sizeof(unsigned long long));
  hipMemcpy(d_in, h.data(), 2048 * sizeof(double), hipMemcpyHostToDevice);
  for (int w : {1, 2, 4}) {
    run<1>(w, d_in, d_out, d_cyc);
    run<2>(w, d_in, d_out, d_cyc);
    run<4>(w, d_in, d_out, d_cyc);
    run<8>(w, d_in, d_out, d_cyc);
  }
  hipFree(d_in);
  hipFree(d_out);
  hipFree(d_cyc);
  return 0;
}
