// store_bench.hip — ceiling of the trajectory-store pattern on MI355X (diagnostic tool).
//
// Each lane owns walker(s), loops over T steps, does a configurable dependent fp64
// chain per step (stand-in for the RK4 arithmetic), and stores S doubles per walker per
// step.  Layouts:
//   L0  [T][S][W]           8 B per lane per store (the engine's layout)
//   L1  [W/64][T][S][64]    8 B per lane, each wave's output contiguous (walker tiles)
//   L2  [T][S][W], 2 walkers per lane, 16 B per lane (dwordx4 stores)
// Build: hipcc -O3 --offload-arch=gfx950 -o store_bench tools/store_bench.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef double d2v __attribute__((ext_vector_type(2)));
#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1);} } while (0)

template <int LAYOUT, bool NT, int S>
__global__ void __launch_bounds__(256) store_kernel(double* out, long W, int T, int work, double a) {
  const long gw = (long)blockIdx.x * blockDim.x + threadIdx.x;
  double y[S];
#pragma unroll
  for (int s = 0; s < S; ++s) y[s] = 1.0 + 1e-3 * s + 1e-9 * (double)gw;
  if (LAYOUT == 2) {
    const long w2 = gw * 2;
    if (w2 >= W) return;
    double z[S];
#pragma unroll
    for (int s = 0; s < S; ++s) z[s] = y[s] * 1.5;
    for (int t = 0; t < T; ++t) {
      for (int k = 0; k < work; ++k) {
#pragma unroll
        for (int s = 0; s < S; ++s) { y[s] = fma(y[s], a, 1e-7); z[s] = fma(z[s], a, 1e-7); }
      }
#pragma unroll
      for (int s = 0; s < S; ++s) {
        d2v* p = reinterpret_cast<d2v*>(out + ((long)t * S + s) * W + w2);
        d2v v = {y[s], z[s]};
        if (NT) __builtin_nontemporal_store(v, p); else *p = v;
      }
    }
    return;
  }
  if (gw >= W) return;
  for (int t = 0; t < T; ++t) {
    for (int k = 0; k < work; ++k) {
#pragma unroll
      for (int s = 0; s < S; ++s) y[s] = fma(y[s], a, 1e-7);
    }
#pragma unroll
    for (int s = 0; s < S; ++s) {
      long idx;
      if (LAYOUT == 0) idx = ((long)t * S + s) * W + gw;
      else idx = (((gw >> 6) * T + t) * S + s) * 64 + (gw & 63);
      if (NT) __builtin_nontemporal_store(y[s], out + idx); else out[idx] = y[s];
    }
  }
}

// L3: [T][S][W] through a per-row buffer descriptor (the engine's current store path),
// cache-policy bits `AUX` (gfx950 aux: sc0=1, nt=2, sc1=16)
template <int AUX, int S>
__global__ void __launch_bounds__(256) buf_kernel(double* out, long W, int T, int work, double a) {
  typedef unsigned int u2 __attribute__((ext_vector_type(2)));
  const long gw = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (gw >= W) return;
  double y[S];
#pragma unroll
  for (int s = 0; s < S; ++s) y[s] = 1.0 + 1e-3 * s + 1e-9 * (double)gw;
  const unsigned off = (unsigned)gw * 8u;
  for (int t = 0; t < T; ++t) {
    for (int k = 0; k < work; ++k) {
#pragma unroll
      for (int s = 0; s < S; ++s) y[s] = fma(y[s], a, 1e-7);
    }
    auto rsrc = __builtin_amdgcn_make_buffer_rsrc((void*)(out + (long)t * S * W), 0, (unsigned)(S * W * 8), 0x00020000);
#pragma unroll
    for (int s = 0; s < S; ++s)
      __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u2, y[s]), rsrc, off, (unsigned)(s * W * 8), AUX);
  }
}

// L4: walker-tiled [W/64][T][S][64] through a per-wave buffer descriptor (contiguous
// 2 KB per wave per step), cache-policy bits AUX
template <int AUX, int S>
__global__ void __launch_bounds__(256) tiled_kernel(double* out, long W, int T, int work, double a) {
  typedef unsigned int u2 __attribute__((ext_vector_type(2)));
  const long gw = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (gw >= W) return;
  double y[S];
#pragma unroll
  for (int s = 0; s < S; ++s) y[s] = 1.0 + 1e-3 * s + 1e-9 * (double)gw;
  const long tile = gw >> 6;
  auto rsrc = __builtin_amdgcn_make_buffer_rsrc((void*)(out + tile * (long)T * S * 64), 0, (unsigned)(T * S * 64 * 8), 0x00020000);
  const unsigned lane_off = (unsigned)(gw & 63) * 8u;
  for (int t = 0; t < T; ++t) {
    for (int k = 0; k < work; ++k) {
#pragma unroll
      for (int s = 0; s < S; ++s) y[s] = fma(y[s], a, 1e-7);
    }
#pragma unroll
    for (int s = 0; s < S; ++s)
      __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u2, y[s]), rsrc, lane_off, (unsigned)((t * S + s) * 512), AUX);
  }
}

template <int AUX>
float runtiled(double* out, long W, int T, int work, int reps) {
  dim3 g((unsigned)((W + 255) / 256)), b(256);
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0)); CHECK(hipEventCreate(&e1));
  hipLaunchKernelGGL((tiled_kernel<AUX, 4>), g, b, 0, 0, out, W, T, work, 0.999999);
  CHECK(hipDeviceSynchronize());
  CHECK(hipEventRecord(e0));
  for (int r = 0; r < reps; ++r) hipLaunchKernelGGL((tiled_kernel<AUX, 4>), g, b, 0, 0, out, W, T, work, 0.999999);
  CHECK(hipEventRecord(e1));
  CHECK(hipEventSynchronize(e1));
  float ms; CHECK(hipEventElapsedTime(&ms, e0, e1));
  return ms / reps;
}

template <int AUX>
float runbuf(double* out, long W, int T, int work, int reps) {
  dim3 g((unsigned)((W + 255) / 256)), b(256);
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0)); CHECK(hipEventCreate(&e1));
  hipLaunchKernelGGL((buf_kernel<AUX, 4>), g, b, 0, 0, out, W, T, work, 0.999999);
  CHECK(hipDeviceSynchronize());
  CHECK(hipEventRecord(e0));
  for (int r = 0; r < reps; ++r) hipLaunchKernelGGL((buf_kernel<AUX, 4>), g, b, 0, 0, out, W, T, work, 0.999999);
  CHECK(hipEventRecord(e1));
  CHECK(hipEventSynchronize(e1));
  float ms; CHECK(hipEventElapsedTime(&ms, e0, e1));
  return ms / reps;
}

template <int LAYOUT, bool NT>
float run(double* out, long W, int T, int work, int reps) {
  constexpr int S = 4;
  const long lanes = LAYOUT == 2 ? W / 2 : W;
  dim3 g((unsigned)((lanes + 255) / 256)), b(256);
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0)); CHECK(hipEventCreate(&e1));
  hipLaunchKernelGGL((store_kernel<LAYOUT, NT, S>), g, b, 0, 0, out, W, T, work, 0.999999);
  CHECK(hipDeviceSynchronize());
  CHECK(hipEventRecord(e0));
  for (int r = 0; r < reps; ++r) hipLaunchKernelGGL((store_kernel<LAYOUT, NT, S>), g, b, 0, 0, out, W, T, work, 0.999999);
  CHECK(hipEventRecord(e1));
  CHECK(hipEventSynchronize(e1));
  float ms; CHECK(hipEventElapsedTime(&ms, e0, e1));
  return ms / reps;
}

int main(int argc, char** argv) {
  const long W = argc > 1 ? atol(argv[1]) : 65536;
  const int T = 1000, S = 4, reps = 10;
  double* out;
  const size_t bytes = (size_t)T * S * W * 8;
  CHECK(hipMalloc(&out, bytes));
  printf("W=%ld T=%d S=%d bytes=%.3f GB\n", W, T, S, bytes / 1e9);
  for (int work : {0, 4, 8, 16}) {
    float t00 = run<0, false>(out, W, T, work, reps), t01 = run<0, true>(out, W, T, work, reps);
    float t10 = run<1, false>(out, W, T, work, reps), t11 = run<1, true>(out, W, T, work, reps);
    float t20 = run<2, false>(out, W, T, work, reps), t21 = run<2, true>(out, W, T, work, reps);
    auto bw = [&](float ms) { return bytes / (ms * 1e-3) / 1e12; };
    printf("work=%2d fma/step/state | L0 %.3f ms %.2f TB/s | L0nt %.3f %.2f | L1 %.3f %.2f | L1nt %.3f %.2f | "
           "L2 %.3f %.2f | L2nt %.3f %.2f\n",
           work, t00, bw(t00), t01, bw(t01), t10, bw(t10), t11, bw(t11), t20, bw(t20), t21, bw(t21));
  }
  for (int work : {0, 8, 14}) {
    auto bw = [&](float ms) { return bytes / (ms * 1e-3) / 1e12; };
    float b0 = runbuf<2>(out, W, T, work, reps), t0 = runtiled<2>(out, W, T, work, reps), t1 = runtiled<0>(out, W, T, work, reps);
    printf("work=%2d | rowbuf nt %.3f ms %.2f | tiled nt %.3f %.2f | tiled cached %.3f %.2f TB/s\n", work, b0, bw(b0), t0, bw(t0), t1, bw(t1));
  }
  for (int work : {0, 14}) {
    auto bw = [&](float ms) { return bytes / (ms * 1e-3) / 1e12; };
    float a0 = runbuf<0>(out, W, T, work, reps), a1 = runbuf<1>(out, W, T, work, reps), a2 = runbuf<2>(out, W, T, work, reps);
    float a3 = runbuf<3>(out, W, T, work, reps), a16 = runbuf<16>(out, W, T, work, reps), a17 = runbuf<17>(out, W, T, work, reps);
    float a18 = runbuf<18>(out, W, T, work, reps), a19 = runbuf<19>(out, W, T, work, reps);
    printf("buffer work=%2d | aux0 %.3f ms %.2f | aux1 %.3f %.2f | aux2(nt) %.3f %.2f | aux3 %.3f %.2f | aux16 %.3f %.2f | "
           "aux17 %.3f %.2f | aux18 %.3f %.2f | aux19 %.3f %.2f TB/s\n", work, a0, bw(a0), a1, bw(a1), a2, bw(a2), a3, bw(a3),
           a16, bw(a16), a17, bw(a17), a18, bw(a18), a19, bw(a19));
  }
  CHECK(hipFree(out));
  return 0;
}
