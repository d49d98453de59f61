// store_waves_bench.hip — does the [T][S][W] trajectory store stream run faster when the
// same bytes are issued by more waves per CU?  (diagnostic for DESIGN.md §6)
//
// Pure stores (no arithmetic) of T x S x W doubles, W = 65 536, S = 4, T = 1000, through
// per-row buffer descriptors with the non-temporal bit, as the engine stores:
//   split 1: one lane per walker stores all S states per step   (4 waves / CU)
//   split 2: two lanes per walker, each stores S/2 states        (8 waves / CU)
//   split 4: four lanes per walker, each stores one state        (16 waves / CU)
// Same bytes, same number of store instructions in total; one JSON line per case with
// the median kernel time and TB/s over back-to-back launches.
//
//   hipcc -O3 --offload-arch=gfx950 -o /tmp/swb tools/store_waves_bench.hip && /tmp/swb
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1);} } while (0)
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));

template <int SPLIT>
__global__ void __launch_bounds__(256) k_store(double* out, int W, int T) {
  constexpr int S = 4, PER = S / SPLIT;
  // lanes of SPLIT consecutive waves share the same 64 walkers: wave j of a group stores
  // states [j*PER, (j+1)*PER) (whole waves, so every store is one 512-B run)
  const int gwave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  const int part = gwave % SPLIT;
  const int w = (gwave / SPLIT) * 64 + lane;
  if (w >= W) return;
  const uint32_t off = (uint32_t)w * 8u;
  double y = 1.0 + 1e-9 * w;
  for (int t = 0; t < T; ++t) {
    const __amdgpu_buffer_rsrc_t rsrc =
        __builtin_amdgcn_make_buffer_rsrc((void*)(out + (long)t * S * W), 0, (unsigned)(S * W * 8), 0x00020000);
#pragma unroll
    for (int k = 0; k < PER; ++k) {
      const int s = part * PER + k;
      __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, y + s), rsrc, off, (unsigned)(s * W * 8), 2);
    }
    y += 1e-12;
  }
}

// linear fill of the same bytes: 16 B per lane, consecutive lanes consecutive addresses,
// grid-stride — the chip's streaming-write ceiling for comparison.  MODE 0: NT stores of
// non-zero data; 1: plain stores of non-zero data; 2: plain stores of zeros; 3: NT zeros
template <int MODE>
__global__ void __launch_bounds__(256) k_fill(double* out, long n2) {
  typedef double d2v __attribute__((ext_vector_type(2)));
  d2v* p = reinterpret_cast<d2v*>(out);
  const long stride = (long)gridDim.x * blockDim.x;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n2; i += stride) {
    d2v v = (MODE >= 2) ? d2v{0.0, 0.0} : d2v{1.0 + i, 2.0};
    if (MODE == 0 || MODE == 3) __builtin_nontemporal_store(v, p + i);
    else p[i] = v;
  }
}

template <class F>
float median_ms(F launch) {
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  std::vector<float> ms;
  for (int r = 0; r < 13; ++r) {  // back to back, one event pair per launch
    CHECK(hipEventRecord(a));
    launch();
    CHECK(hipEventRecord(b));
    CHECK(hipEventSynchronize(b));
    float x;
    CHECK(hipEventElapsedTime(&x, a, b));
    if (r >= 3) ms.push_back(x);
  }
  std::sort(ms.begin(), ms.end());
  CHECK(hipEventDestroy(a));
  CHECK(hipEventDestroy(b));
  return ms[ms.size() / 2];
}

template <int SPLIT>
void run(double* out, int W, int T) {
  const int threads = W * SPLIT;
  const dim3 grid((threads + 255) / 256), block(256);
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  std::vector<float> ms;
  for (int r = 0; r < 13; ++r) {
    CHECK(hipEventRecord(a));
    hipLaunchKernelGGL(k_store<SPLIT>, grid, block, 0, 0, out, W, T);
    CHECK(hipEventRecord(b));
    CHECK(hipEventSynchronize(b));
    float x;
    CHECK(hipEventElapsedTime(&x, a, b));
    if (r >= 3) ms.push_back(x);
  }
  std::sort(ms.begin(), ms.end());
  const double med = ms[ms.size() / 2];
  const double bytes = (double)T * 4 * W * 8;
  printf("{\"split\": %d, \"waves_per_cu\": %d, \"kernel_ms\": %.4f, \"TBps\": %.3f}\n", SPLIT,
         threads / 64 / 256, med, bytes / (med * 1e-3) / 1e12);
  CHECK(hipEventDestroy(a));
  CHECK(hipEventDestroy(b));
}

int main() {
  const int W = 65536, T = 1000;
  double* out;
  CHECK(hipMalloc(&out, sizeof(double) * (size_t)T * 4 * W));
  for (int rep = 0; rep < 2; ++rep) {
    run<1>(out, W, T);
    run<2>(out, W, T);
    run<4>(out, W, T);
  }
  const double bytes = (double)T * 4 * W * 8;
  const long n2 = (long)T * 4 * W / 2;
  for (int mode = 0; mode < 4; ++mode)
    for (int blocks : {1024, 4096}) {
      const float ms = median_ms([&] {
        if (mode == 0) hipLaunchKernelGGL(k_fill<0>, dim3(blocks), dim3(256), 0, 0, out, n2);
        if (mode == 1) hipLaunchKernelGGL(k_fill<1>, dim3(blocks), dim3(256), 0, 0, out, n2);
        if (mode == 2) hipLaunchKernelGGL(k_fill<2>, dim3(blocks), dim3(256), 0, 0, out, n2);
        if (mode == 3) hipLaunchKernelGGL(k_fill<3>, dim3(blocks), dim3(256), 0, 0, out, n2);
      });
      printf("{\"fill_mode\": %d, \"blocks\": %d, \"kernel_ms\": %.4f, \"TBps\": %.3f}\n", mode, blocks, ms,
             bytes / (ms * 1e-3) / 1e12);
    }
  for (int byte : {0, 0x3F}) {
    const float ms = median_ms([&] { CHECK(hipMemsetAsync(out, byte, (size_t)bytes, 0)); });
    printf("{\"memset_byte\": %d, \"ms\": %.4f, \"TBps\": %.3f}\n", byte, ms, bytes / (ms * 1e-3) / 1e12);
  }
  CHECK(hipFree(out));
  return 0;
}
