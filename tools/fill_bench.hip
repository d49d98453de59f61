// fill_bench.hip — what write pattern reaches hipMemset's streaming-write rate?
// (diagnostic for DESIGN.md §6: hipMemset of the C1 trajectory size runs 6.7 TB/s, our
// linear fills 4.6–5.2 and the C1 kernel's [T][S][W] row stores 5.4–5.5 TB/s)
//
// Writes B = 1000 x 4 x 65 536 doubles (2.1 GB, the C1 trajectory) with:
//   chunk<C,AUX>:   one wave per C KiB contiguous chunk, each store instruction one
//                   contiguous KiB (64 lanes x 16 B), no grid stride
//   stride<U,AUX>:  grid-stride loop, U independent 16-B stores per iteration, G blocks
//   rows<AUX>:      the C1 pattern ([T][S][W] 8-B row stores, one lane per walker)
//   memset:         hipMemsetAsync / hipMemsetD32Async
// AUX is the buffer-store cache-policy immediate (0 plain, 2 nt, 16 sc1, 18 nt+sc1).
// Timing as bench.py: >= 60 ms of warm-up launches, then K back-to-back launches between
// two events.  One JSON line per case.
//
//   hipcc -O3 --offload-arch=gfx950 -o /tmp/fb tools/fill_bench.hip && /tmp/fb
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1);} } while (0)
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));

__device__ inline __amdgpu_buffer_rsrc_t rsrc_of(void* p, unsigned bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(p, 0, bytes, 0x00020000);
}

template <int C, int AUX>
__global__ void __launch_bounds__(256) k_chunk(double* out, unsigned bytes) {
  const unsigned wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const unsigned lane = threadIdx.x & 63;
  const unsigned base = wave * (unsigned)C * 1024u;
  if (base >= bytes) return;
  const __amdgpu_buffer_rsrc_t r = rsrc_of(out, bytes);
  u32x4 v = {lane, wave, 1u, 2u};
#pragma unroll
  for (int c = 0; c < C; ++c)
    __builtin_amdgcn_raw_buffer_store_b128(v, r, base + (unsigned)c * 1024u + lane * 16u, 0, AUX);
}

template <int U, int AUX>
__global__ void __launch_bounds__(256) k_stride(double* out, unsigned bytes) {
  const __amdgpu_buffer_rsrc_t r = rsrc_of(out, bytes);
  const unsigned n16 = bytes / 16u;
  const unsigned stride = gridDim.x * blockDim.x;
  u32x4 v = {threadIdx.x, blockIdx.x, 1u, 2u};
  for (unsigned i = blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += U * stride) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const unsigned j = i + (unsigned)u * stride;
      if (j < n16) __builtin_amdgcn_raw_buffer_store_b128(v, r, j * 16u, 0, AUX);
    }
  }
}

template <int AUX>
__global__ void __launch_bounds__(256) k_rows(double* out, int W, int T) {
  constexpr int S = 4;
  const int w = blockIdx.x * blockDim.x + threadIdx.x;
  if (w >= W) return;
  const unsigned off = (unsigned)w * 8u;
  double y = 1.0 + 1e-9 * w;
  for (int t = 0; t < T; ++t) {
    const __amdgpu_buffer_rsrc_t r = rsrc_of(out + (long)t * S * W, (unsigned)(S * W * 8));
#pragma unroll
    for (int s = 0; s < S; ++s)
      __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, y + s), r, off, (unsigned)(s * W * 8), AUX);
    y += 1e-12;
  }
}

// the rows pattern with the engine's XCD-contiguous block order (REMAP) and/or a
// per-wave rotation of the state order (ROT: wave k stores s = (k + j) mod 4 as its j-th)
template <int REMAP, int ROT, int S = 4>
__global__ void __launch_bounds__(256) k_rows_v(double* out, int W, int T) {
  long b = blockIdx.x;
  if (REMAP) {
    const long G = gridDim.x, q = G >> 3, rr = G & 7, x = b & 7, j = b >> 3;
    b = x * q + (x < rr ? x : rr) + j;
  }
  const int w = (int)(b * blockDim.x + threadIdx.x);
  if (w >= W) return;
  const unsigned off = (unsigned)w * 8u;
  const int rot = ROT ? (w >> 6) & 3 : 0;
  double y = 1.0 + 1e-9 * w;
  for (int t = 0; t < T; ++t) {
    const __amdgpu_buffer_rsrc_t r = rsrc_of(out + (long)t * S * W, (unsigned)(S * W * 8));
#pragma unroll
    for (int j = 0; j < S; ++j) {
      const int s = (j + rot) % S;
      __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, y + s), r, off, (unsigned)(s * W * 8), 18);
    }
    y += 1e-12;
  }
}

// rows_remap with the whole grid held in step: every K steps each workgroup checks in at
// a device-scope counter and waits (bounded: at most 4000 short sleeps) until all have
template <int K>
__global__ void __launch_bounds__(256) k_rows_sync(double* out, int W, int T, unsigned* bar) {
  constexpr int S = 4;
  long b = blockIdx.x;
  {
    const long G = gridDim.x, q = G >> 3, rr = G & 7, x = b & 7, j = b >> 3;
    b = x * q + (x < rr ? x : rr) + j;
  }
  const int w = (int)(b * blockDim.x + threadIdx.x);
  const unsigned off = (unsigned)w * 8u;
  double y = 1.0 + 1e-9 * w;
  for (int t = 0; t < T; ++t) {
    if (t % K == 0 && t > 0) {
      if (threadIdx.x == 0) {
        unsigned* c = bar + t / K;
        __hip_atomic_fetch_add(c, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        for (int it = 0; it < 4000; ++it) {
          if (__hip_atomic_load(c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= gridDim.x) break;
          __builtin_amdgcn_s_sleep(1);
        }
      }
      __syncthreads();
    }
    const __amdgpu_buffer_rsrc_t r = rsrc_of(out + (long)t * S * W, (unsigned)(S * W * 8));
#pragma unroll
    for (int s = 0; s < S; ++s)
      __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, y + s), r, off, (unsigned)(s * W * 8), 18);
    y += 1e-12;
  }
}

// n_waves long-lived waves; at step t wave i writes the PIECE-byte run at
// (t * n_waves + i) * PIECE, so every step the chip writes one contiguous region
template <int PIECE>
__global__ void __launch_bounds__(256) k_stream(double* out, unsigned bytes) {
  const unsigned wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const unsigned nw = (gridDim.x * blockDim.x) >> 6;
  const unsigned lane = threadIdx.x & 63;
  const unsigned steps = bytes / (nw * PIECE);
  const __amdgpu_buffer_rsrc_t r = rsrc_of(out, bytes);
  u32x4 v = {lane, wave, 1u, 2u};
  for (unsigned t = 0; t < steps; ++t) {
    const unsigned base = (t * nw + wave) * PIECE + lane * 16u;
#pragma unroll
    for (int k = 0; k < PIECE / 1024; ++k) __builtin_amdgcn_raw_buffer_store_b128(v, r, base + k * 1024u, 0, 18);
    v.z += 1u;
  }
}

// [T][S][W] with 1-KiB store instructions: waves 2k and 2k+1 own walkers
// [128k, 128k+128); each step wave 2k stores states 0,1 and wave 2k+1 states 2,3 of all
// 128 (16 B = two walkers per lane); XCD-contiguous block order
__global__ void __launch_bounds__(256) k_rows_pair(double* out, int W, int T) {
  constexpr int S = 4;
  long b = blockIdx.x;
  {
    const long G = gridDim.x, q = G >> 3, rr = G & 7, x = b & 7, j = b >> 3;
    b = x * q + (x < rr ? x : rr) + j;
  }
  const int wave = (int)(b * 4 + (threadIdx.x >> 6));
  const int lane = threadIdx.x & 63;
  const unsigned off = (unsigned)((wave >> 1) * 128 + 2 * lane) * 8u;
  const int s0 = (wave & 1) * 2;
  u32x4 v = {(unsigned)lane, (unsigned)wave, 1u, 2u};
  for (int t = 0; t < T; ++t) {
    const __amdgpu_buffer_rsrc_t r = rsrc_of(out + (long)t * S * W, (unsigned)(S * W * 8));
    __builtin_amdgcn_raw_buffer_store_b128(v, r, off, (unsigned)(s0 * W * 8), 18);
    __builtin_amdgcn_raw_buffer_store_b128(v, r, off, (unsigned)((s0 + 1) * W * 8), 18);
    v.z += 1u;
  }
}

// rows_remap with XCD chunks of C blocks (C = 1: dispatch order, C = G/8: the engine's
// contiguous ranges) and a padded state stride LD = W + PAD walkers (row stride S * LD)
__global__ void __launch_bounds__(256) k_rows_gp(double* out, int W, int T, int C, int PAD, int R = 0) {
  constexpr int S = 4;
  const long b0 = blockIdx.x, x = (b0 + R) & 7, j = b0 >> 3;
  const long b = ((j / C) * 8 + x) * C + (j % C);
  const int w = (int)(b * blockDim.x + threadIdx.x);
  const long LD = (long)W + PAD;
  const unsigned off = (unsigned)w * 8u;
  double y = 1.0 + 1e-9 * w;
  for (int t = 0; t < T; ++t) {
    const __amdgpu_buffer_rsrc_t r = rsrc_of(out + (long)t * S * LD, (unsigned)(S * LD * 8));
#pragma unroll
    for (int s = 0; s < S; ++s)
      __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, y + s), r, off, (unsigned)(s * LD * 8), 18);
    y += 1e-12;
  }
}

// memset-like: block b writes the 4 KiB run number (b/8)*8 + ((b + R) mod 8), one KiB per wave
__global__ void __launch_bounds__(256) k_chunk_rot(double* out, unsigned bytes, int R) {
  const unsigned b = blockIdx.x;
  const unsigned run = (b >> 3) * 8u + ((b + (unsigned)R) & 7u);
  const unsigned lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const unsigned off = run * 4096u + wave * 1024u + lane * 16u;
  if (off >= bytes) return;
  const __amdgpu_buffer_rsrc_t r = rsrc_of(out, bytes);
  u32x4 v = {lane, b, 1u, 2u};
  __builtin_amdgcn_raw_buffer_store_b128(v, r, off, 0, 18);
}

// [T][W][S]-like: per step each wave writes one contiguous 2 KiB run (two 1-KiB stores)
__global__ void __launch_bounds__(256) k_rows_tws(double* out, int W, int T) {
  constexpr int S = 4;
  const int wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  if (wave * 64 >= W) return;
  u32x4 v = {(unsigned)lane, (unsigned)wave, 1u, 2u};
  for (int t = 0; t < T; ++t) {
    const __amdgpu_buffer_rsrc_t r = rsrc_of(out + (long)t * S * W, (unsigned)(S * W * 8));
    const unsigned base = (unsigned)wave * 2048u + (unsigned)lane * 16u;
    __builtin_amdgcn_raw_buffer_store_b128(v, r, base, 0, 18);
    __builtin_amdgcn_raw_buffer_store_b128(v, r, base + 1024u, 0, 18);
    v.z += 1u;
  }
}

// one KiB per wave like chunk<1>, but the waves take the KiBs in a scattered order
__global__ void __launch_bounds__(256) k_chunk_perm(double* out, unsigned bytes, unsigned mult) {
  const unsigned n = bytes / 1024u;
  const unsigned wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const unsigned lane = threadIdx.x & 63;
  if (wave >= n) return;
  const unsigned c = (unsigned)(((unsigned long long)wave * mult) % n);
  const __amdgpu_buffer_rsrc_t r = rsrc_of(out, bytes);
  u32x4 v = {lane, wave, 1u, 2u};
  __builtin_amdgcn_raw_buffer_store_b128(v, r, c * 1024u + lane * 16u, 0, 18);
}

template <class F>
double b2b_ms(F launch) {
  auto t0 = std::chrono::steady_clock::now();
  do {
    launch();
    CHECK(hipDeviceSynchronize());
  } while (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() < 0.06);
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  const int K = 20;
  CHECK(hipEventRecord(a));
  for (int k = 0; k < K; ++k) launch();
  CHECK(hipEventRecord(b));
  CHECK(hipEventSynchronize(b));
  float ms;
  CHECK(hipEventElapsedTime(&ms, a, b));
  CHECK(hipEventDestroy(a));
  CHECK(hipEventDestroy(b));
  return ms / K;
}

static double g_bytes;
static void report(const char* name, int p1, int p2, double ms) {
  printf("{\"case\": \"%s\", \"p1\": %d, \"p2\": %d, \"ms\": %.4f, \"TBps\": %.3f}\n", name, p1, p2, ms,
         g_bytes / (ms * 1e-3) / 1e12);
  fflush(stdout);
}

template <int C, int AUX>
void chunk(double* out, unsigned bytes) {
  const unsigned waves = bytes / (C * 1024u);
  const dim3 grid((waves * 64u + 255u) / 256u);
  report("chunk", C, AUX, b2b_ms([&] { hipLaunchKernelGGL((k_chunk<C, AUX>), grid, dim3(256), 0, 0, out, bytes); }));
}

template <int U, int AUX>
void stride(double* out, unsigned bytes, int blocks) {
  report(U == 1 ? "stride_u1" : (U == 4 ? "stride_u4" : "stride_u"), blocks, AUX,
         b2b_ms([&] { hipLaunchKernelGGL((k_stride<U, AUX>), dim3(blocks), dim3(256), 0, 0, out, bytes); }));
}

int main() {
  const int W = 65536, T = 1000, S = 4;
  const size_t bytes = (size_t)T * S * W * 8;
  g_bytes = (double)bytes;
  double* out;
  CHECK(hipMalloc(&out, bytes + (size_t)T * S * 4096 * 8));  // room for padded row strides
  if (getenv("FB_ROWS")) {
    for (int rep = 0; rep < 3; ++rep) {
      const dim3 g(W / 256), b(256);
      report("rows", 18, 0, b2b_ms([&] { hipLaunchKernelGGL(k_rows<18>, g, b, 0, 0, out, W, T); }));
      report("rows_remap", 1, 0, b2b_ms([&] { hipLaunchKernelGGL((k_rows_v<1, 0>), g, b, 0, 0, out, W, T); }));
      report("rows_rot", 0, 1, b2b_ms([&] { hipLaunchKernelGGL((k_rows_v<0, 1>), g, b, 0, 0, out, W, T); }));
      report("rows_remap_rot", 1, 1, b2b_ms([&] { hipLaunchKernelGGL((k_rows_v<1, 1>), g, b, 0, 0, out, W, T); }));
      report("rows_tws", 0, 0, b2b_ms([&] { hipLaunchKernelGGL(k_rows_tws, g, b, 0, 0, out, W, T); }));
      report("rows_s1_4w", 0, 0, b2b_ms([&] { hipLaunchKernelGGL((k_rows_v<1, 0, 1>), dim3(W / 64), b, 0, 0, out, 4 * W, T); }));
      for (int rot = 0; rot < 8; ++rot) {
        report("rows_c2_rot", rot, 0, b2b_ms([&] { hipLaunchKernelGGL(k_rows_gp, g, b, 0, 0, out, W, T, 2, 0, rot); }));
        report("chunk_rot", rot, 0, b2b_ms([&] { hipLaunchKernelGGL(k_chunk_rot, dim3((unsigned)(bytes / 4096)), b, 0, 0, out, (unsigned)bytes, rot); }));
      }
      for (int c : {1, 2, 4, 8, 16, 32})
        report("rows_gran", c, 0, b2b_ms([&] { hipLaunchKernelGGL(k_rows_gp, g, b, 0, 0, out, W, T, c, 0); }));
      for (int pad : {64, 256, 512, 1024, 4096}) {
        g_bytes = (double)bytes;  // algorithmic bytes; the padded rows write the same count
        report("rows_pad", pad, 0, b2b_ms([&] { hipLaunchKernelGGL(k_rows_gp, g, b, 0, 0, out, W, T, W / 256 / 8, pad); }));
      }
      report("rows_pair", 0, 0, b2b_ms([&] { hipLaunchKernelGGL(k_rows_pair, g, b, 0, 0, out, W, T); }));
      for (int m : {1, 2, 4, 8, 16}) {
        const dim3 gs(256 * m);  // 4 waves per block: 4m waves per CU
        const double nw = 1024.0 * m;
        g_bytes = (double)(size_t)(bytes / (nw * 1024)) * nw * 1024;  // bytes actually written
        report("stream_1k", 4 * m, 0, b2b_ms([&] { hipLaunchKernelGGL(k_stream<1024>, gs, b, 0, 0, out, (unsigned)bytes); }));
        g_bytes = (double)(size_t)(bytes / (nw * 2048)) * nw * 2048;
        report("stream_2k", 4 * m, 0, b2b_ms([&] { hipLaunchKernelGGL(k_stream<2048>, gs, b, 0, 0, out, (unsigned)bytes); }));
        g_bytes = (double)bytes;
      }
      unsigned* bar;
      CHECK(hipMalloc(&bar, 4 * (T + 1)));
      auto sync = [&](auto kern, int K) {
        report("rows_sync", K, 0, b2b_ms([&] {
          CHECK(hipMemsetAsync(bar, 0, 4 * (T + 1), 0));
          hipLaunchKernelGGL(kern, g, b, 0, 0, out, W, T, bar);
        }));
      };
      sync(k_rows_sync<2>, 2);
      sync(k_rows_sync<8>, 8);
      sync(k_rows_sync<32>, 32);
      sync(k_rows_sync<128>, 128);
      sync(k_rows_sync<2000>, 2000);
      CHECK(hipFree(bar));
      const unsigned n = (unsigned)(bytes / 1024);
      const dim3 gc((n * 64u + 255u) / 256u);
      report("chunk_perm", 1, 0, b2b_ms([&] { hipLaunchKernelGGL(k_chunk_perm, gc, b, 0, 0, out, (unsigned)bytes, 1u); }));
      report("chunk_perm", 257, 0, b2b_ms([&] { hipLaunchKernelGGL(k_chunk_perm, gc, b, 0, 0, out, (unsigned)bytes, 257u); }));
      report("chunk_perm", 1000003, 0, b2b_ms([&] { hipLaunchKernelGGL(k_chunk_perm, gc, b, 0, 0, out, (unsigned)bytes, 1000003u); }));
    }
    CHECK(hipFree(out));
    return 0;
  }
  for (int rep = 0; rep < 2; ++rep) {
    report("memset", 0, 0, b2b_ms([&] { CHECK(hipMemsetAsync(out, 0x3F, bytes, 0)); }));
    report("memsetD32", 0, 0, b2b_ms([&] { CHECK(hipMemsetD32Async((hipDeviceptr_t)out, 0x3F3F3F3F, bytes / 4, 0)); }));
    report("rows", 18, 0, b2b_ms([&] { hipLaunchKernelGGL(k_rows<18>, dim3(W / 256), dim3(256), 0, 0, out, W, T); }));
    report("rows", 0, 0, b2b_ms([&] { hipLaunchKernelGGL(k_rows<0>, dim3(W / 256), dim3(256), 0, 0, out, W, T); }));
    chunk<1, 0>(out, (unsigned)bytes);
    chunk<1, 2>(out, (unsigned)bytes);
    chunk<1, 18>(out, (unsigned)bytes);
    chunk<4, 0>(out, (unsigned)bytes);
    chunk<4, 18>(out, (unsigned)bytes);
    chunk<16, 0>(out, (unsigned)bytes);
    chunk<16, 18>(out, (unsigned)bytes);
    chunk<64, 0>(out, (unsigned)bytes);
    for (int blocks : {1024, 2048, 4096, 8192, 16384}) {
      stride<1, 0>(out, (unsigned)bytes, blocks);
      stride<4, 0>(out, (unsigned)bytes, blocks);
      stride<4, 18>(out, (unsigned)bytes, blocks);
    }
  }
  CHECK(hipFree(out));
  return 0;
}
