// capi.hip — extern "C" implementation of include/odelib_amd.h.
//
// Host-side runtime of the engine: context (device, stream, events, scratch),
// the device copy of the fit problem, the (model, S) → kernel dispatch table,
// and the chunked Metropolis–Hastings driver.  Nothing here computes on the CPU:
// every number the API returns was produced by a kernel in ode_kernels.cuh.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <memory>
#include <mutex>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <new>
#include <string>
#include <vector>

#include "../../include/odelib_amd.h"
#include "dispatch.h"
#include "numpy_rng.cuh"

OE_DECLARE_ENTRY(zero_i);
OE_DECLARE_ENTRY(one_i);
OE_DECLARE_ENTRY(two_i);
OE_DECLARE_ENTRY(chain4);
OE_DECLARE_ENTRY(chain5);
OE_DECLARE_ENTRY(chain6);
OE_DECLARE_ENTRY(chain8);
OE_DECLARE_ENTRY(chain10);
OE_DECLARE_ENTRY(chain12);
OE_DECLARE_ENTRY(chain16);
OE_DECLARE_ENTRY(chain20);
OE_DECLARE_ENTRY(chain24);
OE_DECLARE_ENTRY(chain32);

namespace {

using namespace oe;

const std::vector<Entry>& registry() {
  static const std::vector<Entry> r = {
      oe_entry_zero_i(), oe_entry_one_i(),  oe_entry_two_i(),  oe_entry_chain4(),
      oe_entry_chain5(), oe_entry_chain6(), oe_entry_chain8(), oe_entry_chain10(),
      oe_entry_chain12(), oe_entry_chain16(), oe_entry_chain20(), oe_entry_chain24(),
      oe_entry_chain32(),
  };
  return r;
}

const Entry* find_entry(int32_t model_id, int32_t S) {
  for (const Entry& e : registry()) {
    if (e.model_id != model_id) continue;
    if (model_id == OE_MODEL_CHAIN && e.S != S) continue;
    if (model_id != OE_MODEL_CHAIN && S != 0 && e.S != S) return nullptr;
    return &e;
  }
  return nullptr;
}

constexpr int kBlock = 256;
// per-lane store offsets are 32-bit byte offsets (w*8) into a [..][W] row
constexpr int64_t kMaxWalkers = int64_t(1) << 29;

}  // namespace

struct CustomModel {
  Entry entry{};
  RtcModule rtc;
  std::string body;
};

struct oe_ctx {
  std::vector<std::unique_ptr<CustomModel>> custom;  // user RHS modules (model_id = OE_MODEL_CUSTOM + k)
  std::string arch;
  int n_cu = 256;
  int device = 0;
  hipStream_t own_stream = nullptr;
  hipStream_t stream = nullptr;
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  bool timed = false;
  std::string err;
  // problem
  bool has_problem = false;
  const Entry* entry = nullptr;
  DevProblem dp{};
  int32_t method = 0;
  double* d_times = nullptr;
  double* d_rk4 = nullptr;
  Obs* d_obs = nullptr;
  // scratch
  void* scratch = nullptr;
  size_t scratch_bytes = 0;
  void* draws = nullptr;  // philox / numpy proposal draws of one MH chunk
  size_t draws_bytes = 0;
  void* np_state = nullptr;  // numpy legacy RandomState per chain (key [W][624], pos, gauss, has)
  size_t np_state_bytes = 0;
  // numpy draws of MH chunk j + 1 run on a side stream while chunk j's MH kernels run (one
  // 64-chain block per CU beside them), into the other half of `draws`
  hipStream_t np_stream = nullptr;
  hipEvent_t ev_np[2] = {nullptr, nullptr};  // chunk j's draws written (side stream)
  hipEvent_t ev_mh[2] = {nullptr, nullptr};  // chunk j's MH kernels done with buffer j & 1 (main)
  int32_t* stiff_buf = nullptr;  // wide-model stiff redo: [count][list W][status W]
  size_t stiff_cap = 0;          // walkers it holds
  void* tree = nullptr;          // speculative MH rounds: node proposals and results
  size_t tree_bytes = 0;
  void* obs_buf = nullptr;       // MH 'auto' / 'bdf' (S <= 8): the per-lane BDF pass's deferred
  size_t obs_bytes = 0;          // observations, [n_obs][lanes] (DevProblem::obs_c, bdf.cuh)
  int32_t last_mh_depth = 0;     // iterations per round of the last oe_mh_run (0: sequential)
  // 'auto' integrate through the hand-over queue (ode_kernels.cuh HandQ): the BDF kernel's
  // stream, the events ordering it between the queue's reset and the caller's stream, and the
  // queue [(S + 5) doubles + 6 int32][cap] + 16 int32 of control
  hipStream_t hq_stream = nullptr;
  hipEvent_t ev_hq[2] = {nullptr, nullptr};
  void* hq_buf = nullptr;
  int64_t hq_cap = 0;
  int32_t hq_S = 0;
  int32_t hq_epoch = 0;
  int32_t* hq_ctl = nullptr;  // the last launch's control words (ctl[3]: a BDF wave timed out)
  // OE_TUNE: the RK4 trajectory kernel chosen per shape, with what was measured (built-in
  // models: in a process-wide table shared by every context on the device; hipRTC models here)
  struct Tuned {
    int device;
    const Entry* e;
    int64_t W;
    int32_t T, substeps;
    uint32_t mode;  // nt | xcd flags | OE_HALF_WAVES (the default kernel a candidate must beat)
    int32_t variant;
    double ms[OE_KERNEL_COUNT - 1];
  };
  std::vector<Tuned> tuned;
  int32_t last_variant = -1;
  Tuned last_tune{};          // the choice of the last oe_integrate, if it was tuned
  bool has_last_tune = false;
};

namespace {

thread_local std::string g_err;  // errors of context-free calls (oe_rtc_check)

int fail(oe_ctx* c, int code, const std::string& msg) {
  if (c) c->err = msg;
  else g_err = msg;
  return code;
}

#define OE_HIP(ctx, expr)                                                              \
  do {                                                                                 \
    hipError_t e_ = (expr);                                                            \
    if (e_ != hipSuccess)                                                              \
      return fail(ctx, OE_ERR_HIP, std::string(#expr) + ": " + hipGetErrorString(e_)); \
  } while (0)

// ids of the walkers an 'auto' pass marked ST_STIFF (any order: each is redone on its own)
__global__ void k_stiff_list(const int32_t* __restrict__ status, int64_t W, int32_t* __restrict__ list,
                             int32_t* __restrict__ count) {
  const int64_t w = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (w < W && (status[w] & ST_STIFF)) list[atomicAdd(count, 1)] = (int32_t)w;
}

int ensure_stiff_buf(oe_ctx* c, int64_t W) {
  if ((int64_t)c->stiff_cap >= W) return OE_OK;
  if (c->stiff_buf) {
    OE_HIP(c, hipStreamSynchronize(c->stream));
    OE_HIP(c, hipFree(c->stiff_buf));
    c->stiff_buf = nullptr;
    c->stiff_cap = 0;
  }
  OE_HIP(c, hipMalloc(&c->stiff_buf, sizeof(int32_t) * (size_t)(2 * W + 64)));
  c->stiff_cap = (size_t)W;
  return OE_OK;
}

int ensure_scratch(oe_ctx* c, size_t bytes) {
  if (c->scratch_bytes >= bytes) return OE_OK;
  if (c->scratch) {
    OE_HIP(c, hipStreamSynchronize(c->stream));
    OE_HIP(c, hipFree(c->scratch));
    c->scratch = nullptr;
    c->scratch_bytes = 0;
  }
  OE_HIP(c, hipMalloc(&c->scratch, bytes));
  c->scratch_bytes = bytes;
  return OE_OK;
}

int ensure_obs_buf(oe_ctx* c, size_t bytes) {
  if (c->obs_bytes >= bytes) return OE_OK;
  if (c->obs_buf) {
    OE_HIP(c, hipStreamSynchronize(c->stream));
    OE_HIP(c, hipFree(c->obs_buf));
    c->obs_buf = nullptr;
    c->obs_bytes = 0;
  }
  OE_HIP(c, hipMalloc(&c->obs_buf, bytes));
  c->obs_bytes = bytes;
  return OE_OK;
}

// the hand-over queue for W walkers of S states (zeroed: no slot carries a live epoch)
int ensure_hq(oe_ctx* c, int64_t W, int S, HandQ* q) {
  if (!c->hq_stream) {
    OE_HIP(c, hipStreamCreateWithFlags(&c->hq_stream, hipStreamNonBlocking));
    for (int k = 0; k < 2; ++k) OE_HIP(c, hipEventCreateWithFlags(&c->ev_hq[k], hipEventDisableTiming));
  }
  const auto bytes = [](int64_t cap, int s) { return (size_t)cap * (8 * (size_t)(s + 5) + 4 * 6) + 64; };
  if (c->hq_cap < W || c->hq_S < S) {
    if (c->hq_buf) {
      OE_HIP(c, hipStreamSynchronize(c->stream));
      OE_HIP(c, hipStreamSynchronize(c->hq_stream));
      OE_HIP(c, hipFree(c->hq_buf));
      c->hq_buf = nullptr;
      c->hq_cap = 0;
    }
    OE_HIP(c, hipMalloc(&c->hq_buf, bytes(W, S)));
    OE_HIP(c, hipMemsetAsync(c->hq_buf, 0, bytes(W, S), c->stream));
    c->hq_cap = W;
    c->hq_S = S;
  }
  const int64_t cap = c->hq_cap;
  q->d = static_cast<double*>(c->hq_buf);
  q->n = reinterpret_cast<int32_t*>(q->d + (size_t)(c->hq_S + 5) * cap);
  q->ctl = q->n + 6 * cap;
  q->cap = (int32_t)cap;
  if (++c->hq_epoch <= 0) c->hq_epoch = 1;  // (2^31 launches later: slots of long ago may match)
  q->epoch = c->hq_epoch;
  return OE_OK;
}

int ensure_draws(oe_ctx* c, size_t bytes) {
  if (c->draws_bytes >= bytes) return OE_OK;
  if (c->draws) {
    OE_HIP(c, hipStreamSynchronize(c->stream));
    OE_HIP(c, hipFree(c->draws));
    c->draws = nullptr;
    c->draws_bytes = 0;
  }
  OE_HIP(c, hipMalloc(&c->draws, bytes));
  c->draws_bytes = bytes;
  return OE_OK;
}

int ensure_np_stream(oe_ctx* c) {
  if (c->np_stream) return OE_OK;
  OE_HIP(c, hipStreamCreateWithFlags(&c->np_stream, hipStreamNonBlocking));
  for (int k = 0; k < 2; ++k) {
    OE_HIP(c, hipEventCreateWithFlags(&c->ev_np[k], hipEventDisableTiming));
    OE_HIP(c, hipEventCreateWithFlags(&c->ev_mh[k], hipEventDisableTiming));
  }
  return OE_OK;
}

// per-chain numpy RandomState buffers for W chains
int ensure_np_state(oe_ctx* c, int64_t W, NpState* st) {
  const size_t key_b = sizeof(uint32_t) * (size_t)kMtN * (size_t)W;
  const size_t bytes = key_b + (sizeof(int32_t) * 2 + sizeof(double)) * (size_t)W + 64;
  if (c->np_state_bytes < bytes) {
    if (c->np_state) {
      OE_HIP(c, hipStreamSynchronize(c->stream));
      OE_HIP(c, hipFree(c->np_state));
      c->np_state = nullptr;
      c->np_state_bytes = 0;
    }
    OE_HIP(c, hipMalloc(&c->np_state, bytes));
    c->np_state_bytes = bytes;
  }
  char* b = static_cast<char*>(c->np_state);
  st->key = reinterpret_cast<uint32_t*>(b);
  st->gauss = reinterpret_cast<double*>(b + key_b);
  st->pos = reinterpret_cast<int32_t*>(b + key_b + sizeof(double) * (size_t)W);
  st->has_gauss = st->pos + W;
  return OE_OK;
}

// Switches the calling thread to the context's device for one ABI call and restores the
// caller's device on return: torch (and any other HIP user in the process) reads the same
// thread-current device, so an Engine on device k must not move torch's default device.
struct DeviceGuard {
  int prev = -1;
  hipError_t err = hipSuccess;
  explicit DeviceGuard(int device) {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    if (prev != device) err = hipSetDevice(device);
    else prev = -1;  // already current: nothing to restore
  }
  ~DeviceGuard() {
    if (prev >= 0) (void)hipSetDevice(prev);
  }
  DeviceGuard(const DeviceGuard&) = delete;
  DeviceGuard& operator=(const DeviceGuard&) = delete;
};

#define OE_DEVICE_GUARD(ctx)                                                              \
  DeviceGuard device_guard_((ctx)->device);                                               \
  if (device_guard_.err != hipSuccess)                                                    \
    return fail(ctx, OE_ERR_HIP, std::string("hipSetDevice: ") + hipGetErrorString(device_guard_.err))

// XCD walker runs of the one-lane kernels: 512 consecutive walkers (4 KiB of each state
// row) per XCD in turn (OE_XCD_RUN_WALKERS overrides, for measurements), or one contiguous
// range per XCD, or blockIdx order
int32_t xcd_remap_of(uint32_t flags, const dim3& grid, int64_t per_block) {
  static const int64_t run_walkers = [] {
    const char* v = getenv("OE_XCD_RUN_WALKERS");
    const long n = v ? strtol(v, nullptr, 10) : 0;
    return n > 0 ? (int64_t)n : (int64_t)512;
  }();
  return (flags & OE_NO_XCD_REMAP) ? 0
         : (flags & OE_XCD_RANGES) ? (int32_t)std::max<int64_t>(1, (int64_t)grid.x / 8)
                                   : (int32_t)std::max<int64_t>(1, run_walkers / per_block);
}

// an RK4 trajectory kernel (OE_KERNEL_*) available for this entry and walker count
bool rk4_variant_ok(const Entry* e, int64_t W, int variant, bool nt, uint32_t flags) {
  if (variant == OE_KERNEL_DIRECT || variant == OE_KERNEL_HALF) return true;
  if (variant < OE_KERNEL_PIPE2 || variant > OE_KERNEL_PIPE8X) return false;
  if (variant >= OE_KERNEL_PIPE2X && (flags & (OE_NO_XCD_REMAP | OE_XCD_RANGES))) return false;
  return !e->rtc && W % 2 == 0 && e->rk4_piped[(variant - OE_KERNEL_PIPE2) % 3][nt ? 1 : 0] != nullptr;
}

// one RK4 trajectory launch with the given kernel (same bits for every variant)
hipError_t launch_rk4_traj(oe_ctx* c, const Entry* e, IntegrateArgs ia, int variant, bool nt, uint32_t flags) {
  const int64_t W = ia.W;
  if (variant >= OE_KERNEL_PIPE2) {
    const int pv = (variant - OE_KERNEL_PIPE2) % 3;
    const dim3 grid((unsigned)((W + kPipeWalkers - 1) / kPipeWalkers)), block(256 + 64 * (2 << pv));
    // blockIdx order, or (X) runs of 512 walkers per XCD as the direct kernel's
    ia.xcd_remap = variant >= OE_KERNEL_PIPE2X ? (int32_t)(512 / kPipeWalkers) : 0;
    e->rk4_piped[pv][nt ? 1 : 0](c->dp, ia, grid, block, c->stream);
    return hipGetLastError();
  }
  ia.half = variant == OE_KERNEL_HALF ? 1 : 0;
  const int64_t per_block = ia.half ? kBlock / 2 : kBlock;
  const dim3 grid((unsigned)((W + per_block - 1) / per_block)), block(kBlock);
  ia.xcd_remap = xcd_remap_of(flags, grid, per_block);
  return launch_integrate_entry(e, OE_METHOD_RK4, 1, nt ? 1 : 0, c->dp, ia, grid, block, c->stream);
}

// the process-wide OE_TUNE table of the built-in models (their Entry objects are static)
std::mutex g_tune_mu;
std::vector<oe_ctx::Tuned> g_tuned;

// OE_TUNE: time every available RK4 trajectory kernel for this shape, back to back, after
// the clock has settled under load, and remember the fastest (per device and shape, for the
// process: another context on the device reuses the choice).
int tune_rk4(oe_ctx* c, const Entry* e, const IntegrateArgs& ia, bool nt, uint32_t flags, int dflt,
             oe_ctx::Tuned* out) {
  const uint32_t mode = (nt ? 1u : 0u) | (flags & (OE_NO_XCD_REMAP | OE_XCD_RANGES | OE_HALF_WAVES));
  const bool shared = e->rtc == nullptr;
  auto match = [&](const oe_ctx::Tuned& t) {
    return t.device == c->device && t.e == e && t.W == ia.W && t.T == c->dp.T && t.substeps == c->dp.substeps &&
           t.mode == mode;
  };
  {
    std::lock_guard<std::mutex> lk(g_tune_mu);
    for (const oe_ctx::Tuned& t : shared ? g_tuned : c->tuned)
      if (match(t)) {
        *out = t;
        return OE_OK;
      }
  }
  constexpr int kN = OE_KERNEL_COUNT - 1;
  std::vector<int> cand;
  for (int v = 0; v < kN; ++v)
    if (rk4_variant_ok(e, ia.W, v, nt, flags)) cand.push_back(v);
  // n back-to-back launches timed after one untimed launch of the same kernel: every timed
  // launch then follows a launch of its own kind, as in a series (a launch that ends with
  // part of its output still dirty in the 256 MB MALL pays for it in the next launch, so an
  // isolated or first-after-idle launch flatters the kernels that leave more dirty lines:
  // the piped ones)
  auto batch = [&](int v, int n, float* ms) -> int {
    OE_HIP(c, launch_rk4_traj(c, e, ia, v, nt, flags));
    OE_HIP(c, hipEventRecord(c->ev0, c->stream));
    for (int k = 0; k < n; ++k) OE_HIP(c, launch_rk4_traj(c, e, ia, v, nt, flags));
    OE_HIP(c, hipEventRecord(c->ev1, c->stream));
    OE_HIP(c, hipEventSynchronize(c->ev1));
    OE_HIP(c, hipEventElapsedTime(ms, c->ev0, c->ev1));
    return OE_OK;
  };
  // settle: >= 60 ms of back-to-back launches of the default kernel (the clock and power
  // management take tens of ms to reach the sustained state)
  float ms = 0.f;
  int rc = batch(dflt, 1, &ms);
  if (rc) return rc;
  // launches per measurement: ~15 ms of work, 4..16 launches
  const int per = std::max(4, std::min(16, (int)std::ceil(15.0 / std::max(ms, 1e-3f))));
  // (bounded by a launch count too: a clock that reports no elapsed time must not hang the call)
  double settled = ms;
  for (int n = 0; settled < 60.0 && n < 64; ++n) {
    rc = batch(dflt, per, &ms);
    if (rc) return rc;
    settled += ms;
  }
  oe_ctx::Tuned t{c->device, e, ia.W, c->dp.T, c->dp.substeps, mode, dflt, {}};
  for (int v = 0; v < kN; ++v) t.ms[v] = HUGE_VAL;
  constexpr int kRounds = 3;
  for (int r = 0; r < kRounds; ++r)
    for (size_t j = 0; j < cand.size(); ++j) {
      const int v = cand[(j + r) % cand.size()];  // rotate the order between rounds
      rc = batch(v, per, &ms);
      if (rc) return rc;
      t.ms[v] = std::min(t.ms[v], (double)ms / per);
    }
  int best = dflt;
  for (int v : cand)
    if (t.ms[v] < 0.99 * t.ms[dflt] && t.ms[v] < t.ms[best]) best = v;
  for (int v = 0; v < kN; ++v)
    if (t.ms[v] == HUGE_VAL) t.ms[v] = std::nan("");
  t.variant = best;
  {
    std::lock_guard<std::mutex> lk(g_tune_mu);
    (shared ? g_tuned : c->tuned).push_back(t);
  }
  *out = t;
  return OE_OK;
}

}  // namespace

// numpy legacy RandomState per chain: seeding and one chunk of draws (numpy_rng.cuh)
__global__ void __launch_bounds__(256) k_np_seed(const oe::NpState st, const uint32_t* seeds, int64_t W) {
  const int64_t w = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (w < W) oe::np_seed_lane(st, w, seeds[w]);
}
static dim3 np_grid(int64_t W) { return dim3((unsigned)((W + oe::kNpChainsPerBlock - 1) / oe::kNpChainsPerBlock)); }
__global__ void __launch_bounds__(oe::kNpChainsPerBlock) k_np_draws(const oe::NpDrawArgs d) {
  oe::np_draw_block<oe::kNpChainsPerBlock>(d);
}

// MH proposal draws (philox mode), one lane per (walker, iteration) of the chunk: counter-
// based, so every draw is independent of the others (a few chains no longer draw their
// iterations one after another); see oe::philox_draw_iteration
__global__ void __launch_bounds__(256) k_philox_draws(const oe::DrawArgs d) {
  const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t n_it = d.it1 - d.it0;
  if (g >= d.W * n_it) return;
  const int64_t k = g / d.W;
  oe::philox_draw_iteration(d, g - k * d.W, d.it0 + (int)k);
}

// k_mh_tree's resolution: one lane per chain walks its tree with k_mh's accept test and
// bookkeeping, iteration by iteration, in the reference's arithmetic (Samplers.py:124-153)
__global__ void __launch_bounds__(256) k_mh_resolve(const oe::DevProblem pb, const oe::MHTreeArgs ta, int32_t S) {
  using namespace oe;
  constexpr int kMaxD = 16;  // oe_mh_run caps the depth
  const MHArgs& ma = ta.m;
  const int64_t W = ma.W;
  const int64_t w = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (w >= W) return;
  const int P = pb.P;
  const int PS = P + 5;
  const int D = ta.depth;
  const uint32_t off = (uint32_t)w * 8u;
  double* cur = ma.cur;
  double chi = Row(cur, W).ld(off), rsq = Row(cur + W, W).ld(off), aic = Row(cur + 2 * W, W).ld(off);
  double nacc = Row(cur + 3 * W, W).ld(off);
  // 1. the decisions.  The only loads on the path's dependency chain are the node chis; the
  //    next level's two candidates are loaded before each decision, the uniforms up front.
  //    exp/log inline (the same ocml functions k_mh calls out of line: the same bits).
  double uj[kMaxD], cj[kMaxD], rj[kMaxD], aj[kMaxD], nj[kMaxD];
  int32_t keep[kMaxD];  // node holding the chain's parameters after iteration j (-1: the round's start)
#pragma unroll
  for (int j = 0; j < kMaxD; ++j)
    if (j < D) uj[j] = Row(ma.u + (int64_t)(ma.it0 + j - ma.draw_it0) * W, W).ld(off);
  uint32_t path = 0;
  int32_t last = -1;
  double chin = ta.node_chi[w];
#pragma unroll
  for (int j = 0; j < kMaxD; ++j) {
    if (j >= D) continue;  // (continue, not break: the loop must unroll, the arrays stay in registers)
    const int64_t n = (int64_t)(1u << j) - 1 + path;
    double c0 = 0.0, c1 = 0.0;
    if (j + 1 < D) {
      const int64_t n0 = (int64_t)(2u << j) - 1 + path;
      c0 = ta.node_chi[n0 * W + w];
      c1 = ta.node_chi[(n0 + (int64_t)(1u << j)) * W + w];
    }
    const double lr = exp(chi - chin);
    const double accp = exp(log(lr));
    const bool acc = accp > uj[j];
    if (acc) {
      chi = chin;
      rsq = 1.0 - ta.node_ss[n * W + w] / pb.sstot;
      aic = -2.0 * (-chi) + 2.0 * (double)pb.pnum;
      nacc += 1.0;
      last = (int32_t)n;
    }
    cj[j] = chi;
    rj[j] = rsq;
    aj[j] = aic;
    nj[j] = nacc;
    keep[j] = last;
    path |= (acc ? 1u : 0u) << j;
    chin = acc ? c1 : c0;
  }
  // 2. the sample rows (parameters from the node the chain holds, or from θ, which is
  //    rewritten only after them), then the chain state
#pragma unroll
  for (int j = 0; j < kMaxD; ++j) {
    const int it = ma.it0 + j;
    if (j >= D || it <= ma.burnin) continue;
    const double* src = keep[j] >= 0 ? ta.node_th + (int64_t)keep[j] * P * W : ma.theta;
    double* row = ma.samples + (int64_t)(it - ma.row0) * PS * W;
    for (int q = 0; q < P; ++q) Row(row + (int64_t)q * W, W).st(off, Row(src + (int64_t)q * W, W).ld(off));
    Row(row + (int64_t)P * W, W).st(off, cj[j]);
    Row(row + (int64_t)(P + 1) * W, W).st(off, rj[j]);
    Row(row + (int64_t)(P + 2) * W, W).st(off, aj[j]);
    Row(row + (int64_t)(P + 3) * W, W).st(off, (double)it);
    Row(row + (int64_t)(P + 4) * W, W).st(off, nj[j] / (double)it);
  }
  if (last >= 0) {
    const double* src = ta.node_th + (int64_t)last * P * W;
    for (int q = 0; q < P; ++q) Row(ma.theta + (int64_t)q * W, W).st(off, Row(src + (int64_t)q * W, W).ld(off));
    if (ma.status) ma.status[w] = ta.node_st[(int64_t)last * W + w];
  }
  // linked initial states follow the current parameters (k_mh stores them every iteration:
  // the same final values)
  if (ma.any_walk) {
    const double* src = last >= 0 ? ta.node_th + (int64_t)last * P * W : ma.theta;
    for (int s = 0; s < S; ++s) {
      const int pi = ma.init_param[s];
      if (pi >= 0) Row(ma.y0 + (int64_t)s * W, W).st(off, Row(src + (int64_t)pi * W, W).ld(off));
    }
  }
  Row(cur, W).st(off, chi);
  Row(cur + W, W).st(off, rsq);
  Row(cur + 2 * W, W).st(off, aic);
  Row(cur + 3 * W, W).st(off, nacc);
}

// The same resolution with one wave per chain, for trees of up to 4 095 nodes (depth <= 12):
// the wave loads the chain's node chis into LDS at once, lane 0 walks them (no dependent
// global load per level), then lane j writes iteration j's sample row.  Same arithmetic,
// same outputs as k_mh_resolve.
constexpr int kResolveLdsDepth = 12;
__global__ void __launch_bounds__(64) k_mh_resolve_wave(const oe::DevProblem pb, const oe::MHTreeArgs ta, int32_t S) {
  using namespace oe;
  constexpr int kMaxD = kResolveLdsDepth;
  __shared__ double s_chi[(1 << kMaxD) - 1];
  __shared__ double s_u[kMaxD], s_c[kMaxD], s_r[kMaxD], s_a[kMaxD], s_n[kMaxD];
  __shared__ int32_t s_keep[kMaxD];
  __shared__ int32_t s_last;
  const MHArgs& ma = ta.m;
  const int64_t W = ma.W;
  const int64_t w = blockIdx.x;
  const int t = threadIdx.x;
  const int P = pb.P;
  const int PS = P + 5;
  const int D = ta.depth;
  const int N = (1 << D) - 1;
  const uint32_t off = (uint32_t)w * 8u;
  for (int n = t; n < N; n += 64) s_chi[n] = ta.node_chi[(int64_t)n * W + w];
  if (t < D) s_u[t] = Row(ma.u + (int64_t)(ma.it0 + t - ma.draw_it0) * W, W).ld(off);
  __syncthreads();
  if (t == 0) {
    double* cur = ma.cur;
    double chi = Row(cur, W).ld(off), rsq = Row(cur + W, W).ld(off), aic = Row(cur + 2 * W, W).ld(off);
    double nacc = Row(cur + 3 * W, W).ld(off);
    uint32_t path = 0;
    int32_t last = -1;
    for (int j = 0; j < D; ++j) {
      const int n = (1 << j) - 1 + (int)path;
      const double chin = s_chi[n];
      const double lr = exp(chi - chin);
      const double accp = exp(log(lr));
      const bool acc = accp > s_u[j];
      if (acc) {
        chi = chin;
        rsq = 1.0 - ta.node_ss[(int64_t)n * W + w] / pb.sstot;
        aic = -2.0 * (-chi) + 2.0 * (double)pb.pnum;
        nacc += 1.0;
        last = n;
      }
      s_c[j] = chi;
      s_r[j] = rsq;
      s_a[j] = aic;
      s_n[j] = nacc;
      s_keep[j] = last;
      path |= (acc ? 1u : 0u) << j;
    }
    s_last = last;
    Row(cur, W).st(off, chi);
    Row(cur + W, W).st(off, rsq);
    Row(cur + 2 * W, W).st(off, aic);
    Row(cur + 3 * W, W).st(off, nacc);
    if (last >= 0 && ma.status) ma.status[w] = ta.node_st[(int64_t)last * W + w];
  }
  __syncthreads();
  if (t < D) {  // iteration t's sample row (θ from the node the chain holds, or θ not yet rewritten)
    const int it = ma.it0 + t;
    if (it > ma.burnin) {
      const int k = s_keep[t];
      const double* src = k >= 0 ? ta.node_th + (int64_t)k * P * W : ma.theta;
      double* row = ma.samples + (int64_t)(it - ma.row0) * PS * W;
      for (int q = 0; q < P; ++q) Row(row + (int64_t)q * W, W).st(off, Row(src + (int64_t)q * W, W).ld(off));
      Row(row + (int64_t)P * W, W).st(off, s_c[t]);
      Row(row + (int64_t)(P + 1) * W, W).st(off, s_r[t]);
      Row(row + (int64_t)(P + 2) * W, W).st(off, s_a[t]);
      Row(row + (int64_t)(P + 3) * W, W).st(off, (double)it);
      Row(row + (int64_t)(P + 4) * W, W).st(off, s_n[t] / (double)it);
    }
  }
  __syncthreads();
  if (t == 0) {
    const int32_t last = s_last;
    if (last >= 0) {
      const double* src = ta.node_th + (int64_t)last * P * W;
      for (int q = 0; q < P; ++q) Row(ma.theta + (int64_t)q * W, W).st(off, Row(src + (int64_t)q * W, W).ld(off));
    }
    if (ma.any_walk) {
      const double* src = last >= 0 ? ta.node_th + (int64_t)last * P * W : ma.theta;
      for (int s = 0; s < S; ++s) {
        const int pi = ma.init_param[s];
        if (pi >= 0) Row(ma.y0 + (int64_t)s * W, W).st(off, Row(src + (int64_t)pi * W, W).ld(off));
      }
    }
  }
}

extern "C" {

int oe_abi_version(void) { return OE_ABI_VERSION; }

int oe_model_info(int32_t model_id, int32_t* n_states, int32_t* n_params) {
  if (!n_states || !n_params) return OE_ERR_ARG;
  const Entry* e = find_entry(model_id, *n_states);
  if (!e) return OE_ERR_UNSUPPORTED;
  *n_states = e->S;
  *n_params = e->P;
  return OE_OK;
}

int oe_ctx_create(int32_t device, oe_ctx** out) {
  if (!out) return OE_ERR_ARG;
  *out = nullptr;
  oe_ctx* c = new (std::nothrow) oe_ctx();
  if (!c) return OE_ERR_NOMEM;
  c->device = device;
  int n = 0;
  hipError_t e = hipGetDeviceCount(&n);
  if (e != hipSuccess || device < 0 || device >= n) {
    // keep the context so the caller can read the message
    c->err = std::string("oe_ctx_create: no HIP device ") + std::to_string(device) +
             " (hipGetDeviceCount=" + std::to_string(n) + ", " + hipGetErrorString(e) + ")";
    *out = c;
    return OE_ERR_HIP;
  }
  DeviceGuard dg(device);
  if (dg.err != hipSuccess ||
      hipStreamCreateWithFlags(&c->own_stream, hipStreamNonBlocking) != hipSuccess ||
      hipEventCreate(&c->ev0) != hipSuccess || hipEventCreate(&c->ev1) != hipSuccess) {
    c->err = "oe_ctx_create: HIP initialisation failed";
    *out = c;
    return OE_ERR_HIP;
  }
  c->stream = c->own_stream;
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, device) == hipSuccess) {
    c->arch = prop.gcnArchName;  // e.g. "gfx950:sramecc+:xnack-"
    c->n_cu = prop.multiProcessorCount;
  } else {
    c->arch = "gfx950";
  }
  *out = c;
  return OE_OK;
}

void oe_ctx_destroy(oe_ctx* c) {
  if (!c) return;
  if (c->own_stream) {
    DeviceGuard dg(c->device);
    (void)hipStreamSynchronize(c->stream);
    if (c->d_times) (void)hipFree(c->d_times);
    if (c->d_obs) (void)hipFree(c->d_obs);
    if (c->d_rk4) (void)hipFree(c->d_rk4);
    if (c->scratch) (void)hipFree(c->scratch);
    if (c->obs_buf) (void)hipFree(c->obs_buf);
    if (c->draws) (void)hipFree(c->draws);
    if (c->np_state) (void)hipFree(c->np_state);
    if (c->stiff_buf) (void)hipFree(c->stiff_buf);
    if (c->tree) (void)hipFree(c->tree);
    if (c->hq_stream) {
      (void)hipStreamSynchronize(c->hq_stream);
      (void)hipStreamDestroy(c->hq_stream);
    }
    for (int k = 0; k < 2; ++k)
      if (c->ev_hq[k]) (void)hipEventDestroy(c->ev_hq[k]);
    if (c->hq_buf) (void)hipFree(c->hq_buf);
    if (c->ev0) (void)hipEventDestroy(c->ev0);
    if (c->ev1) (void)hipEventDestroy(c->ev1);
    if (c->np_stream) {
      (void)hipStreamSynchronize(c->np_stream);
      (void)hipStreamDestroy(c->np_stream);
    }
    for (int k = 0; k < 2; ++k) {
      if (c->ev_np[k]) (void)hipEventDestroy(c->ev_np[k]);
      if (c->ev_mh[k]) (void)hipEventDestroy(c->ev_mh[k]);
    }
    for (auto& m : c->custom)
      for (hipModule_t md : {m->rtc.mod, m->rtc.stiff_mod})
        if (md) (void)hipModuleUnload(md);
    (void)hipStreamDestroy(c->own_stream);
  }
  delete c;
}

const char* oe_last_error(const oe_ctx* c) {
  if (c) return c->err.c_str();
  return g_err.empty() ? "null context" : g_err.c_str();
}

int oe_rtc_check(const char* rhs_body, int32_t n_states, int32_t n_params, const char* arch) {
  if (!rhs_body || n_states < 1 || n_states > 64 || n_params < 1 || n_params > 60)
    return fail(nullptr, OE_ERR_ARG, "oe_rtc_check: bad arguments");
  std::string err;
  if (rtc_build(rhs_body, n_states, n_params, arch ? arch : "gfx950", kRtcExplicit, nullptr, err))
    return fail(nullptr, OE_ERR_ARG, err);
  g_err.clear();
  return OE_OK;
}

int oe_model_compile(oe_ctx* c, const char* rhs_body, int32_t n_states, int32_t n_params, int32_t* model_id) {
  if (!c || !c->own_stream) return OE_ERR_STATE;
  if (!rhs_body || !model_id || n_states < 1 || n_states > 64 || n_params < 1 || n_params > 60)
    return fail(c, OE_ERR_ARG, "oe_model_compile: bad arguments");
  for (size_t k = 0; k < c->custom.size(); ++k) {  // cached
    const CustomModel& m = *c->custom[k];
    if (m.body == rhs_body && m.entry.S == n_states && m.entry.P == n_params) {
      *model_id = OE_MODEL_CUSTOM + (int32_t)k;
      return OE_OK;
    }
  }
  OE_DEVICE_GUARD(c);
  auto m = std::make_unique<CustomModel>();
  std::string err;
  if (rtc_build(rhs_body, n_states, n_params, c->arch.c_str(), kRtcExplicit, &m->rtc, err))
    return fail(c, OE_ERR_ARG, err);
  m->body = rhs_body;
  m->entry.model_id = OE_MODEL_CUSTOM + (int32_t)c->custom.size();
  m->entry.S = n_states;
  m->entry.P = n_params;
  m->entry.rtc = &m->rtc;
  *model_id = m->entry.model_id;
  c->custom.push_back(std::move(m));
  return OE_OK;
}

int oe_ctx_set_stream(oe_ctx* c, void* s) {
  if (!c || !c->own_stream) return OE_ERR_STATE;
  c->stream = static_cast<hipStream_t>(s);  // NULL = the null (legacy default) stream
  return OE_OK;
}

int oe_ctx_use_own_stream(oe_ctx* c) {
  if (!c || !c->own_stream) return OE_ERR_STATE;
  c->stream = c->own_stream;
  return OE_OK;
}

int oe_problem_set(oe_ctx* c, const oe_problem* p) {
  if (!c || !c->own_stream) return OE_ERR_STATE;
  if (!p) return fail(c, OE_ERR_ARG, "oe_problem_set: null problem");
  OE_DEVICE_GUARD(c);
  const Entry* e = nullptr;
  CustomModel* cm = nullptr;
  if (p->model_id >= OE_MODEL_CUSTOM) {
    const size_t k = (size_t)(p->model_id - OE_MODEL_CUSTOM);
    if (k < c->custom.size()) {
      cm = c->custom[k].get();
      e = &cm->entry;
    }
  } else {
    e = find_entry(p->model_id, p->n_states);
  }
  if (!e)
    return fail(c, OE_ERR_UNSUPPORTED, "oe_problem_set: model " + std::to_string(p->model_id) +
                                           " with S=" + std::to_string(p->n_states) +
                                           " is not compiled in");
  if (p->n_states != e->S) return fail(c, OE_ERR_ARG, "oe_problem_set: n_states mismatch");
  const int pmax = e->P + (e->S < 4 ? e->S : 4);  // kPmax<M>
  if (p->n_params < e->P || p->n_params > pmax)
    return fail(c, OE_ERR_ARG, "oe_problem_set: n_params must be in [model P, model P + min(S, 4)]");
  if (p->n_times < 2 || !p->times) return fail(c, OE_ERR_ARG, "oe_problem_set: need >= 2 times");
  for (int i = 1; i < p->n_times; ++i)
    if (!(p->times[i] > p->times[i - 1]))
      return fail(c, OE_ERR_ARG, "oe_problem_set: times must be strictly increasing");
  if (p->method < OE_METHOD_RK4 || p->method > OE_METHOD_BDF)
    return fail(c, OE_ERR_ARG, "oe_problem_set: unknown method");
  if (p->method == OE_METHOD_BDF && e->S > kStiffRegS)
    return fail(c, OE_ERR_UNSUPPORTED, "oe_problem_set: bdf needs n_states <= " + std::to_string(kStiffRegS));
  if (p->method == OE_METHOD_AUTO || p->method == OE_METHOD_ROSENBROCK || p->method == OE_METHOD_BDF) {
    if (cm) {  // a user RHS: its stiff kernels are compiled the first time they are asked for
      if (cm->rtc.stiff == 0) {
        std::string err;
        if (rtc_build(cm->body, e->S, e->P, c->arch.c_str(), kRtcStiff, &cm->rtc, err)) {
          cm->rtc.stiff = -1;
          cm->rtc.stiff_err = err;
        }
      }
      if (cm->rtc.stiff != 1) return fail(c, OE_ERR_UNSUPPORTED, "oe_problem_set: " + cm->rtc.stiff_err);
    } else if (e->integrate[p->method][0][0] == nullptr &&
               !(p->method == OE_METHOD_AUTO && e->integrate_hq[0][0][0] != nullptr)) {
      return fail(c, OE_ERR_UNSUPPORTED, "oe_problem_set: the stiff methods (auto, rosenbrock) need n_states <= " +
                                             std::to_string(kStiffMaxS));
    }
  }
  if (p->method == OE_METHOD_RK4 && p->rk4_substeps < 1)
    return fail(c, OE_ERR_ARG, "oe_problem_set: rk4_substeps must be >= 1");
  if (p->method != OE_METHOD_RK4 &&
      (!(p->rtol > 0.0) || !(p->atol >= 0.0) || p->max_steps < 2))
    return fail(c, OE_ERR_ARG, "oe_problem_set: adaptive methods need rtol > 0, atol >= 0, max_steps >= 2");
  if (p->n_obs < 0) return fail(c, OE_ERR_ARG, "oe_problem_set: n_obs < 0");
  if (p->n_obs > 0 && (!p->obs_tidx || !p->obs_mask || !p->obs_log || !p->obs_logsigma || !p->obs_lin))
    return fail(c, OE_ERR_ARG, "oe_problem_set: observation arrays missing");

  std::vector<Obs> obs(p->n_obs);
  const uint64_t valid_mask = (e->S >= 64) ? ~0ull : ((1ull << e->S) - 1ull);
  for (int k = 0; k < p->n_obs; ++k) {
    if (p->obs_tidx[k] < 0 || p->obs_tidx[k] >= p->n_times)
      return fail(c, OE_ERR_ARG, "oe_problem_set: obs_tidx out of range");
    if (p->obs_mask[k] == 0 || (p->obs_mask[k] & ~valid_mask))
      return fail(c, OE_ERR_ARG, "oe_problem_set: obs_mask selects no / unknown states");
    Obs& o = obs[k];
    o.tidx = p->obs_tidx[k];
    o.pad = 0;
    o.mask = p->obs_mask[k];
    o.O = p->obs_log[k];
    const double s = p->obs_logsigma[k];
    o.two_s2 = 2.0 * (s * s);
    o.O_lin = p->obs_lin[k];
  }
  std::stable_sort(obs.begin(), obs.end(), [](const Obs& a, const Obs& b) { return a.tidx < b.tidx; });

  // RK4 per-interval constants: h = (t_i - t_{i-1}) / n, h/2, h/6, t_{i-1}
  // (IEEE-correctly-rounded on host and device alike, so the table is exact)
  const int nsub = p->method == OE_METHOD_RK4 ? p->rk4_substeps : 1;
  std::vector<double> rk4(4 * (size_t)p->n_times);  // + one padding row (the kernel's look-ahead)
  for (int i = 1; i < p->n_times; ++i) {
    const double h = (p->times[i] - p->times[i - 1]) / (double)nsub;
    rk4[4 * (i - 1)] = h;
    rk4[4 * (i - 1) + 1] = 0.5 * h;
    rk4[4 * (i - 1) + 2] = h / 6.0;
    rk4[4 * (i - 1) + 3] = p->times[i - 1];
  }
  for (int j = 0; j < 4; ++j) rk4[4 * (size_t)(p->n_times - 1) + j] = rk4[4 * (size_t)(p->n_times - 2) + j];

  // (re)upload
  OE_HIP(c, hipStreamSynchronize(c->stream));
  if (c->d_times) { OE_HIP(c, hipFree(c->d_times)); c->d_times = nullptr; }
  if (c->d_obs) { OE_HIP(c, hipFree(c->d_obs)); c->d_obs = nullptr; }
  if (c->d_rk4) { OE_HIP(c, hipFree(c->d_rk4)); c->d_rk4 = nullptr; }
  OE_HIP(c, hipMalloc(&c->d_rk4, sizeof(double) * rk4.size()));
  OE_HIP(c, hipMemcpy(c->d_rk4, rk4.data(), sizeof(double) * rk4.size(), hipMemcpyHostToDevice));
  // the grid plus +inf sentinels from index T: the DOPRI5 dense-output loop reads the
  // next grid time one point ahead, the per-lane DOPRI5 (lane.cuh) a window of kGridWin,
  // without clamping the index
  std::vector<double> tg(p->times, p->times + p->n_times);
  tg.insert(tg.end(), oe::kGridWin + 1, HUGE_VAL);
  OE_HIP(c, hipMalloc(&c->d_times, sizeof(double) * tg.size()));
  OE_HIP(c, hipMemcpy(c->d_times, tg.data(), sizeof(double) * tg.size(), hipMemcpyHostToDevice));
  if (p->n_obs > 0) {
    OE_HIP(c, hipMalloc(&c->d_obs, sizeof(Obs) * p->n_obs));
    OE_HIP(c, hipMemcpy(c->d_obs, obs.data(), sizeof(Obs) * p->n_obs, hipMemcpyHostToDevice));
  }
  DevProblem& d = c->dp;
  d.times = c->d_times;
  d.rk4 = c->d_rk4;
  d.obs = c->d_obs;
  d.T = p->n_times;
  d.n_obs = p->n_obs;
  d.P = p->n_params;
  d.substeps = p->method == OE_METHOD_RK4 ? p->rk4_substeps : 1;
  d.rtol = p->rtol;
  d.atol = p->atol;
  d.max_steps = p->max_steps;
  d.pnum = p->pnum;
  d.sstot = p->sstot;
  // scipy's BDF Newton tolerance (oracle/rk_ref.c bdf_newton_tol: the same expression)
  d.newton_tol = std::fmax(10.0 * 2.220446049250313e-16 / p->rtol, std::fmin(0.03, std::sqrt(p->rtol)));
  c->method = p->method;
  c->entry = e;
  c->has_problem = true;
  c->err.clear();
  return OE_OK;
}

int oe_integrate(oe_ctx* c, int64_t W, const double* y0, const double* theta, double* traj,
                 double* chi, double* ssres, int32_t* status, uint32_t flags) {
  if (!c || !c->own_stream) return OE_ERR_STATE;
  if (!c->has_problem) return fail(c, OE_ERR_STATE, "oe_integrate: call oe_problem_set first");
  if (W <= 0 || W > kMaxWalkers) return fail(c, OE_ERR_ARG, "oe_integrate: n_walkers must be in [1, 2^29]");
  if (!y0 || !theta) return fail(c, OE_ERR_ARG, "oe_integrate: y0 and theta are required");
  OE_DEVICE_GUARD(c);
  int rc = OE_OK;
  const Entry* e = c->entry;
  const int S = e->S, P = c->dp.P, T = c->dp.T;
  const bool host = flags & OE_HOST_PTRS;
  const bool nt = flags & OE_NT_STORES;
  if (traj && (int64_t)S * W * 8 >= (int64_t(1) << 32))
    return fail(c, OE_ERR_ARG, "oe_integrate: one trajectory row (S*W*8 bytes) must be < 4 GiB");

  IntegrateArgs ia{};
  ia.W = W;
  const double* h_y0 = y0;
  const double* h_th = theta;
  double* h_traj = traj;
  double *h_chi = chi, *h_ss = ssres;
  int32_t* h_st = status;
  if (host) {
    const size_t n_in = (size_t)(S + P) * W;
    const size_t n_traj = traj ? (size_t)T * S * W : 0;
    const size_t n_out = (size_t)2 * W;
    const size_t bytes = sizeof(double) * (n_in + n_traj + n_out) + sizeof(int32_t) * W + 256;
    rc = ensure_scratch(c, bytes);
    if (rc) return rc;
    double* base = static_cast<double*>(c->scratch);
    double* d_y0 = base;
    double* d_th = d_y0 + (size_t)S * W;
    double* d_traj = traj ? d_th + (size_t)P * W : nullptr;
    double* d_chi = d_th + (size_t)P * W + n_traj;
    double* d_ss = d_chi + W;
    int32_t* d_st = reinterpret_cast<int32_t*>(d_ss + W);
    OE_HIP(c, hipMemcpyAsync(d_y0, h_y0, sizeof(double) * S * W, hipMemcpyHostToDevice, c->stream));
    OE_HIP(c, hipMemcpyAsync(d_th, h_th, sizeof(double) * P * W, hipMemcpyHostToDevice, c->stream));
    ia.y0 = d_y0; ia.theta = d_th; ia.traj = d_traj; ia.chi = d_chi; ia.ssres = d_ss; ia.status = d_st;
  } else {
    ia.y0 = y0; ia.theta = theta; ia.traj = traj; ia.chi = chi; ia.ssres = ssres; ia.status = status;
  }
  // the per-lane BDF pass ('auto' hand-over; S <= 8) defers its observations to a
  // [n_obs][W] scratch (bdf.cuh).  Method 'bdf' runs the wave-lockstep pass here
  // (bdf_wave.cuh), which observes in place (the per-lane one only in OE_LANE_INTEGRATE
  // measurement builds without a trajectory).
  c->dp.obs_c = nullptr;
  const bool lane_bdf = c->method == OE_METHOD_AUTO || (OE_LANE_INTEGRATE && c->method == OE_METHOD_BDF && !traj);
  if (lane_bdf && S <= 8 && c->dp.n_obs > 0) {
    rc = ensure_obs_buf(c, sizeof(double) * (size_t)c->dp.n_obs * (size_t)W);
    if (rc) return rc;
    c->dp.obs_c = static_cast<double*>(c->obs_buf);
  }

  // RK4 trajectories: one of the bitwise-identical kernels (OE_KERNEL_*).
  // * direct: 64 walkers per wave; by default, except:
  // * half: 32 walkers per wave (twice the storing waves).  At <= 1 wave per SIMD a trajectory
  //   of 5+ states is store-issue bound, so the library takes it there (65 536 walkers: chain5
  //   0.508 -> 0.474 ms, chain6 0.694 -> 0.576, chain8 0.89 -> 0.77; two_i 0.394 vs 0.401).
  // * pipe2/4/8 (opt-in): 4 compute waves hand each row to 2, 4 or 8 store waves through a
  //   128 KiB LDS ring, 16-B stores; W even.  Which of these wins back to back differs from
  //   box to box (C1: pipe4 0.349 vs direct 0.379 ms on one box, 0.400 vs 0.391 on another;
  //   DESIGN.md §6), hence OE_TUNE, which measures them on the device at hand.
  const bool rk4_traj = c->method == OE_METHOD_RK4 && ia.traj;
  int variant = OE_KERNEL_OTHER;
  c->has_last_tune = false;
  if (rk4_traj) {
    const bool auto_half = S >= 5 && W <= (int64_t)64 * 4 * c->n_cu;
    const int dflt = ((flags & OE_HALF_WAVES) || auto_half) ? OE_KERNEL_HALF : OE_KERNEL_DIRECT;
    const int xcd = (flags & OE_PIPE_XCD) ? OE_KERNEL_PIPE2X - OE_KERNEL_PIPE2 : 0;
    const int asked = (flags & OE_PIPE_8) ? OE_KERNEL_PIPE8 + xcd : (flags & OE_PIPE_4) ? OE_KERNEL_PIPE4 + xcd
                      : (flags & OE_PIPE) ? OE_KERNEL_PIPE2 + xcd : dflt;
    variant = rk4_variant_ok(e, W, asked, nt, flags) ? asked : dflt;
    if (flags & OE_TUNE) {
      rc = tune_rk4(c, e, ia, nt, flags, dflt, &c->last_tune);
      if (rc) return rc;
      variant = c->last_tune.variant;
      c->has_last_tune = true;
    }
  }
  c->last_variant = variant;
  c->hq_ctl = nullptr;
  const bool timing = !(flags & OE_NO_TIMING);
  if (timing) OE_HIP(c, hipEventRecord(c->ev0, c->stream));
  if (rk4_traj) {
    OE_HIP(c, launch_rk4_traj(c, e, ia, variant, nt, flags));
  } else if (c->method == OE_METHOD_DOPRI5 && ia.traj && !e->rtc && e->dopri5_piped[0] && (flags & OE_PIPE) &&
             (e->split_lanes == 0 || (flags & OE_NO_SPLIT))) {
    // DOPRI5 trajectories through store waves (k_integrate_dopri5_piped): 4 compute + 4 store
    // waves per 256 walkers, blocks dealt to the XCDs in runs of 512 walkers as k_integrate's
    const dim3 grid((unsigned)((W + 255) / 256)), block(512);
    ia.half = 0;
    ia.xcd_remap = xcd_remap_of(flags, grid, 256);
    e->dopri5_piped[nt ? 1 : 0](c->dp, ia, grid, block, c->stream);
  } else if (c->method == OE_METHOD_DOPRI5 && !e->rtc && e->split_lanes > 0 && !(flags & OE_NO_SPLIT)) {
    // wide chain models: one walker over K adjacent lanes (split.cuh), blocks of 256/K
    // walkers dealt to the XCDs in runs of 512 walkers as the one-lane kernel's
    const int K = e->split_lanes;
    const int64_t per_block = kBlock / K;
    const dim3 grid((unsigned)((W + per_block - 1) / per_block)), block(kBlock);
    ia.half = 0;
    ia.xcd_remap = (flags & OE_NO_XCD_REMAP) ? 0
                   : (flags & OE_XCD_RANGES) ? (int32_t)std::max<int64_t>(1, (int64_t)grid.x / 8)
                                             : (int32_t)std::max<int64_t>(1, 512 / per_block);
    e->dopri5_split[ia.traj ? 1 : 0][nt ? 1 : 0](c->dp, ia, grid, block, c->stream);
  } else {
    // RK4 without a trajectory (32 walkers per wave only on request), DOPRI5 (64-lane
    // groups: its step size is shared per wave), the stiff methods
    const bool rk4 = c->method == OE_METHOD_RK4;
    ia.half = (rk4 && (flags & OE_HALF_WAVES)) ? 1 : 0;
    const int64_t per_block = ia.half ? kBlock / 2 : kBlock;
    const dim3 grid((unsigned)((W + per_block - 1) / per_block)), block(kBlock);
    ia.xcd_remap = xcd_remap_of(flags, grid, per_block);
    // Models wider than the register-resident stiff path: 'auto' marks the walkers the
    // DOPRI5 pass evicts, and k_stiff_wave redoes them one wave per walker; 'rosenbrock'
    // is k_stiff_wave for every walker (stiff_wave.cuh).
    const bool wave_stiff = (c->method == OE_METHOD_AUTO || c->method == OE_METHOD_ROSENBROCK) &&
                            S > kStiffRegS && (e->rtc ? e->rtc->stiff_wave[0][0] != nullptr : e->stiff_wave[0][0] != nullptr);
    StiffWaveArgs sa{};
    if (wave_stiff) {
      rc = ensure_stiff_buf(c, W);
      if (rc) return rc;
      sa.y0 = ia.y0; sa.theta = ia.theta; sa.traj = ia.traj; sa.chi = ia.chi; sa.ssres = ia.ssres; sa.W = W;
      if (!ia.status) ia.status = c->stiff_buf + 64 + W;  // the marks need a status array
      sa.status = ia.status;
    }
    // 'auto', S <= kHandMaxS (built-in models): the hand-over queue (ode_kernels.cuh HandQ) —
    // the DOPRI5 kernel on the caller's stream; the BDF kernel beside it on the context's
    // second stream for small ensembles (<= OE_HQ_MAX_W_PER_CU walkers per CU), else after it
    // on the same stream; the caller's stream waits for both
    const int tj = ia.traj ? 1 : 0, nj = nt ? 1 : 0;
    const bool handq = c->method == OE_METHOD_AUTO && !e->rtc && e->integrate_hq[0][tj][nj] && !OE_LANE_INTEGRATE;
    const bool beside = W <= (int64_t)OE_HQ_MAX_W_PER_CU * c->n_cu;  // else: after the DOPRI5 kernel
    if (handq) {
      HandQ q{};
      rc = ensure_hq(c, W, S, &q);
      if (rc) return rc;
      q.n_waves = (int32_t)grid.x * (kBlock / 64);
      OE_HIP(c, hipMemsetAsync(q.ctl, 0, 10 * sizeof(int32_t), c->stream));
      hipStream_t bs = c->stream;
      if (beside) {
        OE_HIP(c, hipEventRecord(c->ev_hq[0], c->stream));
        OE_HIP(c, hipStreamWaitEvent(c->hq_stream, c->ev_hq[0], 0));
        bs = c->hq_stream;
      }
      e->integrate_hq[beside ? 1 : 0][tj][nj](c->dp, ia, q, grid, block, c->stream);
      OE_HIP(c, hipGetLastError());
      // one-wave workgroups, slots dealt statically (k_bdf_hq): one slot per lane of the launch,
      // so the grid covers W slots — beside the DOPRI5 kernel min(W, kHandBdfWaves) waves (W <=
      // 16 per CU there), after it one wave per SIMD, more only past 64 per SIMD (a round of
      // dispatch when nothing was handed).  (One 4-wave workgroup per CU, a lone stiff walker
      // per CU, measured no faster: C2 + 0.1 % stiff 2.37 vs 2.34 ms, profiles/r06/r06y_*.)
      const int64_t G = beside ? std::min<int64_t>((int64_t)kHandBdfWaves, W)
                               : std::max<int64_t>(4 * (int64_t)c->n_cu, (W + 63) / 64);
      static_assert((int64_t)kHandBdfWaves * 64 >= (int64_t)OE_HQ_MAX_W_PER_CU * 1024,
                    "beside the DOPRI5 kernel, the BDF kernel's lanes cover every walker (n_CU <= 1024)");
      e->bdf_hq[beside ? 1 : 0][tj][nj](c->dp, ia, q, dim3((unsigned)G), dim3(64), bs);
      OE_HIP(c, hipGetLastError());
      if (beside) {
        OE_HIP(c, hipEventRecord(c->ev_hq[1], c->hq_stream));
        OE_HIP(c, hipStreamWaitEvent(c->stream, c->ev_hq[1], 0));
      }
      c->hq_ctl = q.ctl;
    } else if (!(wave_stiff && c->method == OE_METHOD_ROSENBROCK)) {
      OE_HIP(c, launch_integrate_entry(e, c->method, ia.traj ? 1 : 0, nt ? 1 : 0, c->dp, ia, grid, block, c->stream));
    }
    if (wave_stiff) {
      const dim3 wgrid((unsigned)std::min<int64_t>(W, (int64_t)16 * c->n_cu)), wblock(64);
      if (c->method == OE_METHOD_AUTO) {
        int32_t* count = c->stiff_buf;
        int32_t* list = c->stiff_buf + 64;
        OE_HIP(c, hipMemsetAsync(count, 0, sizeof(int32_t), c->stream));
        hipLaunchKernelGGL(k_stiff_list, dim3((unsigned)((W + 255) / 256)), dim3(256), 0, c->stream, ia.status, W,
                           list, count);
        OE_HIP(c, hipGetLastError());
        sa.list = list;
        sa.count = count;
      }
      OE_HIP(c, launch_stiff_wave_entry(e, ia.traj ? 1 : 0, nt ? 1 : 0, c->dp, sa, wgrid, wblock, c->stream));
    }
  }
  OE_HIP(c, hipGetLastError());
  if (timing) OE_HIP(c, hipEventRecord(c->ev1, c->stream));
  c->timed = timing;

  if (host) {
    if (h_traj)
      OE_HIP(c, hipMemcpyAsync(h_traj, ia.traj, sizeof(double) * T * S * W, hipMemcpyDeviceToHost, c->stream));
    if (h_chi) OE_HIP(c, hipMemcpyAsync(h_chi, ia.chi, sizeof(double) * W, hipMemcpyDeviceToHost, c->stream));
    if (h_ss) OE_HIP(c, hipMemcpyAsync(h_ss, ia.ssres, sizeof(double) * W, hipMemcpyDeviceToHost, c->stream));
    if (h_st) OE_HIP(c, hipMemcpyAsync(h_st, ia.status, sizeof(int32_t) * W, hipMemcpyDeviceToHost, c->stream));
    OE_HIP(c, hipStreamSynchronize(c->stream));
  } else if (!(flags & OE_ASYNC)) {
    OE_HIP(c, hipStreamSynchronize(c->stream));
  }
  // synchronous calls through the hand-over queue: a BDF wave that gave up waiting (a slot
  // never published within kHandTimeout: a bug, reported rather than hung on)
  if (c->hq_ctl && (host || !(flags & OE_ASYNC))) {
    int32_t timed_out = 0;
    OE_HIP(c, hipMemcpy(&timed_out, c->hq_ctl + 3, sizeof(int32_t), hipMemcpyDeviceToHost));
    if (timed_out) return fail(c, OE_ERR_HIP, "oe_integrate: the hand-over queue's BDF kernel timed out");
  }
  return OE_OK;
}

int oe_mh_run(oe_ctx* c, const oe_mh_args* a, uint32_t flags) {
  if (!c || !c->own_stream) return OE_ERR_STATE;
  if (!c->has_problem) return fail(c, OE_ERR_STATE, "oe_mh_run: call oe_problem_set first");
  if (!a) return fail(c, OE_ERR_ARG, "oe_mh_run: null args");
  if (flags & OE_HOST_PTRS) return fail(c, OE_ERR_ARG, "oe_mh_run: device pointers only");
  const Entry* e = c->entry;
  const int S = e->S, P = c->dp.P;
  const int64_t W = a->n_walkers;
  if (W <= 0 || W > kMaxWalkers) return fail(c, OE_ERR_ARG, "oe_mh_run: n_walkers must be in [1, 2^29]");
  if (a->nits < 1) return fail(c, OE_ERR_ARG, "oe_mh_run: nits must be >= 1");
  if (a->burnin < 0) return fail(c, OE_ERR_ARG, "oe_mh_run: burnin must be >= 0");
  if (!a->theta || !a->y0 || !a->walk_mask || !a->init_param)
    return fail(c, OE_ERR_ARG, "oe_mh_run: theta, y0, walk_mask and init_param are required");
  const int it_start = a->it_start > 1 ? a->it_start : 1;
  const bool resume = it_start > 1;
  if (resume && (it_start > a->nits || !a->final_stats))
    return fail(c, OE_ERR_ARG, "oe_mh_run: resume needs it_start <= nits and the chain state in final_stats");
  const int row0 = std::max(it_start, a->burnin + 1);
  const int kept = std::max(0, a->nits - row0);
  if (kept > 0 && !a->samples) return fail(c, OE_ERR_ARG, "oe_mh_run: samples buffer required");
  if (a->rng_mode == OE_RNG_REPLAY) {
    if (a->nits > 1 && (!a->replay_dz || !a->replay_u))
      return fail(c, OE_ERR_ARG, "oe_mh_run: replay mode needs replay_dz and replay_u");
  } else if (a->rng_mode == OE_RNG_NUMPY) {
    if (!a->numpy_seeds) return fail(c, OE_ERR_ARG, "oe_mh_run: numpy mode needs numpy_seeds");
    if (a->numpy_prior_draws < 0) return fail(c, OE_ERR_ARG, "oe_mh_run: numpy_prior_draws must be >= 0");
  } else if (a->rng_mode != OE_RNG_PHILOX) {
    return fail(c, OE_ERR_ARG, "oe_mh_run: unknown rng_mode");
  }
  if (S > 64) return fail(c, OE_ERR_UNSUPPORTED, "oe_mh_run: S > 64");
  OE_DEVICE_GUARD(c);
  int rc = OE_OK;

  MHArgs m{};
  m.W = W;
  m.walker_offset = a->walker_offset;
  m.burnin = a->burnin;
  m.row0 = row0;
  m.walk_mask = 0;
  for (int p = 0; p < P; ++p)
    if (a->walk_mask[p]) m.walk_mask |= (1ull << p);
  m.any_walk = m.walk_mask != 0;
  for (int s = 0; s < 64; ++s) m.init_param[s] = -1;
  for (int s = 0; s < S; ++s) {
    const int32_t ip = a->init_param[s];
    if (ip < -1 || ip >= P) return fail(c, OE_ERR_ARG, "oe_mh_run: init_param out of range");
    m.init_param[s] = ip;
  }
  m.theta = a->theta;
  m.y0 = a->y0;
  m.samples = a->samples;
  m.n_rows = kept;
  // self-test hook of the debug library's integrity checks (OE_MH_CHECKS): a row bound one
  // short makes the last kept iteration fail the check; the product kernels never read it
  if (getenv("OE_MH_CHECK_SELFTEST")) m.n_rows = kept - 1;
  m.status = a->status;
  // chain state: caller's final_stats buffer if given, else scratch
  if (a->final_stats) {
    m.cur = a->final_stats;
  } else {
    rc = ensure_scratch(c, sizeof(double) * 4 * W);
    if (rc) return rc;
    m.cur = static_cast<double*>(c->scratch);
  }

  const dim3 grid((unsigned)((W + kBlock - 1) / kBlock)), block(kBlock);
  // wide chain models, DOPRI5: the chain over K lanes (split.cuh); the kernel addresses its
  // states in one [S][W] descriptor, so S*W*8 must stay below 4 GiB
  const bool split = c->method == OE_METHOD_DOPRI5 && !e->rtc && e->mh_split && !(flags & OE_NO_SPLIT) &&
                     (int64_t)S * W * 8 < (int64_t(1) << 32);
  const dim3 mh_grid = split ? dim3((unsigned)((W * e->split_lanes + kBlock - 1) / kBlock)) : grid;
  auto launch_mh = [&](const MHArgs& args) -> hipError_t {
    if (split) {
      e->mh_split(c->dp, args, mh_grid, block, c->stream);
      return hipGetLastError();
    }
    return launch_mh_entry(e, c->method, c->dp, args, grid, block, c->stream);
  };
  int chunk = a->chunk > 0 ? a->chunk : 25;
  // Speculative rounds (k_mh_tree + k_mh_resolve): d iterations per round, the tree's
  // (2^d - 1)·W lanes at most about one wave per SIMD, so a round costs about what one
  // iteration of the few chains costs alone
  int depth = 0;
  const bool has_tree = split ? e->mh_split_tree != nullptr
                       : e->rtc ? e->rtc->mh_tree[c->method] != nullptr : e->mh_tree[c->method] != nullptr;
  // the stiff methods of the register-path models have no iteration-loop kernel (kMhRoundsOnly):
  // their chains always run in rounds, one iteration a round at the least
  const bool rounds_only = !split && has_tree && (e->rtc ? e->rtc->mh[c->method] : (const void*)e->mh[c->method]) == nullptr;
  const int lanes_per_walker = split ? e->split_lanes : 1;
  // bytes per tree lane: the node's proposal, chi, R² residual, status, and for the per-lane
  // BDF pass ('auto' / 'bdf', S <= 8) its deferred observations (DevProblem::obs_c)
  const bool lane_bdf = !split && (c->method == OE_METHOD_AUTO || c->method == OE_METHOD_BDF) && S <= 8;
  const double lane_bytes = 8.0 * (P + 2) + 4.0 + (lane_bdf ? 8.0 * c->dp.n_obs : 0.0);
  if (a->speculate != 0 && has_tree && a->nits > 1) {
    const int64_t target = (int64_t)64 * 4 * c->n_cu / lanes_per_walker;
    if (a->speculate < 0) {
      depth = 1;
      while (depth < 16 && ((int64_t(1) << (depth + 1)) - 1) * W <= target) ++depth;
    } else {
      depth = std::min(a->speculate, 16);
    }
    if (depth < 2 || ((int64_t(1) << depth) - 1) * W > kMaxWalkers) depth = 0;
    // the tree buffer ((2^d - 1)·W·(P + 2) doubles) within 4 GiB, like the draw buffers'
    // budget: a deeper explicit request is cut to the deepest tree that fits
    while (depth >= 2 && (double)((int64_t(1) << depth) - 1) * (double)W * lane_bytes > 4294967296.0) --depth;
    if (depth < 2) depth = 0;
  }
  if (rounds_only && depth == 0) depth = 1;
  c->last_mh_depth = depth;
  MHTreeArgs ta{};
  if (depth) {
    chunk = std::max(depth, chunk / depth * depth);  // whole rounds per chunk of draws
    const int64_t nodes = (int64_t(1) << depth) - 1;
    const size_t bytes = sizeof(double) * (size_t)(nodes * W) * (size_t)(P + 2) + sizeof(int32_t) * (size_t)(nodes * W) + 256;
    if (c->tree_bytes < bytes) {
      if (c->tree) {
        OE_HIP(c, hipStreamSynchronize(c->stream));
        OE_HIP(c, hipFree(c->tree));
        c->tree = nullptr;
        c->tree_bytes = 0;
      }
      if (hipMalloc(&c->tree, bytes) != hipSuccess) {  // out of memory: one iteration per step
        (void)hipGetLastError();
        c->tree = nullptr;
        if (rounds_only) return fail(c, OE_ERR_NOMEM, "oe_mh_run: no device memory for the MH round buffer");
        depth = 0;
        c->last_mh_depth = 0;
      } else {
        c->tree_bytes = bytes;
      }
    }
  }
  // the per-lane BDF pass (MH 'auto' / 'bdf', one lane per chain, S <= 8) defers its
  // observations to a [n_obs][lanes] scratch: one column per lane of the largest launch
  c->dp.obs_c = nullptr;
  if (lane_bdf && c->dp.n_obs > 0) {
    const int64_t lanes = depth ? ((int64_t(1) << depth) - 1) * W : W;
    rc = ensure_obs_buf(c, sizeof(double) * (size_t)c->dp.n_obs * (size_t)lanes);
    if (rc && depth >= 2) {  // out of memory for a speculative tree's scratch: one iteration a round
      (void)hipGetLastError();
      depth = rounds_only ? 1 : 0;
      c->last_mh_depth = depth;
      rc = ensure_obs_buf(c, sizeof(double) * (size_t)c->dp.n_obs * (size_t)W);
    }
    if (rc) return rc;
    c->dp.obs_c = static_cast<double*>(c->obs_buf);
  }
  if (depth) {
    const int64_t nodes = (int64_t(1) << depth) - 1;
    double* b = static_cast<double*>(c->tree);
    ta.node_th = b;
    ta.node_chi = b + (size_t)(nodes * W) * P;
    ta.node_ss = ta.node_chi + nodes * W;
    ta.node_st = reinterpret_cast<int32_t*>(ta.node_ss + nodes * W);
  }
  const bool philox = a->rng_mode == OE_RNG_PHILOX, numpy = a->rng_mode == OE_RNG_NUMPY;
  DrawArgs d{};
  NpDrawArgs nd{};
  double* np_dz[2] = {nullptr, nullptr};
  double* np_u[2] = {nullptr, nullptr};
  if ((philox || numpy) && a->nits > 1) {
    // one chunk of draws resident at a time, at most ~1 GiB (at least one iteration)
    const size_t per_it = sizeof(double) * (size_t)(P + 1) * (size_t)W;
    chunk = (int)std::max<int64_t>(1, std::min<int64_t>(chunk, (int64_t)((1ull << 30) / per_it)));
    rc = ensure_draws(c, per_it * (size_t)chunk * (numpy ? 2 : 1));
    if (rc) return rc;
    double* dz = static_cast<double*>(c->draws);
    double* u = dz + (size_t)chunk * P * W;
    m.dz = dz;
    m.u = u;
    np_dz[0] = dz;
    np_u[0] = u;
    np_dz[1] = dz + (size_t)chunk * (P + 1) * W;
    np_u[1] = np_dz[1] + (size_t)chunk * P * W;
    if (philox) {
      d.W = W;
      d.walker_offset = a->walker_offset;
      d.P = P;
      d.seed_lo = (uint32_t)a->seed;
      d.seed_hi = (uint32_t)(a->seed >> 32);
      d.step_sd = a->step_sd;
      d.dz = dz;
      d.u = u;
    } else {
      nd.W = W;
      nd.P = P;
      nd.prior_draws = a->numpy_prior_draws;
      nd.zero_static = 0;
      nd.walk_mask = m.walk_mask;
      nd.step_sd = a->step_sd;
      nd.dz = dz;
      nd.u = u;
      rc = ensure_np_state(c, W, &nd.st);
      if (rc) return rc;
      rc = ensure_np_stream(c);
      if (rc) return rc;
    }
  } else {
    m.dz = a->replay_dz;
    m.u = a->replay_u;
    m.draw_it0 = 1;
  }
  OE_HIP(c, hipEventRecord(c->ev0, c->stream));
  if (numpy && a->nits > 1) {  // np.random.seed(random_seed), Samplers.py:70
    hipLaunchKernelGGL(k_np_seed, grid, block, 0, c->stream, nd.st, a->numpy_seeds, W);
    OE_HIP(c, hipGetLastError());
    for (int f0 = 1; f0 < it_start; f0 += chunk) {  // resume: replay the consumed draws
      nd.it0 = f0;
      nd.it1 = std::min(it_start, f0 + chunk);
      hipLaunchKernelGGL(k_np_draws, np_grid(W), dim3(kNpChainsPerBlock), 0, c->stream, nd);
      OE_HIP(c, hipGetLastError());
    }
  }
  // chunk j's numpy draws on the side stream, into buffer j & 1: after the MT state is ready
  // (j = 0) and after chunk j - 2's MH kernels have read that buffer (j >= 2)
  auto np_draws_chunk = [&](int j) -> int {
    nd.it0 = it_start + j * chunk;
    nd.it1 = std::min(a->nits, nd.it0 + chunk);
    nd.dz = np_dz[j & 1];
    nd.u = np_u[j & 1];
    if (j >= 2) OE_HIP(c, hipStreamWaitEvent(c->np_stream, c->ev_mh[j & 1], 0));
    hipLaunchKernelGGL(k_np_draws, np_grid(W), dim3(kNpChainsPerBlock), 0, c->np_stream, nd);
    OE_HIP(c, hipGetLastError());
    OE_HIP(c, hipEventRecord(c->ev_np[j & 1], c->np_stream));
    return OE_OK;
  };
  if (numpy && a->nits > 1 && it_start < a->nits) {
    OE_HIP(c, hipEventRecord(c->ev_mh[0], c->stream));  // seeded / replayed state
    OE_HIP(c, hipStreamWaitEvent(c->np_stream, c->ev_mh[0], 0));
    rc = np_draws_chunk(0);
    if (rc) return rc;
  }
  if (!resume) {
    m.init = 1;
    m.it0 = 0;
    m.it1 = 0;
    OE_HIP(c, launch_mh(m));
  }
  m.init = 0;
  for (int it0 = it_start; it0 < a->nits; it0 += chunk) {
    m.it0 = it0;
    m.it1 = std::min(a->nits, it0 + chunk);
    if (philox) {
      d.it0 = m.it0;
      d.it1 = m.it1;
      m.draw_it0 = it0;
      hipLaunchKernelGGL(k_philox_draws, dim3((unsigned)((W * (d.it1 - d.it0) + kBlock - 1) / kBlock)), block, 0,
                         c->stream, d);
      OE_HIP(c, hipGetLastError());
    } else if (numpy) {
      const int j = (it0 - it_start) / chunk;
      if (m.it1 < a->nits) {
        rc = np_draws_chunk(j + 1);
        if (rc) return rc;
      }
      OE_HIP(c, hipStreamWaitEvent(c->stream, c->ev_np[j & 1], 0));
      m.dz = np_dz[j & 1];
      m.u = np_u[j & 1];
      m.draw_it0 = it0;
    }
    if (!depth) {
      OE_HIP(c, launch_mh(m));
    } else {
      for (int r0 = m.it0; r0 < m.it1; r0 += ta.depth) {
        ta.m = m;
        ta.m.it0 = r0;
        ta.depth = std::min(depth, m.it1 - r0);
        ta.n_lanes = ((int64_t(1) << ta.depth) - 1) * W;
        // few lanes (<= one per CU): one lane per wave (MHTreeArgs::spread).  The notebook fit's 32
        // chains, sequential: 1.42 -> 0.80 s; 1 024 synthetic chains (one wave per SIMD) ran
        // slower spread, 0.27 -> 0.45 s (profiles/NOTES.md round 6)
        ta.spread = (!split && OE_MH_SPREAD && ta.n_lanes <= (int64_t)c->n_cu) ? 1 : 0;
        const dim3 tgrid = ta.spread ? dim3((unsigned)ta.n_lanes)
                                     : dim3((unsigned)((ta.n_lanes * lanes_per_walker + kBlock - 1) / kBlock));
        const dim3 tblock = ta.spread ? dim3(64) : block;
        if (split) {
          e->mh_split_tree(c->dp, ta, tgrid, tblock, c->stream);
          OE_HIP(c, hipGetLastError());
        } else {
          OE_HIP(c, launch_mh_tree_entry(e, c->method, c->dp, ta, tgrid, tblock, c->stream));
        }
        // one wave per chain pays off for deep trees of few chains (32 chains, d = 11: 0.0311 ->
        // 0.0287 ms per iteration); shallow trees of many chains keep one lane per chain
        // (8 192 chains, d = 3: 0.079 vs 0.099)
        if (ta.depth >= 5 && ta.depth <= kResolveLdsDepth)
          hipLaunchKernelGGL(k_mh_resolve_wave, dim3((unsigned)W), dim3(64), 0, c->stream, c->dp, ta, (int32_t)S);
        else
          hipLaunchKernelGGL(k_mh_resolve, grid, block, 0, c->stream, c->dp, ta, (int32_t)S);
        OE_HIP(c, hipGetLastError());
      }
    }
    if (numpy && m.it1 < a->nits)  // buffer j & 1 is free for chunk j + 2's draws
      OE_HIP(c, hipEventRecord(c->ev_mh[((it0 - it_start) / chunk) & 1], c->stream));
  }
  OE_HIP(c, hipEventRecord(c->ev1, c->stream));
  c->timed = true;
  if (!(flags & OE_ASYNC)) OE_HIP(c, hipStreamSynchronize(c->stream));
  return OE_OK;
}

int oe_numpy_streams(oe_ctx* c, int64_t W, const uint32_t* seeds, int32_t nits, int32_t n_params,
                     const uint8_t* walk_mask, int32_t prior_draws, double step_sd, double* dz, double* u) {
  if (!c || !c->own_stream) return OE_ERR_STATE;
  if (W <= 0 || W > kMaxWalkers) return fail(c, OE_ERR_ARG, "oe_numpy_streams: n_walkers must be in [1, 2^29]");
  if (nits < 1 || n_params < 1 || n_params > 64 || prior_draws < 0)
    return fail(c, OE_ERR_ARG, "oe_numpy_streams: need nits >= 1, 1 <= n_params <= 64, prior_draws >= 0");
  if (!seeds || !walk_mask || (nits > 1 && (!dz || !u)))
    return fail(c, OE_ERR_ARG, "oe_numpy_streams: seeds, walk_mask, dz and u are required");
  OE_DEVICE_GUARD(c);
  int rc = OE_OK;
  if (nits == 1) return OE_OK;
  NpDrawArgs nd{};
  nd.W = W;
  nd.it0 = 1;
  nd.it1 = nits;
  nd.P = n_params;
  nd.prior_draws = prior_draws;
  nd.zero_static = 1;
  for (int p = 0; p < n_params; ++p)
    if (walk_mask[p]) nd.walk_mask |= (1ull << p);
  nd.step_sd = step_sd;
  nd.dz = dz;
  nd.u = u;
  rc = ensure_np_state(c, W, &nd.st);
  if (rc) return rc;
  const dim3 grid((unsigned)((W + kBlock - 1) / kBlock)), block(kBlock);
  OE_HIP(c, hipEventRecord(c->ev0, c->stream));
  hipLaunchKernelGGL(k_np_seed, grid, block, 0, c->stream, nd.st, seeds, W);
  OE_HIP(c, hipGetLastError());
  hipLaunchKernelGGL(k_np_draws, np_grid(W), dim3(kNpChainsPerBlock), 0, c->stream, nd);
  OE_HIP(c, hipGetLastError());
  OE_HIP(c, hipEventRecord(c->ev1, c->stream));
  c->timed = true;
  OE_HIP(c, hipStreamSynchronize(c->stream));
  return OE_OK;
}

int oe_last_kernel_ms(oe_ctx* c, double* ms) {
  if (!c || !ms) return OE_ERR_ARG;
  if (!c->timed) return fail(c, OE_ERR_STATE, "oe_last_kernel_ms: nothing launched yet");
  OE_HIP(c, hipEventSynchronize(c->ev1));
  float f = 0.f;
  OE_HIP(c, hipEventElapsedTime(&f, c->ev0, c->ev1));
  *ms = (double)f;
  return OE_OK;
}

int oe_last_variant(oe_ctx* c, int32_t* variant) {
  if (!c || !variant) return OE_ERR_ARG;
  if (c->last_variant < 0) return fail(c, OE_ERR_STATE, "oe_last_variant: no oe_integrate yet");
  *variant = c->last_variant;
  return OE_OK;
}

int oe_last_mh_depth(oe_ctx* c, int32_t* depth) {
  if (!c || !depth) return OE_ERR_ARG;
  *depth = c->last_mh_depth;
  return OE_OK;
}

int oe_tune_times(oe_ctx* c, double* ms, int32_t n) {
  if (!c || !ms || n < OE_KERNEL_COUNT - 1) return OE_ERR_ARG;
  if (!c->has_last_tune) return fail(c, OE_ERR_STATE, "oe_tune_times: the last oe_integrate was not tuned");
  const oe_ctx::Tuned& t = c->last_tune;
  for (int v = 0; v < OE_KERNEL_COUNT - 1; ++v) ms[v] = t.ms[v];
  return OE_OK;
}

}  // extern "C"
