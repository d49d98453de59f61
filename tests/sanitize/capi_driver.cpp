// TEST INFRASTRUCTURE: the C-ABI's host code (capi.hip, rtc.hip, comm.hip) built with
// AddressSanitizer + UndefinedBehaviorSanitizer on the host side only (device code as in
// the product).  Without a GPU it drives every validation / error path and a
// hipRTC compile check; with one (argv[1] == "device") it also runs problem set-up,
// integrate with host and device pointers for every method, MH with each RNG mode, the
// numpy streams, a run-time compiled model with the lazily built stiff kernels, and
// context teardown.  Any sanitizer report aborts the run.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../../include/odelib_amd.h"

#define CHECK(cond)                                                        \
  do {                                                                     \
    if (!(cond)) {                                                         \
      std::fprintf(stderr, "CHECK failed at line %d: %s\n", __LINE__, #cond); \
      std::exit(1);                                                        \
    }                                                                      \
  } while (0)

static const char* kBody =
    "const R mu = ps[0], phi = ps[1], beta = ps[2], lam = ps[3], tau = ps[4];\n"
    "const R inf = phi * y[0] * y[3];\n"
    "dy[0] = mu * y[0] - inf; dy[1] = inf - tau * y[1];\n"
    "dy[2] = tau * y[1] - lam * y[2]; dy[3] = beta * lam * y[2] - inf;\n";

static void error_paths() {
  CHECK(oe_abi_version() == OE_ABI_VERSION);
  int32_t s = 0, p = 0;
  CHECK(oe_model_info(OE_MODEL_TWO_I, &s, &p) == OE_OK && s == 4 && p == 5);
  s = 20;
  CHECK(oe_model_info(OE_MODEL_CHAIN, &s, &p) == OE_OK && s == 20);
  s = 7;
  CHECK(oe_model_info(OE_MODEL_CHAIN, &s, &p) == OE_ERR_UNSUPPORTED);
  CHECK(oe_model_info(OE_MODEL_TWO_I, nullptr, &p) == OE_ERR_ARG);
  CHECK(oe_ctx_create(0, nullptr) == OE_ERR_ARG);
  CHECK(oe_integrate(nullptr, 1, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, 0) == OE_ERR_STATE);
  CHECK(oe_problem_set(nullptr, nullptr) == OE_ERR_STATE);
  CHECK(oe_mh_run(nullptr, nullptr, 0) == OE_ERR_STATE);
  CHECK(std::strcmp(oe_last_error(nullptr), "null context") == 0);
  double ms = 0;
  CHECK(oe_last_kernel_ms(nullptr, &ms) == OE_ERR_ARG);
  // hipRTC: a good body compiles for gfx950 without a GPU, a bad one reports the log
  CHECK(oe_rtc_check(kBody, 4, 5, "gfx950") == OE_OK);
  CHECK(oe_rtc_check("dy[0] = nope;", 4, 5, "gfx950") == OE_ERR_ARG);
  CHECK(std::strstr(oe_last_error(nullptr), "nope") != nullptr);
  CHECK(oe_rtc_check(nullptr, 4, 5, "gfx950") == OE_ERR_ARG);
  // pooling entry points validate first
  uint8_t id[OE_COMM_ID_BYTES] = {0};
  oe_comm* comm = nullptr;
  CHECK(oe_comm_init(0, 0, 0, id, OE_COMM_ID_BYTES, &comm) == OE_ERR_ARG && comm == nullptr);
  CHECK(oe_comm_init(0, 2, 2, id, OE_COMM_ID_BYTES, &comm) == OE_ERR_ARG);
  CHECK(oe_comm_unique_id(nullptr, OE_COMM_ID_BYTES) == OE_ERR_ARG);
  CHECK(oe_allgather_samples(nullptr, 1, nullptr, nullptr, nullptr, 0) == OE_ERR_ARG);
  oe_comm_destroy(nullptr);
  oe_ctx_destroy(nullptr);
}

static oe_problem two_i_problem(std::vector<double>& t, std::vector<int32_t>& tidx, std::vector<uint64_t>& mask,
                                std::vector<double>& O, std::vector<double>& sig, std::vector<double>& lin,
                                int32_t method) {
  const int T = 200;
  t.resize(T);
  for (int i = 0; i < T; ++i) t[i] = 3.0 * i / (T - 1);
  tidx = {0, 50, 50, 120, 199, 199};
  mask = {7, 8, 7, 8, 7, 8};
  O = {15.47, 16.2, 15.4, 17.0, 14.9, 18.1};
  sig = {0.1, 0.2, 0.1, 0.2, 0.1, 0.2};
  for (double o : O) lin.push_back(std::exp(o));
  oe_problem p{};
  p.model_id = OE_MODEL_TWO_I;
  p.n_states = 4;
  p.n_params = 5;
  p.n_times = T;
  p.times = t.data();
  p.n_obs = (int32_t)tidx.size();
  p.obs_tidx = tidx.data();
  p.obs_mask = mask.data();
  p.obs_log = O.data();
  p.obs_logsigma = sig.data();
  p.obs_lin = lin.data();
  p.method = method;
  p.rk4_substeps = 2;
  p.rtol = p.atol = 1.49012e-8;
  p.max_steps = 500;
  p.sstot = 1.0;
  p.pnum = 5;
  return p;
}

static void device_paths() {
  oe_ctx* c = nullptr;
  CHECK(oe_ctx_create(0, &c) == OE_OK);
  const int64_t W = 130;
  const int S = 4, P = 5, T = 200;
  std::vector<double> y0(S * W), th(P * W);
  const double base[5] = {7.475e-9, 1.069e-7, 19.73, 1.934, 2.799};
  for (int64_t w = 0; w < W; ++w) {
    y0[0 * W + w] = 5236900.0;
    y0[3 * W + w] = 10981000.0;
    for (int j = 0; j < P; ++j) th[j * W + w] = base[j] * (1.0 + 0.01 * std::sin((double)(w * 7 + j)));
  }
  th[4 * W + 5] = 1e5;  // a stiff walker
  std::vector<double> traj((size_t)T * S * W), chi(W), ss(W);
  std::vector<int32_t> st(W);
  for (int32_t method = OE_METHOD_RK4; method <= OE_METHOD_ROSENBROCK; ++method) {
    std::vector<double> t, O, sig, lin;
    std::vector<int32_t> tidx;
    std::vector<uint64_t> mask;
    oe_problem p = two_i_problem(t, tidx, mask, O, sig, lin, method);
    CHECK(oe_problem_set(c, &p) == OE_OK);
    CHECK(oe_integrate(c, W, y0.data(), th.data(), traj.data(), chi.data(), ss.data(), st.data(), OE_HOST_PTRS) ==
          OE_OK);
    CHECK(oe_integrate(c, W, y0.data(), th.data(), nullptr, chi.data(), nullptr, nullptr, OE_HOST_PTRS) == OE_OK);
    double ms = 0;
    CHECK(oe_last_kernel_ms(c, &ms) == OE_OK && ms > 0);
    // bad arguments on a live context
    CHECK(oe_integrate(c, 0, y0.data(), th.data(), nullptr, nullptr, nullptr, nullptr, OE_HOST_PTRS) == OE_ERR_ARG);
    oe_problem bad = p;
    bad.n_times = 1;
    CHECK(oe_problem_set(c, &bad) == OE_ERR_ARG);
    CHECK(oe_problem_set(c, &p) == OE_OK);
    // device-resident MH, every RNG mode
    double *dth, *dy0, *dsamp, *dfin, *ddz, *du;
    int32_t* dst;
    uint32_t* dseeds;
    const int nits = 7, burnin = 2, kept = nits - 1 - burnin;
    CHECK(hipMalloc(&dth, sizeof(double) * P * W) == hipSuccess);
    CHECK(hipMalloc(&dy0, sizeof(double) * S * W) == hipSuccess);
    CHECK(hipMalloc(&dsamp, sizeof(double) * kept * (P + 5) * W) == hipSuccess);
    CHECK(hipMalloc(&dfin, sizeof(double) * 4 * W) == hipSuccess);
    CHECK(hipMalloc(&dst, sizeof(int32_t) * W) == hipSuccess);
    CHECK(hipMalloc(&ddz, sizeof(double) * (nits - 1) * P * W) == hipSuccess);
    CHECK(hipMalloc(&du, sizeof(double) * (nits - 1) * W) == hipSuccess);
    CHECK(hipMalloc(&dseeds, sizeof(uint32_t) * W) == hipSuccess);
    std::vector<uint32_t> seeds(W);
    for (int64_t w = 0; w < W; ++w) seeds[w] = (uint32_t)w;
    CHECK(hipMemcpy(dseeds, seeds.data(), sizeof(uint32_t) * W, hipMemcpyHostToDevice) == hipSuccess);
    uint8_t walk[5] = {1, 1, 0, 1, 1};
    int32_t ip[4] = {-1, -1, -1, -1};
    CHECK(oe_numpy_streams(c, W, dseeds, nits, P, walk, 2, 0.05, ddz, du) == OE_OK);
    for (int32_t mode = OE_RNG_REPLAY; mode <= OE_RNG_NUMPY; ++mode) {
      CHECK(hipMemcpy(dth, th.data(), sizeof(double) * P * W, hipMemcpyHostToDevice) == hipSuccess);
      CHECK(hipMemcpy(dy0, y0.data(), sizeof(double) * S * W, hipMemcpyHostToDevice) == hipSuccess);
      oe_mh_args a{};
      a.n_walkers = W;
      a.nits = nits;
      a.burnin = burnin;
      a.rng_mode = mode;
      a.chunk = 3;
      a.seed = 9;
      a.step_sd = 0.05;
      a.walk_mask = walk;
      a.init_param = ip;
      a.replay_dz = ddz;
      a.replay_u = du;
      a.theta = dth;
      a.y0 = dy0;
      a.samples = dsamp;
      a.final_stats = dfin;
      a.status = dst;
      a.numpy_seeds = dseeds;
      a.numpy_prior_draws = 2;
      CHECK(oe_mh_run(c, &a, 0) == OE_OK);
      oe_mh_args r = a;  // resume from the chain state at iteration 4
      r.it_start = 4;
      CHECK(oe_mh_run(c, &r, 0) == OE_OK);
      oe_mh_args bad_args = a;
      bad_args.nits = 0;
      CHECK(oe_mh_run(c, &bad_args, 0) == OE_ERR_ARG);
    }
    for (void* ptr : {(void*)dth, (void*)dy0, (void*)dsamp, (void*)dfin, (void*)dst, (void*)ddz, (void*)du,
                      (void*)dseeds})
      CHECK(hipFree(ptr) == hipSuccess);
  }
  // a user RHS compiled at run time; its stiff kernels are built on the first 'auto' problem
  int32_t mid = 0;
  CHECK(oe_model_compile(c, kBody, 4, 5, &mid) == OE_OK && mid >= OE_MODEL_CUSTOM);
  std::vector<double> t, O, sig, lin;
  std::vector<int32_t> tidx;
  std::vector<uint64_t> mask;
  oe_problem p = two_i_problem(t, tidx, mask, O, sig, lin, OE_METHOD_AUTO);
  p.model_id = mid;
  CHECK(oe_problem_set(c, &p) == OE_OK);
  CHECK(oe_integrate(c, W, y0.data(), th.data(), traj.data(), chi.data(), ss.data(), st.data(), OE_HOST_PTRS) ==
        OE_OK);
  CHECK(st[5] & OE_STATUS_STIFF);
  oe_ctx_destroy(c);
}

int main(int argc, char** argv) {
  error_paths();
  if (argc > 1 && std::strcmp(argv[1], "device") == 0) device_paths();
  std::puts("SANITIZE OK");
  return 0;
}
