/*
 * odelib_amd.h — C-ABI of the MI355X batched ODE-in-MCMC engine (libodelib_amd.so).
 *
 * This is the drop-in boundary for ODElib's parameter-fitting hot path.  The
 * reference has no FFI: its boundary is Python.  Each entry point
 * below replaces one reference call site; the Python host layer
 * (odelib_amd/_native.py) binds them with ctypes exactly as a maintainer would
 * from ODElib itself.
 *
 *   oe_problem_set   <- ModelFramework.__init__ data setup: times grid
 *                       (ODElib/Framework.py:234), pred_tindex / obs arrays
 *                       (Framework.py:309-329), state summations
 *                       (Framework.py:332-381, applied at :659-664).
 *   oe_integrate     <- ModelFramework.integrate (Framework.py:622-683): the
 *                       scipy odeint call at Framework.py:656, fused with the
 *                       observation gather (:677-682), get_chi
 *                       (Framework.py:685-697 / Statistics/stats.py:22-41)
 *                       and the Rsqrd residual (stats.py:49-56), for W walkers.
 *   oe_mh_run        <- Statistics/Samplers.py:53-174 MetropolisHastings, for W
 *                       independent chains (one per walker), i.e. the
 *                       MCMC(...) chain loop of Framework.py:1013-1030.
 *   oe_allgather_samples <- the pd.concat of the per-process chain posteriors
 *                       (Framework.py:1035-1038) after Pool.starmap (:779-780):
 *                       one RCCL all-gather of the ranks' sample blocks.
 *
 * Conventions
 *   - All buffers are caller-owned.  Pointers are DEVICE pointers unless the
 *     call's flags contain OE_HOST_PTRS (then the library stages through its
 *     own scratch).  The library never frees caller memory.
 *   - Batched layouts are walker-minor ("[state][walker]"): element (s, w) of
 *     a [S][W] array is at s*W + w, so 64 lanes of a wavefront touch 512
 *     contiguous bytes.
 *   - Every call returns OE_OK (0) or a negative OE_ERR_* code; the message is
 *     read with oe_last_error().  Nothing throws or aborts across the ABI.
 *   - Threading: one context per device per host thread.  Calls are
 *     synchronous on return unless OE_ASYNC is passed (then ordered on the
 *     context's stream, see oe_ctx_set_stream).
 */
#ifndef ODELIB_AMD_H
#define ODELIB_AMD_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define OE_ABI_VERSION 6

/* return codes */
enum {
  OE_OK = 0,
  OE_ERR_ARG = -1,         /* invalid argument / shape */
  OE_ERR_HIP = -2,         /* HIP runtime error */
  OE_ERR_STATE = -3,       /* no problem set, etc. */
  OE_ERR_UNSUPPORTED = -4, /* model / method combination not compiled in */
  OE_ERR_NOMEM = -5
};

/* integrators */
enum {
  OE_METHOD_RK4 = 0,    /* fixed-step classical RK4, rk4_substeps steps per output interval */
  OE_METHOD_DOPRI5 = 1, /* Dormand–Prince 5(4), wavefront-shared step, max-norm error,
                           dense output onto the times grid */
  OE_METHOD_AUTO = 2,   /* odeint's LSODA behaviour (Framework.py:656): DOPRI5 with a per-walker
                           stiffness test; a stiff or over-budget walker continues from that point
                           with BDF (n_states <= 8), or is integrated again from t0 by the
                           Rosenbrock method (9..32 states; the Jacobian and LU factors then live
                           in private memory or one wave per walker).  Status bit OE_STATUS_STIFF */
  OE_METHOD_ROSENBROCK = 3, /* stiffly accurate Rosenbrock 4(3) (RODAS) for every walker, exact
                              Jacobian by dual numbers, continuous extension onto the output
                              times.  n_states <= 32 */
  OE_METHOD_BDF = 4      /* LSODA's stiff branch for every walker: variable-order (1..5) BDF in
                            scipy's fixed-leading-coefficient form, max norm, modified Newton on an
                            exact (dual-number) Jacobian.  n_states <= 8.  Trajectory / chi kernels
                            (oe_integrate): walkers share the step size and order per wave.  MH
                            kernels (oe_mh_run): a step size and an order per walker, so a chain
                            does not depend on the chains that share its wavefront */
};

/* built-in right-hand sides (demo notebook models + synthetic chain) */
enum {
  OE_MODEL_ZERO_I = 0, /* S=2 (S,V),        P=3 (mu,phi,beta)         notebook zero_i */
  OE_MODEL_ONE_I = 1,  /* S=3 (S,I1,V),     P=4 (mu,phi,beta,lam)     notebook one_i  */
  OE_MODEL_TWO_I = 2,  /* S=4 (S,I1,I2,V),  P=5 (mu,phi,beta,lam,tau) notebook two_i  */
  OE_MODEL_CHAIN = 3,  /* S=N (S,I1..I_{N-2},V), P=5; N=4 reduces to two_i */
  OE_MODEL_CUSTOM = 1000 /* first id handed out by oe_model_compile (per context) */
};

/* per-walker status bits (OR-ed) */
enum {
  OE_STATUS_NONFINITE = 1, /* a state became NaN/inf */
  OE_STATUS_NEGATIVE = 2,  /* a state went negative at an output time */
  OE_STATUS_MAXSTEP = 4,   /* step budget / step underflow: walker abandoned (NaN output) */
  OE_STATUS_STIFF = 8,     /* OE_METHOD_AUTO: the walker was handed to the stiff method */
  OE_STATUS_INTERNAL = 16  /* oe_mh_run: an internal integrity check failed; the chain stopped storing */
};

/* call flags */
enum {
  OE_HOST_PTRS = 1u, /* buffers are host memory */
  OE_ASYNC = 2u,     /* do not synchronize before returning (device pointers only) */
  OE_NT_STORES = 4u, /* non-temporal trajectory stores */
  OE_PIPE = 8u,      /* RK4 trajectories via the producer/consumer kernel, 2 store waves (built-in models, W even);
                       OE_METHOD_DOPRI5 trajectories (built-in models, S <= 6, one lane per walker): the
                       store-wave kernel (dense output + row stores off the compute waves; same bits) */
  OE_HALF_WAVES = 16u, /* RK4: 32 walkers per wavefront (twice the waves; same results). Chosen
                         automatically for trajectories with S >= 5 at <= 1 wave per SIMD. */
  /* 32u: reserved (was an experimental split-wave layout, measured slower and removed) */
  OE_NO_XCD_REMAP = 64u, /* oe_integrate: keep blockIdx-order walker blocks.  By default the
                           blocks the XCDs receive (round-robin dispatch) take runs of 512
                           consecutive walkers in turn, so each XCD writes 4 KiB runs of every
                           trajectory row (same results, faster trajectory stores) */
  OE_NO_TIMING = 128u,  /* oe_integrate: record no timing events around the launch (back-to-back
                           launches without event markers between them); oe_last_kernel_ms
                           then reports OE_ERR_STATE until a timed call */
  OE_PIPE_4 = 512u,     /* as OE_PIPE with 4 / 8 store waves per 4 compute waves (opt-in) */
  OE_PIPE_8 = 1024u,
  OE_XCD_RANGES = 2048u, /* oe_integrate: one contiguous walker range per XCD instead (the r01
                           mapping; same results) */
  OE_NO_SPLIT = 4096u,  /* oe_integrate / oe_mh_run, OE_METHOD_DOPRI5: one lane per walker even for the models
                           whose DOPRI5 kernel splits a walker over K lanes (built-in chain with
                           14..22 states: K = 2; 24+ states, a multiple of 4: K = 4).  A split
                           wave holds 64/K walkers, which share one step size, so results differ
                           from the one-lane grouping (64 walkers per step size) within tolerance */
  OE_TUNE = 8192u,      /* oe_integrate, OE_METHOD_RK4 with a trajectory: pick the fastest of the
                           RK4 trajectory kernels (OE_KERNEL_*; all produce the same bits) for this
                           shape on this device.  The first call for a shape (model, W, T,
                           substeps, store policy, XCD order) runs each candidate back to back
                           after ~60 ms of launches (the clock settles), three interleaved rounds,
                           and keeps the fastest (the default kernel unless another is > 1 %
                           faster); later calls reuse the choice (built-in models: every
                           context of the process on that device).  The first call synchronizes
                           the stream.  Overrides OE_PIPE*, OE_HALF_WAVES. */
  OE_PIPE_XCD = 16384u  /* with OE_PIPE / OE_PIPE_4 / OE_PIPE_8: the piped kernel's workgroups dealt
                           to the XCDs in runs of 512 walkers (OE_KERNEL_PIPE*X) */
};

/* RK4 trajectory kernels (oe_last_variant; all bitwise identical; OE_TUNE times those
 * available for the shape: the piped ones need W even and a built-in model,
 * the X ones the default XCD order) */
enum {
  OE_KERNEL_DIRECT = 0, /* one walker per lane, 64 walkers per wavefront, stores from the compute waves */
  OE_KERNEL_HALF = 1,   /* 32 walkers per wavefront (OE_HALF_WAVES) */
  OE_KERNEL_PIPE2 = 2,  /* producer/consumer: 4 compute waves + 2 / 4 / 8 store waves per workgroup */
  OE_KERNEL_PIPE4 = 3,  /*   through an LDS ring (OE_PIPE / OE_PIPE_4 / OE_PIPE_8) */
  OE_KERNEL_PIPE8 = 4,
  OE_KERNEL_PIPE2X = 5, /* the same with the workgroups dealt to the XCDs in runs of 512 walkers */
  OE_KERNEL_PIPE4X = 6, /*   (the piped kernels' default is blockIdx order) */
  OE_KERNEL_PIPE8X = 7,
  OE_KERNEL_OTHER = 8,  /* not an RK4 trajectory launch (DOPRI5, stiff, no trajectory, MH) */
  OE_KERNEL_COUNT = 9
};

/* RNG modes for oe_mh_run */
enum {
  OE_RNG_REPLAY = 0, /* caller supplies the proposal increments and uniforms */
  OE_RNG_PHILOX = 1, /* counter-based Philox4x32-10 keyed by (seed, global walker id) */
  OE_RNG_NUMPY = 2   /* per chain numpy legacy RandomState(numpy_seeds[w]) on the device, drawn in
                        the reference's order (Samplers.py:70, 104-127): normal(0, step_sd) per
                        walking parameter, numpy_prior_draws standard normals (the prior pdf()
                        calls' lognorm rvs, Framework.py:103), one random_sample() */
};

typedef struct oe_ctx oe_ctx;

/* The fit problem: everything ModelFramework.__init__ derives from the data. */
typedef struct {
  int32_t model_id;          /* OE_MODEL_* */
  int32_t n_states;          /* S (for OE_MODEL_CHAIN: N) */
  int32_t n_params;          /* model's own P <= n_params <= P + min(S, 4); extra entries
                                are e.g. '<state>0' initial-condition parameters */
  int32_t n_times;           /* T >= 2 */
  const double* times;       /* [T] host, strictly increasing (np.linspace grid) */
  int32_t n_obs;             /* number of observations (0 = no likelihood) */
  const int32_t* obs_tidx;   /* [n_obs] host: grid index (first-nearest, Framework.py:316) */
  const uint64_t* obs_mask;  /* [n_obs] host: bitmask of ODE states summed into the
                                observed column (Framework.py:659-664), S <= 64 */
  const double* obs_log;     /* [n_obs] host: observed log abundance O */
  const double* obs_logsigma;/* [n_obs] host: log sigma S */
  const double* obs_lin;     /* [n_obs] host: exp(O) as numpy computes it (Framework.py:700) */
  int32_t method;            /* OE_METHOD_* */
  int32_t rk4_substeps;      /* >= 1 */
  double rtol, atol;         /* DOPRI5 tolerances (odeint defaults 1.49012e-8) */
  int32_t max_steps;         /* DOPRI5 steps per output interval (odeint mxstep 500) */
  double sstot;              /* Σ n_s·var(O_s) for R² (stats.py:49-56) */
  int32_t pnum;              /* parameter count used by AIC (Framework.py:261-263) */
} oe_problem;

/* Metropolis–Hastings over W independent chains (Samplers.py:53-174). */
typedef struct {
  int64_t n_walkers;          /* W (walkers on this device) */
  int64_t walker_offset;      /* global id of walker 0 (Philox key; sharding across ranks) */
  int32_t nits;               /* reference nits: iterations 1..nits-1 are run (Samplers.py:84) */
  int32_t burnin;             /* samples kept for it > burnin (Samplers.py:147) */
  int32_t rng_mode;           /* OE_RNG_* */
  int32_t chunk;              /* iterations per kernel launch (0 = library default) */
  uint64_t seed;              /* Philox seed */
  double step_sd;             /* log-normal walk sd (Framework.py:107: 0.05) */
  const uint8_t* walk_mask;   /* [P] host: 1 = parameter walks, 0 = static */
  const int32_t* init_param;  /* [S] host: -1, or p for a '<state>0' parameter
                                 (Samplers.py:110-114, :139-143) */
  const double* replay_dz;    /* [nits-1][P][W] proposal increments (REPLAY) */
  const double* replay_u;     /* [nits-1][W] acceptance uniforms (REPLAY) */
  double* theta;              /* [P][W] in: initial θ; out: final θ */
  double* y0;                 /* [S][W] in: initial states; out: final states */
  double* samples;            /* [nits-1-burnin][P+5][W] out: θ, chi, rsquared, aic,
                                 iteration, acceptance_ratio (Samplers.py:160-165)
                                 (resume: [nits-max(it_start, burnin+1)][P+5][W]) */
  double* final_stats;        /* [4][W] out (may be NULL): chi, rsquared, aic, n_accepted */
  int32_t* status;            /* [W] out (may be NULL): status bits of the integration of the
                                 chain's current (last accepted / initial) state */
  const uint32_t* numpy_seeds;/* [W] device: per chain seed (NUMPY; MCMC uses the chain index,
                                 Framework.py:1015/1020) */
  int32_t numpy_prior_draws;  /* NUMPY: standard normals consumed per iteration after the
                                 proposal normals */
  int32_t it_start;           /* 0 or 1: fresh run (a-priori fit first, Samplers.py:88-91).
                                 k > 1: RESUME at reference iteration k from a checkpoint:
                                 theta, y0, final_stats and status hold the chain state after
                                 iteration k-1 (inputs); samples receives the rows of iterations
                                 max(k, burnin+1)..nits-1.  Philox counters and replay arrays
                                 are indexed by iteration; NUMPY streams are re-seeded and
                                 fast-forwarded on the device.  Same results as one run. */
  int32_t speculate;          /* (ABI 5) speculative rounds for small ensembles: 0 = off (one
                                 iteration per step), -1 = depth chosen by the library (off when
                                 the chains fill the device), d >= 2: d iterations per round.  A
                                 round integrates every proposal the next d accept/reject
                                 decisions can lead to (2^d - 1 per chain) at once, then keeps
                                 each chain's actual path: the same Markov chain, the same draws
                                 in the same order.  RK4, and DOPRI5 / auto / BDF with
                                 n_states <= 8 (a step size per lane): bitwise the chains of
                                 speculate = 0; larger models: within the integration tolerance
                                 (a wave's 64 lanes share one step size, and they are other
                                 proposals here).
                                 Every MH kernel: built-in and hipRTC models, one lane or split
                                 over K lanes per chain (the depth then counts K lanes per
                                 proposal). */
} oe_mh_args;

int oe_abi_version(void);

/* Model registry query: fills S (for CHAIN pass the wanted N in *n_states) and the
 * model's own parameter count.  Returns OE_ERR_UNSUPPORTED if not compiled in. */
int oe_model_info(int32_t model_id, int32_t* n_states, int32_t* n_params);

/* User right-hand side compiled at run time (hipRTC) for this context's device.
 * rhs_body is the body of
 *     template <class R> __device__ void rhs(const R* y, R t, const R* ps, R* dy)
 * (C++; y[0..n_states), ps[0..n_params), t; must assign dy[0..n_states)), i.e. the
 * reference's ODE(y, t, ps) callable (Framework.py:177-180) re-declared in C.  On success
 * *model_id (>= OE_MODEL_CUSTOM) is usable in oe_problem.model_id with this context.
 * Compile errors are returned as OE_ERR_ARG with the compiler log in oe_last_error. */
int oe_model_compile(oe_ctx* ctx, const char* rhs_body, int32_t n_states, int32_t n_params, int32_t* model_id);
/* Compile-only check of a user RHS for target `arch` (e.g. "gfx950"); needs no GPU.
 * Errors: oe_last_error(NULL). */
int oe_rtc_check(const char* rhs_body, int32_t n_states, int32_t n_params, const char* arch);

int oe_ctx_create(int32_t device, oe_ctx** out);
void oe_ctx_destroy(oe_ctx* ctx);
const char* oe_last_error(const oe_ctx* ctx);
/* Launch on an existing hipStream_t (e.g. torch.cuda.current_stream().cuda_stream),
 * used as given: NULL is the null (legacy default) stream. */
int oe_ctx_set_stream(oe_ctx* ctx, void* hip_stream);
/* Launch on the context's own non-blocking stream (the default after oe_ctx_create). */
int oe_ctx_use_own_stream(oe_ctx* ctx);

int oe_problem_set(oe_ctx* ctx, const oe_problem* problem);

/* Batched integrate + fused likelihood.
 *   y0     [S][W]    initial states            (Framework.py:647-650)
 *   theta  [P][W]    parameters                (Framework.py:651-654)
 *   traj   [T][S][W] full trajectory, or NULL  (the odeint [T,S] output, :656)
 *   chi    [W] or NULL   Σ_finite (O − log C)²/(2S²)   (stats.py:41), NaN if all masked
 *   ssres  [W] or NULL   Σ_nan-skipping (C − exp O)²     (stats.py:52)
 *   status [W] or NULL
 * OE_METHOD_AUTO with S <= 8 also keeps an n_obs * W * 8-byte device scratch in the context
 * (the BDF pass's deferred observations), allocated on first use and grown as W grows;
 * OE_ERR_HIP if that allocation fails. */
int oe_integrate(oe_ctx* ctx, int64_t n_walkers, const double* y0, const double* theta,
                 double* traj, double* chi, double* ssres, int32_t* status, uint32_t flags);

/* Batched Metropolis–Hastings; device pointers only. */
int oe_mh_run(oe_ctx* ctx, const oe_mh_args* args, uint32_t flags);

/* The reference's proposal streams on the device: for chain w, numpy legacy
 * RandomState(seeds[w]) (MT19937, Box–Muller polar gauss with its cached second value,
 * 53-bit random_sample) consumed per iteration as in OE_RNG_NUMPY.  Writes
 * dz [nits-1][P][W] (step_sd·N(0,1) for walking parameters, 0 for static ones) and
 * u [nits-1][W]: the replay_dz / replay_u inputs of OE_RNG_REPLAY.  Device pointers. */
int oe_numpy_streams(oe_ctx* ctx, int64_t n_walkers, const uint32_t* seeds, int32_t nits, int32_t n_params,
                     const uint8_t* walk_mask, int32_t prior_draws, double step_sd, double* dz, double* u);

/* ---- multi-GPU posterior pooling (one process per GPU, RCCL over xGMI) ----------------
 * Ranks own contiguous global walker ids (rank r: counts[r] walkers after those of ranks
 * < r) and run oe_mh_run with walker_offset = their first id.  Their sample blocks are
 * pooled by ONE all-gather, the analogue of Framework.py:1037's pd.concat.
 * The communicator is RCCL's (librccl.so opened at first use).  Rank 0 creates the id
 * with oe_comm_unique_id and hands the 128 bytes to the other ranks by any channel (MPI,
 * torch.distributed broadcast, a file); every rank then calls oe_comm_init with it. */
#define OE_COMM_ID_BYTES 128
typedef struct oe_comm oe_comm;
int oe_comm_unique_id(uint8_t* id, int32_t id_bytes);
int oe_comm_init(int32_t device, int32_t n_ranks, int32_t rank, const uint8_t* id, int32_t id_bytes,
                 oe_comm** out);
void oe_comm_destroy(oe_comm* comm);
const char* oe_comm_last_error(const oe_comm* comm); /* NULL: the last oe_comm_init / unique_id error */
/* Launch the collective on this hipStream_t (NULL = the null stream, the default). */
int oe_comm_set_stream(oe_comm* comm, void* hip_stream);
/* Every rank's block [rows][counts[rank]] (device, walker-minor, e.g. oe_mh_run's samples
 * viewed as rows = kept*(P+5)) gathered into out [rows][sum(counts)] (device) on every
 * rank, in global walker order.  Uneven counts are padded for the collective.  Flags:
 * OE_ASYNC (do not synchronize the stream before returning). */
int oe_allgather_samples(oe_comm* comm, int64_t rows, const double* block, const int64_t* counts, double* out,
                         uint32_t flags);
/* The two data movements of oe_allgather_samples, callable without a communicator (one
 * device; tests drive the n-rank layout with a synthetic gathered buffer):
 *   oe_pool_pad:      block [rows][count] -> padded [rows][cmax] (zeros beyond count), the
 *                     send block of a rank with fewer walkers than the largest;
 *   oe_pool_relayout: the collective's rank-major result gathered [n_ranks][rows][cmax]
 *                     (cmax = max counts) -> out [rows][sum(counts)], rank r's walkers at
 *                     columns sum(counts[:r]) .. + counts[r] (global walker order).
 * Device pointers; hip_stream NULL = the null stream; synchronous unless OE_ASYNC.  Errors
 * read with oe_comm_last_error(NULL). */
int oe_pool_pad(int64_t rows, const double* block, int64_t count, int64_t cmax, double* padded, void* hip_stream,
                uint32_t flags);
int oe_pool_relayout(int32_t n_ranks, int64_t rows, const int64_t* counts, const double* gathered, double* out,
                     void* hip_stream, uint32_t flags);

/* Device time (ms) of the kernel launches of the last oe_integrate / oe_mh_run,
 * from HIP events recorded on the context's stream around them (waits for them). */
int oe_last_kernel_ms(oe_ctx* ctx, double* ms);

/* Iterations per speculative round of the last oe_mh_run (oe_mh_args.speculate); 0 = it ran
 * one iteration per step. */
int oe_last_mh_depth(oe_ctx* ctx, int32_t* depth);
/* The kernel (OE_KERNEL_*) the last oe_integrate launched.  OE_ERR_STATE before any call. */
int oe_last_variant(oe_ctx* ctx, int32_t* variant);
/* OE_TUNE's measurements for the shape of the last oe_integrate: ms[k] = mean launch time of
 * kernel k (back to back, best of the rounds), NaN for kernels not measured (not available for
 * the shape).  n >= OE_KERNEL_COUNT - 1 entries.  OE_ERR_STATE if that call was not tuned. */
int oe_tune_times(oe_ctx* ctx, double* ms, int32_t n);

#ifdef __cplusplus
}
#endif

#endif /* ODELIB_AMD_H */
