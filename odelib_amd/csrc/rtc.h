// rtc.h — user right-hand sides compiled at run time (see rtc.hip).
#pragma once
#include <hip/hip_runtime.h>

#include <string>

namespace oe {

// The kernels of one user RHS, built in two parts on demand: the explicit methods (RK4,
// DOPRI5) when the model is compiled, the stiff ones (auto, Rosenbrock, BDF: the body
// instantiated with dual numbers, plus the one-wave-per-walker kernel for S > 8) the first
// time a problem asks for them.
struct RtcModule {
  hipModule_t mod = nullptr;              // RK4 + DOPRI5
  hipModule_t stiff_mod = nullptr;        // auto + Rosenbrock + BDF (+ k_stiff_wave)
  hipFunction_t integrate[5][2][2] = {};  // [method][traj][nt]; the stiff methods null until built
  hipFunction_t mh[5] = {};
  hipFunction_t mh_init[5] = {};           // the a-priori pass (k_mh<.., INIT = true>)
  hipFunction_t mh_tree[5] = {};          // speculative MH rounds (k_mh_tree)
  hipFunction_t stiff_wave[2][2] = {};    // [traj][nt]: S > kStiffRegS with the stiff methods
  int stiff = 0;                          // 0: not built yet, 1: built, -1: unavailable (stiff_err)
  std::string stiff_err;
};

enum RtcPart { kRtcExplicit = 0, kRtcStiff = 1 };

// Compile (and, if out != null, load into *out) one part of the kernels of a user RHS
// body; 0 on success, else -1 with the compiler log in err.  The stiff part needs
// S <= kStiffMaxS and a body that compiles for dual numbers (templated on R, no `double`
// temporaries).
int rtc_build(const std::string& body, int S, int P, const char* arch, RtcPart part, RtcModule* out,
              std::string& err);

}  // namespace oe
