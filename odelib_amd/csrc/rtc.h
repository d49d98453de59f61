// rtc.h — user right-hand sides compiled at run time (see rtc.hip).
#pragma once
#include <hip/hip_runtime.h>

#include <string>

namespace oe {

struct RtcModule {
  hipModule_t mod = nullptr;
  hipFunction_t integrate[4][2][2] = {};  // [method][traj][nt]; the stiff methods may be null
  hipFunction_t mh[4] = {};
  hipFunction_t stiff_wave[2][2] = {};    // [traj][nt]: S > 8 with the stiff methods
  int n_methods = 0;                      // 4: RK4, DOPRI5, auto, Rosenbrock; 2: no stiff methods
};

// Compile (and, if out != null, load) the kernels for a user RHS body; 0 on success.
// The stiff methods (auto, Rosenbrock) instantiate the body with dual numbers: when the
// body does not compile for them (e.g. it declares `double` temporaries) or S > 8, the
// module has RK4 and DOPRI5 only (n_methods = 2).
int rtc_build(const std::string& body, int S, int P, const char* arch, RtcModule* out, std::string& err);

}  // namespace oe
