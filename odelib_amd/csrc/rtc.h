// rtc.h — user right-hand sides compiled at run time (see rtc.hip).
#pragma once
#include <hip/hip_runtime.h>

#include <string>

namespace oe {

struct RtcModule {
  hipModule_t mod = nullptr;
  hipFunction_t integrate[2][2][2] = {};  // [method][traj][nt]
  hipFunction_t mh[2] = {};
};

// Compile (and, if out != null, load) the kernels for a user RHS body; 0 on success.
int rtc_build(const std::string& body, int S, int P, const char* arch, RtcModule* out, std::string& err);

}  // namespace oe
