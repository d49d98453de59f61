// rtc.hip — run-time compilation of user right-hand sides (hipRTC).
//
// The reference integrates any user Python callable ODE(y, t, ps) (Framework.py:177-180,
// :656).  Built-in models are compiled ahead of time (models.cuh); any other RHS is
// given as the body of
//     template <class R> __device__ void rhs(const R* y, R t, const R* ps, R* dy)
// (C source, or transpiled from the Python callable by odelib_amd/transpile.py) and the
// SAME kernel templates (ode_kernels.cuh, embedded at build time) are instantiated for
// it with hiprtc for the device's gfx950 target, loaded as a module and launched with
// hipModuleLaunchKernel.  The explicit methods are compiled with the model; the stiff
// ones (dual-number Jacobian, the larger kernels) only when a problem first asks for them.
#include <hip/hip_runtime.h>
#include <hip/hiprtc.h>

#include <cstdio>
#include <string>
#include <vector>

#include "dispatch.h"
#include "rtc.h"
#include "rtc_source.inc"

namespace oe {

static const char* kMethodName[5] = {"0", "1", "2", "3", "4"};
static const char* kBool[2] = {"false", "true"};

std::string rtc_integrate_name(int method, int traj, int nt) {
  return std::string("oe::k_integrate<UserModel, ") + kMethodName[method] + ", " + kBool[traj] + ", " + kBool[nt] + ">";
}
std::string rtc_mh_name(int method) { return std::string("oe::k_mh<UserModel, ") + kMethodName[method] + ">"; }
std::string rtc_mh_init_name(int method) {
  return std::string("oe::k_mh<UserModel, ") + kMethodName[method] + ", true>";
}
std::string rtc_mh_tree_name(int method) {
  return std::string("oe::k_mh_tree<UserModel, ") + kMethodName[method] + ">";
}
std::string rtc_stiff_wave_name(int traj, int nt) {
  return std::string("oe::k_stiff_wave<UserModel, ") + kBool[traj] + ", " + kBool[nt] + ">";
}
static bool has_stiff_wave(int S, RtcPart part) { return part == kRtcStiff && S > kStiffRegS; }
// k_mh's iteration loop for method m (ode_kernels.cuh kMhRoundsOnly: the stiff methods of
// register-path models run their chains as k_mh_tree rounds only)
static bool has_mh_loop(int S, int m) { return !((m == 2 || m == 4) && S <= kStiffRegS); }
static int first_method(RtcPart part) { return part == kRtcStiff ? 2 : 0; }
// the methods of a part: RK4 + DOPRI5; auto + Rosenbrock (+ BDF up to kStiffRegS states)
static int end_method(int S, RtcPart part) { return part == kRtcStiff ? (S <= kStiffRegS ? 5 : 4) : 2; }

std::string rtc_source(const std::string& body, int S, int P, RtcPart part) {
  std::string src;
  src += "typedef unsigned long long uint64_t; typedef long long int64_t;\n";
  src += "typedef unsigned int uint32_t; typedef int int32_t;\n";
  src += kRtcKernelSource;
  char hdr[256];
  snprintf(hdr, sizeof(hdr), "\nstruct UserModel {\n  static constexpr int S = %d, P = %d;\n", S, P);
  src += hdr;
  src += "  template <class R>\n  __device__ static inline void rhs(const R* y, R t, const R* ps, R* dy) {\n";
  src += "    (void)t;\n";
  src += body;
  src += "\n  }\n};\n";
  for (int m = first_method(part); m < end_method(S, part); ++m) {
    for (int tr = 0; tr < 2; ++tr)
      for (int nt = 0; nt < 2; ++nt)
        src += "template __global__ void " + rtc_integrate_name(m, tr, nt) + "(const oe::DevProblem, const oe::IntegrateArgs);\n";
    if (has_mh_loop(S, m)) src += "template __global__ void " + rtc_mh_name(m) + "(const oe::DevProblem, const oe::MHArgs);\n";
    src += "template __global__ void " + rtc_mh_init_name(m) + "(const oe::DevProblem, const oe::MHArgs);\n";
    src += "template __global__ void " + rtc_mh_tree_name(m) + "(const oe::DevProblem, const oe::MHTreeArgs);\n";
  }
  if (has_stiff_wave(S, part))
    for (int tr = 0; tr < 2; ++tr)
      for (int nt = 0; nt < 2; ++nt)
        src += "template __global__ void " + rtc_stiff_wave_name(tr, nt) +
               "(const oe::DevProblem, const oe::StiffWaveArgs);\n";
  return src;
}

static int compile_program(const std::string& src, const char* arch, std::vector<std::string>& names,
                           std::vector<std::string>& lowered, std::vector<char>& code, std::string& log) {
  hiprtcProgram prog;
  if (hiprtcCreateProgram(&prog, src.c_str(), "odelib_user_rhs.hip", 0, nullptr, nullptr) != HIPRTC_SUCCESS) {
    log = "hiprtcCreateProgram failed";
    return -1;
  }
  for (auto& n : names) hiprtcAddNameExpression(prog, n.c_str());
  std::string archopt = std::string("--offload-arch=") + arch;
  const char* opts[] = {archopt.c_str(), "-O3", "-ffp-contract=off", "-std=c++17"};
  const hiprtcResult r = hiprtcCompileProgram(prog, 4, opts);
  size_t ls = 0;
  hiprtcGetProgramLogSize(prog, &ls);
  log.assign(ls, '\0');
  if (ls) hiprtcGetProgramLog(prog, &log[0]);
  if (r != HIPRTC_SUCCESS) {
    hiprtcDestroyProgram(&prog);
    return -1;
  }
  lowered.clear();
  for (auto& n : names) {
    const char* lw = nullptr;
    if (hiprtcGetLoweredName(prog, n.c_str(), &lw) != HIPRTC_SUCCESS || !lw) {
      log += "\nno lowered name for " + n;
      hiprtcDestroyProgram(&prog);
      return -1;
    }
    lowered.emplace_back(lw);
  }
  size_t cs = 0;
  hiprtcGetCodeSize(prog, &cs);
  code.resize(cs);
  hiprtcGetCode(prog, code.data());
  hiprtcDestroyProgram(&prog);
  return 0;
}

static std::vector<std::string> all_names(int S, RtcPart part) {
  std::vector<std::string> names;
  const int m0 = first_method(part);
  for (int m = m0; m < end_method(S, part); ++m)
    for (int tr = 0; tr < 2; ++tr)
      for (int nt = 0; nt < 2; ++nt) names.push_back(rtc_integrate_name(m, tr, nt));
  for (int m = m0; m < end_method(S, part); ++m)
    if (has_mh_loop(S, m)) names.push_back(rtc_mh_name(m));
  for (int m = m0; m < end_method(S, part); ++m) names.push_back(rtc_mh_init_name(m));
  for (int m = m0; m < end_method(S, part); ++m) names.push_back(rtc_mh_tree_name(m));
  if (has_stiff_wave(S, part))
    for (int tr = 0; tr < 2; ++tr)
      for (int nt = 0; nt < 2; ++nt) names.push_back(rtc_stiff_wave_name(tr, nt));
  return names;
}

int rtc_build(const std::string& body, int S, int P, const char* arch, RtcPart part, RtcModule* out,
              std::string& err) {
  if (part == kRtcStiff && S > kStiffMaxS) {
    err = "the stiff methods (auto, rosenbrock) need n_states <= " + std::to_string(kStiffMaxS);
    return -1;
  }
  std::vector<std::string> names = all_names(S, part), lowered;
  std::vector<char> code;
  std::string log;
  if (compile_program(rtc_source(body, S, P, part), arch, names, lowered, code, log)) {
    err = part == kRtcStiff
              ? "the stiff methods (auto, rosenbrock) need a right-hand side that compiles for dual numbers "
                "(templated on its scalar type R); hipRTC said:\n" + log
              : "hipRTC compilation of the user RHS failed:\n" + log;
    return -1;
  }
  if (!out) return 0;  // compile check only
  hipModule_t mod;
  if (hipModuleLoadData(&mod, code.data()) != hipSuccess) {
    err = "hipModuleLoadData failed for the user RHS";
    return -1;
  }
  (part == kRtcStiff ? out->stiff_mod : out->mod) = mod;
  size_t idx = 0;
  const int m0 = first_method(part);
  auto get = [&](hipFunction_t* f) {
    if (hipModuleGetFunction(f, mod, lowered[idx++].c_str()) != hipSuccess) {
      err = "hipModuleGetFunction failed for the user RHS";
      return false;
    }
    return true;
  };
  for (int m = m0; m < end_method(S, part); ++m)
    for (int tr = 0; tr < 2; ++tr)
      for (int nt = 0; nt < 2; ++nt)
        if (!get(&out->integrate[m][tr][nt])) return -1;
  for (int m = m0; m < end_method(S, part); ++m)
    if (has_mh_loop(S, m) && !get(&out->mh[m])) return -1;
  for (int m = m0; m < end_method(S, part); ++m)
    if (!get(&out->mh_init[m])) return -1;
  for (int m = m0; m < end_method(S, part); ++m)
    if (!get(&out->mh_tree[m])) return -1;
  if (has_stiff_wave(S, part))
    for (int tr = 0; tr < 2; ++tr)
      for (int nt = 0; nt < 2; ++nt)
        if (!get(&out->stiff_wave[tr][nt])) return -1;
  if (part == kRtcStiff) out->stiff = 1;
  return 0;
}

}  // namespace oe
