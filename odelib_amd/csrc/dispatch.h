// dispatch.h — (model, method, trajectory, store-policy) → kernel launcher table.
// Each built-in model is instantiated in its own translation unit (inst_*.hip) so the
// library builds in parallel.
#pragma once
#include <hip/hip_runtime.h>
#include "ode_kernels.cuh"
#include "rtc.h"

namespace oe {

// ---- dispatch table ---------------------------------------------------------
using IntegrateLaunch = void (*)(const DevProblem&, const IntegrateArgs&, dim3, dim3, hipStream_t);
using MHLaunch = void (*)(const DevProblem&, const MHArgs&, dim3, dim3, hipStream_t);

struct Entry {
  int32_t model_id;
  int32_t S;
  int32_t P;  // the model's own parameter count
  // [method][traj][nt]
  IntegrateLaunch integrate[2][2][2];
  IntegrateLaunch rk4_piped[2];  // [nt]; null when S > 8 (LDS ring too large)
  MHLaunch mh[2];
  const RtcModule* rtc = nullptr;  // user RHS compiled at run time (launchers above unused)
};

// launch through the ahead-of-time launcher or the hipRTC module function
inline hipError_t launch_integrate_entry(const Entry* e, int method, int traj, int nt, const DevProblem& dp,
                                         const IntegrateArgs& ia, dim3 g, dim3 b, hipStream_t s) {
  if (e->rtc) {
    DevProblem a0 = dp;
    IntegrateArgs a1 = ia;
    void* args[] = {(void*)&a0, (void*)&a1};
    return hipModuleLaunchKernel(e->rtc->integrate[method][traj][nt], g.x, g.y, g.z, b.x, b.y, b.z, 0, s, args, nullptr);
  }
  e->integrate[method][traj][nt](dp, ia, g, b, s);
  return hipGetLastError();
}
inline hipError_t launch_mh_entry(const Entry* e, int method, const DevProblem& dp, const MHArgs& ma, dim3 g, dim3 b,
                                  hipStream_t s) {
  if (e->rtc) {
    DevProblem a0 = dp;
    MHArgs a1 = ma;
    void* args[] = {(void*)&a0, (void*)&a1};
    return hipModuleLaunchKernel(e->rtc->mh[method], g.x, g.y, g.z, b.x, b.y, b.z, 0, s, args, nullptr);
  }
  e->mh[method](dp, ma, g, b, s);
  return hipGetLastError();
}

template <class M, int METHOD, bool TRAJ, bool NT>
void launch_integrate(const DevProblem& pb, const IntegrateArgs& ia, dim3 g, dim3 b, hipStream_t s) {
  hipLaunchKernelGGL((k_integrate<M, METHOD, TRAJ, NT>), g, b, 0, s, pb, ia);
}
template <class M, bool NT>
void launch_rk4_piped(const DevProblem& pb, const IntegrateArgs& ia, dim3 g, dim3 b, hipStream_t s) {
  hipLaunchKernelGGL((k_integrate_rk4_piped<M, NT>), g, b, 0, s, pb, ia);
}
template <class M, int METHOD>
void launch_mh(const DevProblem& pb, const MHArgs& ma, dim3 g, dim3 b, hipStream_t s) {
  hipLaunchKernelGGL((k_mh<M, METHOD>), g, b, 0, s, pb, ma);
}

template <class M>
Entry make_entry(int32_t model_id) {
  Entry e{};
  e.model_id = model_id;
  e.S = M::S;
  e.P = M::P;
  e.integrate[0][0][0] = launch_integrate<M, 0, false, false>;
  e.integrate[0][1][0] = launch_integrate<M, 0, true, false>;
  e.integrate[0][1][1] = launch_integrate<M, 0, true, true>;
  e.integrate[0][0][1] = launch_integrate<M, 0, false, false>;
  e.integrate[1][0][0] = launch_integrate<M, 1, false, false>;
  e.integrate[1][1][0] = launch_integrate<M, 1, true, false>;
  e.integrate[1][1][1] = launch_integrate<M, 1, true, true>;
  e.integrate[1][0][1] = launch_integrate<M, 1, false, false>;
  if constexpr (M::S <= 8) {
    e.rk4_piped[0] = launch_rk4_piped<M, false>;
    e.rk4_piped[1] = launch_rk4_piped<M, true>;
  }
  e.mh[0] = launch_mh<M, 0>;
  e.mh[1] = launch_mh<M, 1>;
  return e;
}


}  // namespace oe

// one factory per instantiation unit
#define OE_DECLARE_ENTRY(NAME) oe::Entry oe_entry_##NAME()
