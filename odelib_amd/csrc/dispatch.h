// dispatch.h — (model, method, trajectory, store-policy) → kernel launcher table.
// Each built-in model is instantiated in its own translation unit (inst_*.hip) so the
// library builds in parallel.
#pragma once
#include <hip/hip_runtime.h>
#include "ode_kernels.cuh"
#include "rtc.h"

namespace oe {

// widest model with the producer/consumer RK4 trajectory kernels
#ifndef OE_PIPE_MAX_S
#define OE_PIPE_MAX_S 32  // every built-in (A/B: the piped XCD-ordered kernels win up to chain20)
#endif

// ---- dispatch table ---------------------------------------------------------
using IntegrateLaunch = void (*)(const DevProblem&, const IntegrateArgs&, dim3, dim3, hipStream_t);
using MHLaunch = void (*)(const DevProblem&, const MHArgs&, dim3, dim3, hipStream_t);
using StiffWaveLaunch = void (*)(const DevProblem&, const StiffWaveArgs&, dim3, dim3, hipStream_t);
using MHTreeLaunch = void (*)(const DevProblem&, const MHTreeArgs&, dim3, dim3, hipStream_t);
using HandQLaunch = void (*)(const DevProblem&, const IntegrateArgs&, const HandQ&, dim3, dim3, hipStream_t);

struct Entry {
  int32_t model_id;
  int32_t S;
  int32_t P;  // the model's own parameter count
  // [method][traj][nt]; methods kAuto / kRosenbrock are null when S > kStiffMaxS, kBdf when
  // S > kStiffRegS
  IntegrateLaunch integrate[kMethods][2][2];
  IntegrateLaunch rk4_piped[3][2];  // [2, 4, 8 store waves][nt]; null when S > OE_PIPE_MAX_S
  IntegrateLaunch dopri5_piped[2];  // [nt]: DOPRI5 trajectories through store waves; null when S > 6
  // 'auto' through the hand-over queue (S <= kHandMaxS): the DOPRI5 kernel, [beside][traj][nt]
  // (beside: its register budget leaves room for the BDF kernel on the same SIMDs), and the
  // BDF kernel, [beside][traj][nt] (after the DOPRI5 kernel: its difference table in registers)
  HandQLaunch integrate_hq[2][2][2];
  HandQLaunch bdf_hq[2][2][2];  // [beside][traj][nt]
  MHLaunch mh[kMethods];
  MHLaunch mh_init[kMethods];  // the a-priori pass (MHArgs::init)
  MHTreeLaunch mh_tree[kMethods];  // speculative MH rounds (k_mh_tree); the resolve kernel is shared
  StiffWaveLaunch stiff_wave[2][2];  // [traj][nt]: S > kStiffRegS stiff redo, one wave per walker
  IntegrateLaunch dopri5_split[2][2];  // [traj][nt]: DOPRI5 with split_lanes lanes per walker (split.cuh)
  MHLaunch mh_split = nullptr;         // DOPRI5 Metropolis–Hastings, split_lanes lanes per walker
  MHTreeLaunch mh_split_tree = nullptr;  // its speculative rounds (k_mh_split_tree)
  int32_t split_lanes = 0;             // 0: the model has no split kernel
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
    return hipModuleLaunchKernel(ma.init ? e->rtc->mh_init[method] : e->rtc->mh[method], g.x, g.y, g.z, b.x, b.y, b.z,
                                 0, s, args, nullptr);
  }
  (ma.init ? e->mh_init : e->mh)[method](dp, ma, g, b, s);
  return hipGetLastError();
}

template <class M, int METHOD, bool TRAJ, bool NT>
void launch_integrate(const DevProblem& pb, const IntegrateArgs& ia, dim3 g, dim3 b, hipStream_t s) {
  hipLaunchKernelGGL((k_integrate<M, METHOD, TRAJ, NT>), g, b, 0, s, pb, ia);
}
template <class M, bool NT, int NSW>
void launch_rk4_piped(const DevProblem& pb, const IntegrateArgs& ia, dim3 g, dim3 b, hipStream_t s) {
  hipLaunchKernelGGL((k_integrate_rk4_piped<M, NT, NSW>), g, b, 0, s, pb, ia);
}
template <class M, bool NT>
void launch_dopri5_piped(const DevProblem& pb, const IntegrateArgs& ia, dim3 g, dim3 b, hipStream_t s) {
  hipLaunchKernelGGL((k_integrate_dopri5_piped<M, NT>), g, b, 0, s, pb, ia);
}
template <class M, bool TRAJ, bool NT, bool MIX>
void launch_integrate_hq(const DevProblem& pb, const IntegrateArgs& ia, const HandQ& q, dim3 g, dim3 b, hipStream_t s) {
  hipLaunchKernelGGL((k_integrate_hq<M, TRAJ, NT, MIX>), g, b, 0, s, pb, ia, q);
}
template <class M, bool TRAJ, bool NT, bool DREG>
void launch_bdf_hq(const DevProblem& pb, const IntegrateArgs& ia, const HandQ& q, dim3 g, dim3 b, hipStream_t s) {
  hipLaunchKernelGGL((k_bdf_hq<M, TRAJ, NT, DREG>), g, b, 0, s, pb, ia, q);
}
template <class M, int METHOD, bool INIT = false>
void launch_mh(const DevProblem& pb, const MHArgs& ma, dim3 g, dim3 b, hipStream_t s) {
  hipLaunchKernelGGL((k_mh<M, METHOD, INIT>), g, b, 0, s, pb, ma);
}
inline hipError_t launch_mh_tree_entry(const Entry* e, int method, const DevProblem& dp, const MHTreeArgs& ta,
                                       dim3 g, dim3 b, hipStream_t s) {
  if (e->rtc) {
    DevProblem a0 = dp;
    MHTreeArgs a1 = ta;
    void* args[] = {(void*)&a0, (void*)&a1};
    return hipModuleLaunchKernel(e->rtc->mh_tree[method], g.x, g.y, g.z, b.x, b.y, b.z, 0, s, args, nullptr);
  }
  e->mh_tree[method](dp, ta, g, b, s);
  return hipGetLastError();
}
template <class M, int METHOD>
void launch_mh_tree(const DevProblem& pb, const MHTreeArgs& ta, dim3 g, dim3 b, hipStream_t s) {
  hipLaunchKernelGGL((k_mh_tree<M, METHOD>), g, b, 0, s, pb, ta);
}
template <class M, bool TRAJ, bool NT>
void launch_stiff_wave(const DevProblem& pb, const StiffWaveArgs& sa, dim3 g, dim3 b, hipStream_t s) {
  hipLaunchKernelGGL((k_stiff_wave<M, TRAJ, NT>), g, b, 0, s, pb, sa);
}
inline hipError_t launch_stiff_wave_entry(const Entry* e, int traj, int nt, const DevProblem& dp,
                                          const StiffWaveArgs& sa, dim3 g, dim3 b, hipStream_t s) {
  if (e->rtc) {
    DevProblem a0 = dp;
    StiffWaveArgs a1 = sa;
    void* args[] = {(void*)&a0, (void*)&a1};
    return hipModuleLaunchKernel(e->rtc->stiff_wave[traj][nt], g.x, g.y, g.z, b.x, b.y, b.z, 0, s, args, nullptr);
  }
  e->stiff_wave[traj][nt](dp, sa, g, b, s);
  return hipGetLastError();
}

template <int N, int K, bool TRAJ, bool NT>
void launch_split(const DevProblem& pb, const IntegrateArgs& ia, dim3 g, dim3 b, hipStream_t s) {
  hipLaunchKernelGGL((k_integrate_split<N, K, TRAJ, NT>), g, b, 0, s, pb, ia);
}
template <int N, int K>
void launch_mh_split(const DevProblem& pb, const MHArgs& ma, dim3 g, dim3 b, hipStream_t s) {
  hipLaunchKernelGGL((k_mh_split<N, K>), g, b, 0, s, pb, ma);
}
template <int N, int K>
void launch_mh_split_tree(const DevProblem& pb, const MHTreeArgs& ta, dim3 g, dim3 b, hipStream_t s) {
  hipLaunchKernelGGL((k_mh_split_tree<N, K>), g, b, 0, s, pb, ta);
}
// lanes per walker of a model's split DOPRI5 kernel (split.cuh): the built-in chain only
template <class M>
struct SplitOf { static constexpr int K = 0; };
template <int N>
struct SplitOf<Chain<N>> { static constexpr int K = split_lanes_chain<N>(); };
#ifdef OE_SPLIT_TWOI  // measurement builds: two_i (Chain<4>'s RHS, operation for operation) over 2 or 4 lanes
static_assert(OE_SPLIT_TWOI == 2 || OE_SPLIT_TWOI == 4, "OE_SPLIT_TWOI: 2 or 4 lanes per walker (=2 or =4, not bare)");
template <>
struct SplitOf<TwoI> { static constexpr int K = OE_SPLIT_TWOI; };
#endif
// The split kernels are DOPRI5's only (mh_split / dopri5_split): no 'auto' / 'bdf' launch takes
// them, so the per-lane BDF pass and its deferred-observation scratch (DevProblem::obs_c,
// which oe_mh_run leaves null for split launches) never meet a split walker.

template <class M, int METHOD>
void fill_method(Entry& e) {
  // 'auto' with S <= kHandMaxS integrates through the hand-over queue (integrate_hq / bdf_hq)
  if constexpr (!kHandQueue<M, METHOD>) {
    e.integrate[METHOD][0][0] = launch_integrate<M, METHOD, false, false>;
    e.integrate[METHOD][0][1] = launch_integrate<M, METHOD, false, false>;  // NT only matters with a trajectory
    e.integrate[METHOD][1][0] = launch_integrate<M, METHOD, true, false>;
    e.integrate[METHOD][1][1] = launch_integrate<M, METHOD, true, true>;
  }
  // the stiff methods' MH chains with one lane per chain (S <= kStiffRegS) run as rounds of
  // k_mh_tree + k_mh_resolve, one iteration a round when not speculating (kMhRoundsOnly)
  if constexpr (!kMhRoundsOnly<M, METHOD>) e.mh[METHOD] = launch_mh<M, METHOD>;
  e.mh_init[METHOD] = launch_mh<M, METHOD, true>;
  e.mh_tree[METHOD] = launch_mh_tree<M, METHOD>;
}

template <class M>
Entry make_entry(int32_t model_id) {
  Entry e{};
  e.model_id = model_id;
  e.S = M::S;
  e.P = M::P;
  fill_method<M, kRK4>(e);
  fill_method<M, kDOPRI5>(e);
  if constexpr (M::S <= kStiffMaxS) {
    fill_method<M, kAuto>(e);
    fill_method<M, kRosenbrock>(e);
  }
  if constexpr (M::S <= kStiffRegS) fill_method<M, kBdf>(e);
  if constexpr (M::S <= kHandMaxS) {
    e.integrate_hq[1][0][0] = e.integrate_hq[1][0][1] = launch_integrate_hq<M, false, false, true>;
    e.integrate_hq[1][1][0] = launch_integrate_hq<M, true, false, true>;
    e.integrate_hq[1][1][1] = launch_integrate_hq<M, true, true, true>;
    e.integrate_hq[0][0][0] = e.integrate_hq[0][0][1] = launch_integrate_hq<M, false, false, false>;
    e.integrate_hq[0][1][0] = launch_integrate_hq<M, true, false, false>;
    e.integrate_hq[0][1][1] = launch_integrate_hq<M, true, true, false>;
    e.bdf_hq[1][0][0] = e.bdf_hq[1][0][1] = launch_bdf_hq<M, false, false, false>;
    e.bdf_hq[1][1][0] = launch_bdf_hq<M, true, false, false>;
    e.bdf_hq[1][1][1] = launch_bdf_hq<M, true, true, false>;
    e.bdf_hq[0][0][0] = e.bdf_hq[0][0][1] = launch_bdf_hq<M, false, false, true>;
    e.bdf_hq[0][1][0] = launch_bdf_hq<M, true, false, true>;
    e.bdf_hq[0][1][1] = launch_bdf_hq<M, true, true, true>;
  }
  if constexpr (M::S <= 8 && dp_pipe_slots<M::S>() >= 2) {  // a slot ring of >= 2 steps fits (S <= 6)
    e.dopri5_piped[0] = launch_dopri5_piped<M, false>;
    e.dopri5_piped[1] = launch_dopri5_piped<M, true>;
  }
  if constexpr (M::S > kStiffRegS && M::S <= kStiffMaxS) {
    e.stiff_wave[0][0] = launch_stiff_wave<M, false, false>;
    e.stiff_wave[0][1] = launch_stiff_wave<M, false, false>;
    e.stiff_wave[1][0] = launch_stiff_wave<M, true, false>;
    e.stiff_wave[1][1] = launch_stiff_wave<M, true, true>;
  }
  if constexpr (SplitOf<M>::K > 0) {
    constexpr int K = SplitOf<M>::K;
    e.split_lanes = K;
    e.dopri5_split[0][0] = launch_split<M::S, K, false, false>;
    e.dopri5_split[0][1] = launch_split<M::S, K, false, false>;
    e.dopri5_split[1][0] = launch_split<M::S, K, true, false>;
    e.dopri5_split[1][1] = launch_split<M::S, K, true, true>;
    e.mh_split = launch_mh_split<M::S, K>;
    e.mh_split_tree = launch_mh_split_tree<M::S, K>;
  }
  if constexpr (M::S <= OE_PIPE_MAX_S) {
    e.rk4_piped[0][0] = launch_rk4_piped<M, false, 2>;
    e.rk4_piped[0][1] = launch_rk4_piped<M, true, 2>;
    e.rk4_piped[1][0] = launch_rk4_piped<M, false, 4>;
    e.rk4_piped[1][1] = launch_rk4_piped<M, true, 4>;
    e.rk4_piped[2][0] = launch_rk4_piped<M, false, 8>;
    e.rk4_piped[2][1] = launch_rk4_piped<M, true, 8>;
  }
  return e;
}


}  // namespace oe

// one factory per instantiation unit
#define OE_DECLARE_ENTRY(NAME) oe::Entry oe_entry_##NAME()
