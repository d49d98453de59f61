"""Register / scratch budgets of the hot kernels, read from the compiler (CPU, no GPU).

A kernel that starts spilling is still bitwise correct, so parity tests do not see it;
the chain20 DOPRI5 MH kernel once doubled in time (13.4 vs 6.3 ms per iteration,
DESIGN.md §3.4 r01k) after unrelated integrator changes pushed it to 432 B/lane of
scratch.  These budgets catch that at build time: hipcc's kernel-resource-usage remarks
for the translation units the bench and the C3 configs use, and for the stiff methods' MH
kernels (k_mh / k_mh_tree with 'auto' and 'bdf', the per-lane BDF pass of csrc/bdf.cuh)
of every built-in model with at most 8 states.
"""
import os
import re
import shutil
import subprocess

import pytest

CSRC = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "odelib_amd", "csrc")
HIPCC = "/opt/rocm/bin/hipcc"
FLAGS = ["-O3", "-std=c++17", "-fPIC", "-ffp-contract=off", "--offload-arch=gfx950", "--cuda-device-only",
         "-Rpass-analysis=kernel-resource-usage", "-c", "-o", os.devnull]
SMALL_UNITS = ["inst_zero_i.hip", "inst_one_i.hip", "inst_two_i.hip", "inst_chain4.hip"]  # S <= 4
WIDE_REG_UNITS = ["inst_chain5.hip", "inst_chain6.hip", "inst_chain8.hip"]  # the register path's widest

_FIELDS = {"VGPRs": "vgpr", "AGPRs": "agpr", "ScratchSize [bytes/lane]": "scratch",
           "Occupancy [waves/SIMD]": "occupancy", "SGPRs Spill": "sgpr_spill", "VGPRs Spill": "vgpr_spill"}


def _parse(text):
    kernels, cur = {}, None
    for line in text.splitlines():
        m = re.search(r"remark: Function Name: (\S+)", line)
        if m:
            cur = kernels.setdefault(m.group(1), {})
            continue
        m = re.search(r"remark:\s+([^:]+): (\d+)", line)
        if m and cur is not None and m.group(1).strip() in _FIELDS:
            cur[_FIELDS[m.group(1).strip()]] = int(m.group(2))
    return kernels


@pytest.fixture(scope="module")
def resources():
    if not os.path.exists(HIPCC) and shutil.which("hipcc") is None:
        pytest.skip("hipcc not available")
    units = sorted(set(SMALL_UNITS + WIDE_REG_UNITS + ["inst_chain20.hip"]))
    procs = {u: subprocess.Popen([HIPCC, *FLAGS, u], cwd=CSRC, stdout=subprocess.PIPE,
                                 stderr=subprocess.STDOUT, text=True) for u in units}
    out = {}
    for u, p in procs.items():
        text, _ = p.communicate(timeout=600)
        assert p.returncode == 0, text[-2000:]
        out[u] = _parse(text)
    return out


def _find(kernels, *needles):
    hits = [v for k, v in kernels.items() if all(n in k for n in needles)]
    assert len(hits) == 1, (needles, list(kernels))
    return hits[0]


# mangled-name fragments: k_integrate<M, METHOD(0 RK4, 1 DOPRI5), TRAJ, NT>, k_mh<M, METHOD, INIT>
C1 = ("k_integrateINS_4TwoIELi0ELb1ELb1E",)
C2 = ("k_integrateINS_4TwoIELi1ELb1ELb1E",)
C3 = ("k_integrateINS_5ChainILi20EEELi0ELb1ELb1E",)
# k_mh<M, METHOD, INIT>: the iteration-loop kernel (INIT false)
MH_TWO_I_RK4 = ("k_mhINS_4TwoIELi0ELb0E",)
MH_TWO_I_DOPRI5 = ("k_mhINS_4TwoIELi1ELb0E",)
MH_CHAIN20_RK4 = ("k_mhINS_5ChainILi20EEELi0ELb0E",)
MH_CHAIN20_DOPRI5 = ("k_mhINS_5ChainILi20EEELi1ELb0E",)
# speculative MH rounds (k_mh_tree<M, METHOD>): the sequential MH kernel's occupancy
TREE_TWO_I_RK4 = ("k_mh_treeINS_4TwoIELi0E",)
TREE_TWO_I_DOPRI5 = ("k_mh_treeINS_4TwoIELi1E",)


def test_two_i_kernels_never_spill(resources):
    """No two_i kernel touches scratch; the kernels without a stiff method do not spill at
    all (the 'auto' / 'bdf' kernels run at one wave per SIMD, where a spill lands in AGPRs)."""
    for name, r in resources["inst_two_i.hip"].items():
        assert r["scratch"] == 0, (name, r)
        if not re.search(r"ELi[24]E", name):
            assert r["vgpr_spill"] == 0, (name, r)


@pytest.mark.parametrize("needles,min_occ", [(C1, 4), (C2, 2), (MH_TWO_I_RK4, 4), (MH_TWO_I_DOPRI5, 2),
                                             (TREE_TWO_I_RK4, 4), (TREE_TWO_I_DOPRI5, 2)])
def test_two_i_occupancy(resources, needles, min_occ):
    r = _find(resources["inst_two_i.hip"], *needles)
    assert r["occupancy"] >= min_occ, r


def test_chain20_rk4_kernels_fit_registers(resources):
    for needles in (C3, MH_CHAIN20_RK4):
        r = _find(resources["inst_chain20.hip"], *needles)
        assert r["scratch"] == 0 and r["vgpr_spill"] == 0 and r["occupancy"] >= 2, (needles, r)


def test_chain20_dopri5_mh_scratch_budget(resources):
    r = _find(resources["inst_chain20.hip"], *MH_CHAIN20_DOPRI5)
    assert r["scratch"] <= 192, r  # 160 B/lane at r01k; 432 when it ran 2x slower


def _stiff_mh(kernels):
    """the MH kernels of the stiff methods: k_mh<M, METHOD, INIT> / k_mh_tree<M, METHOD> with
    METHOD 2 ('auto') or 4 ('bdf')"""
    return {k: v for k, v in kernels.items() if re.search(r"k_mh(_tree)?I.*?ELi[24]E", k)}


def _stiff(kernels):
    """every kernel of the stiff methods: the MH kernels above, k_integrate<M, 2 | 4, ...> and
    the hand-over queue's k_integrate_hq / k_bdf_hq ('auto', S <= 4)"""
    return {k: v for k, v in kernels.items()
            if re.search(r"k_mh(_tree)?I.*?ELi[24]E|k_integrateI.*?ELi[24]ELb|k_integrate_hq|k_bdf_hq", k)}


@pytest.mark.parametrize("unit", SMALL_UNITS)
def test_small_models_never_spill(resources, unit):
    """Up to 4 states every kernel — the stiff methods' MH, integrate and hand-over-queue kernels
    with the per-lane BDF pass included — runs without scratch."""
    ks = resources[unit]
    assert len(_stiff_mh(ks)) == 4, list(ks)
    for name, r in ks.items():
        assert r["scratch"] == 0, (name, r)


def test_two_i_stiff_kernels_spill_budget(resources):
    """the drop-in default's kernels out of the SGPR-spill regime of round 4's
    unexplained failures (k_mh<TwoI, auto> carried 510 spilled SGPRs at 256 VGPR + 67 AGPR).
    Every two_i kernel of 'auto' and 'bdf': no VGPR spill, no scratch, at most 64 SGPRs spilled
    to VGPR lanes — except the trajectory kernels of method 'bdf' (the wave-lockstep pass,
    bdf_wave.cuh: 67 in r06), held at 72.  The MH chains of the stiff methods run as k_mh_tree
    rounds (no iteration-loop kernel is built for them, kMhRoundsOnly), 'auto' trajectories
    through the hand-over queue (no in-wave k_integrate<TwoI, auto>, kHandQueue)."""
    ks = _stiff(resources["inst_two_i.hip"])
    names = " ".join(ks)
    assert "k_integrate_hq" in names and "k_bdf_hq" in names, names
    assert not re.search(r"k_mhINS_4TwoIELi[24]ELb0E", names), names          # no MH loop kernel
    assert not re.search(r"k_integrateINS_4TwoIELi2ELb", names), names       # no in-wave 'auto'
    for name, r in ks.items():
        assert r["scratch"] == 0 and r["vgpr_spill"] == 0, (name, r)
        budget = 72 if re.search(r"k_integrateINS_4TwoIELi4ELb1", name) else 64
        assert r["sgpr_spill"] <= budget, (name, r)


def test_hand_over_queue_co_residency_budget(resources):
    """k_bdf_hq runs beside k_integrate_hq on the SIMDs (small ensembles): the two register
    allocations (arch VGPRs rounded to 4, plus AGPRs, in granules of 8) must fit 512 together."""
    def alloc(r):
        v = (r["vgpr"] + 3) // 4 * 4 + r.get("agpr", 0)
        return (v + 7) // 8 * 8
    ks = resources["inst_two_i.hip"]
    for traj in ("ELb0ELb0E", "ELb1ELb0E", "ELb1ELb1E"):
        prod = _find(ks, "k_integrate_hqINS_4TwoI" + traj + "Lb1E")  # MIX: the beside variant
        cons = _find(ks, "k_bdf_hqINS_4TwoI" + traj + "Lb0E")  # beside: the LDS-table variant
        assert alloc(prod) + alloc(cons) <= 512, (traj, prod, cons)


@pytest.mark.parametrize("unit", WIDE_REG_UNITS)
def test_stiff_mh_kernels_scratch_budget_up_to_8_states(resources, unit):
    """5..8 states: the per-lane BDF pass (difference table in LDS, LU in registers) keeps the
    'auto' / 'bdf' MH kernels within 256 B/lane of scratch (chain8 'auto' k_mh was 1 296-1 376
    with the lockstep pass; 0-80 now) and their spills within the r06 counts (chain8: ~120
    SGPRs, 32 VGPRs to AGPRs)."""
    ks = _stiff_mh(resources[unit])
    assert len(ks) == 4, list(resources[unit])
    for name, r in ks.items():
        assert r["scratch"] <= 256, (name, r)
        assert r["sgpr_spill"] <= 160 and r["vgpr_spill"] <= 64, (name, r)
