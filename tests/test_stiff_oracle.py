"""Pin the stiff methods' C restatement (oracle/rk_ref.c: 'rosenbrock' = the stiffly
accurate RODAS method, 'auto' = DOPRI5 + per-walker stiffness test + BDF from the eviction
point for n_states <= 8, a Rosenbrock restart for wider models — the kernels' algorithms,
DESIGN.md §3.6) against the reference's algorithm on stiff draws:
odeint's LSODA switches to BDF there (Framework.py:656), so the yardstick is a tight
implicit solution (scipy Radau, rtol 1e-13) and the reference's own odeint."""
import os
import re

import numpy as np
import pytest
from scipy.integrate import solve_ivp

from helpers import CONFIGS, ROOT, chain_problem, product_model, walker_thetas
from oracle import cpu_ref, rk_ref

STIFF_H = os.path.join(ROOT, "odelib_amd", "csrc", "stiff.cuh")
# two_i parameter sets: the demo posterior, then tau / lam raised so that the I1/I2
# compartments relax 1e4..1e9 times faster than the rest (explicit methods crawl)
BASE = [7.475e-9, 1.069e-7, 19.73, 1.934, 2.799]
STIFF_SETS = {
    "nonstiff": BASE,
    "tau1e5": BASE[:4] + [1e5],
    "tau1e6_lam1e4": BASE[:3] + [1e4, 1e6],
    "tau1e9": BASE[:4] + [1e9],
}
ODEINT_TOL = 1.49012e-8


def _ros_constants():
    src = open(STIFF_H).read()
    block = src[src.index("namespace ros {"):src.index("constexpr double safe")]
    vals = dict((k, float(v)) for k, v in re.findall(r"(\w+) = (-?[0-9.eE+-]+)", block))
    return vals


def _rodas_tableau():
    """The shipped RODAS set (stiff.cuh) in matrix form: stage-argument weights A (stage 6
    = the embedded solution), increment couplings C, solution weights m (y_new = stage-6
    argument + k6) and embedded weights mh."""
    c = _ros_constants()
    n = 6
    A = np.zeros((n, n)); C = np.zeros((n, n))
    for i in range(2, 6):
        for j in range(1, i):
            A[i - 1, j - 1] = c[f"a{i}{j}"]
    A[5, :4] = A[4, :4]; A[5, 4] = 1.0
    for i in range(2, 7):
        for j in range(1, i):
            C[i - 1, j - 1] = c[f"c{i}{j}"]
    m = np.array([c["a51"], c["a52"], c["a53"], c["a54"], 1.0, 1.0])
    mh = np.array([c["a51"], c["a52"], c["a53"], c["a54"], 1.0, 0.0])
    return c, A, C, m, mh


def test_rodas_coefficients_order_and_l_stability():
    """The shipped RODAS set (stiff.cuh) satisfies the eight order-4 conditions of a
    Rosenbrock method, its embedded method the four order-3 ones (Hairer & Wanner II,
    §VI.4, in the transformed form of the code); BOTH are L-stable (R(∞) = 0) and
    A-stable — the embedded estimate being L-stable is what keeps the step size of a
    stiff walker on its slow manifold large; the stage times are Σα_ij and the ∂f/∂t
    weights Σγ_ij."""
    c, A, C, m, mh = _rodas_tableau()
    gam, n = c["gam"], 6
    assert c["inv_gam"] == 1.0 / gam
    G = np.linalg.inv(np.diag(np.full(n, 1 / gam)) - C)
    alpha = A @ G
    beta = np.tril(alpha + G, -1)
    bp, al = beta.sum(1), alpha.sum(1)

    def conds(b):
        return np.array([b.sum() - 1, b @ bp - (0.5 - gam), b @ al ** 2 - 1 / 3, b @ beta @ bp - (1 / 6 - gam + gam ** 2),
                         b @ al ** 3 - 1 / 4, (b * al) @ alpha @ bp - (1 / 8 - gam / 3),
                         b @ beta @ al ** 2 - (1 / 12 - gam / 3),
                         b @ beta @ beta @ bp - (1 / 24 - gam / 2 + 1.5 * gam ** 2 - gam ** 3)])
    assert np.abs(conds(m @ G)).max() < 1e-13
    assert np.abs(conds(mh @ G)[:4]).max() < 1e-13
    assert np.abs(conds(mh @ G)[4:]).max() > 1e-3  # the estimate is genuinely order 3
    B = alpha + G
    for w in (m @ G, mh @ G):
        assert abs(1 - w @ np.linalg.solve(B, np.ones(n))) < 1e-13          # R(∞) = 0
        R = lambda z: 1 + z * (w @ np.linalg.solve(np.eye(n) - z * B, np.ones(n)))
        assert max(abs(R(1j * y)) for y in np.logspace(-3, 6, 400)) <= 1 + 1e-12
    np.testing.assert_allclose(al, [0, c["c2x"], c["c3x"], c["c4x"], 1, 1], atol=1e-14)
    np.testing.assert_allclose(G.sum(1), [c["d1"], c["d2"], c["d3"], c["d4"], 0, 0], atol=1e-14)


def test_rodas_continuous_extension_order():
    """The dense-output weights h2j, h3j: y(θ) = (1−θ)·y0 + θ·(y1 + (1−θ)·(q3 + θ·q4)) on
    y' = λy reproduces exp(θz) to third order in z for every θ (the extension's order)."""
    c, A, C, m, mh = _rodas_tableau()
    gam, n = c["gam"], 6
    h2 = np.array([c[f"h2{j}"] for j in range(1, 6)] + [0.0])
    h3 = np.array([c[f"h3{j}"] for j in range(1, 6)] + [0.0])
    G = np.linalg.inv(np.diag(np.full(n, 1 / gam)) - C)
    B = A @ G + G

    def dense(z, th):  # one step of y' = λy from y0 = 1 (z = hλ); increments K = z·(I − zB)^{-1}·G·1…
        # k_i solves (1/(γh) − λ) k_i = λ(y0 + Σ a_ij k_j) + Σ (c_ij/h) k_j, in units of y0
        K = np.zeros(n)
        for i in range(n):
            rhs = z * (1 + A[i, :i] @ K[:i]) + C[i, :i] @ K[:i]
            K[i] = rhs / (1 / gam - z)
        y1 = 1 + m @ K
        return (1 - th) + th * (y1 + (1 - th) * (h2 @ K + th * (h3 @ K)))

    for th in (0.2, 0.5, 0.9):
        errs = [abs(dense(z, th) - np.exp(th * z)) for z in (1e-2, 5e-3)]
        assert errs[0] / errs[1] > 2 ** 3.7, (th, errs)  # local error O(z^4)


def test_inv_fourth_root_accuracy():
    xs = np.concatenate([[5e-324, 1e-310, 2.2250738585072014e-308, 1e-30, 1.0, 1e30],
                         np.logspace(-300, 300, 4001), np.random.RandomState(2).uniform(0.5, 40.0, 2000)])
    for x in xs:
        got = rk_ref.inv_fourth_root(x)
        want = float(np.exp(-0.25 * np.log(np.longdouble(x))))
        assert abs(got / want - 1.0) < 1e-14, (x, got, want)


def _problem(method, W_sets):
    m = product_model("two_i")
    fp = m.fit_problem()
    fp.method = method
    theta = np.array([STIFF_SETS[k] for k in W_sets], float).T.copy()
    y0 = np.repeat(np.asarray(m.get_inits(), float)[:, None], theta.shape[1], axis=1)
    return fp, theta, y0


def _radau(fp, y0, th):
    f = CONFIGS["two_i"]["ode"]
    sol = solve_ivp(lambda t, y: f(y, t, th), (fp.times[0], fp.times[-1]), y0, method="Radau",
                    t_eval=fp.times, rtol=1e-13, atol=1e-10)
    assert sol.success
    return sol.y.T


@pytest.mark.parametrize("method", ["rosenbrock", "auto", "bdf"])
def test_stiff_methods_match_tight_implicit_solution(method):
    """odeint's default tolerances; every walker — stiff or not — within
    1e-6·|y| + 1e-6 of the tight implicit solution, the bar the explicit methods meet on
    non-stiff draws.  'auto' flags exactly the stiff walkers (OE_STATUS_STIFF)."""
    sets = list(STIFF_SETS)
    fp, theta, y0 = _problem(method, sets)
    out = rk_ref.integrate(fp, y0, theta)
    for w, k in enumerate(sets):
        ref = _radau(fp, y0[:, w], theta[:, w])
        np.testing.assert_allclose(out["traj"][:, :, w], ref, rtol=1e-6, atol=1e-6, err_msg=k)
    st = out["status"]
    assert not (st & 4).any()  # no walker abandoned
    if method == "auto":
        assert [bool(s & 8) for s in st] == [k != "nonstiff" for k in sets]


def test_auto_switch_is_scale_invariant_and_cost_aware():
    """The stiffness test weighs each component by the error control's scale, so a stiff
    mode in a small compartment is seen next to the 1e7-sized host/virus states
    (unweighted, tau = 1e4 and 3e4 were never flagged and DOPRI5 crawled 10-30x the normal
    work).  The hand-over to BDF continues from the eviction point, so it is taken whenever
    DOPRI5 would need more than 300 more steps at h|lambda| > 2.5, or more than 1500 at
    h|lambda| > 0.5: tau = 1e2 stays with DOPRI5, tau = 1e3 (accuracy-limited at
    h|lambda| ~ 0.9: 2 359 DOPRI5 steps) and up are handed over.  Every walker within the
    1e-6 bar of tight Radau, and the hand-over costs far fewer steps than DOPRI5 alone."""
    taus = [1e2, 1e3, 3e3, 1e4, 3e4]
    fp, theta, y0 = _problem("auto", ["nonstiff"] * len(taus))
    theta[4, :] = taus
    out = rk_ref.integrate(fp, y0, theta)
    assert [bool(s & 8) for s in out["status"]] == [False, True, True, True, True]
    for w, tau in enumerate(taus[1:], 1):
        th = theta[:, w:w + 1].copy()
        steps = {}
        for meth in ("dopri5", "auto"):
            fp.method = meth
            rk_ref.dopri5_stats(True), rk_ref.bdf_stats(True)
            rk_ref.integrate(fp, y0[:, w:w + 1].copy(), th, trajectory=False)
            steps[meth] = sum(rk_ref.dopri5_stats(True)[k] for k in ("accepted", "rejected")) + \
                rk_ref.bdf_stats(True)["steps"]
        assert steps["auto"] < 0.3 * steps["dopri5"], (tau, steps)
    fp.method = "auto"
    assert not (out["status"] & 4).any()
    for w in range(len(taus)):
        ref = _radau(fp, y0[:, w], theta[:, w])
        np.testing.assert_allclose(out["traj"][:, :, w], ref, rtol=1e-6, atol=1e-6, err_msg=str(taus[w]))


def test_auto_equals_dopri5_bitwise_without_stiff_walkers():
    """The stiffness test changes no arithmetic: with no walker evicted, 'auto' is DOPRI5."""
    m = product_model("two_i")
    fp = m.fit_problem()
    W = 70  # two groups, the second ragged
    theta = walker_thetas("two_i", W).T.copy()
    y0 = np.repeat(np.asarray(m.get_inits(), float)[:, None], W, axis=1)
    fp.method = "dopri5"
    a = rk_ref.integrate(fp, y0, theta)
    fp.method = "auto"
    b = rk_ref.integrate(fp, y0, theta)
    assert np.array_equal(a["traj"], b["traj"]) and np.array_equal(a["chi"], b["chi"])
    assert np.array_equal(a["status"], b["status"])


def test_auto_chi_at_least_as_accurate_as_reference_odeint():
    """The fused likelihood of stiff walkers against the reference's own pipeline
    (scipy odeint = LSODA at default tolerances + summation + masked chi,
    Framework.py:656-697) and the same pipeline on the tight implicit trajectory: 'auto'
    is within 1e-6 of the tight chi, or at least as close to it as the reference itself
    (with lam = 1e4 the host compartment H dips to 3e-8 and LSODA's absolute error moves
    its chi by 5e-4 while ours stays within 4e-7)."""
    from helpers import oracle_model
    sets = list(STIFF_SETS)
    fp, theta, y0 = _problem("auto", sets)
    out = rk_ref.integrate(fp, y0, theta)
    for w, k in enumerate(sets):
        ref_m, tight_m = oracle_model("two_i"), oracle_model("two_i")
        for om in (ref_m, tight_m):
            for p, v in zip(om.get_pnames(), theta[:, w]):
                om.parameters[p].val = v
        ref_chi = float(ref_m.get_chi(ref_m.integrate_obs()))
        tr = _radau(fp, y0[:, w], theta[:, w])
        tight_m.integrator = lambda yy, ps, tr=tr: tr
        tight_chi = float(tight_m.get_chi(tight_m.integrate_obs()))
        ours = abs(out["chi"][w] / tight_chi - 1)
        assert ours <= max(1e-6, abs(ref_chi / tight_chi - 1)), (k, out["chi"][w], ref_chi, tight_chi)


def test_stiff_walker_in_a_wave_of_nonstiff_ones():
    """One stiff walker among 63 demo draws: it is evicted from the shared DOPRI5 step and
    continues with BDF; every walker stays within tolerance of the tight solution, and the
    wave's step count stays that of the non-stiff draws (the stiff lane does not pin it)."""
    m = product_model("two_i")
    fp = m.fit_problem()
    fp.method = "auto"
    W = 64
    theta = walker_thetas("two_i", W).T.copy()
    theta[4, 17] = 1e6  # tau
    y0 = np.repeat(np.asarray(m.get_inits(), float)[:, None], W, axis=1)
    out = rk_ref.integrate(fp, y0, theta)
    assert [w for w in range(W) if out["status"][w] & 8] == [17]
    for w in (0, 17, 40):
        ref = _radau(fp, y0[:, w], theta[:, w])
        np.testing.assert_allclose(out["traj"][:, :, w], ref, rtol=1e-6, atol=1e-6)


@pytest.mark.parametrize("n", [10, 20])
def test_wide_chain_stiff_walkers_match_tight_implicit_solution(n):
    """Chains wider than the register-resident stiff path (S > 8: the device keeps J and
    the LU factors in private memory, same arithmetic): 'auto' on the C restatement flags
    exactly the stiff walkers, abandons none, and every walker is within
    1e-6·|y| + 1e-5 of tight Radau (the downstream compartments of a long chain start at
    0 and carry odeint-sized absolute errors)."""
    from odelib_amd.models import chain_rhs
    m = chain_problem(n, method="auto")
    fp = m.fit_problem()
    sets = ["nonstiff", "tau1e5", "tau1e9"]
    theta = np.array([STIFF_SETS[k] for k in sets], float).T.copy()
    y0 = np.repeat(np.asarray(m.get_inits(), float)[:, None], len(sets), axis=1)
    out = rk_ref.integrate(fp, y0, theta)
    f = chain_rhs(n)
    for w, k in enumerate(sets):
        sol = solve_ivp(lambda t, y: f(y, t, theta[:, w]), (fp.times[0], fp.times[-1]), y0[:, w], method="Radau",
                        t_eval=fp.times, rtol=1e-13, atol=1e-10)
        assert sol.success
        np.testing.assert_allclose(out["traj"][:, :, w], sol.y.T, rtol=1e-6, atol=1e-5, err_msg=k)
    st = out["status"]
    assert not (st & 4).any()
    assert [bool(s & 8) for s in st] == [k != "nonstiff" for k in sets]


def test_inv_root_accuracy():
    """x^(-1/q), q = 1..6, of the BDF step controller (frexp/ldexp + Newton, bit-identical on
    the device): within 1e-15 relative of the long-double value; 0 -> inf, inf -> 0."""
    xs = np.concatenate([[5e-324, 1e-310, 2.2250738585072014e-308, 1e-30, 1.0, 1e30, 1.7e308],
                         np.logspace(-300, 300, 2001), np.random.RandomState(3).uniform(0.5, 40.0, 1000)])
    for q in range(1, 7):
        for x in xs:
            got = rk_ref.inv_root(x, q)
            want = float(np.exp(-np.log(np.longdouble(x)) / q))
            if np.isinf(want):  # 1/x beyond the double range: overflows alike
                assert got == want, (q, x, got)
                continue
            assert abs(got / want - 1.0) < 2e-15, (q, x, got, want)
    assert rk_ref.inv_root(0.0, 3) == np.inf and rk_ref.inv_root(np.inf, 2) == 0.0


def test_bdf_step_counts_are_lsoda_like_where_explicit_and_rosenbrock_methods_are_not():
    """The reason 'auto' hands stiff lanes to BDF and not to RODAS: on a
    stiff component sitting on its quasi-steady state (two_i, tau = 1e4) the one-step
    Rosenbrock method suffers order reduction (~3 700 steps at odeint's tolerances) and DOPRI5
    crawls at its stability limit (~12 000), while BDF takes LSODA-like step counts (~600;
    scipy's BDF: 546, LSODA: 734).  Measured on the C restatement."""
    fp, theta, y0 = _problem("bdf", ["nonstiff"])
    theta[4, 0] = 1e4
    steps = {}
    for meth in ("dopri5", "rosenbrock", "bdf"):
        fp.method = meth
        rk_ref.dopri5_stats(True), rk_ref.rosenbrock_stats(True), rk_ref.bdf_stats(True)
        rk_ref.integrate(fp, y0, theta, trajectory=False)
        d, r, b = rk_ref.dopri5_stats(True), rk_ref.rosenbrock_stats(True), rk_ref.bdf_stats(True)
        steps[meth] = d["accepted"] + d["rejected"] + r["steps"] + b["steps"]
    assert steps["bdf"] < 700 and steps["rosenbrock"] > 3000 and steps["dopri5"] > 10000, steps


def test_bdf_handover_in_a_lockstep_group_matches_tight_solution():
    """'auto' lanes handed over at different times (tau = 1e3 .. 1e5, the demo's phi ~ 1e-4
    region) continue with their own time and a shared BDF step: all within the 1e-6 bar
    of tight Radau, the others untouched by the hand-over (DOPRI5's own trajectory)."""
    m = product_model("two_i")
    fp = m.fit_problem()
    W = 64
    theta = walker_thetas("two_i", W).T.copy()
    lanes = {3: (4, 1e3), 17: (4, 1e5), 30: (1, 1.0e-4), 31: (4, 3e4), 50: (1, 6e-6)}
    for w, (j, v) in lanes.items():
        theta[j, w] = v
    y0 = np.repeat(np.asarray(m.get_inits(), float)[:, None], W, axis=1)
    fp.method = "auto"
    out = rk_ref.integrate(fp, y0, theta)
    flagged = [w for w in range(W) if out["status"][w] & 8]
    assert set(flagged) >= {3, 17, 30, 31}, flagged
    assert not (out["status"] & 4).any()
    for w in list(lanes) + [0, 63]:
        ref = _radau(fp, y0[:, w], theta[:, w])
        np.testing.assert_allclose(out["traj"][:, :, w], ref, rtol=1e-6, atol=1e-6, err_msg=str(w))


def test_step_counts_against_lsoda_on_the_reference_draws():
    """the device's DOPRI5 + BDF hand-over against odeint's LSODA on the stiff
    draws and the stiff MH starts of the golden set (tests/golden/lsoda_counts.json: LSODA's
    own nst / nfe / nje from the reference's integrate call, Framework.py:656).  Steps are the
    stiff workload's cost model; no draw may take more than 1.5x LSODA's steps (a regression
    in the hand-over or the BDF controller shows here first).  Prints the table
    (profiles/NOTES.md round 6)."""
    import json
    with open(os.path.join(ROOT, "tests", "golden", "lsoda_counts.json")) as f:
        lsoda = json.load(f)
    m = product_model("two_i", method="auto")
    fp = m.fit_problem()
    y0 = np.asarray(m.get_inits(), float)[:, None].copy()
    rows = []
    for lab, ref in sorted(lsoda.items()):
        rk_ref.dopri5_stats(); rk_ref.bdf_stats(); rk_ref.bdf_detail()
        out = rk_ref.integrate(fp, y0, np.asarray(ref["theta"], float)[:, None].copy(), trajectory=False, lane=True)
        dp, bs, bd = rk_ref.dopri5_stats(), rk_ref.bdf_stats(), rk_ref.bdf_detail()
        dsteps = dp["accepted"] + dp["rejected"]
        rhs = 3 + 6 * dsteps + ((2 + bd["newton_iterations"] + 4 * bs["jacobians"]) if bs["steps"] else 0)
        steps = dsteps + bs["steps"]
        rows.append((lab, steps, dsteps, bs["steps"], rhs, bs["jacobians"], ref["nst"], ref["nfe"], ref["nje"]))
        assert out["status"][0] & 8, lab  # every one of them is handed to BDF, as LSODA switches
        assert steps <= 1.5 * ref["nst"], (lab, steps, ref["nst"])
    print("\n%-20s %6s %7s %5s %6s %4s | %6s %6s %4s" % ("draw", "steps", "dopri5", "bdf", "rhs", "jac", "nst",
                                                         "nfe", "nje"))
    for r in rows:
        print("%-20s %6d %7d %5d %6d %4d | %6d %6d %4d" % r)
