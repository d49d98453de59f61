"""Python RHS -> C transpiler for the hipRTC path (CPU: translation, validation,
compile check with hipRTC for gfx950 — no GPU needed)."""
import math

import numpy as np
import pytest

from helpers import CONFIGS
from odelib_amd import _native as N
from odelib_amd.models import resolve_model
from odelib_amd.transpile import Unsupported, transpile

K_HALF = 1e6


def sat_infection(y, t, ps):
    """host growth, saturating infection, virus decay, a time-forced term"""
    mu, phi, beta, delta = ps[0], ps[1], ps[2], ps[3]
    S, V = y
    inf = phi * S * V / (1.0 + S / K_HALF)
    dS = mu * S * (1 - S / 1e7) - inf
    dV = beta * inf - delta * V + 0.1 * math.sin(2 * np.pi * t) ** 2
    return [dS, dV]


def piecewise(y, t, ps):
    x = y[0]
    rate = ps[0] if x < 5.0 else ps[1]
    out = -rate * x
    out += np.exp(-x) * 0.0
    return np.array([out, abs(y[-1]) - np.maximum(x, 1.0) ** 1.5])


def hill_power(y, t, ps):
    """Hill-type activation with a fitted exponent: a state that starts at 0 raised to a
    parameter power (pow(y, p) in the translation)."""
    k, K, n, d = ps[0], ps[1], ps[2], ps[3]
    X = y[0]
    Y = y[1]
    dX = k - d * X
    dY = k * X ** n / (K ** n + X ** n) - d * Y
    return [dX, dY]


def test_power_of_state_translates_to_pow():
    tr = transpile(hill_power, 2, 4)
    assert "pow(y[0], ps[2])" in tr.c_body.replace("X", "y[0]") or "pow(" in tr.c_body
    rs = np.random.RandomState(2)
    for _ in range(10):
        y = rs.uniform(0, 5, 2)
        ps = rs.uniform(0.5, 3, 4)
        np.testing.assert_allclose(tr.evaluate(y, 0.0, ps), hill_power(y, 0.0, ps), rtol=1e-14)
    np.testing.assert_array_equal(tr.evaluate(np.zeros(2), 0.0, [2.0, 1.5, 2.5, 0.7]), [2.0, 0.0])


@pytest.mark.parametrize("name", ["zero_i", "one_i", "two_i"])
def test_demo_models_translate_exactly(name):
    f = CONFIGS[name]["ode"]
    S, P = len(CONFIGS[name]["snames"]), len(CONFIGS[name]["pnames"])
    tr = transpile(f, S, P)
    rs = np.random.RandomState(0)
    for _ in range(20):
        y = rs.uniform(0, 1e7, S)
        ps = rs.uniform(0, 2, P) * 10.0 ** rs.uniform(-8, 1, P)
        assert np.array_equal(tr.evaluate(y, 0.5, ps), np.asarray(f(y, 0.5, ps)))
    assert "dy[%d]" % (S - 1) in tr.c_body


def test_general_subset_translates():
    tr = transpile(sat_infection, 2, 4)
    tr2 = transpile(piecewise, 2, 2)
    rs = np.random.RandomState(1)
    for _ in range(20):
        y = rs.uniform(0, 1e7, 2)
        ps = rs.uniform(0, 1, 4) * [1, 1e-7, 50, 1]
        t = rs.uniform(0, 3)
        np.testing.assert_allclose(tr.evaluate(y, t, ps), sat_infection(y, t, ps), rtol=1e-14)
        y2 = rs.uniform(0, 10, 2)
        np.testing.assert_allclose(tr2.evaluate(y2, t, ps[:2]), piecewise(y2, t, ps[:2]), rtol=1e-14)
    assert "1000000.0" in tr.c_body and "sin(" in tr.c_body
    assert "?" in tr2.c_body and "pow(" in tr2.c_body


def chain_loop(y, t, ps):
    """The synthetic N-state chain as a user would write it: a loop
    over the compartments into a preallocated array."""
    mu, phi, beta, lam, tau = ps
    n = len(y)
    dy = np.zeros(n)
    inf = phi * y[0] * y[-1]
    dy[0] = mu * y[0] - inf
    dy[1] = inf - tau * y[1]
    for k in range(2, n - 2):
        dy[k] = tau * y[k - 1] - tau * y[k]
    dy[n - 2] = tau * y[n - 3] - lam * y[n - 2]
    dy[-1] = beta * lam * y[n - 2] - inf
    return dy


def chain_branchy(y, t, ps):
    """The chain model with the boundary compartments picked by `if` on the loop index."""
    mu, phi, beta, lam, tau = ps
    n = len(y)
    inf = phi * y[0] * y[n - 1]
    out = [0.0] * n
    for k in range(n):
        if k == 0:
            out[k] = mu * y[0] - inf
        elif k == 1:
            out[k] = inf - tau * y[1]
        elif k < n - 2:
            out[k] = tau * y[k - 1] - tau * y[k]
        elif k == n - 2 and not n < 4:
            out[k] = tau * y[k - 1] - lam * y[k]
        else:
            out[k] = beta * lam * y[n - 2] - inf
    return out


def thresholds(y, t, ps):
    """`if`/`elif`/`else` on data (evaluated as selects), a literal local reused as an
    index, and array elements set in both branches."""
    a, b = ps
    x = 0
    if y[0] < 1.0 and t > 0.5:
        x = y[0] * a
        f = 2.0
    elif y[1] > 3.0 or not y[0] < 2.0:
        f = b
    else:
        f = a * b
        x += 1.5
    out = np.zeros(2)
    out[0] = -f * y[0] + x
    if 0.0 < y[1] <= 4.0:
        out[1] = y[1] * f
    else:
        out[1] = -y[1]
    i = 1
    out[i] += 0.25
    return out


def test_if_on_data_translates_to_selects():
    tr = transpile(thresholds, 2, 2)
    assert "?" in tr.c_body and "&&" in tr.c_body and "||" in tr.c_body
    rs = np.random.RandomState(5)
    for _ in range(3000):
        y, t, ps = rs.uniform(0, 5, 2), rs.uniform(0, 1), rs.uniform(0, 1, 2)
        assert np.array_equal(tr.evaluate(y, t, ps), thresholds(y, t, ps))


def pooled(y, t, ps):
    """Sums over slices (built-in sum and numpy's pairwise np.sum), augmented element
    updates and a loop variable used as a number."""
    d = np.zeros_like(y)
    total = np.sum(y)
    head = sum(y[: len(y) // 2])
    for i in range(len(y)):
        d[i] = ps[0] * total - ps[1] * y[i]
        d[i] += head * (i + 1) * 1e-3
    return d


def vec_chain(y, t, ps):
    """The chain model in numpy slice style (whole-array arithmetic, slice assignment)."""
    mu, phi, beta, lam, tau = ps
    inf = phi * y[0] * y[-1]
    dy = np.empty_like(y)
    dy[0] = mu * y[0] - inf
    dy[1] = inf - tau * y[1]
    dy[2:-2] = tau * y[1:-3] - tau * y[2:-2]
    dy[-2] = tau * y[-3] - lam * y[-2]
    dy[-1] = beta * lam * y[-2] - inf
    return dy


def vec_misc(y, t, ps):
    k = np.array([ps[0], ps[1]] + [ps[0] * ps[1]] * (len(y) - 2))
    out = -k * y + np.exp(-y / 10.0) * t
    out[1:] += 0.5 * y[:-1] ** 2
    out *= 1.5
    return out


@pytest.mark.parametrize("n", [4, 7, 8, 12, 20, 33])
def test_loops_arrays_and_sums_translate_exactly(n):
    """Unrolled loops, local arrays and sums keep Python's operation order: the
    translation evaluates bit-for-bit like the callable (np.sum in numpy's pairwise
    order: sequential below 8 elements, 8 strided accumulators above)."""
    tr = transpile(chain_loop, n, 5)
    tp = transpile(pooled, n, 2)
    tv = transpile(vec_chain, n, 5)
    tm = transpile(vec_misc, n, 2)
    tb = transpile(chain_branchy, n, 5)
    rs = np.random.RandomState(n)
    for _ in range(25):
        y = rs.uniform(0, 1, n) * 10.0 ** rs.uniform(-3, 7, n)
        ps = rs.uniform(0.1, 3, 5)
        t = rs.uniform(0, 3)
        assert np.array_equal(tr.evaluate(y, t, ps), chain_loop(y, t, ps))
        assert np.array_equal(tp.evaluate(y, t, ps[:2]), pooled(y, t, ps[:2]))
        assert np.array_equal(tv.evaluate(y, t, ps), vec_chain(y, t, ps))
        assert np.array_equal(tm.evaluate(y, t, ps[:2]), vec_misc(y, t, ps[:2]))
        assert np.array_equal(tb.evaluate(y, t, ps), np.array(chain_branchy(y, t, ps)))
    assert "for" not in tr.c_body and f"dy[{n - 1}]" in tr.c_body


def test_unsupported_constructs_are_rejected():
    def loop(y, t, ps):
        out = []
        for v in y:
            out.append(-v)
        return out

    def dyn_index(y, t, ps):
        i = int(ps[0])
        return [y[i]]

    def wrong_len(y, t, ps):
        return [y[0]]

    def data_if(y, t, ps):
        if y[0] > 1.0:
            return [-y[0]]
        return [y[0]]

    for f, S in ((loop, 2), (dyn_index, 1), (wrong_len, 2), (data_if, 1)):
        with pytest.raises(Unsupported):
            transpile(f, S, 1)
    with pytest.raises(Unsupported):
        transpile(lambda y, t, ps: y, 1, 1)


def test_resolution_prefers_builtins_then_rtc():
    dm = resolve_model(CONFIGS["two_i"]["ode"], 4, 5)
    assert dm.model_id == N.OE_MODEL_TWO_I and dm.source is None
    dm = resolve_model(CONFIGS["two_i"]["ode"], 4, 5, device_model="rtc")
    assert dm.model_id is None and "dy[3]" in dm.source
    dm = resolve_model(sat_infection, 2, 4)
    assert dm.model_id is None and dm.name == "rtc:sat_infection"
    dm = resolve_model(None, 3, 2, device_rhs="dy[0] = 0.0; dy[1] = 0.0; dy[2] = 0.0;")
    assert dm.source.startswith("dy[0]")


def test_transpiled_rhs_compiles_with_hiprtc_for_gfx950():
    N.rtc_check(transpile(sat_infection, 2, 4).c_body, 2, 4, "gfx950")
    N.rtc_check(transpile(vec_misc, 6, 2).c_body, 6, 2, "gfx950")
    N.rtc_check(transpile(thresholds, 2, 2).c_body, 2, 2, "gfx950")
    with pytest.raises(ValueError, match="hipRTC compilation"):
        N.rtc_check("dy[0] = no_such_symbol;", 1, 1, "gfx950")
