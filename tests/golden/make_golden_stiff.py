"""Golden fixtures of the REFERENCE on stiff draws and near-posterior walkers (stiff.npz).

Run in the build container only (needs /root/reference, read-only), after make_golden.py:

    python tests/golden/make_golden_stiff.py

The reference is imported exactly as make_golden.py does (pyDOE2 stub that raises,
pandas Series.iteritems alias).  Everything below is the reference's own pipeline —
``ModelFramework.integrate`` (odeint = LSODA, Framework.py:656, then the summation and the
observation gather, :659-682), ``get_chi`` (masked chi, stats.py:41), ``get_Rsqrd`` and
``get_AIC`` — at two tolerances:
  * default: odeint's own (rtol = atol = 1.49012e-8), what a reference chain sees;
  * tight: the same call with rtol = atol = 1e-13, by rebinding the ``odeint`` name the
    reference's Framework module imported (``functools.partial(odeint, rtol=.., atol=..)``);
    nothing else of the pipeline changes.
Draws (two_i, the notebook's 4-state model):
  * near/: 16 near-posterior walkers (theta* · exp(0.05 z), seed 1);
  * stiff/: theta* with tau = 1e3, 1e4, 1e5, with lam = 1e3, and the notebook fit's slow
    region (phi = 1.06e-4, the host infected within ~1e-3 time units), where LSODA runs BDF.
Stored (numbers only): theta, trajectories [W][T][S] (states before summation), the
predictions at the observations, chi, R², AIC, per tolerance.

LSODA's step / RHS / Jacobian counts on the same stiff draws and the MH starts below
(lsoda_counts.json; ``--lsoda-counts`` writes only these): odeint's ``full_output`` info of
the reference's own integrate call.

Metropolis–Hastings chains in the stiff region (mh_stiff.npz + mh_stiff.json): the
reference's own ``Statistics.Samplers.MetropolisHastings`` (Samplers.py:53-174: LSODA for
every proposal, Framework.py:656; its global numpy stream seeded with random_seed) from the
notebook fit's slow starts — phi ~ 1.5e-5, beta ~ 50 (where the fit's LHS survey starts its
slowest chains) and tau = 1e3 — with the notebook's priors, 200 iterations each.  Stored:
the posterior columns, and from the oracle's restatement of the same chains (bit-equal to
the reference's, asserted here) each iteration's decision and margin acc − u.
"""
from __future__ import annotations

import functools
import os
import sys
import warnings

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from make_golden import THETA, build_model, import_reference, walker_thetas  # noqa: E402

TIGHT = 1e-13


def stiff_thetas():
    base = [THETA["two_i"][p] for p in ("mu", "phi", "beta", "lam", "tau")]
    rows, labels = [], []
    for tau in (1e3, 1e4, 1e5):
        rows.append(base[:4] + [tau])
        labels.append(f"tau={tau:g}")
    rows.append(base[:3] + [1e3, base[4]])
    labels.append("lam=1e3")
    rows.append([base[0], 1.06e-4] + base[2:])
    labels.append("phi=1.06e-4")
    return np.array(rows), labels


def run(ODElib, m, TH, tol):
    from scipy.integrate import odeint
    fw = sys.modules["ODElib.Framework"]
    saved = fw.odeint
    if tol is not None:
        fw.odeint = functools.partial(odeint, rtol=tol, atol=tol)
    try:
        trajs, preds, chis, rsqs, aics = [], [], [], [], []
        for w in range(TH.shape[0]):
            ps = list(TH[w])
            trajs.append(m.integrate(parameters=(ps,), as_dataframe=False, sum_subpopulations=False))
            d = m.integrate(parameters=(ps,), predict_obs=True, as_dataframe=False)
            preds.append(np.concatenate([d[s] for s in d]))
            c = m.get_chi(d)
            chis.append(float(np.ma.filled(c, np.nan)))
            rsqs.append(float(m.get_Rsqrd(d)))
            aics.append(float(np.ma.filled(m.get_AIC(c), np.nan)))
    finally:
        fw.odeint = saved
    return dict(traj=np.array(trajs), pred=np.array(preds), chi=np.array(chis), rsq=np.array(rsqs),
                aic=np.array(aics))


# (key, start, random_seed, nits): the notebook fit's slow region and a tau = 1e3 start
MH_STIFF = [
    ("slow_phi1.5e-5_s11", {"mu": 6.1e-9, "phi": 1.5e-5, "beta": 50.0, "lam": 2.0, "tau": 3.0}, 11, 200),
    ("slow_phi1.2e-5_s12", {"mu": 8.0e-9, "phi": 1.2e-5, "beta": 55.0, "lam": 1.5, "tau": 2.5}, 12, 200),
    ("tau1e3_s13", dict(THETA["two_i"], tau=1e3), 13, 200),
]


def mh_chains(ODElib):
    import contextlib
    import io
    import json
    sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
    sys.path.insert(0, os.path.dirname(HERE))
    from helpers import oracle_model  # noqa: E402
    from oracle import cpu_ref  # noqa: E402
    out, meta = {}, {}
    for key, th, seed, nits in MH_STIFF:
        m = build_model(ODElib, "two_i", theta=th, seed=seed)
        with contextlib.redirect_stdout(io.StringIO()):
            post = ODElib.Statistics.Samplers.MetropolisHastings(m, nits=nits, print_progress=False)
        ref = cpu_ref.metropolis_hastings(oracle_model("two_i", theta=th, seed=seed), nits=nits)
        for c in post.columns:
            v = np.asarray(post[c].to_numpy(), dtype=float)
            assert np.array_equal(v, np.asarray(ref[c], dtype=float), equal_nan=True), (key, c)
            out[f"{key}/{c}"] = v
        out[f"{key}/margin"] = np.asarray(ref["margin"], dtype=float)
        out[f"{key}/accepted"] = np.asarray(ref["accepted"], dtype=float)
        meta[key] = dict(model="two_i", theta=th, seed=seed, nits=nits, columns=list(post.columns),
                         accept_ratio=float(post["acceptance_ratio"].to_numpy()[-1]))
    np.savez_compressed(os.path.join(HERE, "mh_stiff.npz"), **out)
    with open(os.path.join(HERE, "mh_stiff.json"), "w") as f:
        json.dump(meta, f, indent=1, sort_keys=True)
    print("stiff MH chains written:", meta)


def lsoda_counts(ODElib):
    """LSODA's own work on the stiff draws and the stiff MH starts (lsoda_counts.json): the
    reference's ``ModelFramework.integrate`` with its ``odeint`` name rebound to a wrapper that
    makes the same call with ``full_output=True`` and keeps the info dict (Framework.py:656;
    nothing else of the call changes, the wrapper returns the trajectory the reference gets).
    Per draw: steps (nst), RHS evaluations (nfe), Jacobian evaluations (nje), the output
    points LSODA reached on BDF (mused == 2) and the first such time — the cost model the
    device's DOPRI5 + BDF hand-over is compared against (tests/test_stiff_oracle.py)."""
    import json
    from scipy.integrate import odeint
    fw = sys.modules["ODElib.Framework"]
    saved = fw.odeint
    info = {}

    def wrapped(*a, **k):
        y, d = odeint(*a, full_output=True, **k)
        info.update(d)
        return y

    rows = {}
    st, labels = stiff_thetas()
    draws = [(lab, list(st[w])) for w, lab in enumerate(labels)]
    draws += [(key, [th[p] for p in ("mu", "phi", "beta", "lam", "tau")]) for key, th, _, _ in MH_STIFF]
    m = build_model(ODElib, "two_i")
    fw.odeint = wrapped
    try:
        for lab, ps in draws:
            info.clear()
            m.integrate(parameters=(ps,), as_dataframe=False, sum_subpopulations=False)
            mused = np.asarray(info["mused"])
            tcur = np.asarray(info["tcur"])
            bdf = np.nonzero(mused == 2)[0]
            rows[lab] = dict(theta=[float(v) for v in ps], nst=int(info["nst"][-1]), nfe=int(info["nfe"][-1]),
                             nje=int(info["nje"][-1]), bdf_outputs=int(bdf.size), outputs=int(mused.size),
                             first_bdf_t=float(tcur[bdf[0]]) if bdf.size else None)
    finally:
        fw.odeint = saved
    with open(os.path.join(HERE, "lsoda_counts.json"), "w") as f:
        json.dump(rows, f, indent=1, sort_keys=True)
    print("LSODA counts written:", rows)


def main():
    ODElib = import_reference()
    warnings.filterwarnings("ignore")
    if "--mh-only" in sys.argv:
        mh_chains(ODElib)
        return
    if "--lsoda-counts" in sys.argv:
        lsoda_counts(ODElib)
        return
    lsoda_counts(ODElib)
    mh_chains(ODElib)
    m = build_model(ODElib, "two_i")
    out = {}
    near = walker_thetas("two_i", W=16, seed=1)
    st, labels = stiff_thetas()
    for group, TH in (("near", near), ("stiff", st)):
        out[f"{group}/theta"] = TH
        for tag, tol in (("default", None), ("tight", TIGHT)):
            r = run(ODElib, m, TH, tol)
            for k, v in r.items():
                out[f"{group}/{tag}/{k}"] = v
    out["stiff/labels"] = np.array(labels)
    np.savez_compressed(os.path.join(HERE, "stiff.npz"), **out)
    print("stiff fixtures written:", {k: v.shape for k, v in out.items()})


if __name__ == "__main__":
    main()
