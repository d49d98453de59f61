"""CPU restatement of ODElib's fitting hot path — TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg
may import this module, and only as the checker / the timed CPU baseline.  The
product (``odelib_amd``) never imports it and has no CPU fallback.

Every function restates one reference call site of SEpapoulis/ODElib (citations are
into /root/reference, which is NOT available on the GPU box — nothing here reads it):

* ``times_grid``          ODElib/Framework.py:234 / :241
* ``format_df``           Framework.py:281-307   (_formatdf)
* ``fit_setup``           Framework.py:309-329   (_df_fitsetup, first-nearest pred_tindex)
* ``summation_index``     Framework.py:332-381   (_get_summation_index)
* ``integrate``           Framework.py:622-683   (odeint call at :656 with scipy defaults)
* ``chi`` / ``rsqrd`` / ``aic``   Statistics/stats.py:22-56
* ``get_chi`` / ``get_rsqrd``     Framework.py:685-706
* ``metropolis_hastings`` Statistics/Samplers.py:53-174 (global numpy RNG, same draw order)
* ``rawstats``            Framework.py:11-17

Parity pin: ``tests/test_oracle_golden.py`` checks every function here against golden
vectors produced by importing the reference itself in the build container
(``tests/golden/make_golden.py``).  The integration is the very same scipy ``odeint``
call, so trajectories are bit-identical to the reference's.

Third-party algorithm on the path: ``scipy.integrate.odeint`` (ODEPACK LSODA,
requirements.txt pins ``scipy>=1.5.1``; 1.15.3 in this image) and numpy's legacy
``RandomState`` (MT19937 + polar Box–Muller, ``numpy>=1.19.0``; 2.2.6 here).
"""
from __future__ import annotations

import warnings

import numpy as np
import pandas as pd
from scipy.integrate import odeint


# ---------------------------------------------------------------- data setup (Framework.py)
def times_grid(t_end: float, t_steps: int) -> np.ndarray:
    return np.linspace(0, t_end, t_steps)


def format_df(df: pd.DataFrame, snames) -> pd.DataFrame:
    """_formatdf (Framework.py:281-307), non-replicate and replicate branches."""
    df = df.sort_values(by=["organism", "time"])
    if "replicate" in df:
        _df = df[["organism", "time", "abundance"]].copy()
        _df["log_abundance"] = np.log(_df["abundance"])
        dfagg = _df.groupby(by=["time", "organism"]).mean()
        dfagg["log_sigma"] = _df.groupby(by=["time", "organism"]).std()["log_abundance"]
        dfagg = dfagg.reset_index(level="time")
        return dfagg
    df = df.set_index("organism")
    if "abundance" in df and "log_abundance" not in df:
        df["log_abundance"] = np.log(df["abundance"].to_numpy())
    if "log_sigma" not in df:
        df["log_sigma"] = 1
        warnings.warn("log_sigma not found, setting log variance to 1")
    return df


def fit_setup(df: pd.DataFrame, times: np.ndarray):
    """_df_fitsetup (Framework.py:309-329): first index minimising |t_obs - t|."""
    pred_tindex, obs_log, obs_logsigma = {}, {}, {}
    for pred in set(df.index):
        tv = df.loc[pred]["time"]
        if isinstance(tv, pd.Series):
            pred_tindex[pred] = np.r_[[np.where(abs(a - times) == min(abs(a - times)))[0][0] for a in tv]]
        else:
            pred_tindex[pred] = np.r_[np.where(abs(tv - times) == min(abs(tv - times)))[0][0]]
    for sname in df.index:
        obs_log[sname] = df.loc[sname]["log_abundance"].to_numpy()
        obs_logsigma[sname] = df.loc[sname]["log_sigma"].to_numpy()
    return pred_tindex, obs_log, obs_logsigma


def summation_index(snames, mapping):
    """_get_summation_index (Framework.py:332-381)."""
    if not mapping:
        return {}, tuple(), tuple(), {}
    sname_i = {s: i for i, s in enumerate(snames)}
    isum, summed, newname = {}, set(), {}
    for sumpop, pops in mapping.items():
        idx = []
        for pop in pops:
            if pop in summed:
                raise ValueError(f"{pop} state varaiable cannot be used in two summations")
            if pop not in snames:
                raise ValueError(f"{pop} state varaiable is not a valid state name")
            summed.add(pop)
            idx.append(sname_i[pop])
        idx.sort()
        newname[idx[0]] = sumpop
        isum[idx[0]] = tuple(idx)
    out_names, keep = [], []
    for i, s in enumerate(snames):
        if i in newname:
            out_names.append(newname[i]); keep.append(i)
        elif s not in summed:
            out_names.append(s); keep.append(i)
    return isum, tuple(out_names), tuple(keep), newname


# ---------------------------------------------------------------- integrate + likelihood
def odeint_traj(rhs, y0, times, ps, rtol=None, atol=None):
    """The reference's integrator call (Framework.py:656): full [T, S] float64."""
    kw = {}
    if rtol is not None:
        kw["rtol"] = rtol
    if atol is not None:
        kw["atol"] = atol
    return odeint(rhs, y0=list(y0), t=times, args=(list(ps),), **kw)


def integrate(rhs, y0, times, ps, sum_index=None, sumkeep=(), out_names=(), pred_tindex=None,
              predict_obs=False, sum_subpopulations=True, rtol=None, atol=None):
    """ModelFramework.integrate(as_dataframe=False) (Framework.py:622-683)."""
    mod = odeint_traj(rhs, y0, times, ps, rtol, atol)
    if sum_subpopulations and sum_index:
        for sumi in sum_index:
            mod[:, sumi] = mod[:, sum_index[sumi]].sum(axis=1)
        mod = mod[:, sumkeep]
    if predict_obs:
        d = {}
        for i, s in enumerate(out_names):
            if s in pred_tindex:
                d[s] = mod[:, i][pred_tindex[s]]
        return d
    return mod


def chi(O, C, S):
    """stats.chi (stats.py:22-41): non-finite terms are masked out of the sum."""
    return ((np.ma.masked_invalid(O) - C) ** 2 / (2 * (S ** 2))).sum()


def aic(chi_v, num_parameters):
    """stats.AIC (stats.py:44-47)."""
    return -2 * (-chi_v) + 2 * num_parameters


def rsqrd(C_dict, O_dict):
    """stats.Rsqrd (stats.py:49-56), linear space."""
    sstot = 0
    ssres = 0
    for s in C_dict:
        ssres += np.nansum((C_dict[s] - O_dict[s]) ** 2)
        sstot += C_dict[s].shape[0] * np.var(O_dict[s])
    return 1 - ssres / sstot


def get_chi(mod_dict, obs_log, obs_logsigma):
    """ModelFramework.get_chi (Framework.py:685-697): concatenation in mod_dict order."""
    O, Cc, S = [], [], []
    for s in mod_dict:
        O.append(obs_log[s]); Cc.append(np.log(mod_dict[s])); S.append(obs_logsigma[s])
    return chi(np.concatenate(O, axis=0), np.concatenate(Cc, axis=0), np.concatenate(S, axis=0))


def get_rsqrd(mod_dict, obs_log):
    """ModelFramework.get_Rsqrd (Framework.py:699-702)."""
    return rsqrd(mod_dict, {k: np.exp(v) for k, v in obs_log.items()})


def rawstats(series):
    """rawstats (Framework.py:11-17): log-normal median and std (pandas ddof=1)."""
    log_mean = np.log(series).mean()
    median = np.exp(log_mean)
    log_std = np.log(series).std()
    std = ((np.exp(log_std ** 2) - 1) * np.exp(2 * log_mean + log_std ** 2.0)) ** 0.5
    return median, std


# ---------------------------------------------------------------- Metropolis–Hastings
class Param:
    """Minimal restatement of ODElib.parameter (Framework.py:50-163) for the MH loop."""

    def __init__(self, val, dist=None, hp=None):
        self.val = np.array(val)
        self.dist = dist
        self.hp = hp or {}
        self._dim = self.val.shape

    def pdf(self, val=None):  # Framework.py:97-105 (no-arg form draws rvs)
        if self.dist:
            if val:
                return self.dist.pdf(val, **self.hp)
            return self.dist.pdf(self.dist.rvs(**self.hp), **self.hp)
        return 1.0

    def rwalk(self, std=0.05):  # Framework.py:107-122
        stds = np.full(self._dim, std)
        self.val = np.exp(np.log(self.val) + np.random.normal(0, stds))


class Model:
    """The slice of ModelFramework that MetropolisHastings touches (duck typing,
    Samplers.py:72-153)."""

    def __init__(self, rhs, pnames, snames, params, istates, times, pred_tindex, obs_log, obs_logsigma,
                 sum_index=None, sumkeep=(), out_names=None, random_seed=0, integrator=None):
        self.rhs = rhs
        self._pnames = tuple(pnames)
        self._snames = tuple(snames)
        self.parameters = params            # name -> Param
        self.istates = dict(istates)
        self.times = times
        self._pred_tindex = pred_tindex
        self._obs_logabundance = obs_log
        self._obs_logsigma = obs_logsigma
        self.sum_index = sum_index or {}
        self.sumkeep = sumkeep
        self.out_names = tuple(out_names) if out_names is not None else tuple(snames)
        self.random_seed = random_seed
        self._pnum = sum(1 for p in pnames if params.get(p) is not None)
        # integrator(y0, ps) -> full [T,S] trajectory; default = the reference's odeint
        self.integrator = integrator or (lambda y0, ps: odeint_traj(self.rhs, y0, self.times, ps))

    def get_pnames(self):
        return list(self._pnames)

    def get_parameters(self, as_dict=False):
        if as_dict:
            return {p: self.parameters[p].val for p in self._pnames}
        return (tuple(self.parameters[p].val for p in self._pnames),)

    def set_parameters(self, **kw):
        for p, v in kw.items():
            self.parameters[p].val = v

    def set_inits(self, **kw):
        for s, v in kw.items():
            if s in self.istates:
                self.istates[s] = v

    def integrate_obs(self):
        y0 = [self.istates[s] for s in self._snames]
        ps = [self.parameters[p].val for p in self._pnames]
        mod = np.array(self.integrator(y0, ps), dtype=float)
        if self.sum_index:
            for sumi in self.sum_index:
                mod[:, sumi] = mod[:, self.sum_index[sumi]].sum(axis=1)
            mod = mod[:, self.sumkeep]
        d = {}
        for i, s in enumerate(self.out_names):
            if s in self._pred_tindex:
                d[s] = mod[:, i][self._pred_tindex[s]]
        return d

    def get_chi(self, mod_dict):
        return get_chi(mod_dict, self._obs_logabundance, self._obs_logsigma)

    def get_Rsqrd(self, mod_dict):
        return get_rsqrd(mod_dict, self._obs_logabundance)

    def get_AIC(self, chi_v):
        return aic(chi_v, self._pnum)


def metropolis_hastings(model: Model, nits=1000, burnin=None, static_parameters=(), replay=None):
    """Samplers.MetropolisHastings (Samplers.py:53-174), printing removed.

    With ``replay=(dz [nits-1][P], u [nits-1])`` the proposal increments and the
    acceptance uniforms come from the arrays instead of the global numpy RNG (and the
    prior ``rvs`` draws, whose values are unused at Samplers.py:118-121, are skipped).
    Returns a dict of columns: pnames..., chi, rsquared, aic, iteration,
    acceptance_ratio, plus 'accepted' (per-iteration decisions, all iterations),
    'margin' (acc - u per iteration, for borderline analysis), 'a_priori' (the initial
    chi, printed as 'a priori error') and 'printed' (the value the reference prints on
    every iteration, exp(-chi) of the current state before the decision, Samplers.py:123;
    NaN where it prints a masked value)."""
    if replay is None:
        np.random.seed(model.random_seed)
    pnames = model.get_pnames()
    reject = set(static_parameters)
    ps = model.get_parameters(as_dict=True)
    oldpar = {p: ps[p] for p in ps if p not in reject}
    iterations = np.arange(1, nits, 1)
    if not burnin:
        burnin = int(nits / 2)
    modcalc = model.integrate_obs()
    chi_v = model.get_chi(modcalc)
    rsq = model.get_Rsqrd(modcalc)
    aic_v = model.get_AIC(chi_v)
    rows, chis, its, rsqs, aics, ars_out = [], [], [], [], [], []
    ars, accepted, margins, printed = [], [], [], []
    a_priori = float(np.ma.filled(chi_v, np.nan)) if np.ma.is_masked(chi_v) else float(chi_v)
    pidx = {p: i for i, p in enumerate(pnames)}
    for it in iterations:
        for p in oldpar:
            if replay is None:
                model.parameters[p].rwalk()
            else:
                v = model.parameters[p].val
                model.parameters[p].val = np.exp(np.log(v) + replay[0][it - 1][pidx[p]])
            _is = {}
            for s in model._snames:
                if s + "0" in pnames:
                    _is[s] = model.parameters[s + "0"].val
            model.set_inits(**_is)
        modcalc = model.integrate_obs()
        chinew = model.get_chi(modcalc)
        if replay is None:
            [model.parameters[p].pdf(oldpar[p]) for p in oldpar]
            [model.parameters[p].pdf() for p in oldpar]
        shown = np.exp(-chi_v)
        printed.append(float(np.ma.filled(shown, np.nan)) if np.ma.is_masked(shown) else float(shown))
        lr = np.exp(chi_v - chinew)
        acc = np.exp(np.log(lr))
        u = np.random.rand() if replay is None else replay[1][it - 1]
        take = acc > u
        margins.append(float(np.ma.filled(acc - u, np.nan)) if np.ma.is_masked(acc - u) else float(acc - u))
        if take:
            chi_v = chinew
            rsq = model.get_Rsqrd(modcalc)
            aic_v = model.get_AIC(chi_v)
            ps = model.get_parameters(as_dict=True)
            for p in oldpar:
                oldpar[p] = ps[p]
            ars.append(1)
        else:
            model.set_parameters(**oldpar)
            _is = {}
            for s in model._snames:
                if (s + "0" in pnames) and (s + "0" not in reject):
                    _is[s] = oldpar[s + "0"]
            model.set_inits(**_is)
            ars.append(0)
        accepted.append(bool(take))
        if it > burnin:
            rows.append({p: float(v) for p, v in model.get_parameters(as_dict=True).items()})
            chis.append(float(chi_v))
            its.append(int(it))
            rsqs.append(float(rsq))
            aics.append(float(aic_v))
            ars_out.append(np.array(ars).mean())
    out = {p: np.array([r[p] for r in rows], dtype=float) for p in pnames}
    for p in static_parameters:  # Samplers.py:166-170 (reports hp['scale'])
        out[p] = np.full(len(rows), model.parameters[p].hp["scale"], dtype=float)
    out.update(chi=np.array(chis, float), rsquared=np.array(rsqs, float), aic=np.array(aics, float),
               iteration=np.array(its, float), acceptance_ratio=np.array(ars_out, float),
               accepted=np.array(accepted, bool), margin=np.array(margins, float), a_priori=a_priori,
               printed=np.array(printed, float))
    return out
