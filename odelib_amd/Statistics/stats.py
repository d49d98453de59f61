"""Fit statistics with the reference's formulas (ODElib/Statistics/stats.py:3-63).

These evaluate a handful of numbers on host arrays the caller already holds (a
prediction dict); the per-walker likelihood inside integration / MCMC is computed in
the HIP kernels (ode_kernels.cuh ``emit``) with the same formula.
"""
import numpy as np


def predict_logsigma(sigma, mean):
    """log-space standard deviation from linear mean / sd (stats.py:3-20)"""
    return np.log(1.0 + sigma ** 2.0 / mean ** 2.0) ** 0.5


def chi(O, C, S):
    """Σ (O − C)² / (2 S²) with non-finite terms masked out (stats.py:22-41)"""
    return ((np.ma.masked_invalid(O) - C) ** 2 / (2 * (S ** 2))).sum()


def AIC(chi, num_parameters):
    """stats.py:44-47"""
    return -2 * (-chi) + 2 * num_parameters


def Rsqrd(C_dict, O_dict):
    """linear-space R² (stats.py:49-56)"""
    sstot = 0
    ssres = 0
    for sname in C_dict:
        ssres += np.nansum((C_dict[sname] - O_dict[sname]) ** 2)
        sstot += C_dict[sname].shape[0] * np.var(O_dict[sname])
    return 1 - ssres / sstot


def get_adjusted_rsquared(Rsqrd, num_samples, num_parameters):
    """stats.py:58-63"""
    n, p = num_samples, num_parameters
    return 1 - (1 - Rsqrd) * (n - 1) / (n - p - 1)
