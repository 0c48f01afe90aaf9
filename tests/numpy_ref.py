"""Independent float64 numpy restatement of the reference's per-entity math
(dev-only checker for the C oracle; never used by the product).

Written from the reference sources, not from oracle/frecsys_oracle.c:
  iALS Project                ials.h:88-144
  ProjectU / ProjectU_eval    safer2.h:104-163, cvar_mf.h:182-229
  ProjectV (+ tail quirk)     safer2.h:166-221 (quirk :200-204)
  CVaR gradient steps         cvar_mf.h:88-180
  ComputeLoss                 ials.h:70-86, safer2.h:85-101
  SAFER2 smoothed quantile    safer2.h:598-742
"""
import math

import numpy as np


def ials(hist, X, G, reg, w):
    Xh = X[hist].astype(np.float64)
    A = w * G.astype(np.float64) + reg * np.eye(X.shape[1]) + Xh.T @ Xh
    return np.linalg.solve(A, Xh.sum(0))


def _quirk_rows(h):
    if h > 128 and h % 128:
        r = h % 128
        return np.arange(h - 128, h - r)
    return np.arange(0)


def assemble_u(hist, X, G, reg, w, omega):
    h = len(hist)
    Xh = X[hist].astype(np.float64)
    A = omega * (Xh.T @ Xh / h + w * G.astype(np.float64)) + reg * np.eye(X.shape[1])
    b = omega / h * Xh.sum(0)
    return A, b


def assemble_v(hist, X, G, reg, w, nu, quirk):
    h = len(hist)
    Xh = X[hist].astype(np.float64)
    nh = nu[hist].astype(np.float64)
    A = w * G.astype(np.float64) + (Xh * nh[:, None]).T @ Xh + reg * np.eye(X.shape[1])
    if quirk:
        q = _quirk_rows(h)
        if len(q):
            Xq = Xh[q]
            A += (Xq * nh[q][:, None]).T @ Xq
    b = (Xh * nh[:, None]).sum(0)
    return A, b


def project_u(hist, X, G, reg, w, omega):
    A, b = assemble_u(hist, X, G, reg, w, omega)
    return np.linalg.solve(A, b)


def project_v(hist, X, G, reg, w, nu, quirk):
    A, b = assemble_v(hist, X, G, reg, w, nu, quirk)
    return np.linalg.solve(A, b)


def _stale_upper(A, upper_vals):
    """Full matrix whose strict upper triangle holds `upper_vals` (the
    rank updates only wrote the lower part: SelfAdjointView<Lower>)."""
    L = np.tril(A)
    return L + np.triu(upper_vals, 1)


def cvar_u(hist, e, X, G, reg, w, eta, omega):
    A, b = assemble_u(hist, X, G, reg, w, omega)
    Af = _stale_upper(A, omega * w * G.astype(np.float64))
    return e - eta * (Af @ e - b)


def cvar_v(hist, e, X, G, reg, w, nu, eta, quirk):
    A, b = assemble_v(hist, X, G, reg, w, nu, quirk)
    Af = _stale_upper(A, w * G.astype(np.float64))
    return e - eta * (Af @ e - b)


def user_loss(hist, u, X, G, beta, half):
    p = X[hist].astype(np.float64) @ u.astype(np.float64)
    l = np.mean((p - 1.0) ** 2) + beta * (u @ G.astype(np.float64) @ u)
    return l / 2 if half else l


# ---- SAFER2 smoothed quantile, float64 throughout ----
def _phi(u, h):
    return math.exp(-0.5 * (u / h) ** 2) / (h * math.sqrt(2 * math.pi))


def _Phi(u, h):
    return 0.5 * math.erfc(-(u / h) / math.sqrt(2))


def _gloss(u, h, alpha):
    ell = h * _phi(u, h) + (u / h) * (1 - 2 * _Phi(-u, h))
    return (h / 2) * ell + ((1 - alpha) - 0.5) * u


def _epan_k(u, h):
    uh = u / h
    return 0.75 * (1 - uh * uh) * (abs(uh) < 1) / h


def _epan_cdf(u, h):
    uh = u / h
    ins = abs(uh) <= 1
    pos = uh > 1
    return (h ** -3 / 4.0) * ((3 * u * h * h - u ** 3) + 2 * h ** 3) * ins + (1 - ins) * pos


def _epan_loss(u, h, alpha):
    uh = u / h
    ins = abs(uh) <= 1
    pos = uh > 1
    ell = (0.75 * uh ** 2 - uh ** 4 / 8 + 3 / 8) * ins + abs(uh) * pos
    return 0.5 * h * ell + ((1 - alpha) - 0.5) * u


def safer2_weight(loss, xi, bw, epan=False):
    r = loss - xi
    return 1 - (_epan_cdf(-r, bw) if epan else _Phi(-r, bw))


def _quantile(xi, losses, alpha, bw, epan):
    r = losses - xi
    if epan:
        g = (-(1 - alpha) + np.mean([_epan_cdf(-u, bw) for u in r])) / alpha
        H = np.mean([_epan_k(-u, bw) for u in r]) / alpha
        f = np.mean([_epan_loss(u, bw, alpha) for u in r]) / alpha
    else:
        g = (-(1 - alpha) + np.mean([_Phi(-u, bw) for u in r])) / alpha
        H = np.mean([_phi(-u, bw) for u in r]) / alpha
        f = np.mean([_gloss(u, bw, alpha) for u in r]) / alpha
    return f, g, H


def safer2_xi(losses, prev_xi, iters, alpha, bw, epan=False):
    xi = prev_xi
    for _ in range(iters):
        f0, g0, H = _quantile(xi, losses, alpha, bw, epan)
        d = g0 / H
        gamma = 1.0
        x = xi - gamma * d
        for _ in range(32):
            fx, gx, _ = _quantile(x, losses, alpha, bw, epan)
            if fx > f0 + 1e-4 * gamma * gx * (-d):
                gamma *= 0.5
                x = xi - gamma * d
            else:
                break
        xi = xi - gamma * d
    return xi
