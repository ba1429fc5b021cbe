"""CPU model of the Newton-basis Kalman step (csrc/kalman_core.h, kstep_nb2) against the oracle.

StepKalman4D (L/WaveSpecZZ_1.0.3-pla-kalman-fast.mq5:2031-2125) predicts with the constant-jerk
transition F = exp(N) (N the shift).  F = T Jd T^-1 with Jd = I + N the Jordan block and

    T^-1 = [[1, 0, 0, 0], [0, 1, 1/2, 1/6], [0, 0, 1, 1], [0, 0, 0, 1]]

(u = T^-1 x = the forward differences of the cubic: u0 = pos, u1 = vel + acc/2 + jerk/6,
u2 = acc + jerk, u3 = jerk).  In u the predict is three neighbour sums for the state and
P' <- Jd P' Jd^T (15 adds) for the covariance, instead of 6 and 35 operations.  What carries over:
  * the measurement row stays e0 (T's first row is e0): S, the gain, boost and clip are unchanged;
  * the reference's P11 prediction (:2052) is not (F P F^T)_11 -- it adds
    e = P12 + P22 + (P13 + P23)/2 of the ORIGINAL basis; T^-1 e1 = e1, so in u it is e added to
    P'11, with e a fixed linear form of P' (E_COEF below);
  * Q = diag(Qp, Qv, Qa, Qj) becomes Q' = T^-1 Q T^-T (7 entries, Q'0j = 0 for j > 0);
  * the diagonal floors max(1e-12, P_ii) (:2110-2114) act on the ORIGINAL basis.  They are
    dropped, and their being no-ops is guarded: if every step has e >= -Qv/2, the predicted P
    dominates diag(Qp, Qv/2, Qa, Qj) > 0 (P PSD by induction: F P F^T and bQ are PSD, and e e1e1^T
    removes at most Qv/2 from the Qv the predict adds), so after the update
    P_n = (P_p^-1 + h h^T / R)^-1 >= diag(Qp R/(Qp + R), Qv/2, Qa, Qj) and no floor binds when those
    exceed 1e-12 (the host gate, nb2_gate below).  A wave with any e < -Qv/2 re-runs in the
    original basis with the floors (kernel side).
This file checks the algebra in fp64 against the oracle's filter (1e-10 of the price level), the guard's
premises on the C3 data, and that the guard fires where it should.
"""
import numpy as np
import pytest

import oracle
from wavespec_amd import synth

TINV = np.array([[1, 0, 0, 0], [0, 1, 0.5, 1 / 6], [0, 0, 1, 1], [0, 0, 0, 1]], dtype=np.float64)
T = np.linalg.inv(TINV)
F = np.array([[1, 1, 0.5, 1 / 6], [0, 1, 1, 0.5], [0, 0, 1, 1], [0, 0, 0, 1]], dtype=np.float64)
JD = np.eye(4) + np.eye(4, k=1)
# e = P12 + P22 + (P13 + P23)/2 (original basis) as a linear form of P' (u basis):
#   P'12 - P'13/2 + P'22/2 - 11/12 P'23 + P'33/3
E_COEF = {(1, 2): 1.0, (1, 3): -0.5, (2, 2): 0.5, (2, 3): -11.0 / 12.0, (3, 3): 1.0 / 3.0}


def q_newton(q):
    """Q' = T^-1 diag(q) T^-T as the 7 entries the kernel adds (00, 11, 12, 13, 22, 23, 33)."""
    m = TINV @ np.diag(q) @ TINV.T
    return m


def nb2_gate(params) -> bool:
    """The host's condition for the floor-free Newton-basis kernel (mtbridge / kalman_kernels.hip):
    the reference default flags and the lower bounds of the docstring comfortably above 1e-12
    (2^-20: fp32 rounding of P stays far below them)."""
    kp = [float(v) for v in params]
    qs = max(0.05, kp[0])
    Qp, Qv, Qa, Qj = (max(1e-9, kp[i] * qs) for i in (1, 2, 3, 4))
    R = max(1e-9, kp[6])
    return min(Qp * R / (Qp + R), Qv / 2, Qa, Qj) >= 2.0 ** -20


def newton_trend(X, params=None):
    """fp64 model of kstep_nb2: returns (trend, min over steps of e + Qv/2 per window)."""
    kp = [float(v) for v in (oracle.KALMAN_DEFAULTS if params is None else params)]
    (follow, q_pos, q_vel, q_acc, q_jerk, adapt, meas, vp, vv, va, vj, iv, ia, ij, clip, ema) = kp
    assert ema == 0.0
    X = np.atleast_2d(np.asarray(X, dtype=np.float64))
    W, n = X.shape
    qs = max(0.05, follow)
    q = np.array([max(1e-9, v * qs) for v in (q_pos, q_vel, q_acc, q_jerk)])
    R = max(1e-9, meas)
    Qn = q_newton(q)
    u = np.zeros((W, 4))
    u[:, 0] = X[:, 0]
    u[:, 1:] = (TINV @ np.array([0.0, iv, ia, ij]))[1:]
    P = np.broadcast_to(TINV @ np.diag([max(1e-9, v) for v in (vp, vv, va, vj)]) @ TINV.T, (W, 4, 4)).copy()
    trend = np.empty((W, n))
    emin = np.full(W, np.inf)
    for t in range(n):
        z = X[:, t]
        e = sum(c * P[:, i, j] for (i, j), c in E_COEF.items())
        emin = np.minimum(emin, e + q[1] / 2)
        up = u.copy()
        up[:, 0] += u[:, 1]
        up[:, 1] += u[:, 2]
        up[:, 2] += u[:, 3]
        Pp = np.einsum("ab,wbc,dc->wad", JD, P, JD)
        Pp[:, 1, 1] += e
        y = z - up[:, 0]
        S = Pp[:, 0, 0] + Qn[0, 0] + R
        if adapt > 0:
            k = np.minimum(5.0, np.abs(y) / np.sqrt(S)) * adapt
        else:
            k = np.zeros(W)
        Pp = Pp + (1.0 + k)[:, None, None] * Qn[None]
        S = Pp[:, 0, 0] + R
        rs = 1.0 / np.sqrt(S)
        yn = y * rs
        if clip > 0:
            yn = np.clip(yn, -clip, clip)
        g = Pp[:, 0, :] * rs[:, None]
        u = up + g * yn[:, None]
        P = Pp - g[:, :, None] * g[:, None, :]
        trend[:, t] = u[:, 0]
    return trend, emin


def test_jordan_factorisation():
    assert np.allclose(T @ JD @ TINV, F, atol=1e-15)
    assert np.allclose(T[0], [1, 0, 0, 0])  # the measurement row stays e0
    assert np.allclose(TINV @ np.eye(4)[1], np.eye(4)[1])  # the P11 extra term stays on P'11
    # e's linear form: (T P' T^T) entries 12 + 22 + (13 + 23)/2 for random symmetric P'
    rng = np.random.default_rng(3)
    for _ in range(5):
        a = rng.standard_normal((4, 4))
        Pn = a + a.T
        Po = T @ Pn @ T.T
        e_orig = Po[1, 2] + Po[2, 2] + 0.5 * (Po[1, 3] + Po[2, 3])
        e_new = sum(c * Pn[i, j] for (i, j), c in E_COEF.items())
        assert abs(e_orig - e_new) < 1e-12 * (1 + abs(e_orig))
    Qn = q_newton(np.array([0.01, 0.003, 0.0008, 0.0002]))
    assert np.allclose(Qn[0, 1:], 0.0) and np.allclose(Qn[1:, 0], 0.0)


@pytest.mark.parametrize("case", ["default", "jumps", "adapt0", "noclip", "slow"])
def test_newton_trend_matches_oracle(case):
    kp = list(oracle.KALMAN_DEFAULTS)
    n, W = 1024, 48
    s = synth.random_walk(W * 64 + n, seed=41)
    X = np.stack([s[w * 64:w * 64 + n] for w in range(W)])
    if case == "jumps":
        X[::3, n // 3:] += 0.5
        X[1::3, n // 2:] -= 0.5
    if case == "adapt0":
        kp[5] = 0.0
    if case == "noclip":
        kp[14] = 0.0
    if case == "slow":
        kp[1:5] = [1e-3, 2e-4, 5e-5, 1e-5]
    ref = oracle.numpy_kalman_trend(X, kp)
    got, emin = newton_trend(X, kp)
    assert nb2_gate(kp)
    assert np.all(emin > 0), "the floor guard holds on these inputs"
    # fp64 rounding at the price level (~1.1) accumulates to ~1e-12; an algebra slip shows at the
    # residual's own scale (~1e-4)
    assert np.abs(got - ref).max() <= 1e-10 * np.abs(X).max()


def test_floor_guard_premise_c3_data():
    """On the C3 series (BASELINE config 3) the guard e >= -Qv/2 holds with room to spare."""
    n = 4096
    s = synth.random_walk(64 * 257 + n, seed=7)
    X = np.stack([s[w * 257:w * 257 + n] for w in range(64)])
    _, emin = newton_trend(X)
    q_v = oracle.KALMAN_DEFAULTS[2] * max(0.05, oracle.KALMAN_DEFAULTS[0])
    assert emin.min() > 0.25 * q_v


def test_gate_rejects_tiny_noise():
    kp = list(oracle.KALMAN_DEFAULTS)
    assert nb2_gate(kp)
    kp[4] = 1e-9  # q_jerk at its floor: P33 may approach 1e-12 in fp32 terms
    assert not nb2_gate(kp)
    kp = list(oracle.KALMAN_DEFAULTS)
    kp[6] = 1e-9  # measurement noise at its floor
    assert not nb2_gate(kp)
