"""Synthetic line-landmark worlds and scans (host side, numpy).

Produces the inputs of `Robot::localize` (slam_ros/Robot.cpp:126): per instance an encoder
pose (main.cpp:84-89, topic realRoboPose) and a list of observed lines {alfa, r, C_AR}
(simplifyPath.h:62-79, produced by LineExtraction, lineFitting.cpp:650-702).

Benchmark world (tuned so that association is robust):
  * s = N - 10 active landmarks on a jittered (alpha, r) grid with A = ceil(sqrt(s)) columns;
  * P0 = diag(pose, heading, landmark variances) + U·Uᵀ (U: n×32 Gaussian, inactive rows 0);
  * the robot drives slowly along +x with a small heading wobble; the encoder reports the true
    pose plus noise; each scan observes L distinct landmarks with small Gaussian noise and
    C_AR = diag(var_alpha, var_r) (off-diagonals zero, as lineFitting.cpp:446-448 forces).
Instance k of an ensemble perturbs the encoder and the observations with its own stream.

Two parameter profiles. "bench" (default, above): small noise, so that the association is
unambiguous at the reference's 0.4 Mahalanobis gate. "survey": SURVEY.md §8d literally — P0 pose /
heading / landmark variances 0.05 / 1e-3 / 1e-3 plus U·Uᵀ with U_ik ~ N(0, (1e-2/√32)²), 0.05 m and
0.01 rad per step, encoder noise σ = 1e-3, observation noise σ_z = 1e-2, R = diag(9e-4, 9e-4)
(LINENOISE² = 0.03², Robot.h:16). Under the survey profile a true match has sqrt(d²) ≈ σ_z·√2/0.03
≈ 0.47 on average — above the 0.4 gate — so many lines are not matched and become new landmarks
(DESIGN §5 reports what that does to the association and the throughput).
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import numpy as np

LINE_FIELDS = 6  # alpha, r, R00, R01, R10, R11  (== struct ekf_line)


def wrap_pi(a):
    """main.cpp:63-66 style wrap of an observed line angle into (-pi, pi]."""
    a = np.mod(np.asarray(a, dtype=np.float64) + np.pi, 2.0 * np.pi) - np.pi
    return np.where(a <= -np.pi, a + 2.0 * np.pi, a)


@dataclass
class World:
    capacity: int
    alpha: np.ndarray  # world-frame line angles of the active landmarks
    r: np.ndarray      # world-frame line distances

    @property
    def active(self) -> int:
        return int(self.alpha.shape[0])

    @property
    def n(self) -> int:
        return 3 + 2 * self.capacity


def make_world(capacity: int, active: int | None = None, seed: int = 42) -> World:
    s = capacity - 10 if active is None else int(active)
    s = max(0, min(s, capacity))
    A = max(1, math.ceil(math.sqrt(max(s, 1))))
    rows = max(1, math.ceil(s / A))
    rng = np.random.default_rng(seed)
    j = np.arange(s)
    alpha = -np.pi + 2.0 * np.pi * ((j % A) + 0.5) / A + rng.uniform(-0.2 / A, 0.2 / A, s)
    r = 0.5 + 7.5 * (j // A) / rows + rng.uniform(-0.01, 0.01, s)
    return World(capacity, alpha.astype(np.float64), r.astype(np.float64))


@dataclass
class InitialState:
    diag: np.ndarray   # (n,)
    U: np.ndarray      # (n, rank)
    y: np.ndarray      # (n,)
    saved: int
    pose: np.ndarray   # (3,)

    def dense_P(self) -> np.ndarray:
        P = self.U @ self.U.T
        P[np.diag_indices_from(P)] += self.diag
        return P


PROFILES = {
    # P0 variances, U column sigma, step (m, rad), noise sigmas, line covariance
    "bench": dict(pose_var=1e-4, heading_var=1e-5, landmark_var=1e-5, u_sigma=None, speed=1e-3,
                  turn=None, enc_noise=1e-4, z_noise=5e-4, var_alpha=1e-4, var_r=1e-4),
    "survey": dict(pose_var=0.05, heading_var=1e-3, landmark_var=1e-3, u_sigma=1e-2 / math.sqrt(32),
                   speed=0.05, turn=0.01, enc_noise=1e-3, z_noise=1e-2, var_alpha=9e-4, var_r=9e-4),
}


def initial_state(world: World, seed: int = 43, rank: int = 32, pose_var: float = 1e-4,
                  heading_var: float = 1e-5, landmark_var: float = 1e-5,
                  profile: str | None = None) -> InitialState:
    n, s = world.n, world.active
    rng = np.random.default_rng(seed)
    sigma = None
    if profile is not None:
        pr = PROFILES[profile]
        pose_var, heading_var, landmark_var, sigma = (pr["pose_var"], pr["heading_var"],
                                                      pr["landmark_var"], pr["u_sigma"])
    diag = np.zeros(n)
    diag[0] = diag[1] = pose_var
    diag[2] = heading_var
    diag[3:3 + 2 * s] = landmark_var
    if sigma is None:
        sigma = math.sqrt(0.5 * landmark_var / rank)
    U = rng.normal(0.0, sigma, size=(n, rank))
    U[3 + 2 * s:] = 0.0
    y = np.zeros(n)
    y[3:3 + 2 * s:2] = world.alpha
    y[4:3 + 2 * s:2] = world.r
    return InitialState(diag, U, y, s, np.zeros(3))


def truth_pose(step: int, speed: float = 1e-3, wobble: float = 2e-4, turn: float | None = None) -> np.ndarray:
    if turn is None:
        return np.array([speed * step, 0.0, wobble * math.sin(step / 10.0)])
    # constant speed and turn rate: a circle of radius speed / turn (0.05 m, 0.01 rad)
    th = turn * step
    if turn == 0.0:
        return np.array([speed * step, 0.0, 0.0])
    R = speed / turn
    return np.array([R * math.sin(th), R * (1.0 - math.cos(th)), th])


def _noise(rng: np.random.Generator, sigma: float, size, clip: float = 2.5) -> np.ndarray:
    """Gaussian noise truncated at ±clip·sigma, so that no draw lands near the 0.4 gate
    (association must be precision-robust)."""
    return np.clip(rng.normal(0.0, sigma, size), -clip * sigma, clip * sigma)


def make_scan(world: World, step: int, instances: int = 1, lines: int = 8, seed: int = 7,
              z_noise: float = 5e-4, enc_noise: float = 1e-4, var_alpha: float = 1e-4,
              var_r: float = 1e-4, first_instance: int = 0, profile: str | None = None,
              redraw: int = 0):
    """Returns (encoder[E,3], lines[E,L,6], nlines[E]) for one scan of `instances` EKFs.
    redraw > 0 draws another scan for the same step (the gate-margin rejection of SURVEY §8d)."""
    s = world.active
    L = min(lines, s)
    speed, turn = 1e-3, None
    if profile is not None:
        pr = PROFILES[profile]
        z_noise, enc_noise, var_alpha, var_r = pr["z_noise"], pr["enc_noise"], pr["var_alpha"], pr["var_r"]
        speed, turn = pr["speed"], pr["turn"]
    pick = np.random.default_rng([seed + step, redraw] if redraw else seed + step).choice(s, size=L, replace=False)
    pose = truth_pose(step, speed=speed, turn=turn)
    enc = np.zeros((instances, 3))
    out = np.zeros((instances, lines, LINE_FIELDS))
    for e in range(instances):
        rng = np.random.default_rng([1000 + first_instance + e, step] + ([redraw] if redraw else []))
        enc[e] = pose + _noise(rng, enc_noise, 3) * np.array([1.0, 1.0, 0.1])
        a = world.alpha[pick]
        z_a = wrap_pi(a - pose[2] + _noise(rng, z_noise, L))
        z_r = world.r[pick] - (pose[0] * np.cos(a) + pose[1] * np.sin(a)) + _noise(rng, z_noise, L)
        out[e, :L, 0] = z_a
        out[e, :L, 1] = z_r
        out[e, :L, 2] = var_alpha
        out[e, :L, 5] = var_r
    return enc, out, np.full(instances, L, dtype=np.int32)


def random_lines(rng: np.random.Generator, count: int, var=(1e-4, 1e-4)) -> np.ndarray:
    """Unstructured observations (first scans / augmentation tests)."""
    out = np.zeros((count, LINE_FIELDS))
    out[:, 0] = rng.uniform(-np.pi, np.pi, count)
    out[:, 1] = rng.uniform(0.3, 6.0, count)
    out[:, 2] = var[0]
    out[:, 5] = var[1]
    return out
