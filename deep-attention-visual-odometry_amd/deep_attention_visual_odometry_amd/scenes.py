"""Seeded synthetic multi-view calibration scenes.

Replaces the reference's random scene generator
(``data/camera_and_parameters_dataset.py:48-151``, which does not parse in the
reference snapshot) with a deterministic one: problem ``i`` of a batch is a
pure function of ``(seed, i)``, so any contiguous shard of a batch can be
generated on its own rank with no scatter.

Distributions (per problem), in camera 0's frame:

* f = 1/tan(a/2), a ~ U(pi/6, 2pi/3)                 (dataset ``:148-150``)
* cx, cy ~ clamp(0.2 N(0,1), -0.5, 0.5)               (``:149``)
* views m >= 1 look at the cloud, like the dataset's look-at construction
  (``:100-133``): centre C_m ~ N(0, 3^2), target (0, 0, 20) + N(0, 1), roll
  ~ N(0, 0.1^2); stored as axis-angle w_m and t_m = -R(w_m) C_m
* points X_xy ~ N(0, 3^2), X_z = 20 + 5 clip(N(0,1), -2, 2)   (``:90-94``),
  REJECTION-SAMPLED until every point projects inside |u|, |v| < 0.9 in every
  view (the dataset's visibility window ``:194-197``)
* k1 ~ N(0, 1e-2^2), k2 ~ N(0, 1e-3^2), k3 ~ N(0, 1e-4^2), p1, p2 ~ N(0, 1e-3^2)
* observations: noise-free projection of the truth (fp64, then fp32)
* visibility: all ones, or each (m, n) dropped with probability ``drop``
  (the pair stays in-image, so its residual is finite)
* initial guess x0 = truth + N(0, 0.01^2) on the pinhole block; the five
  distortion coefficients get 10 % of their own spread
  (N(0, [1e-3, 1e-4, 1e-5, 1e-4, 1e-4]^2)).

Why every point is in-image: the reference objective masks with
``(residual^2 * vis).sum()``, so an invisible pair whose projection overflows
at a trial point gives inf * 0 = NaN, and the reference line search (all of
whose tests are NaN-false) then widens or bisects for its full 1000 trials
and walks to inf.  With independent random rotations ~20 % of the
Brown-Conrady problems did exactly that -- in the oracle as well as on the
GPU.  Look-at views + in-image points keep every residual finite.

Parameter layout: see ``camera_model.layout``.
"""
from typing import NamedTuple

import numpy as np
from scipy.spatial.transform import Rotation


class SceneBatch(NamedTuple):
    truth: np.ndarray  # (B, P) float64
    initial: np.ndarray  # (B, P) float32
    observations: np.ndarray  # (B, M, N, 2) float32
    visibility: np.ndarray  # (B, M, N) bool
    num_views: int
    num_points: int
    distortion: bool


def parameter_count(num_views: int, num_points: int, distortion: bool) -> int:
    return 3 + 3 * num_points + 6 * (num_views - 1) + (5 if distortion else 0)


def _rotate(v: np.ndarray, w: np.ndarray) -> np.ndarray:
    """Rodrigues in fp64, v (N,3), w (3,)."""
    theta = np.linalg.norm(w)
    if theta < 1e-12:
        return v.copy()
    k = w / theta
    c, s = np.cos(theta), np.sin(theta)
    return v * c + np.cross(k, v) * s + np.outer(v @ k, k) * (1.0 - c)


def _look_at(forward: np.ndarray, roll: float) -> Rotation:
    """Rotation R with R forward/|forward| = +z, followed by a roll about +z."""
    f = forward / np.linalg.norm(forward)
    axis = np.cross(f, np.array([0.0, 0.0, 1.0]))
    sin_a = np.linalg.norm(axis)
    angle = np.arctan2(sin_a, f[2])
    align = Rotation.from_rotvec(axis / sin_a * angle) if sin_a > 1e-12 else Rotation.identity()
    return Rotation.from_rotvec([0.0, 0.0, roll]) * align


def _pack(f, c, pts, t, w, k) -> np.ndarray:
    row = [np.array([f, c[0], c[1]]), pts.ravel(), t.ravel(), w.ravel()]
    if k is not None:
        row.append(k)
    return np.concatenate(row)


def project_truth(x: np.ndarray, num_views: int, num_points: int, distortion: bool) -> np.ndarray:
    """(M, N, 2) fp64 projection of one parameter vector (no scale normalisation:
    the projection is invariant to it)."""
    f, cx, cy = x[0], x[1], x[2]
    pts = x[3:3 + 3 * num_points].reshape(num_points, 3)
    base = 3 + 3 * num_points
    ts = x[base:base + 3 * (num_views - 1)].reshape(num_views - 1, 3)
    ws = x[base + 3 * (num_views - 1):base + 6 * (num_views - 1)].reshape(num_views - 1, 3)
    out = np.empty((num_views, num_points, 2))
    for m in range(num_views):
        p = pts if m == 0 else _rotate(pts, ws[m - 1]) + ts[m - 1]
        u = f * p[:, 0] / p[:, 2]
        v = f * p[:, 1] / p[:, 2]
        if distortion:
            k1, k2, k3, p1, p2 = x[base + 6 * (num_views - 1):base + 6 * (num_views - 1) + 5]
            r2 = u * u + v * v
            radial = 1.0 + k1 * r2 + k2 * r2 * r2 + k3 * r2 * r2 * r2
            u, v = (u * radial + 2.0 * p1 * u * v + p2 * (r2 + 2 * u * u),
                    v * radial + 2.0 * p2 * u * v + p1 * (r2 + 2 * v * v))
        out[m, :, 0] = u + cx
        out[m, :, 1] = v + cy
    return out


def make_scenes(
    batch: int,
    num_views: int,
    num_points: int,
    distortion: bool = False,
    seed: int = 20251015,
    first_index: int = 0,
    initial_noise: float = 0.01,
    drop: float = 0.0,
    ray_angle: bool = False,
) -> SceneBatch:
    """Problems ``first_index .. first_index + batch - 1`` of the stream ``seed``.

    ``ray_angle=True`` stores the focal slot in the parameterisation of the ray-angle
    objective (focal = elu(x[0]) + 1, ``geometry/homogeneous_projection.py:21-44``), so
    the truth is an exact zero of ``RayAngleError``; the observations are unchanged.
    """
    if num_views < 2:
        raise ValueError("num_views must be >= 2 (the scale normalisation needs a translation)")
    if ray_angle and distortion:
        raise ValueError("the ray-angle objective is pinhole only")
    p = parameter_count(num_views, num_points, distortion)
    truth = np.empty((batch, p))
    initial = np.empty((batch, p), dtype=np.float32)
    obs = np.empty((batch, num_views, num_points, 2), dtype=np.float32)
    vis = np.empty((batch, num_views, num_points), dtype=bool)
    for b in range(batch):
        rng = np.random.default_rng([seed, first_index + b])
        a = np.pi / 6 + (np.pi / 2) * rng.random()
        f = 1.0 / np.tan(a / 2.0)
        c = np.clip(0.2 * rng.standard_normal(2), -0.5, 0.5)
        t = np.empty((num_views - 1, 3))
        w = np.empty((num_views - 1, 3))
        for m in range(num_views - 1):
            centre = 3.0 * rng.standard_normal(3)
            target = np.array([0.0, 0.0, 20.0]) + rng.standard_normal(3)
            rot = _look_at(target - centre, 0.1 * rng.standard_normal())
            w[m] = rot.as_rotvec()
            t[m] = -rot.apply(centre)
        k = rng.standard_normal(5) * np.array([1e-2, 1e-3, 1e-4, 1e-3, 1e-3]) if distortion else None
        pts = np.empty((0, 3))
        for _ in range(1000):
            cand = np.concatenate([3.0 * rng.standard_normal((2 * num_points, 2)),
                                   20.0 + 5.0 * np.clip(rng.standard_normal((2 * num_points, 1)), -2.0, 2.0)], axis=1)
            x = _pack(f, c, cand, t, w, k)
            uv = project_truth(x, num_views, cand.shape[0], distortion)
            inside = (np.abs(uv) < 0.9).all(axis=(0, 2))
            pts = np.concatenate([pts, cand[inside]])
            if pts.shape[0] >= num_points:
                break
        else:
            raise RuntimeError("could not place points inside every view")
        x = _pack(f, c, pts[:num_points], t, w, k)
        obs[b] = project_truth(x, num_views, num_points, distortion)
        if ray_angle:  # elu(x0) + 1 == f
            x[0] = f - 1.0 if f > 1.0 else np.log(f)
        truth[b] = x
        vis[b] = True if drop <= 0.0 else rng.random((num_views, num_points)) >= drop
        kick = initial_noise * rng.standard_normal(p)
        if distortion:
            kick[-5:] *= np.array([1e-1, 1e-2, 1e-3, 1e-2, 1e-2])
        initial[b] = x + kick
    return SceneBatch(truth, initial, obs, vis, num_views, num_points, distortion)
