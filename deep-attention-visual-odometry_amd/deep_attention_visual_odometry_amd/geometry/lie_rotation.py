"""``LieRotation`` (reference: ``geometry/lie_rotation.py``), the rotation parameter of the
legacy ``PinholeCameraModelL1``.

The model itself evaluates rotations, their parameter Jacobians and the rotated-vector
Jacobians inside its HIP kernel (csrc/camera_l1.hip); this class carries the axis-angle
vector with the reference's API (construction, ``add_lie_parameters`` with the optional
[-pi, pi) constraint, ``masked_update``, ``slice``, ``as_parameters_vector``,
``from_quaternion``) plus ``rotate_vector`` / ``parameter_gradient`` /
``vector_gradient`` for callers that use them directly.  Same formulas and Taylor
thresholds as the reference (``utils/func_*.py``: 0.01, 0.05, 0.01, 0.25).
"""
import torch


def _series(x, threshold, series, direct):
    near = x.abs() < threshold
    safe = torch.where(near, torch.ones_like(x), x)
    return torch.where(near, series(x), direct(safe))


def _sinc(x):
    return _series(x, 0.01, lambda t: 1.0 - t.square() / 6.0 + t.square().square() / 120
                   - t.square().square() * t.square() / 5040, lambda t: torch.sin(t) / t)


def _versine(x):
    return _series(x, 0.05, lambda t: 0.5 - t.square() / 24 + t.square().square() / 720
                   - t.square().square() * t.square() / 40320, lambda t: (1.0 - torch.cos(t)) / t.square())


def _c_term(x):
    return _series(x, 0.01, lambda t: -1.0 / 3.0 + t.square() / 30.0 - t.square().square() / 840
                   + t.square().square() * t.square() / 45360,
                   lambda t: torch.cos(t) / t.square() - torch.sin(t) / (t * t.square()))


def _d_term(x):
    return _series(x, 0.25, lambda t: -1.0 / 12.0 + t.square() / 180.0 - t.square().square() / 6720.0
                   + t.square().square() * t.square() / 362880.0,
                   lambda t: torch.sin(t) / (t * t.square()) - 2.0 * (1.0 - torch.cos(t)) / t.square().square())


class LieRotation:
    """Axis-angle rotation; ``lie_vector`` (..., 3)."""

    def __init__(self, lie_vector: torch.Tensor):
        self._lie_vector = lie_vector

    @property
    def lie_vector(self) -> torch.Tensor:
        return self._lie_vector

    def angle(self) -> torch.Tensor:
        return torch.linalg.norm(self._lie_vector, dim=-1, keepdim=True)

    def rotate_vector(self, vector: torch.Tensor) -> torch.Tensor:
        w = self._lie_vector
        th = self.angle()
        dot = (vector * w).sum(dim=-1, keepdims=True)
        cross = torch.linalg.cross(w, vector, dim=-1)
        return vector * torch.cos(th) + _versine(th) * dot * w + cross * _sinc(th)

    def parameter_gradient(self, vector: torch.Tensor) -> torch.Tensor:
        """d R(w) v / d w, (..., 3, 3): first axis coordinate, second parameter."""
        w = self._lie_vector
        th = self.angle()
        sinc, vers = _sinc(th), _versine(th)
        dot = (vector * w).sum(dim=-1, keepdims=True)
        cross = torch.linalg.cross(w, vector, dim=-1)
        outer = w.unsqueeze(-2) * vector.unsqueeze(-1)
        term1 = -1.0 * outer * sinc.unsqueeze(-1)
        term2 = (dot * _d_term(th)).unsqueeze(-1) * (w.unsqueeze(-2) * w.unsqueeze(-1))
        term3 = vers.unsqueeze(-1) * (outer.transpose(-2, -1) + dot.unsqueeze(-1) * torch.eye(3, device=w.device,
                                                                                             dtype=w.dtype))
        term4 = (w.unsqueeze(-2) * cross.unsqueeze(-1)) * _c_term(th).unsqueeze(-1)
        x, y, z = vector[..., 0:1], vector[..., 1:2], vector[..., 2:3]
        zero = torch.zeros_like(x)
        term5 = torch.stack([torch.cat([zero, -z, y], dim=-1), torch.cat([z, zero, -x], dim=-1),
                             torch.cat([-y, x, zero], dim=-1)], dim=-1) * sinc.unsqueeze(-1)
        return term1 + term2 + term3 + term4 + term5

    def vector_gradient(self) -> torch.Tensor:
        """d R(w) v / d v = R(w), (..., 3, 3)."""
        w = self._lie_vector
        th = self.angle()
        cos_t, sinc = torch.cos(th), _sinc(th)
        outer = (w.unsqueeze(-2) * w.unsqueeze(-1)) * _versine(th).unsqueeze(-1)
        a, b, c = w[..., 0:1] * sinc, w[..., 1:2] * sinc, w[..., 2:3] * sinc
        cross = torch.stack([torch.cat([cos_t, c, -b], dim=-1), torch.cat([-c, cos_t, a], dim=-1),
                             torch.cat([b, -a, cos_t], dim=-1)], dim=-1)
        return outer + cross

    def slice(self, mask: torch.Tensor) -> "LieRotation":
        sliced = self._lie_vector[mask]
        for _ in range(mask.ndim - 1):
            sliced = sliced.unsqueeze(1)
        return type(self)(sliced)

    def add_lie_parameters(self, lie_vector: torch.Tensor, constrain: bool = False) -> "LieRotation":
        new = self._lie_vector + lie_vector
        if constrain:  # keep the angle in [-pi, pi)
            angles = torch.linalg.norm(new, dim=-1, keepdim=True)
            axes = new / angles.clamp(min=1e-8)
            angles = torch.fmod(angles + torch.pi, 2 * torch.pi) - torch.pi
            new = angles * axes
        return type(self)(new)

    def masked_update(self, other: "LieRotation", mask: torch.Tensor) -> "LieRotation":
        return type(self)(torch.where(mask, other._lie_vector, self._lie_vector))

    def as_parameters_vector(self) -> torch.Tensor:
        return self._lie_vector

    @classmethod
    def from_quaternion(cls, quaternion: torch.Tensor) -> "LieRotation":
        scalar = quaternion[..., 0:1]
        vector = quaternion[..., 1:4]
        half = torch.atan2(torch.linalg.norm(vector, dim=-1, keepdim=True), scalar)
        return cls(torch.nan_to_num(2 * half / torch.sin(half), nan=0.0) * vector)
