"""``IOptimisableFunction`` (reference: ``solvers/i_optimisable_function.py:6-65``): a batched
function of B x E parameter estimates with lazily evaluated error (B, E) and gradient
(B, E, P), functional ``add`` and ``masked_update``."""
from abc import ABC, abstractmethod

import torch


class IOptimisableFunction(ABC):
    @property
    @abstractmethod
    def batch_size(self) -> int:
        ...

    @property
    @abstractmethod
    def num_estimates(self) -> int:
        ...

    @property
    @abstractmethod
    def num_parameters(self) -> int:
        ...

    @property
    @abstractmethod
    def device(self) -> torch.device:
        ...

    @abstractmethod
    def get_error(self) -> torch.Tensor:
        """(B, E) error at the current parameters."""

    @abstractmethod
    def get_gradient(self) -> torch.Tensor:
        """(B, E, P) gradient at the current parameters."""

    def as_parameters_vector(self) -> torch.Tensor:
        """(B, E, P) parameters, for networks."""

    @abstractmethod
    def add(self, parameters: torch.Tensor) -> "IOptimisableFunction":
        """A new instance at current + parameters (B, E, P)."""

    @abstractmethod
    def masked_update(self, other: "IOptimisableFunction", mask: torch.Tensor) -> "IOptimisableFunction":
        """A new instance with ``other``'s values where ``mask`` (B, E) is true."""
