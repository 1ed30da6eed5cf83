"""The legacy solver path over :class:`IOptimisableFunction` objects (reference: ``solvers/``)."""
from .bfgs_camera_solver import BFGSCameraSolver
from .i_optimisable_function import IOptimisableFunction
from .line_search_strong_wolfe_conditions import LineSearchStrongWolfeConditions

__all__ = ["BFGSCameraSolver", "IOptimisableFunction", "LineSearchStrongWolfeConditions"]
