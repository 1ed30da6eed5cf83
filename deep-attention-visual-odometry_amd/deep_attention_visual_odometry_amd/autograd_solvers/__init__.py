from .bfgs_solver import BFGSSolver
from .line_search import line_search_wolfe_conditions

__all__ = ["BFGSSolver", "line_search_wolfe_conditions"]
