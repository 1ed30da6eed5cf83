from .wolfe_conditions import line_search_wolfe_conditions

__all__ = ["line_search_wolfe_conditions"]
