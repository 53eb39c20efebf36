"""The problem family and its solvers (one per reference stage)."""
from .problem import STAGES, PoissonEllipse, stage_problem  # noqa: F401
from .solvers import Result, make_session, solve, solve_cpu, solve_cpu_decomposed, solve_hip  # noqa: F401
