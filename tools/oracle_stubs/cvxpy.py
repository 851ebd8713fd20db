class SolverError(Exception):
    pass
