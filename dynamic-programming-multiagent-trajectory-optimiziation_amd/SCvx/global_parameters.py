"""Global SCvx constants -- identical values to the reference SCvx/global_parameters.py:4-18."""
K = 100
MAX_ITER = 30
TRUST_RADIUS0 = 100.0
CONV_TOL = 1e-3
WEIGHT_NU = 1e4
WEIGHT_SLACK = 1e6
WEIGHT_SIGMA = 100.0
