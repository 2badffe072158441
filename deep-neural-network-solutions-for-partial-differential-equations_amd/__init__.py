"""MI355X-native deep-BSDE (FBSNN) training step.

The hot path -- Euler-Maruyama rollout, NAIS-Net/FC subnetwork forward with
Z = grad_x u, residual loss, second-order backward, clip + Adam -- runs as
hand-written HIP kernels for gfx950 behind the C ABI of include/dbsde.h
(lib/libdbsde.so).  This package is the host side: the reference's FBSNN
class surface (nd_BSPDE_case.py / DeepBSDE.py) over that ABI.

Import it with importlib (the directory name is not a Python identifier):
    pkg = importlib.import_module(
        "deep-neural-network-solutions-for-partial-differential-equations_amd")
"""
from . import _lib
from .deepbsde import BlackScholesBarenblatt, u_exact
from .fbsnn import FBSNN, PredictionGenerator
from .problems import BasketCallOption, BSPDETestCase, CallOption, CallOption1D, HamiltonJacobiBellman, HestonFBSNN
from .solver import NativeSolver, ProblemSpec, exact, hjb_mc

__all__ = ["FBSNN", "PredictionGenerator", "BlackScholesBarenblatt", "u_exact", "CallOption", "CallOption1D",
           "BasketCallOption", "BSPDETestCase", "HamiltonJacobiBellman", "HestonFBSNN", "NativeSolver",
           "ProblemSpec", "exact", "hjb_mc", "_lib"]
