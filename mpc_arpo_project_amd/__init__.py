"""mpc_arpo_project_amd -- MI355X-native batched MPC-QP engine.

The drop-in replacement for the OSQP solve on the reference's hot path
(reference src/trajectorySimulate.py:242-348): a C-ABI HIP library (`libmpcqp.so`, header
include/mpcqp.h) driven from Python through ctypes, with PyTorch-ROCm tensors as batch containers.
"""
from .mpcsim import Debris, FailsafeParams, MPCParams, Noise, SimConditions, SimRun  # noqa: F401

__version__ = "0.1.0"
