"""MI355X-native per-grid-cell full-GP regression (OptimalInterpolation hot path).

Submodules:
  gpr        reference-shaped API: SMLII, GPR3D, GPR3D_batch (GPR_CS2S3.py:107-191)
  _lib       ctypes binding of liboi.so (include/oi.h)
  synthetic  seeded synthetic 25 km workloads
  driver     multi-GPU day driver (pass 1 sharding + RCCL gather)
"""
__version__ = "0.1.0"
