"""superlu_dist_amd -- MI355X-native numeric factorization (pdgstrf / psgstrf /
pzgstrf) for SuperLU_DIST.  See DESIGN.md.

Layout:
  csrc/        HIP kernels (kernels.h), engine (engine.hip), C ABI (abi.cpp),
               front-end (frontend.cpp) -> lib/libslu_mi355x.so
  lib.py       ctypes binding of include/slu_mi355x.h
  frontend.py  stencil matrices, nested dissection, symbolic, distribution
  engine.py    Plan / Comm drivers of the device factorization
  hbio.py      Harwell-Boeing reader (EXAMPLE/*.rua inputs)
"""
from .lib import SLU_D, SLU_S, SLU_Z, lib  # noqa: F401
