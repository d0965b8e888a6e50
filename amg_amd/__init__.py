"""MI355X-native AMG solve-phase engine (drop-in for the SSS_SOLVE path of txthpc/amg).

The product is the C-ABI library ``amg_amd/lib/libsss_amg.so`` (host C + gfx950 HIP kernels)
and the ``amg_amd/bin/amg`` CLI; this package is the Python binding used by tests and bench.py.
"""
from ._native import (  # noqa: F401
    ABI_SYMBOLS, COARSE, SMOOTH, SPMV, Comm, DeviceHierarchy, DistHierarchy, Hierarchy, NumpyCSR, PartPlan,
    SSS_AMG, SSS_AMG_COMP,
    SSS_AMG_PARS, SSS_HIP_OPTS, SSS_MAT, SSS_RTN, SSS_SMTR, SSS_VEC, csr_arrays, default_pars, device_count,
    hbm_used_bytes,
    generate, lib, part_save, read_mtx,
)
