"""CPU: the drop-in ABI — struct layouts, exported symbols, header declarations,
and that the product path fails loudly (no CPU fallback) when no GPU is visible."""
from __future__ import annotations

import ctypes as C
import re
import subprocess
from pathlib import Path

import pytest

import amg_amd as A
from amg_amd import _native as N

ROOT = Path(__file__).resolve().parent.parent


@pytest.mark.parametrize("struct,size,offsets", [
    (N.SSS_MAT, 40, {"row_ptr": 16, "col_idx": 24, "val": 32}),
    (N.SSS_VEC, 16, {"d": 8}),
    (N.SSS_IVEC, 16, {"d": 8}),
    (N.SSS_RTN, 24, {"nits": 16}),
    (N.SSS_AMG_PARS, 104, {"tol": 8, "ctol": 16, "max_it": 24, "smoother": 40, "relax": 48, "cf_order": 56,
                           "pre_iter": 60, "post_iter": 64, "interp_type": 72, "strong_threshold": 80,
                           "trunc_threshold": 96}),
    (N.SSS_AMG_COMP, 184, {"R": 40, "P": 80, "b": 120, "x": 136, "cfmark": 152, "wp": 168}),
    (N.SSS_AMG, 144, {"cg": 8, "pars": 16, "rtn": 120}),
    (N.SSS_SMTR, 72, {}),
    (N.SSS_KRYLOV, 48, {}),
])
def test_struct_layout_matches_reference(struct, size, offsets):
    assert C.sizeof(struct) == size
    for field, off in offsets.items():
        assert getattr(struct, field).offset == off, field


def test_c_header_layout_compiles_to_reference_sizes(tmp_path):
    """The C header itself (not only the ctypes mirror) has the reference layout."""
    src = tmp_path / "chk.c"
    src.write_text('#include "sss_amg.h"\n#include <stddef.h>\n'
                   '_Static_assert(sizeof(SSS_MAT) == 40, "MAT");\n'
                   '_Static_assert(sizeof(SSS_AMG_PARS) == 104, "PARS");\n'
                   '_Static_assert(sizeof(SSS_AMG_COMP) == 184, "COMP");\n'
                   '_Static_assert(sizeof(SSS_AMG) == 144, "AMG");\n'
                   '_Static_assert(sizeof(SSS_SMTR) == 72, "SMTR");\n'
                   '_Static_assert(sizeof(SSS_KRYLOV) == 48, "KRYLOV");\n'
                   '_Static_assert(offsetof(SSS_AMG_COMP, wp) == 168, "wp");\n'
                   '_Static_assert(offsetof(SSS_AMG, rtn) == 120, "rtn");\n'
                   'int main(void) { return 0; }\n')
    subprocess.run(["gcc", "-std=c11", "-I", str(ROOT / "include"), "-c", str(src), "-o", str(tmp_path / "chk.o")],
                   check=True)


def test_library_exports_every_declared_symbol():
    lib = A.lib()
    for name in N.ABI_SYMBOLS:
        assert hasattr(lib, name), name
    out = subprocess.run(["nm", "-D", "--defined-only", str(N.LIB_PATH)], capture_output=True, text=True,
                         check=True).stdout
    exported = {line.split()[-1] for line in out.splitlines() if " T " in line}
    missing = [s for s in N.ABI_SYMBOLS if s not in exported]
    assert not missing, missing


def test_headers_declare_every_symbol():
    text = (ROOT / "include" / "sss_amg.h").read_text() + (ROOT / "include" / "sss_hip.h").read_text()
    for name in N.ABI_SYMBOLS:
        assert re.search(r"\b%s\s*\(" % re.escape(name), text), name


def test_cli_binary_built():
    assert N.BIN_PATH.exists()


@pytest.mark.skipif(A.device_count() > 0, reason="a GPU is present")
def test_product_fails_loudly_without_gpu(tmp_path):
    """SSS_solver_amg must not silently fall back to a CPU path (exit ERROR_MISC = -14)."""
    env = {"SSS_GEN": "poisson7:8", "PATH": "/usr/bin:/bin"}
    r = subprocess.run([str(N.BIN_PATH)], capture_output=True, text=True, env=env, timeout=120)
    assert r.returncode == (-14) % 256
    assert "### ERROR" in r.stdout + r.stderr
    # the setup table (host C, as in the reference) was printed before the solve refused
    assert "Operator complexity" in r.stdout


@pytest.mark.skipif(A.device_count() > 0, reason="a GPU is present")
def test_spmv_entry_fails_loudly_without_gpu():
    code = ("import sys; sys.path.insert(0, %r)\n"
            "import numpy as np, ctypes as C, amg_amd as A\n"
            "from amg_amd._native import dptr\n"
            "M = A.generate(7, 4); x = np.ones(64); y = np.zeros(64)\n"
            "A.lib().SSS_blas_mv_mxy(C.byref(M), C.byref(A.SSS_VEC(64, dptr(x))), C.byref(A.SSS_VEC(64, dptr(y))))\n"
            "print('returned')\n") % str(ROOT)
    r = subprocess.run(["python", "-c", code], capture_output=True, text=True, timeout=120)
    assert r.returncode == (-14) % 256 and "returned" not in r.stdout


@pytest.mark.parametrize("env,want", [(None, -1), ("full", 0), ("lean", 1), ("bogus", -1)])
def test_opts_formats_default_and_env(env, want, monkeypatch):
    """sss_hip_opts.formats: auto (-1) by default -- plain tiles for the exact smoother, every
    qualifying format otherwise -- SSS_HIP_FORMATS=full|lean force either; the struct's size and the
    field's offset are the C header's (sss_hip.h)."""
    if env is None:
        monkeypatch.delenv("SSS_HIP_FORMATS", raising=False)
    else:
        monkeypatch.setenv("SSS_HIP_FORMATS", env)
    o = N.SSS_HIP_OPTS()
    A.lib().sss_hip_opts_default(C.byref(o))
    assert o.formats == want
    # the ctypes mirror matches the C header's layout (compiled here)
    import subprocess as sp
    import tempfile
    with tempfile.TemporaryDirectory() as d:
        src = Path(d) / "o.c"
        src.write_text('#include "sss_hip.h"\n#include <stddef.h>\n'
                       '_Static_assert(sizeof(sss_hip_opts) == %d, "size");\n'
                       '_Static_assert(offsetof(sss_hip_opts, formats) == %d, "formats");\n'
                       % (C.sizeof(N.SSS_HIP_OPTS), N.SSS_HIP_OPTS.formats.offset))
        sp.run(["gcc", "-std=c11", "-I", str(ROOT / "include"), "-c", str(src), "-o", str(Path(d) / "o.o")], check=True)


def test_huge_page_hint_is_harmless():
    """sss_huge_hint (transparent huge pages for the large host arrays) accepts any pointer and size:
    small and unaligned ranges are ignored, a large one is advised, and the memory stays intact."""
    import numpy as np
    A.lib().sss_huge_hint.argtypes = [C.c_void_p, C.c_size_t]
    a = np.arange(3 << 20, dtype=np.float64)   # 24 MiB
    A.lib().sss_huge_hint(a.ctypes.data, a.nbytes)
    A.lib().sss_huge_hint(a.ctypes.data + 3, 1000)
    A.lib().sss_huge_hint(None, 0)
    assert a[12345] == 12345.0 and a[-1] == (3 << 20) - 1
