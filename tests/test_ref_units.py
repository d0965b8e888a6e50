"""CPU: product host code and oracle kernels vs the reference's OWN compiled C units.

The reference's pure-C translation units (SSS_utils.c, SSS_matvec.c, Solve/SSS_smooth.c,
Setup/SSS_coarsen.c, SSS_main.c) are built from /root/reference by oracle/Makefile into
oracle/_ref/libsss_ref.so.  Where that library is absent (the GPU box has no reference tree unless
the .so travelled), the same checks run against the committed fixtures in tests/golden/golden.json
(`ref_units`, produced by tests/golden/make_golden.py from that library).
"""
from __future__ import annotations

import ctypes as C
import hashlib
import json
from pathlib import Path

import numpy as np
import pytest

import amg_amd as A
import oracle
from amg_amd._native import SSS_IMAT, SSS_MAT, SSS_SMTR, SSS_VEC, dptr
from conftest import BUS_MTX, build_hierarchy, oracle_solve

HERE = Path(__file__).resolve().parent
REFG = json.loads((HERE / "golden" / "golden.json").read_text())["ref_units"]


class _LazyRef:
    """oracle/_ref/libsss_ref.so, loaded on first use only (so a `-m gpu` run, which deselects
    these CPU tests, never maps the compiled reference).  Only the reference's own symbols (SSS_*)
    load it: pytest's collection probes module attributes (`__test__`, `_pytestfixturefunction`,
    ...), and those must not map the library."""

    def __getattr__(self, name):
        if not name.startswith("SSS_"):
            raise AttributeError(name)
        return getattr(oracle.load_ref(), name)


REF = _LazyRef()
needs_ref = pytest.mark.skipif(not oracle.REF_PATH.exists(), reason="reference units not built (no /root/reference)")


def seq(a) -> str:
    return "%.17g" % (float(np.cumsum(np.asarray(a, dtype=np.float64))[-1]) if len(a) else 0.0)


def ihash(a) -> str:
    return hashlib.sha256(np.ascontiguousarray(a, dtype=np.int32).tobytes()).hexdigest()[:24]


def csr_summary(M) -> dict:
    rp, ci, v = A.csr_arrays(M)
    return {"rows": M.num_rows, "cols": M.num_cols, "nnz": M.num_nnzs, "rp": ihash(rp), "ci": ihash(ci),
            "v_sum": seq(v), "v_abs_sum": seq(np.abs(v)), "v_weighted": seq(v * (np.arange(len(v)) % 97 + 1))}


def same_csr(M1, M2):
    a, b = A.csr_arrays(M1), A.csr_arrays(M2)
    return (M1.num_rows, M1.num_cols, M1.num_nnzs) == (M2.num_rows, M2.num_cols, M2.num_nnzs) and all(
        np.array_equal(x.view(np.uint8), y.view(np.uint8)) for x, y in zip(a, b))


# ---------------------------------------------------------------- golden (always runs)
def test_mtx_ingest_golden():
    assert csr_summary(A.read_mtx(BUS_MTX)) == REFG["bus_csr"]


def test_coarsen_golden(quiet):
    M = A.read_mtx(BUS_MTX)
    pars = A.default_pars()
    verts = A.lib().SSS_ivec_create(M.num_rows)
    P, S = SSS_MAT(), SSS_IMAT()
    with quiet():
        rc = A.lib().SSS_amg_coarsen(C.byref(M), C.byref(verts), C.byref(P), C.byref(S), C.byref(pars))
    mark = np.ctypeslib.as_array(verts.d, shape=(M.num_rows,))
    prp = np.ctypeslib.as_array(P.row_ptr, shape=(P.num_rows + 1,))
    pci = np.ctypeslib.as_array(P.col_idx, shape=(P.num_nnzs,))
    got = {"rc": rc, "mark": ihash(mark), "nC_col": P.num_cols, "n_c_points": int((mark == 1).sum()),
           "P_rp": ihash(prp), "P_ci": ihash(pci), "P_nnz": P.num_nnzs}
    assert got == REFG["bus_coarsen"]


def test_transpose_rap_golden(bus_matrix, quiet):
    H = build_hierarchy(bus_matrix, quiet)
    L0 = H.level(0)
    assert csr_summary(L0.R) == REFG["bus_R"]
    assert csr_summary(H.level(1).A) == REFG["bus_RAP"]


def test_oracle_kernels_golden(bus_matrix, quiet):
    H = build_hierarchy(bus_matrix, quiet)
    L0 = H.level(0)
    n = bus_matrix.num_rows
    ora = oracle.load()
    x = np.cos(np.arange(n) * 0.37)
    y = np.sin(np.arange(n) * 0.11)
    ora.ora_mv_amxpy(-1.0, C.byref(L0.A), dptr(x), dptr(y), 0)
    assert seq(y) == REFG["bus_amxpy"]
    z = np.zeros(n)
    ora.ora_mv_mxy(C.byref(L0.A), dptr(x), dptr(z))
    assert seq(z) == REFG["bus_mxy"]
    for post in (0, 1):
        u = np.cos(np.arange(n) * 0.05)
        ora.ora_gs_cf(dptr(u), C.byref(L0.A), dptr(np.ones(n)), 2, L0.cfmark.d, -1 if post else 1)
        assert seq(u) == REFG["bus_gscf_post" if post else "bus_gscf_pre"]


# ---------------------------------------------------------------- live reference units
def _write_mtx(path, n, entries, field="real", sym="general"):
    with open(path, "w") as f:
        f.write(f"%%MatrixMarket matrix coordinate {field} {sym}\n% generated\n{n} {n} {len(entries)}\n")
        for (i, j, v) in entries:
            if field == "pattern":
                f.write(f"{i + 1} {j + 1}\n")
            elif field == "integer":
                f.write(f"{i + 1} {j + 1} {int(v)}\n")
            else:
                f.write(f"{i + 1} {j + 1} {v!r}\n")


@needs_ref
@pytest.mark.parametrize("field,sym", [("real", "general"), ("real", "symmetric"), ("pattern", "symmetric"),
                                       ("integer", "general"), ("real", "skew-symmetric"), ("complex", "hermitian")])
def test_mtx_variants_vs_reference(tmp_path, field, sym, quiet):
    rng = np.random.default_rng(4)
    n = 37
    ent = []
    for _ in range(150):
        i, j = int(rng.integers(0, n)), int(rng.integers(0, n))
        if sym != "general" and j > i:
            i, j = j, i
        ent.append((i, j, float(rng.standard_normal()) * 10))
    ent += [(i, i, 4.0 + i) for i in range(n)]
    rng.shuffle(ent)
    p = tmp_path / "m.mtx"
    if field == "complex":
        with open(p, "w") as f:
            f.write(f"%%MatrixMarket matrix coordinate complex {sym}\n{n} {n} {len(ent)}\n")
            for (i, j, v) in ent:
                f.write(f"{i + 1} {j + 1} {v!r} {v / 3!r}\n")
    else:
        _write_mtx(p, n, ent, field, sym)
    M1, M2 = SSS_MAT(), SSS_MAT()
    with quiet():
        A.lib().SSS_mat_read(str(p).encode(), C.byref(M1))
        REF.SSS_mat_read(str(p).encode(), C.byref(M2))
    assert same_csr(M1, M2)


def _write_big_mtx(path, n, nent, field, sym, seed, layout="lines"):
    """A Matrix Market file above the parallel-parse threshold (4 MiB of data)."""
    rng = np.random.default_rng(seed)
    i = rng.integers(0, n, nent)
    j = rng.integers(0, n, nent)
    if sym != "general":
        i, j = np.maximum(i, j), np.minimum(i, j)
    v = (rng.standard_normal(nent) * 10).tolist()
    i, j = i.tolist(), j.tolist()
    with open(path, "w") as f:
        f.write(f"%%MatrixMarket matrix coordinate {field} {sym}\n% generated\n{n} {n} {nent}\n")
        if field == "pattern":
            body = "\n".join(f"{a + 1} {b + 1}" for a, b in zip(i, j))
        elif field == "integer":
            body = "\n".join(f"{a + 1} {b + 1} {int(c)}" for a, b, c in zip(i, j, v))
        else:
            body = "\n".join(f"{a + 1}  {b + 1}\t{c!r}  " for a, b, c in zip(i, j, v))
        if layout == "split":   # an entry spread over two lines: only the sequential parser reads it
            body = body.replace("\n", " \n", 1).replace(" \n", "\n\n", 1)
            k = body.index("\n", 1000)
            body = body[:k] + body[k:].replace(" ", "\n", 1)
        f.write(body + "\n\n")


@needs_ref
@pytest.mark.parametrize("field,sym,layout", [("real", "general", "lines"), ("real", "symmetric", "lines"),
                                              ("pattern", "general", "lines"), ("integer", "symmetric", "lines"),
                                              ("real", "general", "split")])
def test_mtx_large_vs_reference(tmp_path, field, sym, layout, quiet):
    """Files above the parallel-parse threshold (sss_mmio.c parse_parallel, chunked at line ends):
    the same CSR as the reference's sequential mmio_info/mmio_data, also when the data section is
    laid out so that only the sequential parser applies (an entry split over two lines)."""
    p = tmp_path / "big.mtx"
    _write_big_mtx(p, 20000, 450000, field, sym, seed=7, layout=layout)
    assert p.stat().st_size > (4 << 20)
    M1, M2 = SSS_MAT(), SSS_MAT()
    with quiet():
        A.lib().SSS_mat_read(str(p).encode(), C.byref(M1))
        REF.SSS_mat_read(str(p).encode(), C.byref(M2))
    assert same_csr(M1, M2)


@needs_ref
def test_generator_equals_mtx_ingest(tmp_path, quiet):
    """The in-memory 7-pt generator == reference ingest of the same operator written as .mtx."""
    for kind, n in [(7, 6), (27, 5)]:
        G = A.generate(kind, n)
        rp, ci, v = A.csr_arrays(G)
        ent = [(i, int(ci[k]), float(v[k])) for i in range(G.num_rows) for k in range(rp[i], rp[i + 1])]
        p = tmp_path / f"g{kind}.mtx"
        _write_mtx(p, G.num_rows, ent)
        M = SSS_MAT()
        with quiet():
            REF.SSS_mat_read(str(p).encode(), C.byref(M))
        assert same_csr(G, M)


@needs_ref
@pytest.mark.parametrize("gen", ["bus", "p7_12", "a27_8"])
def test_coarsen_transpose_rap_vs_reference(gen, quiet):
    M = A.read_mtx(BUS_MTX) if gen == "bus" else A.generate(7, 12) if gen == "p7_12" else A.generate(27, 8)
    pars = A.default_pars()
    v1, v2 = A.lib().SSS_ivec_create(M.num_rows), REF.SSS_ivec_create(M.num_rows)
    P1, S1, P2, S2 = SSS_MAT(), SSS_IMAT(), SSS_MAT(), SSS_IMAT()
    with quiet():
        r1 = A.lib().SSS_amg_coarsen(C.byref(M), C.byref(v1), C.byref(P1), C.byref(S1), C.byref(pars))
        r2 = REF.SSS_amg_coarsen(C.byref(M), C.byref(v2), C.byref(P2), C.byref(S2), C.cast(C.byref(pars), C.c_void_p))
    assert r1 == r2
    m1 = np.ctypeslib.as_array(v1.d, shape=(M.num_rows,))
    m2 = np.ctypeslib.as_array(v2.d, shape=(M.num_rows,))
    assert np.array_equal(m1, m2)
    assert P1.num_cols == P2.num_cols
    # transpose + RAP on the product hierarchy's operators
    H = build_hierarchy(M, quiet)
    for l in range(H.num_levels - 1):
        L = H.level(l)
        assert same_csr(L.R, REF.SSS_mat_trans(C.byref(L.P)))
        assert same_csr(H.level(l + 1).A, REF.SSS_blas_mat_rap(C.byref(L.R), C.byref(L.A), C.byref(L.P)))


@needs_ref
@pytest.mark.parametrize("gen", ["bus", "p7_12"])
def test_oracle_spmv_and_smoother_vs_reference(gen, quiet):
    M = A.read_mtx(BUS_MTX) if gen == "bus" else A.generate(7, 12)
    H = build_hierarchy(M, quiet)
    ora = oracle.load()
    rng = np.random.default_rng(0)
    for l in range(H.num_levels - 1):
        L = H.level(l)
        n = L.A.num_rows
        for Mop in (L.A, L.P, L.R):
            x = rng.standard_normal(Mop.num_cols)
            y1 = rng.standard_normal(Mop.num_rows)
            y2 = y1.copy()
            ora.ora_mv_amxpy(-1.0, C.byref(Mop), dptr(x), dptr(y1), 0)
            REF.SSS_blas_mv_amxpy(-1.0, C.byref(Mop), C.byref(SSS_VEC(Mop.num_cols, dptr(x))),
                                  C.byref(SSS_VEC(Mop.num_rows, dptr(y2))))
            assert np.array_equal(y1.view(np.uint64), y2.view(np.uint64))
            ora.ora_mv_mxy(C.byref(Mop), dptr(x), dptr(y1))
            REF.SSS_blas_mv_mxy(C.byref(Mop), C.byref(SSS_VEC(Mop.num_cols, dptr(x))),
                                C.byref(SSS_VEC(Mop.num_rows, dptr(y2))))
            assert np.array_equal(y1.view(np.uint64), y2.view(np.uint64))
        for post in (0, 1):
            for cf in (1, 0):
                b = rng.standard_normal(n)
                u0 = rng.standard_normal(n)
                us = [u0.copy(), u0.copy()]
                for who, u in zip(("ora", "ref"), us):
                    s = SSS_SMTR()
                    s.smoother = 2
                    s.A = C.pointer(L.A)
                    s.b = C.pointer(SSS_VEC(n, dptr(b)))
                    s.x = C.pointer(SSS_VEC(n, dptr(u)))
                    s.nsweeps = 2
                    s.istart, s.iend, s.istep = 0, n - 1, -1 if post else 1
                    s.cf_order = cf
                    s.ordering = L.cfmark.d
                    fn = (ora.ora_smoother_post if post else ora.ora_smoother_pre) if who == "ora" else \
                        (REF.SSS_amg_smoother_post if post else REF.SSS_amg_smoother_pre)
                    fn(C.byref(s))
                assert np.array_equal(us[0].view(np.uint64), us[1].view(np.uint64)), (gen, l, post, cf)


@needs_ref
def test_blas1_vs_reference():
    rng = np.random.default_rng(1)
    x, y = rng.standard_normal(1001), rng.standard_normal(1001)
    lib = A.lib()
    lib.SSS_blas_array_dot.restype = C.c_double
    lib.SSS_blas_array_dot.argtypes = [C.c_int, C.POINTER(C.c_double), C.POINTER(C.c_double)]
    lib.SSS_blas_array_norm2.restype = C.c_double
    lib.SSS_blas_array_norm2.argtypes = [C.c_int, C.POINTER(C.c_double)]
    assert lib.SSS_blas_array_dot(1001, dptr(x), dptr(y)) == REF.SSS_blas_array_dot(1001, dptr(x), dptr(y))
    assert lib.SSS_blas_array_norm2(1001, dptr(x)) == REF.SSS_blas_array_norm2(1001, dptr(x))


class _capture_fd1:
    """Capture what C code writes to fd 1 (printf) into a string."""

    def __enter__(self):
        import os
        import tempfile
        C.CDLL(None).fflush(None)
        self.f = tempfile.TemporaryFile(mode="w+b")
        self.saved = os.dup(1)
        os.dup2(self.f.fileno(), 1)
        return self

    def __exit__(self, *a):
        import os
        C.CDLL(None).fflush(None)
        os.dup2(self.saved, 1)
        os.close(self.saved)
        self.f.seek(0)
        self.text = self.f.read().decode()
        self.f.close()


@needs_ref
@pytest.mark.parametrize("case", ["bus", "p16", "p32"])
def test_outer_loop_vs_reference_solve(case, quiet):
    """The reference's own SSS_amg_solve (Solve/SSS_SOLVE.c, compiled from the reference tree; its
    SSS_amg_cycle resolved to the oracle cycle) against the oracle's restated loop (ora_solve) and
    the product's iteration print (SSS_print_itinfo, amg_amd/host/sss_util.c): same rtn bitwise,
    same x bitwise, same printed table (timing line excluded)."""
    M = A.read_mtx(BUS_MTX) if case == "bus" else A.generate(7, 16 if case == "p16" else 32)
    H = build_hierarchy(M, quiet)
    n = M.num_rows
    x_ref, b = np.ones(n), np.ones(n)
    with _capture_fd1() as cap:
        rtn_ref = REF.SSS_amg_solve(C.byref(H.mg), C.byref(SSS_VEC(n, dptr(x_ref))), C.byref(SSS_VEC(n, dptr(b))))
    H2 = build_hierarchy(M, quiet)
    x_ora = np.ones(n)
    rtn_ora, rel, ab = oracle_solve(H2, np.ones(n), x_ora)
    assert (rtn_ref.nits, rtn_ref.ares, rtn_ref.rres) == (rtn_ora.nits, rtn_ora.ares, rtn_ora.rres)
    assert np.array_equal(x_ref.view(np.uint64), x_ora.view(np.uint64))
    # the printed table: the product's SSS_print_itinfo over the oracle history reproduces it
    lines = [l for l in cap.text.splitlines() if l.strip() and "solve time" not in l and "WARNING" not in l]
    sumb = float(np.sqrt(n))
    with _capture_fd1() as mine:
        A.lib().SSS_print_itinfo(1, 0, 1.0, sumb, 0.0)
        prev = sumb
        for it, (r, a) in enumerate(zip(rel, ab), start=1):
            A.lib().SSS_print_itinfo(1, it, r, a, a / prev)
            prev = a
    mine_lines = [l for l in mine.text.splitlines() if l.strip()]
    ref_rows = [l for l in lines if not l.startswith("###")]
    assert ref_rows == mine_lines


@needs_ref
@pytest.mark.parametrize("transpose", ["chunked", "atomic", "chunk-fallback"])
@pytest.mark.parametrize("gen", ["p7_64", "circuit", "scrambled"])
def test_parallel_setup_paths_vs_reference(gen, transpose, quiet, monkeypatch):
    """Matrices above the parallel threshold (>= 2^20 entries): both OpenMP transposes
    (transpose_pattern_chunked, and transpose_pattern_par under SSS_TRANSPOSE_ATOMIC) and the
    weak-coupling compaction give the reference's results exactly -- SSS_mat_trans of A and the RS
    C/F marks (SSS_amg_coarsen) against the compiled reference.  chunk-fallback: the chunked
    transpose's window cap lowered to 0 (SSS_TRANSPOSE_CHUNK_CAP), so on the scrambled matrix (windows
    wider than 4 x ncols) it declines and the atomic transpose runs from inside transpose_pattern."""
    from amg_amd import workloads as W
    monkeypatch.delenv("SSS_TRANSPOSE_CHUNK_CAP", raising=False)
    if transpose == "atomic":
        monkeypatch.setenv("SSS_TRANSPOSE_ATOMIC", "1")
    else:
        monkeypatch.delenv("SSS_TRANSPOSE_ATOMIC", raising=False)
    if transpose == "chunk-fallback":
        monkeypatch.setenv("SSS_TRANSPOSE_CHUNK_CAP", "0")
    keep = None
    if gen == "p7_64":
        M = A.generate(7, 64)
    elif gen == "scrambled":   # rows and columns randomly permuted: every chunk's window is wide
        import scipy.sparse as sp
        ia, ja, va = A.csr_arrays(A.generate(7, 64))
        n = len(ia) - 1
        perm = np.random.default_rng(3).permutation(n)
        S = sp.csr_matrix((va, ja, ia), shape=(n, n))[perm][:, perm].tocsr()
        S.sort_indices()
        keep = A.NumpyCSR(S.indptr.astype(np.int32), S.indices.astype(np.int32), S.data.astype(np.float64))
        M = keep.mat
    else:
        keep = W.circuit_csr(300000)
        M = keep.mat
    assert M.num_nnzs >= 1 << 20
    assert same_csr(A.lib().SSS_mat_trans(C.byref(M)), REF.SSS_mat_trans(C.byref(M)))
    pars = A.default_pars()
    v1, v2 = A.lib().SSS_ivec_create(M.num_rows), REF.SSS_ivec_create(M.num_rows)
    P1, S1, P2, S2 = SSS_MAT(), SSS_IMAT(), SSS_MAT(), SSS_IMAT()
    with quiet():
        r1 = A.lib().SSS_amg_coarsen(C.byref(M), C.byref(v1), C.byref(P1), C.byref(S1), C.byref(pars))
        r2 = REF.SSS_amg_coarsen(C.byref(M), C.byref(v2), C.byref(P2), C.byref(S2), C.cast(C.byref(pars), C.c_void_p))
    assert r1 == r2
    assert np.array_equal(np.ctypeslib.as_array(v1.d, shape=(M.num_rows,)),
                          np.ctypeslib.as_array(v2.d, shape=(M.num_rows,)))
    assert (P1.num_cols, P1.num_nnzs) == (P2.num_cols, P2.num_nnzs)
    del keep
