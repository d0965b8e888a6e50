"""Regenerates tests/golden/golden.json (run in the survey container, where /root/reference exists).

Two kinds of fixtures:
  * "survey": known answers measured from the reference (oracle build of SURVEY.md Appendix B) and
    published in SURVEY.md §4 / §8 — typed in verbatim, with the section they come from.
  * "ref_units": outputs of the reference's OWN C units compiled from /root/reference by
    oracle/Makefile (oracle/_ref/libsss_ref.so): .mtx ingest, RS coarsening, transposes, RAP,
    SpMV and the GS-CF smoother on 1138_bus level 0 — stored as sizes + exact checksums
    (sequential sums printed with 17 significant digits, integer hashes) so the GPU box, which has
    no reference tree, can still check against them.

usage: python tests/golden/make_golden.py
"""
from __future__ import annotations

import ctypes as C
import hashlib
import json
import sys
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
ROOT = HERE.parent.parent
sys.path.insert(0, str(ROOT))

import amg_amd as A  # noqa: E402
import oracle  # noqa: E402
from amg_amd._native import SSS_IMAT, SSS_MAT, SSS_SMTR, SSS_VEC, dptr  # noqa: E402

SURVEY = {
    "bus_levels": {"source": "SURVEY.md §4 (1138_bus)", "n_nnz": [[1138, 4054], [511, 2465], [230, 1416],
                                                                   [111, 939], [59, 733]],
                   "nC": [511, 230, 111, 59], "nnzP": [1489, 721, 329, 176],
                   "sumA": ["1460.0402678999981", "14.756851884984847", "7.5745127147709592",
                            "5.3247174423655004"],
                   "grid_complexity": "1.801", "operator_complexity": "2.370"},
    "bus_history": {"source": "SURVEY.md §4 outer-loop history",
                    "relres": ["1.000000e+00", "2.907170e+00", "4.389125e-01", "1.321964e-01", "4.453643e-02",
                               "1.213532e-02", "3.537244e-03", "1.358532e-03", "3.614966e-04", "1.381984e-04",
                               "2.328166e-05", "9.120090e-06", "2.602226e-06", "8.230269e-07"],
                    "absres": ["3.373426e+01", "9.807122e+01", "1.480639e+01", "4.459547e+00", "1.502403e+00",
                               "4.093760e-01", "1.193263e-01", "4.582905e-02", "1.219482e-02", "4.662022e-03",
                               "7.853895e-04", "3.076594e-04", "8.778417e-05", "2.776420e-05"]},
    "bus_cycles": {"source": "SURVEY.md §4 x after V-cycles 1-3",
                   "sum_x": ["273808.28646897391", "308065.47596590512", "317674.07232719049"],
                   "x0": ["0.67613404160134516", "0.74542614008909491", "0.76721282946757596"]},
    "poisson16": {"source": "SURVEY.md §4 7-pt 16^3", "n_nnz": [[4096, 27136], [2048, 34400], [445, 13171],
                                                                 [137, 7419]],
                  "relres": ["3.073047e-02", "8.588788e-04", "2.338000e-05", "6.215931e-07"]},
    "poisson32": {"source": "SURVEY.md §4 7-pt 32^3",
                  "relres": ["6.349449e-02", "3.369243e-03", "1.791682e-04", "9.449950e-06", "4.943019e-07"]},
    "poisson64": {"source": "SURVEY.md §4 7-pt 64^3", "nC": [131072, 23792, 5104, 1981, 944],
                  "coarsest": [944, 225862], "sum_x_cycle1": "21950404.365244035", "iterations": 6,
                  "final_relres": "1.30597e-07"},
    "poisson128": {"source": "SURVEY.md §4 7-pt 128^3", "coarsest": [2120, 1414166], "iterations": 8,
                   "final_relres": "3.47652e-07"},
    "poisson256": {"source": "SURVEY.md §4/§8 uncapped 7-pt 256^3",
                   "n_nnz": [[16777216, 117047296], [8388608, 158205440], [1430459, 49708321], [257139, 16563015],
                             [82546, 16348210], [47117, 19176721], [28240, 20751416], [16858, 19236648],
                             [9585, 13212471], [5041, 6430621]],
                   "relres": ["4.265988e-01", "1.588871e-01", "6.021087e-02", "2.284404e-02", "8.665959e-03",
                              "3.287038e-03", "1.246711e-03", "4.728411e-04", "1.793326e-04", "6.801437e-05",
                              "2.579531e-05", "9.783176e-06", "3.710381e-06", "1.407204e-06", "5.336973e-07"]},
}


def seq(a) -> str:
    return "%.17g" % (float(np.cumsum(np.asarray(a, dtype=np.float64))[-1]) if len(a) else 0.0)


def ihash(a) -> str:
    return hashlib.sha256(np.ascontiguousarray(a, dtype=np.int32).tobytes()).hexdigest()[:24]


def csr_summary(M: SSS_MAT) -> dict:
    rp, ci, v = A.csr_arrays(M)
    return {"rows": M.num_rows, "cols": M.num_cols, "nnz": M.num_nnzs, "rp": ihash(rp), "ci": ihash(ci),
            "v_sum": seq(v), "v_abs_sum": seq(np.abs(v)),
            "v_weighted": seq(v * (np.arange(len(v)) % 97 + 1))}


def ref_units() -> dict:
    ref = oracle.load_ref()
    assert ref is not None, "oracle/_ref/libsss_ref.so missing: run `make oracle` with /root/reference present"
    out = {}
    path = str(HERE / "1138_bus.mtx").encode()
    M = SSS_MAT()
    ref.SSS_mat_read(path, C.byref(M))
    out["bus_csr"] = csr_summary(M)
    # coarsening of level 0 (reference SSS_amg_coarsen, default pars)
    pars = A.default_pars()
    verts = ref.SSS_ivec_create(M.num_rows)
    P = SSS_MAT()
    S = SSS_IMAT()
    rc = ref.SSS_amg_coarsen(C.byref(M), C.byref(verts), C.byref(P), C.byref(S), C.cast(C.byref(pars), C.c_void_p))
    mark = np.ctypeslib.as_array(verts.d, shape=(M.num_rows,)).copy()
    prp = np.ctypeslib.as_array(P.row_ptr, shape=(P.num_rows + 1,)).copy()
    pci = np.ctypeslib.as_array(P.col_idx, shape=(P.num_nnzs,)).copy()
    out["bus_coarsen"] = {"rc": rc, "mark": ihash(mark), "nC_col": P.num_cols, "n_c_points": int((mark == 1).sum()),
                          "P_rp": ihash(prp), "P_ci": ihash(pci), "P_nnz": P.num_nnzs}
    # the standard-interpolation pattern (SSS_coarsen.c:633-725 through SSS_amg_coarsen, interp_type 2)
    pars = A.default_pars()
    pars.interp_type = 2
    verts = ref.SSS_ivec_create(M.num_rows)
    P = SSS_MAT()
    S = SSS_IMAT()
    rc = ref.SSS_amg_coarsen(C.byref(M), C.byref(verts), C.byref(P), C.byref(S), C.cast(C.byref(pars), C.c_void_p))
    mark = np.ctypeslib.as_array(verts.d, shape=(M.num_rows,)).copy()
    prp = np.ctypeslib.as_array(P.row_ptr, shape=(P.num_rows + 1,)).copy()
    pci = np.ctypeslib.as_array(P.col_idx, shape=(P.num_nnzs,)).copy()
    out["bus_coarsen_std"] = {"rc": rc, "mark": ihash(mark), "nC_col": P.num_cols,
                              "n_c_points": int((mark == 1).sum()), "P_rp": ihash(prp), "P_ci": ihash(pci),
                              "P_nnz": P.num_nnzs}
    # transpose + RAP on the product hierarchy's level-0 P (values from the product's interp_DIR)
    H = A.Hierarchy(M)
    L0 = H.level(0)
    RT = ref.SSS_mat_trans(C.byref(L0.P))
    out["bus_R"] = csr_summary(RT)
    Ac = ref.SSS_blas_mat_rap(C.byref(L0.R), C.byref(L0.A), C.byref(L0.P))
    out["bus_RAP"] = csr_summary(Ac)
    # SpMV and smoother on level 0 with deterministic inputs
    n = M.num_rows
    x = np.cos(np.arange(n) * 0.37)
    y = np.sin(np.arange(n) * 0.11)
    ref.SSS_blas_mv_amxpy(-1.0, C.byref(L0.A), C.byref(SSS_VEC(n, dptr(x))), C.byref(SSS_VEC(n, dptr(y))))
    out["bus_amxpy"] = seq(y)
    z = np.zeros(n)
    ref.SSS_blas_mv_mxy(C.byref(L0.A), C.byref(SSS_VEC(n, dptr(x))), C.byref(SSS_VEC(n, dptr(z))))
    out["bus_mxy"] = seq(z)
    for post in (0, 1):
        u = np.cos(np.arange(n) * 0.05)
        b = np.ones(n)
        s = SSS_SMTR()
        s.smoother = 2
        s.A = C.pointer(L0.A)
        s.b = C.pointer(SSS_VEC(n, dptr(b)))
        s.x = C.pointer(SSS_VEC(n, dptr(u)))
        s.nsweeps = 2
        s.istart, s.iend, s.istep = 0, n - 1, -1 if post else 1
        s.cf_order = 1
        s.ordering = L0.cfmark.d
        (ref.SSS_amg_smoother_post if post else ref.SSS_amg_smoother_pre)(C.byref(s))
        out[f"bus_gscf_{'post' if post else 'pre'}"] = seq(u)
    return out


def main():
    data = {"survey": SURVEY, "ref_units": ref_units()}
    (HERE / "golden.json").write_text(json.dumps(data, indent=1, sort_keys=True) + "\n")
    print("wrote", HERE / "golden.json")


if __name__ == "__main__":
    main()
