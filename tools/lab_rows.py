"""Drive tools/liblab_rows.so over every level of a 7-pt Poisson hierarchy (see lab_rows.hip)."""
import ctypes as C
import os
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
import amg_amd as A  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 256
lab = C.CDLL(str(ROOT / "tools" / "liblab_rows.so"))
lab.lab_time.restype = C.c_double
t = time.time()
fd = os.dup(1)
nul = os.open(os.devnull, os.O_WRONLY)
os.dup2(nul, 1)
H = A.Hierarchy(A.generate(7, N))
os.dup2(fd, 1)
print(f"setup {time.time() - t:.1f}s levels={H.num_levels}", flush=True)
names = ["tile", "wave256", "wave512", "wave1024", "wavedb256", "wavedb512", "mrow4", "mrow8", "mrow16", "mrow32", "lane16", "lane16pf", "lane8pf", "lane32pf", "tilepipe", "wdb256p", "wdb512p", "wdb1024p", "tilesort", "wavesort", "ts2k", "ts4k", "ts8k512", "ts8k1024", "ts16k", "chain2k", "v8u", "v8s", "v16s", "v32s", "v64s", "v64u", "v4s", "v64s8", "lx8k512", "lx8k1024", "lx16k", "lx16kR2Q4", "lx16kR8Q1", "lx16k512", "mg4", "mg8", "mg16", "mg8u2", "mlds16", "mlds32", "mlds8"]
sel = [int(a) for a in os.environ.get("LAB_VARIANTS", "0,20,4,26,27,28,29,30,31,32,33").split(",")]
for l in range(int(os.environ.get('LAB_FROM', '0')), H.num_levels):
    M = H.level(l).A
    rp, ci, v = A.csr_arrays(M)
    n, nnz = M.num_rows, M.num_nnzs
    assert lab.lab_load(n, rp.ctypes.data_as(C.c_void_p), ci.ctypes.data_as(C.c_void_p), v.ctypes.data_as(C.c_void_p)) == 0
    by = 12.0 * nnz + 4.0 * (n + 1) + 24.0 * n
    ref = None
    line = [f"L{l} n={n} nnz/row={nnz / n:.1f}"]
    for vi in sel:
        nm = names[vi]
        y = np.zeros(n)
        ms = lab.lab_time(vi, 10, y.ctypes.data_as(C.c_void_p))
        ok = ""
        if ref is None:
            ref = y.copy()
        elif not np.array_equal(ref.view(np.uint64), y.view(np.uint64)):
            d = float(np.max(np.abs(ref - y) / np.maximum(np.abs(ref), 1e-300)))
            ok = "!MISMATCH" if d > 1e-11 else f"(rel {d:.0e})"
        line.append(f"{nm}={ms * 1e3:.0f}us/{by / ms / 1e6:.0f}GB/s{ok}")
    print("  ".join(line), flush=True)
    lab.lab_free()
