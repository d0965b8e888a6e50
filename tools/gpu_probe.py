"""Quick GPU probe: per-level shapes, level-0 SpMV time, iteration time for a Poisson size.

usage: python tools/gpu_probe.py N [smoother] [coarse]
"""
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
import numpy as np  # noqa: E402

import amg_amd as A  # noqa: E402

n = int(sys.argv[1])
smoother = sys.argv[2] if len(sys.argv) > 2 else "exact"
coarse = sys.argv[3] if len(sys.argv) > 3 else "direct"
t0 = time.time()
M = A.generate(7, n)
H = A.Hierarchy(M)
print(f"setup {time.time() - t0:.1f}s", flush=True)
t0 = time.time()
D = A.DeviceHierarchy(H, smoother=smoother, coarse=coarse)
print(f"upload {time.time() - t0:.1f}s", flush=True)
for l in range(H.num_levels):
    i = D.level_info(l)
    print(f"level {l}: rows={i.rows} nnz={i.nnz} nnzP={i.nnz_p} dagF={i.dag_f} dagC={i.dag_c} kind={i.smoother_kind}")
N = M.num_rows
D.upload(0, "b", np.ones(N))
D.upload(0, "x", np.ones(N))
nnz = M.num_nnzs
ms = D.time_level0_spmv(20)
B = 12 * nnz + 4 * (N + 1) + 8 * N + 8 * N + 8 * N
print(f"level0 resid spmv {ms:.4f} ms  {B / ms / 1e6:.1f} GB/s ({B / ms / 1e6 / 8000 * 100:.1f}% of 8 TB/s)", flush=True)
sumb = np.sqrt(N)
for it in range(3):
    ms, ares = D.time_iterations(1)
    print(f"iter {it}: {ms:.2f} ms relres {ares / sumb:.6e}", flush=True)
ms, ares = D.time_iterations(5)
print(f"avg iteration {ms:.2f} ms -> {1000 / ms:.1f} it/s", flush=True)
