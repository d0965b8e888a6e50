"""Run only the level-0 residual SpMV of the bench workload (for rocprofv3 --pmc passes).

    rocprofv3 --pmc FETCH_SIZE --output-format csv -d OUT -o run -- python3 tools/pmc_level0.py 400
"""
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
import numpy as np  # noqa: E402

import amg_amd as A  # noqa: E402

import threading  # noqa: E402
import time  # noqa: E402


def _heartbeat():   # gpurun kills a command that prints nothing for 3 minutes (setup + upload)
    t0 = time.time()
    while True:
        time.sleep(60)
        print(f"[pmc_level0] working ({time.time() - t0:.0f} s)", file=sys.stderr, flush=True)


threading.Thread(target=_heartbeat, daemon=True).start()
n = int(sys.argv[1]) if len(sys.argv) > 1 else 400
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
fd = os.dup(1)
nul = os.open(os.devnull, os.O_WRONLY)
os.dup2(nul, 1)
H = A.Hierarchy(A.generate(7, n))
os.dup2(fd, 1)
D = A.DeviceHierarchy(H, smoother="hybrid", coarse="direct")
N = H.level(0).A.num_rows
D.upload(0, "b", np.ones(N))
D.upload(0, "x", np.ones(N))
ms_csr = D.time_level0_spmv_csr(reps)   # spmv_adaptive<2, false, 0>: A_0's CSR arrays
ms = D.time_level0_spmv(reps)           # the cycle's storage of A_0
info = D.level_info(0)
print(f"level0 n={N} nnz={H.level(0).A.num_nnzs} avg_ms={ms:.4f}", flush=True)
import json  # noqa: E402
print(json.dumps({"n": n, "rows": N, "nnz": H.level(0).A.num_nnzs, "avg_ms": ms, "avg_ms_csr": ms_csr,
                  "a_format": A._native.a_format_name(info.a_format),
                  "algorithmic_bytes_per_launch": int(info.a_stream_bytes) + 24 * N}), flush=True)
