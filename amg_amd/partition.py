"""Partition set of a stencil hierarchy for a row-partitioned multi-GPU solve (host only).

    python -m amg_amd.partition --stencil 7 --n 512 --ranks 8 --prefix /tmp/sss_parts/part

Builds the global hierarchy once (the reference-semantics host setup), writes one partition file
per rank (prefix.r<rank>: its rows, ghosts and halo lists of every partitioned level) and the
replicated coarse tail (prefix.tail), then a manifest (prefix.json: global level sizes, timings,
this process's peak host memory).  Run as its own process so that no solve rank ever holds the
global hierarchy (sss_hip_dist_create_from_files); it never touches the GPU.
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import os
import resource
import sys
import threading
import time
from pathlib import Path

# The partition file layout's version (sss_part.hip kPartVersion; readers reject any other).  A set on
# disk records it in its manifest and bench.py puts it in the set's directory name, so a set written
# by an older layout is regenerated instead of failing the run with ERROR_WRONG_FILE.
PART_FORMAT = 2


def level_table(H) -> list:
    out = []
    for l in range(H.num_levels):
        L = H.level(l)
        last = l + 1 == H.num_levels
        out.append({"rows": L.A.num_rows, "nnz": L.A.num_nnzs, "nnz_p": 0 if last else L.P.num_nnzs,
                    "rows_next": 0 if last else H.level(l + 1).A.num_rows})
    return out


def rank_summary(prefix: Path, ranks: int) -> list:
    """Per rank: its partition file's size and, per partitioned level, own rows, ghosts and the
    peers it receives from / sends to (read back from the files, one at a time)."""
    from . import _native as N
    out = []
    for r in range(ranks):
        f = Path(f"{prefix}.r{r}")
        P = N.PartPlan.load(f)
        lv = []
        for l in range(P.nagg):
            _, _, m, g = P.level(l)
            h = P.halo(l)
            lv.append({"m": m, "g": g, "recv_peers": h["rsrc"].tolist(), "send_peers": h["sdst"].tolist()})
        out.append({"rank": r, "file_bytes": f.stat().st_size, "nagg": P.nagg, "levels": lv})
        P.close()
    return out


def _heartbeat(stop: threading.Event, t0: float, what: list):
    while not stop.wait(30.0):
        print(f"[partition] {what[0]} ({time.perf_counter() - t0:.0f} s)", file=sys.stderr, flush=True)


def build(stencil: int, n: int, ranks: int, prefix: Path, agg_rows: int = 0, summary: bool = True) -> dict:
    from . import _native as N
    t0 = time.perf_counter()
    phase = ["generating the operator"]
    stop = threading.Event()
    threading.Thread(target=_heartbeat, args=(stop, t0, phase), daemon=True).start()
    M = N.generate(stencil, n)
    sys.stdout.flush()
    saved = os.dup(1)
    os.dup2(2, 1)   # the setup's level table goes to stderr
    try:
        phase[0] = "setup"
        H = N.Hierarchy(M)
    finally:
        C.CDLL(None).fflush(None)
        os.dup2(saved, 1)
        os.close(saved)
    N.lib().SSS_mat_destroy(C.byref(M))
    t1 = time.perf_counter()
    prefix.parent.mkdir(parents=True, exist_ok=True)
    phase[0] = "writing the partition set"
    N.part_save(H, ranks, prefix, agg_rows)
    t2 = time.perf_counter()
    man = {"format": PART_FORMAT, "stencil": stencil, "n": n, "ranks": ranks, "agg_rows": agg_rows,
           "levels": level_table(H),
           "pars": {"pre_iter": H.pars.pre_iter, "post_iter": H.pars.post_iter, "tol": H.pars.tol},
           "setup_s": t1 - t0, "partition_s": t2 - t1,
           "peak_rss_gb": resource.getrusage(resource.RUSAGE_SELF).ru_maxrss / 2**20}
    H.close()
    man["rank_file_bytes"] = [Path(f"{prefix}.r{r}").stat().st_size for r in range(ranks)]
    man["tail_file_bytes"] = Path(f"{prefix}.tail").stat().st_size
    if summary:
        phase[0] = "reading the partition files back"
        t3 = time.perf_counter()
        man["ranks_detail"] = rank_summary(prefix, ranks)
        man["readback_s"] = time.perf_counter() - t3
    stop.set()
    Path(str(prefix) + ".json").write_text(json.dumps(man))
    return man


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--stencil", type=int, default=7)
    p.add_argument("--n", type=int, required=True)
    p.add_argument("--ranks", type=int, required=True)
    p.add_argument("--prefix", required=True)
    p.add_argument("--agg-rows", type=int, default=0)
    p.add_argument("--no-readback", action="store_true",
                   help="skip reading every rank file back for the per-rank halo summary (bench.py)")
    a = p.parse_args()
    man = build(a.stencil, a.n, a.ranks, Path(a.prefix), a.agg_rows, summary=not a.no_readback)
    print(json.dumps({k: v for k, v in man.items() if k not in ("levels", "ranks_detail")}), flush=True)


if __name__ == "__main__":
    main()
