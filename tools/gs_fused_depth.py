"""Lab tool (CPU): critical path of the exact GS-CF smoother per level, one launch per class pass
(today's flow engine) against one dataflow over all passes of a smoother call.

    python tools/gs_fused_depth.py --n 160 [--levels 4,5,6] [--sweeps 2]

Model (DESIGN.md §8 "Parity mode"): a row finishes at
    max( max_k avail(j_k) + c * (len - k),  c * len ) + h
over its stored entries k whose value is produced by an update this smoother call makes (a same-class
lower neighbour in the same pass, or -- fused only -- any neighbour's update in an earlier pass), with
c the chain cost per entry and h the granule hand-off.  Separate passes: a pass starts when the
previous one has finished.  Fused: rows of later passes start as soon as the versions they read exist
(valid when the coupling is structurally symmetric: a row cannot be overwritten before every reader of
its previous value has read it, because each such reader is one of its dependencies).
"""
from __future__ import annotations

import argparse
import ctypes as C
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def passes(sweeps, post):
    seq = []
    for _ in range(sweeps):
        seq += [1, 0] if post else [0, 1]   # class of each pass: 0 = F, 1 = C
    return seq


def critical_fast(rp, ci, cls, seq, c_ns, h_ns, fused):
    """Finish time of the smoother call under the model above (ns); longest path by relaxation."""
    n = len(rp) - 1
    last_t = np.zeros(n)
    t_pass_end = 0.0
    lens = np.diff(rp)
    row_of = np.repeat(np.arange(n), lens)
    pos_from_end = (rp[1:][row_of] - np.arange(len(ci))).astype(np.float64)   # L - k
    for k in seq:
        start = 0.0 if fused else t_pass_end
        cur = np.zeros(n)
        # same-class lower neighbours need row order: process rows in increasing index, but in
        # waves of rows whose lower same-class neighbours are already done (DAG levels)
        same_lower = (cls[row_of] == k) & (cls[ci] == k) & (ci < row_of)
        # contribution from other rows' earlier versions (fused) is known up front
        base = start + c_ns * lens.astype(np.float64)
        if fused:
            other = (ci != row_of) & ~same_lower
            v = np.where(other, last_t[ci] + c_ns * pos_from_end, 0.0)
            base = np.maximum(base, np.maximum.reduceat(np.concatenate([v, [0.0]]), rp[:-1]) if len(ci) else base)
            base = np.where(lens > 0, base, start)
        rows = np.nonzero(cls == k)[0]
        sl_r, sl_c = row_of[same_lower], ci[same_lower]
        sl_w = pos_from_end[same_lower]
        order = np.argsort(sl_r, kind="stable")
        sl_r, sl_c, sl_w = sl_r[order], sl_c[order], sl_w[order]
        # iterate: relax until fixed point (longest path by repeated max; depth bounded)
        cur = np.where(cls == k, base + h_ns, 0.0)
        for _ in range(100000):
            cand = cur[sl_c] + c_ns * sl_w
            upd = np.zeros(n)
            np.maximum.at(upd, sl_r, cand)
            new = np.where(cls == k, np.maximum(base, upd) + h_ns, 0.0)
            if np.array_equal(new, cur):
                break
            cur = new
        t_end = cur[rows].max() if len(rows) else start
        t_pass_end = max(t_pass_end, t_end)
        last_t = np.where(cls == k, cur, last_t)
    return t_pass_end


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--n", type=int, default=128)
    p.add_argument("--stencil", type=int, default=7)
    p.add_argument("--levels", default="")
    p.add_argument("--sweeps", type=int, default=2)
    p.add_argument("--c-ns", type=float, default=4.2)   # 10 cycles per entry at 2.4 GHz
    p.add_argument("--h-ns", type=float, default=2000.0)
    a = p.parse_args()
    import amg_amd as A
    from amg_amd._native import csr_arrays
    t0 = time.perf_counter()
    M = A.generate(a.stencil, a.n)
    H = A.Hierarchy(M)
    A.lib().SSS_mat_destroy(C.byref(M))
    print(f"setup {time.perf_counter() - t0:.1f} s, {H.num_levels} levels", flush=True)
    levels = [int(x) for x in a.levels.split(",")] if a.levels else list(range(1, H.num_levels - 1))
    for l in levels:
        comp = H.level(l)
        rp, ci, _ = csr_arrays(comp.A)
        rp = rp.astype(np.int64)
        ci = ci.astype(np.int64)
        n = len(rp) - 1
        mk = np.ctypeslib.as_array(comp.cfmark.d, shape=(comp.cfmark.n,)).copy()
        cls = (mk[:n] == 1).astype(np.int64)
        t1 = time.perf_counter()
        res = {}
        for post in (False, True):
            seq = passes(a.sweeps, post)
            sep = critical_fast(rp, ci, cls, seq, a.c_ns, a.h_ns, False)
            fus = critical_fast(rp, ci, cls, seq, a.c_ns, a.h_ns, True)
            res["post" if post else "pre"] = (sep, fus)
        print(f"L{l} rows {n:8d} nnz/row {len(ci) / max(n, 1):7.1f}  pre sep {res['pre'][0] / 1e6:8.3f} ms "
              f"fused {res['pre'][1] / 1e6:8.3f} ms ({res['pre'][1] / max(res['pre'][0], 1e-9):.2f})  "
              f"post sep {res['post'][0] / 1e6:8.3f} fused {res['post'][1] / 1e6:8.3f} "
              f"({res['post'][1] / max(res['post'][0], 1e-9):.2f})  [{time.perf_counter() - t1:.1f} s]", flush=True)


if __name__ == "__main__":
    main()
