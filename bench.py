"""bench.py — V-cycle iterations/s + fine-level SpMV HBM GB/s on the 7-pt Poisson problem.

BASELINE.json metric: "V-cycle iters/sec + fine-level SpMV GB/s (%HBM peak), 64M-row 7pt Poisson".
A step = one outer iteration of SSS_amg_solve (Solve/SSS_SOLVE.c:53-80): one V-cycle, r = b - A0 x,
||r|| read back to the host.  Workload at N=1: 7-pt Poisson 400^3 (64,000,000 rows), FP64, b = x0 = 1
(SSS_main.c:141-145), synthetic operator generated in memory (a 400^3 .mtx would be ~60 GB of text).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--n 400] [--mode throughput|parity]
                    [--no-cpu-baseline]

Modes:
  throughput : exact GS-CF on level 0 (red-black -> fully parallel), two-stage GS-CF on coarser
               levels (a Jacobi step + `--inner` Jacobi-Richardson steps on each pass's lower
               triangle), explicit-inverse coarse solve.  Converges to the same tolerance.
  parity     : exact GS-CF on every level + the reference CG(beta=1)+GMRES coarse solve; x is bitwise
               identical to the reference after every V-cycle (tests/test_gpu_parity.py).

N > 1 (launched by torch.distributed.run): one global 400^3 problem, row-partitioned over the
ranks (sss_hip_dist_*: halos and the norm over RCCL/xGMI, levels below SSS_HIP_AGG_ROWS rows
replicated); strong scaling, `value` = global V-cycles / max-over-ranks time.
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import os
import sys
import threading
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

PEAK_HBM_GBS = 8000.0       # MI355X HBM3E spec (MI355X_MICROARCH.md:36)
COPY_PEAK_GBS = 6290.0      # measured float4 copy peak (same source)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=None,
                   help="ranks (one per GPU); without WORLD_SIZE in the environment and N > 1 the bench "
                        "launches N ranks itself (torch.distributed.run) before touching the GPU")
    p.add_argument("--steps", type=int, default=10)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--grid", "--n", dest="n", type=int, default=None,
                   help="grid edge (default 400: the metric's 64M-row problem at every rank count, so that "
                        "--gpus 1/2/4/8 form one strong-scaling curve; BASELINE.json's other configs: "
                        "--n 512 --gpus 8, --stencil 27 --n 256 --gpus 4)")
    p.add_argument("--probe-ranks", action="store_true",
                   help="print one line per rank (rank, world size) and exit before any GPU call (tests)")
    p.add_argument("--hier-cache", default=None,
                   help="binary hierarchy file (SSS_amg_save): loaded when present, else written after setup "
                        "(rank 0; the other ranks load it)")
    p.add_argument("--stencil", type=int, default=None, choices=[7, 27],
                   help="7: 7-pt Poisson (the metric's workload, the default); 27: the 27-pt anisotropic "
                        "operator of BASELINE.json configs[4] (SURVEY.md 8(d))")
    p.add_argument("--workload", default="stencil", choices=["stencil", "circuit"],
                   help="stencil: the --stencil operator on an --n grid; circuit: the G3_circuit stand-in "
                        "(BASELINE.json configs[3], amg_amd/workloads.py; --n = rows, default 1,585,478; 1 GPU)")
    p.add_argument("--mtx", default=None,
                   help="a Matrix Market file read by the reference's ingest (SSS_mat_read: SSS_main.c:12-22, "
                        "mmio_highlevel.h:10-305) instead of a generated operator, b = x0 = 1 as ./amg sets them "
                        "(SSS_main.c:141-145): BASELINE.json configs[0] (nos5) and configs[3] (G3_circuit) when the "
                        "SuiteSparse file is supplied; 1 GPU")
    p.add_argument("--parity-converge", type=int, default=None,
                   help="run the parity-mode mirror to tol (the reference-semantics iteration count measured in "
                        "this run, beside the throughput count); default 1 at N = 1")
    p.add_argument("--mode", default="throughput", choices=["throughput", "parity"])
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--sequential-upload", action="store_true",
                   help="build the HBM mirror after the setup instead of while it runs")
    p.add_argument("--cpu-threads", type=int, default=0,
                   help="threads of the multi-core CPU baseline in the GPU's mode (default: every CPU this "
                        "process may run on -- affinity mask, capped by the cgroup CPU quota)")
    p.add_argument("--cpu-iters", type=int, default=5, help="timed CPU-baseline iterations (median reported)")
    p.add_argument("--cpu-warmup", type=int, default=1, help="untimed CPU-baseline iterations first")
    p.add_argument("--cpu-n", type=int, default=0, help="grid edge of the CPU sample (default: same workload)")
    p.add_argument("--mode-smoother", default=None, help="override: exact|hybrid|jacobi")
    p.add_argument("--mode-coarse", default=None, help="override: krylov|direct")
    p.add_argument("--inner", type=int, default=None,
                   help="two-stage inner steps on C/F-Jacobi levels (default: SSS_HIP_INNER or 1; 0 = plain C/F-Jacobi)")
    p.add_argument("--inner-long", type=int, default=None,
                   help="extra inner steps on the two-stage levels of long rows (>= 300 entries per row; default: "
                        "SSS_HIP_INNER_LONG or 1)")
    p.add_argument("--inner-from", type=int, default=None,
                   help="first level with the two-stage form (default: SSS_HIP_INNER_FROM or 2)")
    p.add_argument("--converge-max", type=int, default=100, help="max V-cycles of the iterations-to-tol run (0: skip)")
    p.add_argument("--parity-cycles", type=int, default=2,
                   help="N=1: V-cycles timed on a second mirror in parity mode (the drop-in default: exact GS-CF "
                        "on every level, reference CG(beta=1)+GMRES coarse solve; 0 skips it)")
    p.add_argument("--sum-order", type=int, default=None,
                   help="0: stored CSR order everywhere (bitwise kernels); 1: tree-summed long rows "
                        "(default: 1 in throughput mode, 0 in parity mode)")
    p.add_argument("--sorted-tiles", type=int, default=None, help="column-sorted tile staging (default 1)")
    p.add_argument("--keep-parts", action="store_true",
                   help="N > 1: keep a partition set this run wrote (default: removed at the end unless "
                        "SSS_PART_DIR is set; a set found already present is always kept)")
    p.add_argument("--single-ref", default=None,
                   help="N > 1: a 1-GPU bench record (JSON) of the same workload for parallel_efficiency "
                        "(default: the record the last N = 1 run on this host left in the temp directory, "
                        "else the newest committed profiles/r*_bench400_throughput.json of that workload)")
    argv = None
    if "WORLD_SIZE" in os.environ and "SSS_BENCH_ARGV" in os.environ:   # ranks spawned by spawn_ranks()
        argv = json.loads(os.environ["SSS_BENCH_ARGV"])
    return p.parse_args(argv)


class Dist:
    """torch.distributed (gloo, host-side barrier / max only) when launched with WORLD_SIZE > 1."""

    def __init__(self):
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        self.local_rank = int(os.environ.get("LOCAL_RANK", "0"))
        self.pg = None
        if self.world > 1:
            import torch.distributed as dist
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            dist.init_process_group("gloo")
            self.dist = dist

    def barrier(self):
        if self.world > 1:
            self.dist.barrier()

    def max(self, v: float) -> float:
        if self.world == 1:
            return v
        import torch
        t = torch.tensor([v], dtype=torch.float64)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
        return float(t.item())

    def min(self, v: float) -> float:
        if self.world == 1:
            return v
        import torch
        t = torch.tensor([v], dtype=torch.float64)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MIN)
        return float(t.item())

    def gather(self, v: float) -> list:
        """Every rank's value, in rank order (on every rank)."""
        if self.world == 1:
            return [v]
        out = [None] * self.world
        self.dist.all_gather_object(out, v)
        return out

    def close(self):
        if self.world > 1:
            self.dist.destroy_process_group()


def quiet_call(fn, *a, **kw):
    """Run fn with the C library's stdout (setup tables) sent to stderr."""
    sys.stdout.flush()
    saved = os.dup(1)
    os.dup2(2, 1)
    try:
        return fn(*a, **kw)
    finally:
        C.CDLL(None).fflush(None)
        os.dup2(saved, 1)
        os.close(saved)


def cpu_iterations(H, out: dict, threads: int = 1, iters: int = 1, warmup: int = 0, **mode):
    """Outer iterations (V-cycle, r = b - A0 x, ||r||) of the CPU restatement oracle/sss_oracle.c.
    threads = 1 with no mode keys: exactly the reference's serial host path (GS-CF everywhere,
    CG(beta=1)+GMRES coarse solve).  threads > 1: its row loops on that many host threads (results
    unchanged).  mode: oracle options, e.g. the GPU throughput mode (smoother=1, inner=1,
    inner_mask, coarse_mode=1)."""
    import oracle
    ora = oracle.load()
    ora.ora_set_threads(threads)
    n = H.level(0).A.num_rows
    b = np.ones(n)
    x = np.ones(n)
    from amg_amd._native import SSS_VEC, dptr
    H.mg.cg[0].x = SSS_VEC(n, dptr(x))
    H.mg.cg[0].b = SSS_VEC(n, dptr(b))
    opts = oracle.opts(**mode)
    r = np.empty(n)

    def one():
        ora.ora_cycle(C.byref(H.mg), C.byref(opts))
        r[:] = b
        ora.ora_mv_amxpy(-1.0, C.byref(H.level(0).A), dptr(x), dptr(r), 0)
        return float(np.sqrt(np.dot(r, r)))

    for _ in range(warmup):
        one()
    per, coarse = [], []
    for _ in range(iters):
        ora.ora_reset_timers()
        t0 = time.perf_counter()
        one()
        per.append(time.perf_counter() - t0)
        coarse.append(ora.ora_coarse_seconds())
    # the fine-level SpMV of the CPU path, for the GB/s column (one r = b - A0 x), median of 3
    sp = []
    for _ in range(3):
        t1 = time.perf_counter()
        ora.ora_mv_amxpy(-1.0, C.byref(H.level(0).A), dptr(x), dptr(r), 0)
        sp.append(time.perf_counter() - t1)
    out.update(seconds=float(np.median(per)), seconds_all=per, coarse_seconds=float(np.median(coarse)),
               threads=ora.ora_get_threads(), spmv_seconds=float(np.median(sp)), iters=iters, warmup=warmup)


def host_cpus() -> dict:
    """What the CPU baseline ran on: logical CPUs of the machine, the ones this process may use
    (affinity mask, capped by the cgroup v2 CPU quota), the CPU model and the NUMA node count."""
    info = {"nproc_machine": os.cpu_count()}
    try:
        usable = len(os.sched_getaffinity(0))
    except AttributeError:
        usable = os.cpu_count() or 1
    try:
        q, per = Path("/sys/fs/cgroup/cpu.max").read_text().split()[:2]
        if q != "max":
            info["cgroup_cpu_quota"] = int(q) / int(per)
            usable = max(1, min(usable, int(int(q) // int(per))))
    except (OSError, ValueError):
        pass
    info["usable_cpus"] = usable
    try:
        for line in Path("/proc/cpuinfo").read_text().splitlines():
            if line.startswith("model name"):
                info["model"] = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    try:
        info["numa_nodes"] = len([d for d in os.listdir("/sys/devices/system/node") if d.startswith("node")])
    except OSError:
        pass
    return info


def spawn_ranks(n: int) -> int:
    """Launch this script as n ranks under torch.distributed.run (child process; this process
    never initialises the GPU) and return its exit code."""
    import socket
    import subprocess
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    # the ranks get this command line through the environment: torch.distributed.run would try to
    # parse options such as --n itself
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={port}", str(Path(__file__).resolve())]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY=os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY", "0"),
               SSS_BENCH_ARGV=json.dumps(sys.argv[1:]))
    return subprocess.call(cmd, env=env)


class Single:
    """N = 1: the single-GPU engine (sss_hip_hier_*)."""

    def __init__(self, DH, N):
        self.DH, self.N = DH, N
        self.rows, self.ghosts = N, 0

    def set_ones(self):
        self.DH.upload(0, "b", np.ones(self.N))
        self.DH.upload(0, "x", np.ones(self.N))

    def set_x_ones(self):
        self.DH.upload(0, "x", np.ones(self.N))

    def cycle(self):
        self.DH.cycle()

    def residual_norm(self):
        return self.DH.residual_norm()

    def sync(self):
        self.DH.sync()

    def time_level0_spmv(self, reps):
        return self.DH.time_level0_spmv(reps)

    def close(self):
        self.DH.close()


class Distributed(Single):
    """N > 1: this rank's rows of the row-partitioned engine (sss_hip_dist_*)."""

    def __init__(self, DD):
        self.DH = DD
        self.rows, self.ghosts, self.nnz = DD.level_size(0)

    def set_ones(self):
        self.DH.upload("b", np.ones(self.rows))
        self.DH.upload("x", np.ones(self.rows))

    def set_x_ones(self):
        self.DH.upload("x", np.ones(self.rows))


def vcycle_bytes(levels: list, sweeps: int) -> int:
    """Algorithmic HBM bytes of one outer iteration, SURVEY.md 8(d): per level l < coarsest, with
    z = nnz(A_l), p = nnz(P_l) = nnz(R_l), n = n_l, m = n_{l+1}:
      GS-CF sweep   12z + 4(n+1) + 8n + 8n + 16n + 8n      (x (pre_iter + post_iter) sweeps)
      residual      12z + 4(n+1) + 24n
      restriction   12p + 4(m+1) + 8n + 8m
      prolongation  12p + 4(n+1) + 8m + 16n
      zero-fill     8m
    plus the outer residual and norm 12z0 + 4(n0+1) + 24n0 + 8n0; the coarse solve is excluded.
    levels: per level {"rows", "nnz", "nnz_p", "rows_next"} (amg_amd.partition.level_table)."""
    tot = 0
    for L in levels[:-1]:
        z, n, m, p = L["nnz"], L["rows"], L["rows_next"], L["nnz_p"]
        tot += sweeps * (12 * z + 4 * (n + 1) + 40 * n)
        tot += 12 * z + 4 * (n + 1) + 24 * n
        tot += 12 * p + 4 * (m + 1) + 8 * n + 8 * m
        tot += 12 * p + 4 * (n + 1) + 8 * m + 16 * n
        tot += 8 * m
    L0 = levels[0]
    tot += 12 * L0["nnz"] + 4 * (L0["rows"] + 1) + 32 * L0["rows"]
    return int(tot)


def select_workload(args, world: int):
    """(stencil, n) of this run: the metric's 7-pt 400^3 problem at every rank count unless
    --stencil / --n say otherwise, so that the driver's --gpus 1, 2, 4, 8 runs measure one problem
    (a strong-scaling curve).  --workload circuit: the G3_circuit stand-in's row count."""
    stencil = args.stencil if args.stencil is not None else 7
    if args.n is not None:
        return stencil, args.n
    if args.workload == "circuit":
        from amg_amd.workloads import G3_CIRCUIT_ROWS
        return stencil, G3_CIRCUIT_ROWS
    return stencil, 256 if stencil == 27 else 400


def workload_name(args, circuit: bool, mtx) -> str:
    """config.workload of this run: the stencil and grid, the circuit stand-in's rows, or the .mtx
    file's name (mtx_<stem>)."""
    if mtx is not None:
        return f"mtx_{Path(mtx).stem}"
    return f"g3_circuit_standin_{args.n}" if circuit else f"poisson{args.stencil}_{args.n}^3"


def load_mtx(A, path):
    """The .mtx file as the reference's ./amg reads it (SSS_mat_read -> mmio_info + mmio_data: symmetric
    expansion, file order within rows, SSS_main.c:12-22); refuses an empty or unreadable matrix."""
    M = A.read_mtx(path)
    if M.num_rows <= 0 or M.num_rows != M.num_cols or not M.row_ptr:
        raise SystemExit(f"bench.py: --mtx {path}: not a square sparse matrix ({M.num_rows} x {M.num_cols})")
    return M


def transport_policy(world: int, devices: int, rccl_ok_everywhere: bool) -> str:
    """The halo transport of a multi-rank run: "rccl" when every rank created its communicator;
    "host" (gloo) only when the ranks share GPUs (fewer visible devices than ranks: RCCL refuses
    two ranks on one device, e.g. the one-GPU test box); "fail" when each rank owns a GPU and RCCL
    still failed somewhere -- that is a broken node, not a configuration to measure around."""
    if rccl_ok_everywhere:
        return "rccl"
    return "host" if devices < world else "fail"


def part_set_name(stencil: int, n: int, world: int) -> str:
    """Directory name of a partition set: the file layout's version (amg_amd.partition.PART_FORMAT)
    and the replicated-tail threshold are part of it, so a set written by an older layout or for
    another threshold is never picked up (it would fail the run with ERROR_WRONG_FILE, or silently
    measure another tail)."""
    from amg_amd.partition import PART_FORMAT
    agg = int(os.environ.get("SSS_HIP_AGG_ROWS", "0") or 0)
    return f"sss_parts_v{PART_FORMAT}_{stencil}pt_{n}_{world}r" + (f"_agg{agg}" if agg > 0 else "")


def part_set_usable(manifest: Path) -> bool:
    """A set on disk is reused only if its manifest records this layout version."""
    from amg_amd.partition import PART_FORMAT
    try:
        return json.loads(manifest.read_text()).get("format") == PART_FORMAT
    except (OSError, ValueError):
        return False


def part_prefix(stencil: int, n: int, world: int) -> Path:
    """Where the partition set of a multi-rank run lives (reused by later runs of the same
    configuration): SSS_PART_DIR if set; else an existing set of this configuration in any of /tmp,
    /dev/shm, the home directory and the repository's parent; else the first of them with room for
    it -- the set takes ~490 B per row for the 7-point operator and ~870 B per row for the 27-point
    one (profiles/r03_partition_*.json: 65 GB at 512^3; r04_partition_p7_400_*.json at 400^3)."""
    import shutil
    name = part_set_name(stencil, n, world)
    if os.environ.get("SSS_PART_DIR"):
        return Path(os.environ["SSS_PART_DIR"]) / name / "part"
    need = 1.25 * (870 if stencil == 27 else 490) * float(n) ** 3
    cands = [Path("/tmp"), Path("/dev/shm"), Path.home(), ROOT.parent]
    for c in cands:   # an existing set of this configuration anywhere wins over free space
        if part_set_usable(c / name / "part.json"):
            return c / name / "part"
    best, room = None, -1.0
    for c in cands:
        try:
            free = float(shutil.disk_usage(c).free)
        except OSError:
            continue
        if free >= need:
            return c / name / "part"
        if free > room:
            best, room = c, free
    print(f"[bench] no scratch directory has {need / 1e9:.0f} GB free; using {best} ({room / 1e9:.0f} GB free)",
          file=sys.stderr, flush=True)
    return (best or Path("/tmp")) / name / "part"


def single_ref_path(workload: str, mode: str) -> Path:
    import tempfile
    return Path(tempfile.gettempdir()) / f"sss_bench_single_{workload.replace('^', '')}_{mode}.json"


REF_KEYS = ("workload", "mode", "smoother", "sum_order")   # what a 1-GPU reference record must share


def single_gpu_reference(explicit, cfg: dict):
    """The 1-GPU rate of the same configuration for parallel_efficiency = value / (N x rate):
    --single-ref, else the record the last N = 1 run on this host left (single_ref_path), else the
    newest committed profiles/r*_bench*_throughput.json -- only a record whose workload, mode,
    smoother and sum order all equal this run's (a parity-mode or differently smoothed 1-GPU rate is
    no denominator).  None if there is none."""
    cands = [Path(explicit)] if explicit else []
    cands.append(single_ref_path(cfg["workload"], cfg["mode"]))
    cands += sorted((ROOT / "profiles").glob("r*_bench*_throughput.json"), reverse=True)
    for c in cands:
        try:
            r = json.loads(c.read_text())
        except (OSError, ValueError):
            continue
        rc = r.get("config", {})
        if all(rc.get(k) == cfg.get(k) for k in REF_KEYS) and r.get("n_gpus", 1) == 1 and r.get("value"):
            return {"value": r["value"], "ms_per_step": r.get("ms_per_step"), "source": str(c)}
    return None


def heartbeat(stop: threading.Event, t0: float):
    """A progress line on stderr every 60 s through the long host phases (setup, upload)."""
    while not stop.wait(60.0):
        print(f"[bench] working ({time.perf_counter() - t0:.0f} s)", file=sys.stderr, flush=True)


def make_comm(A, D):
    """N > 1: this rank's communicator, created before any setup so that a broken node fails in
    seconds.  RCCL (xGMI) when every rank created it; the host transport only when the ranks share
    GPUs (transport_policy); otherwise every rank exits non-zero."""
    ndev = int(os.environ.get("SSS_BENCH_FAKE_DEVICES", "0")) or A.device_count()   # (tests: fake a node)
    dev = D.local_rank % max(ndev, 1)
    comm, ok, why = None, 1, ""
    try:
        comm = A.Comm(D.world, D.rank, "rccl", device=dev)
    except Exception as e:  # noqa: BLE001
        why = str(e)
        print(f"[bench] rank {D.rank}: RCCL communicator failed on device {dev} ({e})", file=sys.stderr, flush=True)
        ok = 0
    policy = transport_policy(D.world, ndev, D.min(ok) >= 1)   # every rank decides the same
    if policy == "fail":
        if comm is not None:
            comm.close()
        D.close()
        raise SystemExit(f"bench.py: rank {D.rank}: RCCL communicator creation failed with {ndev} GPUs for "
                         f"{D.world} ranks{' (' + why + ')' if why else ' (on another rank)'}; no host-transport "
                         f"fallback when every rank owns a device")
    if policy == "host":   # ranks share GPUs (e.g. several ranks on the one-GPU test box)
        if comm is not None:
            comm.close()
        print(f"[bench] rank {D.rank}: {D.world} ranks on {ndev} GPU(s): using the host transport (gloo)",
              file=sys.stderr, flush=True)
        return A.Comm(D.world, D.rank, "host"), dev, "host-gloo"
    return comm, dev, "rccl"


def main():
    args = parse()
    ws = os.environ.get("WORLD_SIZE")
    if ws is None and args.gpus is not None and args.gpus > 1:
        sys.exit(spawn_ranks(args.gpus))   # before anything touches the GPU
    # stdout carries the JSON record only: library banners (gloo's peer lines at the process group's
    # start, RCCL's version block) and the C setup tables go to stderr
    sys.stdout.flush()
    json_fd = os.dup(1)
    os.dup2(2, 1)
    D = Dist()
    if args.gpus is not None and args.gpus != D.world:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={D.world}")
    circuit = args.workload == "circuit"
    if circuit and D.world > 1:
        raise SystemExit("bench.py: --workload circuit is a single-GPU configuration (BASELINE.json configs[3])")
    mtx = Path(args.mtx) if args.mtx else None
    if mtx is not None and D.world > 1:
        raise SystemExit("bench.py: --mtx runs on one GPU (BASELINE.json configs[0] and configs[3])")
    if mtx is not None and not mtx.is_file():
        raise SystemExit(f"bench.py: --mtx {mtx}: no such file")
    irregular = circuit or mtx is not None   # no stencil: no grid edge, no stencil-only records
    # one problem at every rank count (the metric's 7-pt 400^3 unless --stencil / --n): the driver's
    # --gpus 1, 2, 4, 8 runs form one strong-scaling curve
    args.stencil, args.n = select_workload(args, D.world)
    workload = workload_name(args, circuit, mtx)
    if args.probe_ranks:
        # one write() per line: the ranks share the launcher's stdout pipe
        os.write(json_fd, (json.dumps({"rank": D.rank, "world": D.world, "local_rank": D.local_rank,
                                       "workload": workload}) + "\n").encode())
        D.close()
        return
    if args.parity_converge is None:
        args.parity_converge = 1 if D.world == 1 else 0
    hb_stop = threading.Event()
    threading.Thread(target=heartbeat, args=(hb_stop, time.perf_counter()), daemon=True).start()
    import amg_amd as A
    comm, dev, transport = make_comm(A, D) if D.world > 1 else (None, 0, None)

    n = args.n
    smoother, coarse = ("hybrid", "direct") if args.mode == "throughput" else ("exact", "krylov")
    smoother = args.mode_smoother or smoother
    if args.mode_smoother is None and D.world > 1 and args.stencil == 27 and smoother == "hybrid":
        # level 0 of the 27-point operator is not red-black: its exact GS-CF has intra-class chains
        # that cannot be split across ranks; the row-partitioned engine smooths it by C/F-Jacobi
        smoother = "jacobi"
    coarse = args.mode_coarse or coarse
    sum_order = args.sum_order if args.sum_order is not None else (1 if args.mode == "throughput" else 0)
    sorted_tiles = args.sorted_tiles if args.sorted_tiles is not None else int(os.environ.get("SSS_HIP_SORTED_TILES", "1"))

    t0 = time.perf_counter()
    hier_src = None
    made_parts = False
    part_rec = None
    H = None
    DH = None   # set here when the mirror is built while the setup runs (sss_hip_setup_create)
    dh_kw = dict(smoother=smoother, coarse=coarse, device=-1, inner=args.inner, inner_from=args.inner_from,
                 inner_long=args.inner_long,
                 sum_order=sum_order, sorted_tiles=sorted_tiles)
    if D.world == 1:
        cache = Path(args.hier_cache) if args.hier_cache else None
        if cache is not None and cache.exists():
            H = A.Hierarchy.load(cache)
            hier_src = f"loaded from {cache}"
        elif mtx is not None:
            M = load_mtx(A, mtx)
            if args.sequential_upload:
                H = quiet_call(A.Hierarchy, M)
            else:
                DH = quiet_call(A.DeviceHierarchy, None, setup_from=M, **dh_kw)
                H = DH.H
            A.lib().SSS_mat_destroy(C.byref(M))
            hier_src = f"setup of {mtx.name} (SSS_mat_read)"
        elif circuit:
            from amg_amd.workloads import circuit_csr
            M = circuit_csr(n)
            if args.sequential_upload:
                H = quiet_call(A.Hierarchy, M.mat)
            else:
                DH = quiet_call(A.DeviceHierarchy, None, setup_from=M.mat, **dh_kw)
                H = DH.H
            del M
            hier_src = "setup"
        else:
            M = A.generate(args.stencil, n)
            if args.sequential_upload:
                H = quiet_call(A.Hierarchy, M)
            else:
                DH = quiet_call(A.DeviceHierarchy, None, setup_from=M, **dh_kw)
                H = DH.H
            A.lib().SSS_mat_destroy(C.byref(M))
            hier_src = "setup"
            if cache is not None:
                H.save(cache)
                hier_src = "setup (saved)"
        from amg_amd.partition import level_table
        table = level_table(H)
        pars = {"pre_iter": H.pars.pre_iter, "post_iter": H.pars.post_iter, "tol": H.pars.tol}
    else:
        # rows partitioned over the ranks: a separate host process builds the global hierarchy and
        # writes one partition file per rank (amg_amd/partition.py); each rank then reads only its
        # rows, ghosts and the replicated coarse tail -- no rank ever holds the global hierarchy
        # rank 0 chooses the directory (free space changes once the set is being written)
        box = [str(part_prefix(args.stencil, n, D.world)) if D.rank == 0 else None]
        D.dist.broadcast_object_list(box, src=0)
        prefix = Path(box[0])
        manifest = Path(str(prefix) + ".json")
        if D.rank == 0 and not part_set_usable(manifest):
            import subprocess
            subprocess.run([sys.executable, "-m", "amg_amd.partition", "--stencil", str(args.stencil), "--n", str(n),
                            "--ranks", str(D.world), "--prefix", str(prefix), "--no-readback",
                            "--agg-rows", str(int(os.environ.get("SSS_HIP_AGG_ROWS", "0") or 0))], check=True,
                           cwd=str(ROOT), stdout=sys.stderr)
            hier_src = f"partition set written to {prefix.parent}"
            # a set this run wrote is removed at the end (tens of GB of scratch per rank count)
            made_parts = not args.keep_parts and not os.environ.get("SSS_PART_DIR")
        D.barrier()
        man = json.loads(manifest.read_text())
        table, pars = man["levels"], man["pars"]
        part_rec = {k: man.get(k) for k in ("setup_s", "partition_s", "peak_rss_gb", "rank_file_bytes",
                                            "tail_file_bytes", "agg_rows")}
        hier_src = hier_src or f"partition set read from {prefix.parent}"
        if D.rank == 0:
            print(f"[bench] partition set: setup {man['setup_s']:.1f} s, partition {man['partition_s']:.1f} s, "
                  f"peak host memory of the partitioning process {man['peak_rss_gb']:.1f} GB", file=sys.stderr, flush=True)
    setup_s = time.perf_counter() - t0 if DH is None else DH.times[0]
    N = table[0]["rows"]
    nnz = table[0]["nnz"]

    t0 = time.perf_counter()
    inner = args.inner if args.inner is not None else int(os.environ.get("SSS_HIP_INNER", "1"))
    inner_from = args.inner_from if args.inner_from is not None else int(os.environ.get("SSS_HIP_INNER_FROM", "2"))
    inner_long = args.inner_long if args.inner_long is not None else int(os.environ.get("SSS_HIP_INNER_LONG", "1"))
    if D.world == 1:
        if DH is None:
            DH = A.DeviceHierarchy(H, **dh_kw)
        eng = Single(DH, N)
    else:
        # row-partitioned solve over RCCL (xGMI): each rank reads only its own partition file
        DD = A.DistHierarchy(None, comm, smoother=smoother, coarse=coarse, device=dev, inner=args.inner,
                             inner_long=args.inner_long,
                             inner_from=args.inner_from, sum_order=sum_order, sorted_tiles=sorted_tiles, parts=prefix)
        eng = Distributed(DD)
        D.barrier()   # every rank has read its file: the set is no longer needed
        if made_parts:
            import shutil
            shutil.rmtree(prefix.parent, ignore_errors=True)
            print(f"[bench] removed the partition set {prefix.parent}", file=sys.stderr, flush=True)
    upload_s = time.perf_counter() - t0
    # HBM in use on each rank's device once its mirror is resident (ranks sharing one GPU all see
    # the device total)
    hbm_ranks = D.gather(A.hbm_used_bytes() / 1e9)
    hbm_gb = max(hbm_ranks)
    overlapped = D.world == 1 and getattr(DH, "times", None) is not None
    if overlapped:   # levels were uploaded during the setup: what is left after it returned
        upload_s = DH.times[1]
    print(f"[bench] setup {setup_s:.1f} s, upload {upload_s:.1f} s"
          f"{' (after the setup; the rest overlapped it)' if overlapped else ''}", file=sys.stderr, flush=True)
    eng.set_ones()
    DH = eng

    for _ in range(args.warmup):
        DH.cycle()
        DH.residual_norm()
    DH.sync()
    # N > 1: the distributed cycle replays one captured hipGraph over RCCL unless the capture failed
    # (then eager launches; SSS_HIP_DIST_GRAPH=0 forces them)
    cycle_graph = DH.DH.level_flags(0)["cycle_graph"] if D.world > 1 else None
    D.barrier()
    t0 = time.perf_counter()
    absres = 0.0
    for it in range(args.steps):
        DH.cycle()
        absres = DH.residual_norm()      # synchronises (8-byte D2H per iteration, as the reference)
        if args.steps <= 4:
            print(f"[bench] timed step {it + 1}", file=sys.stderr, flush=True)
    DH.sync()
    t1 = time.perf_counter()
    D.barrier()
    elapsed = D.max(t1 - t0)
    ms_per_step = elapsed * 1e3 / args.steps
    value = args.steps / elapsed   # global V-cycles per second (strong scaling at N > 1)
    # the stored-format bytes the timed step's kernels read and write (the next cycle as it would run
    # now -- the steady state of the loop above -- and the residual + norm; sss_hip_cycle_bytes)
    cyc_bytes = DH.DH.cycle_bytes() if D.world == 1 else None

    # roofline of the dominant streaming kernel: level-0 fused residual SpMV (wp = b - A0 x);
    # N > 1: rank 0's share (its rows, x with ghosts), no exchange inside the timed launches
    spmv_ms = DH.time_level0_spmv(20)   # the cycle's own storage of A_0
    a_format = None
    launches, tail_from = None, None
    level_formats = None
    transfer_formats = None
    level_smoothers = None
    csr_bytes = 12 * nnz + 4 * (N + 1) + 8 * N + 8 * N + 8 * N   # val+col, row_ptr, x, b, y
    if D.world == 1:
        info0 = DH.DH.level_info(0)
        a_format = A._native.a_format_name(info0.a_format)
        level_formats = [DH.DH.level_info(l).a_format for l in range(len(table) - 1)]
        transfer_formats = [[DH.DH.level_info(l).r_format, DH.DH.level_info(l).p_format] for l in range(len(table) - 1)]
        level_smoothers = [(DH.DH.level_info(l).smoother_kind, DH.DH.level_info(l).inner) for l in range(len(table) - 1)]
        # the stored format's own bytes (dictionary ELL: 8 B per row + block dictionaries) + vectors
        spmv_bytes = info0.a_stream_bytes + 8 * N + 8 * N + 8 * N
        # SURVEY.md 8(d)'s kernel: the same residual SpMV from A_0's CSR arrays
        csr_ms = DH.DH.time_level0_spmv_csr(20)
        launches = A.lib().sss_hip_cycle_launches(DH.DH.h)   # kernels per V-cycle (captured graph)
        tail_from = A.lib().sss_hip_tail_from(DH.DH.h)
    else:
        m, g = DH.rows, DH.ghosts
        spmv_bytes = 12 * DH.nnz + 4 * (m + 1) + 8 * (m + g) + 8 * m + 8 * m
        csr_bytes = spmv_bytes
        csr_ms = spmv_ms
    # roofline: SURVEY.md 8(d)'s algorithmic bytes of the CSR SpMV over the CSR kernel's time; the
    # cycle's own (compressed) storage of A_0 is reported beside it with its own bytes
    achieved = csr_bytes / (csr_ms * 1e-3) / 1e9
    format_gbps = spmv_bytes / (spmv_ms * 1e-3) / 1e9

    # iterations to tol from x0 = 1 (the CLI's problem), and time to solution
    DH.set_x_ones()
    sumb = float(np.sqrt(N))
    its = 0
    t0 = time.perf_counter()
    relres = 1.0
    history = []
    while its < args.converge_max:
        DH.cycle()
        relres = DH.residual_norm() / sumb
        history.append(relres)
        its += 1
        print(f"[bench] converge iteration {its}: relres {relres:.6e}", file=sys.stderr, flush=True)
        if relres < pars["tol"]:
            break
    solve_s = time.perf_counter() - t0
    pcg = None
    if D.world == 1 and args.converge_max > 0:
        # AMG as a CG preconditioner: same problem, same x0, same tolerance
        DH.set_x_ones()
        t0 = time.perf_counter()
        pits, phist = DH.DH.pcg(pars["tol"], args.converge_max)
        pcg = {"iterations_to_tol": pits, "final_relres": float(phist[-1]) if len(phist) else None,
               "time_to_solution_s": time.perf_counter() - t0}
        print(f"[bench] AMG-PCG: {pits} iterations, relres {pcg['final_relres']:.3e}, "
              f"{pcg['time_to_solution_s']:.3f} s", file=sys.stderr, flush=True)
    # the drop-in default (parity mode) on the same problem: V-cycles/s of the engine whose x is
    # bitwise the reference's after every cycle
    parity = None
    converge_parity = bool(args.parity_converge) and args.converge_max > 0
    if D.world == 1 and args.parity_cycles > 0 and args.mode == "throughput":
        DH.close()   # one mirror at a time
        t0 = time.perf_counter()
        PD = A.DeviceHierarchy(H, smoother="exact", coarse="krylov", device=-1, sum_order=0)
        up = time.perf_counter() - t0
        PD.upload(0, "b", np.ones(N))
        PD.upload(0, "x", np.ones(N))
        PD.cycle()   # warm-up (graph capture)
        PD.residual_norm()
        PD.upload(0, "x", np.ones(N))
        t0 = time.perf_counter()
        prel = []
        ncyc = args.converge_max if converge_parity else args.parity_cycles
        for _ in range(ncyc):
            PD.cycle()
            prel.append(PD.residual_norm() / float(np.sqrt(N)))
            if converge_parity and prel[-1] < pars["tol"]:
                break
        pdt = (time.perf_counter() - t0) / len(prel)
        info = [PD.level_info(l) for l in range(len(table) - 1)]
        PD.close()
        parity = {"value": 1.0 / pdt, "unit": "V-cycle iter/s", "ms_per_step": pdt * 1e3, "upload_s": up,
                  "relres_first_cycles": prel[:4], "gs_engines": [[i.gs_engine_f, i.gs_engine_c] for i in info],
                  "gs_stall": any(i.gs_stall for i in info)}
        if converge_parity:
            parity.update(iterations_to_tol=len(prel), final_relres=prel[-1], time_to_solution_s=pdt * len(prel))
        print(f"[bench] parity mode: {pdt * 1e3:.1f} ms per V-cycle (upload {up:.1f} s)", file=sys.stderr, flush=True)
    # reference-semantics iteration counts measured with the parity engine (tools/conv_study.py; the
    # parity engine's printed history equals the reference's, tests/test_gpu_at_size.py)
    ref_conv = None
    conv = ROOT / "profiles" / f"r02_conv{n}_parity_vs_throughput.json"
    if parity and converge_parity:
        ref_conv = {"iterations_to_tol_reference": parity["iterations_to_tol"],
                    "iterations_to_tol_throughput_same_run": its,
                    "parity_ms_per_cycle_same_run": parity["ms_per_step"],
                    "source": "this run (parity-mode mirror to tol)"}
        # throughput mode must converge within the reference's count + 2
        ref_conv["ladder"] = ("ok" if parity["final_relres"] < pars["tol"] and relres < pars["tol"]
                              and its <= parity["iterations_to_tol"] + 2 else "violated")
    elif conv.exists() and args.stencil == 7 and not irregular:
        try:
            cj = json.loads(conv.read_text())["modes"]
            ref_conv = {"iterations_to_tol_reference": cj["parity"]["iters"],
                        "iterations_to_tol_throughput_same_run": cj["throughput"]["iters"],
                        "parity_ms_per_cycle_same_run": cj["parity"]["ms_per_iter_median"],
                        "source": f"profiles/{conv.name}"}
        except Exception:
            ref_conv = None

    levels = [(L["rows"], L["nnz"]) for L in table]
    vbytes = vcycle_bytes(table, pars["pre_iter"] + pars["post_iter"])
    import resource
    rss_ranks = D.gather(resource.getrusage(resource.RUSAGE_SELF).ru_maxrss / 2**20)
    rss_gb = max(rss_ranks)   # peak over the ranks

    # {"csr": bytes, "stored": bytes} per launch: the newest committed PMC record of this workload and
    # format (tools/gpu/pmc.sh: separate rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes cannot run
    # inside this process), with the commit it was measured at
    traffic, traffic_src = None, None
    pmcs = sorted((ROOT / "profiles").glob("r*_level0_spmv_pmc.json"))
    if pmcs and D.world == 1 and not irregular:
        try:
            rec = json.loads(pmcs[-1].read_text())
            if rec.get("n") == n and rec.get("a_format") == a_format:
                traffic = {k: rec[k]["hbm_bytes_per_launch"] for k in ("csr", "stored") if k in rec}
                traffic_src = f"profiles/{pmcs[-1].name} (commit {rec.get('commit', 'unknown')})"
        except Exception:
            traffic = None

    # CPU baselines, rank 0 at N = 1 only, after every GPU measurement: the
    # median of --cpu-iters outer iterations after --cpu-warmup, on the same hierarchy
    cpu_baseline = None
    cpu_mt = None
    if D.rank == 0 and D.world == 1 and not args.no_cpu_baseline:
        hb_stop.set()
        hb_stop = threading.Event()
        threading.Thread(target=heartbeat, args=(hb_stop, time.perf_counter()), daemon=True).start()
        Hc = H
        if args.cpu_n and args.cpu_n != n and not irregular:
            Mc = A.generate(args.stencil, args.cpu_n)
            Hc = quiet_call(A.Hierarchy, Mc)
        cpu_n = n if irregular else (args.cpu_n or n)
        wname = (f"{mtx.name} ({N} rows)" if mtx is not None else f"G3_circuit stand-in ({n} rows)" if circuit
                 else f"{args.stencil}-pt {cpu_n}^3")
        hostinfo = host_cpus()
        a0_bytes = 12 * nnz + 4 * (N + 1) + 24 * N
        print("[bench] CPU baseline: reference semantics, 1 thread", file=sys.stderr, flush=True)
        cpu = {}
        cpu_iterations(Hc, cpu, threads=1, iters=args.cpu_iters, warmup=args.cpu_warmup)
        cpu_baseline = {
            "value": 1.0 / cpu["seconds"], "unit": "V-cycle iter/s", "cores": 1, "kind": "port",
            "sample": f"median of {args.cpu_iters} outer iterations after {args.cpu_warmup} warm-up (V-cycle incl. the "
                      f"reference CG(beta=1)+GMRES coarse solve, residual, norm) of oracle/sss_oracle.c with the "
                      f"reference semantics on the same {wname} hierarchy, 1 host thread, run "
                      f"after the GPU measurements; coarse solve {cpu['coarse_seconds']:.1f} s of {cpu['seconds']:.1f} s",
            "seconds": cpu["seconds"], "seconds_all": cpu["seconds_all"], "coarse_seconds": cpu["coarse_seconds"],
            "fine_spmv_GBps": a0_bytes / cpu["spmv_seconds"] / 1e9 if cpu_n == n else None,
            "host": hostinfo,
        }
        # the same restatement in the GPU's own mode, its row loops on every usable host CPU
        thr = args.cpu_threads or hostinfo["usable_cpus"]
        print(f"[bench] CPU baseline: GPU's mode, {thr} threads", file=sys.stderr, flush=True)
        mt = {}
        mode = {}
        if args.mode == "throughput":
            # the device's per-level smoothers (hybrid: level 0 exact only where chain-free)
            jac = [l for l, (k, _) in enumerate(level_smoothers) if k == 2]   # SSS_HIP_SMOOTH_JACOBI
            mask = sum(1 << l for l, (_, i) in enumerate(level_smoothers) if i > 0)
            steps = sorted({i for _, i in level_smoothers if i > 0})   # base, and the long-row levels'
            base = steps[0] if steps else 0
            mode = dict(smoother=1, jacobi_from=jac[0] if jac else len(level_smoothers),
                        coarse_mode=1 if coarse == "direct" else 0, inner=base, inner_mask=mask if mask else 1 << 30,
                        inner_long=steps[-1] - base if steps else 0,
                        long_mask=sum(1 << l for l, (_, i) in enumerate(level_smoothers) if steps and i == steps[-1] > base))
        cpu_iterations(Hc, mt, threads=thr, iters=args.cpu_iters, warmup=args.cpu_warmup, **mode)
        cpu_mt = {
            "value": 1.0 / mt["seconds"], "unit": "V-cycle iter/s", "cores": mt["threads"], "kind": "port",
            "sample": f"median of {args.cpu_iters} outer iterations after {args.cpu_warmup} warm-up, "
                      f"oracle/sss_oracle.c in the GPU's mode ({smoother} smoother, {coarse} coarse solve) on the same "
                      f"{wname} hierarchy, row loops on {mt['threads']} host threads; coarse solve "
                      f"{mt['coarse_seconds']:.2f} s of {mt['seconds']:.2f} s",
            "seconds": mt["seconds"], "seconds_all": mt["seconds_all"], "coarse_seconds": mt["coarse_seconds"],
            "fine_spmv_GBps": a0_bytes / mt["spmv_seconds"] / 1e9 if cpu_n == n else None,
            "host": hostinfo,
        }

    rec = {
        "metric": "V-cycle iters/sec + fine-level SpMV GB/s (%HBM peak), 64M-row 7pt Poisson",
        "value": value, "unit": "V-cycle iter/s", "n_gpus": D.world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": ms_per_step, "higher_is_better": True,
        "scaling": "strong" if D.world > 1 else None, "vs_baseline": None,
        "dtype": "f64",
        "data": (f"{mtx} read by SSS_mat_read (the reference's .mtx ingest), b = x0 = 1" if mtx is not None else
                 "synthetic (G3_circuit stand-in: weighted graph Laplacian + shift, amg_amd/workloads.py; b = x0 = 1)"
                 if circuit else f"synthetic ({args.stencil}-pt Poisson generated in memory, b = x0 = 1)"),
        "config": {"workload": workload, "rows": N, "nnz": nnz, "levels": len(levels),
                   "hierarchy": [list(t) for t in levels],
                   "mode": args.mode, "smoother": smoother, "coarse": coarse,
                   "inner": inner if smoother != "exact" else None,
                   "inner_from": inner_from if smoother != "exact" else None,
                   "inner_long": inner_long if smoother != "exact" else None,
                   "sum_order": "tree (long rows)" if sum_order == 1 else "stored CSR order",
                   "sorted_tiles": bool(sorted_tiles),
                   "level_storage_bits": level_formats,
                   "transfer_storage_bits_r_p": transfer_formats,
                   "kernel_launches_per_cycle": launches,
                   "single_workgroup_tail_from_level": tail_from if tail_from is not None and tail_from >= 0 else None,
                   "level_smoothers": [["exact", "hybrid", "jacobi"][k] + (f"+inner{i}" if i else "")
                                       for k, i in level_smoothers] if level_smoothers else None,
                   "iterations_to_tol": its, "final_relres": relres, "time_to_solution_s": solve_s,
                   "amg_pcg": pcg,
                   "reference_convergence": ref_conv,
                   "time_to_solution_reference_semantics_s": (ref_conv["iterations_to_tol_reference"] / parity["value"])
                   if (ref_conv and parity) else None,
                   "setup_s": setup_s, "hierarchy_source": hier_src, "upload_s": upload_s,
                   "upload_overlapped_with_setup": overlapped,
                   "setup_plus_upload_s": setup_s + upload_s,
                   "parallelism": f"rowpart{D.world}" if D.world > 1 else "single-gpu",
                   "host_peak_rss_gb_max_over_ranks": rss_gb,
                   "host_peak_rss_gb_per_rank": rss_ranks,
                   "hbm_used_gb_max_over_ranks": hbm_gb,
                   "hbm_used_gb_per_rank": hbm_ranks,
                   "partition_set": part_rec,
                   "relres_history": history,
                   "transport": transport},
        "roofline": {"bound": "hbm", "kernel": "spmv_adaptive<RESID> level 0 from its CSR arrays (y = b - A0 x)",
                     "achieved": achieved, "peak": PEAK_HBM_GBS, "unit": "GB/s", "frac": achieved / PEAK_HBM_GBS,
                     # the same residual as the V-cycle runs it, from its own (compressed) storage
                     "cycle_storage_frac": format_gbps / PEAK_HBM_GBS,
                     "frac_of_copy_peak": achieved / COPY_PEAK_GBS, "avg_launch_ms": csr_ms,
                     "bytes_per_launch": csr_bytes, "traffic": traffic.get("csr") if traffic else None,
                     "traffic_source": traffic_src,
                     "algorithmic_bytes": "SURVEY.md 8(d): 12 nnz + 4 (n + 1) + 8 n_cols + 16 n",
                     "cycle_storage": {
                         "a_format": a_format, "kernel": "the same residual from the storage the V-cycle uses",
                         "avg_launch_ms": spmv_ms, "bytes_per_launch": spmv_bytes, "GBps": format_gbps,
                         "frac": format_gbps / PEAK_HBM_GBS,
                         "traffic": traffic.get("stored") if traffic else None,
                         "csr_equivalent_rate_GBps": csr_bytes / (spmv_ms * 1e-3) / 1e9,
                         "note": "bytes = the stored format of A_0 (dictionary ELL: 8 B per row of codes + block "
                                 "dictionaries) + x, b, y; csr_equivalent = SURVEY 8(d) CSR bytes over this "
                                 "kernel's time, the rate a CSR SpMV would need to match it"}},
        # the V-cycle's roofline: the bytes its kernels actually move in their stored formats
        "vcycle_stored": ({
            "bytes_per_step": cyc_bytes["total"], "GBps": cyc_bytes["total"] / (ms_per_step * 1e-3) / 1e9,
            "peak": PEAK_HBM_GBS, "unit": "GB/s",
            "frac": cyc_bytes["total"] / (ms_per_step * 1e-3) / 1e9 / PEAK_HBM_GBS,
            "bytes_per_level": [round(b) for b in cyc_bytes["levels"]],
            "bytes_outer_residual": round(cyc_bytes["outer"]), "bytes_coarse": round(cyc_bytes["coarse"]),
            "definition": "sum over the launches of one outer iteration (the captured V-cycle + residual + "
                          "norm, sss_hip_cycle_bytes) of the bytes each reads and writes in the engine's stored "
                          "formats: the matrix storage of the rows it covers (codes, dictionaries, values, row "
                          "bounds), the x it gathers counted once per covered row, 8 B per covered row of every "
                          "row vector it streams (b, y, divisors, iterates); divided by ms_per_step"}
                          if cyc_bytes else None),
        # SURVEY.md 8(d)'s CSR-storage V-cycle bytes over the step time: the rate a CSR engine would need
        "vcycle_csr_equivalent": {
            "bytes_per_step": vbytes, "csr_equivalent_rate_GBps": vbytes / (ms_per_step * 1e-3) / 1e9,
            "definition": "SURVEY.md 8(d) V-cycle algorithmic bytes of CSR storage (12 B/entry): per smoothed "
                          "level 4 GS-CF sweeps, residual, restriction, prolongation, zero-fill; plus the outer "
                          "residual+norm; coarse solve excluded -- divided by the measured time per outer "
                          "iteration (whole-job bytes / max-over-ranks time at N > 1).  The engine stores the "
                          "stencil levels in compressed formats and skips exactly-dead work, so it moves fewer "
                          "bytes than this: a CSR-equivalent rate, not a roofline fraction (vcycle_stored is)",
        },
        "parity_mode": parity,
        "cpu_baseline": cpu_baseline,
        "cpu_baseline_same_mode": cpu_mt,
    }
    if D.world == 1 and not irregular:
        # left for the N > 1 runs of the same workload on this host (parallel_efficiency)
        try:
            single_ref_path(workload, args.mode).write_text(
                json.dumps({k: rec[k] for k in ("value", "ms_per_step", "config", "n_gpus")}))
        except OSError:
            pass
    else:
        rec["config"]["cycle_graph"] = cycle_graph
        ref = single_gpu_reference(args.single_ref, rec["config"])
        rec["single_gpu_reference"] = ref
        rec["parallel_efficiency"] = value / (D.world * ref["value"]) if ref else None
    # speed-ups on the same basis only: the drop-in default (parity mode, x bitwise the
    # reference's) against the reference semantics on 1 host thread, and this line's throughput mode
    # against the CPU running that same mode on every usable core
    if cpu_baseline and parity:
        rec["speedup_parity_vs_cpu_reference_semantics_1_thread"] = parity["value"] / cpu_baseline["value"]
    if cpu_mt:
        rec["speedup_throughput_vs_cpu_same_mode_all_cores"] = value / cpu_mt["value"]
    DH.close()
    if comm is not None:
        comm.close()
    hb_stop.set()
    if D.rank == 0:
        sys.stdout.flush()
        os.write(json_fd, (json.dumps(rec) + "\n").encode())
    D.close()


if __name__ == "__main__":
    main()
