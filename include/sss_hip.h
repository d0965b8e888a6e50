/*
 * sss_hip.h — C ABI of the gfx950 device engine behind the drop-in solve path.
 *
 * The host C side (amg_amd/host/sss_solve.c) implements the reference's SSS_amg_solve loop
 * (Solve/SSS_SOLVE.c:53-80) on top of these calls; bench.py and the GPU tests call them
 * through ctypes.  Plain pointers and sizes only.  All functions return 0 on success and a
 * negative SSS_ERROR_CODE on failure (ERROR_MISC for HIP/RCCL errors, with a message on
 * stderr), except where noted.
 *
 * Reference interfaces these replace (amg/ tree):
 *   sss_hip_cycle ............ SSS_amg_cycle                Solve/SSS_cycle.cu:848-967
 *   sss_hip_residual_norm .... r = b - A*x; ||r||            Solve/SSS_SOLVE.c:59-64
 *   sss_hip_coarse_solve ..... SSS_amg_coarest_solve        Solve/SSS_cycle.cu:819-846
 *   sss_hip_smooth ........... SSS_amg_smoother_pre/post    Solve/SSS_smooth.c:138-304
 *   sss_hip_csr_spmv ......... SSS_blas_mv_amxpy/_mxy, spmv_cuda/alpha_spmv_cuda
 *                              SSS_utils.c:161-201, Solve/SSS_cuda.cu:77-165
 */
#ifndef SSS_HIP_H
#define SSS_HIP_H

#include "sss_amg.h"

#ifdef __cplusplus
extern "C" {
#endif

/* ---- engine options ------------------------------------------------------------------ */
enum {
    SSS_HIP_SMOOTH_EXACT = 0,    /* reference GS-CF on every level (level-scheduled, bitwise) */
    SSS_HIP_SMOOTH_HYBRID = 1,   /* exact GS-CF on level 0 when its C and F classes are independent
                                    sets (red-black: no chains), else two-stage GS-CF there;
                                    C/F-Jacobi (two-stage from inner_from) below */
    SSS_HIP_SMOOTH_JACOBI = 2    /* C/F-Jacobi on every level */
};
enum {
    SSS_HIP_COARSE_KRYLOV = 0,   /* reference CG(beta==1)+GMRES(30), on device */
    SSS_HIP_COARSE_DIRECT = 1    /* explicit inverse of the coarsest operator, one GEMV */
};
enum { SSS_HIP_VEC_B = 0, SSS_HIP_VEC_X = 1, SSS_HIP_VEC_WP = 2 };

typedef struct sss_hip_opts {
    int device;        /* HIP device ordinal; -1 = keep current */
    int smoother;      /* SSS_HIP_SMOOTH_* */
    int coarse;        /* SSS_HIP_COARSE_* */
    int row_cap;       /* 0 = uncapped coarse SpMV; 4096 reproduces <<<64,64>>> (as shipped) */
    int use_graph;     /* capture the V-cycle into a hipGraph once and replay it */
    int verbose;       /* engine diagnostics on stderr */
    int inner;         /* C/F-Jacobi levels: 0 = plain C/F-Jacobi; k > 0 = two-stage GS-CF with k
                          Jacobi-Richardson steps on each pass's same-class lower triangle */
    int inner_from;    /* first level that uses the two-stage form (plain C/F-Jacobi above it) */
    int relabel;       /* renumber levels F-first/C-second on the device (bitwise-neutral):
                          0 off, 1 every level but the coarsest, 2 as 1 but level 0 kept */
    int sorted_tiles;  /* store each SpMV/relaxation staging tile column-sorted with its stored
                          positions (x gathers coalesce across rows; sums unchanged, bitwise) */
    int sum_order;     /* 0: every row sum in the reference's stored CSR order (bitwise);
                          1: rows of long-row levels (>= SSS_HIP_WAVE_MIN entries on average)
                          summed by a wave in a fixed tree order over column-sorted rows --
                          deterministic, within the reordered-summation bound of the reference,
                          not bitwise (throughput mode) */
    int inner_long;    /* extra Jacobi-Richardson steps on the two-stage levels of long rows (at least
                          SSS_HIP_LONG_ROW_MIN = 300 entries per row on average over the whole level):
                          their lower triangles are the densest, and the extra step keeps throughput
                          mode within the reference's iteration count + 2 at 7-pt 512^3 (default 1) */
    int formats;       /* storage formats of the uploaded operators (all bitwise-neutral): 0 = every
                          format a level qualifies for (dictionary / column ELL, dictionary and
                          column-sorted tiles); 1 = plain CSR tiles only (cheapest to build); -1 = auto
                          (default): 1 for the exact smoother, whose cycle is bound by the GS-CF chains,
                          so the formats would only lengthen the mirror's construction, else 0 */
} sss_hip_opts;

#define SSS_HIP_LONG_ROW_MIN 300
/* Defaults, overridable by environment: SSS_HIP_SMOOTHER=exact|hybrid|jacobi,
 * SSS_HIP_COARSE=krylov|direct, SSS_HIP_ROWCAP=<n>, SSS_HIP_GRAPH=0|1, SSS_HIP_DEVICE=<n>,
 * SSS_HIP_VERBOSE=0|1, SSS_HIP_RELABEL=0|1|2 (default 1), SSS_HIP_INNER=<k> (default 1),
 * SSS_HIP_SORTED_TILES=0|1 (default 1), SSS_HIP_SUM_ORDER=0|1 (default 0),
 * SSS_HIP_INNER_FROM=<level> (default 2), SSS_HIP_INNER_LONG=<k> (default 1),
 * SSS_HIP_FORMATS=auto|full|lean (default auto). */
void sss_hip_opts_default(sss_hip_opts *o);

/* Number of usable HIP devices (0 when none; never exits). */
int sss_hip_device_count(void);
/* Free and total HBM of the current device, in bytes (hipMemGetInfo). */
int sss_hip_mem_info(size_t *free_bytes, size_t *total_bytes);

/* ---- hierarchy mirror -------------------------------------------------------------- */
typedef struct sss_hip_hier sss_hip_hier;

/* Uploads every level of mg (A, P, R, cfmark; b/x/wp allocated) to HBM and builds the
 * smoother schedules.  mg->cg[0].x/.b may be unset. Returns NULL on failure. */
sss_hip_hier *sss_hip_hier_create(const SSS_AMG *mg, const sss_hip_opts *o);
void sss_hip_hier_destroy(sss_hip_hier *h);

/* SSS_amg_setup (Setup/SSS_SETUP.cu:36-178 semantics, same printed output, same mg) with the
 * mirror built while the setup runs: every level is relabeled and uploaded on a worker thread as
 * soon as the setup has moved past it, so the uploads overlap the setup's serial RS passes.
 * Equivalent to SSS_amg_setup(mg, A, pars) followed by sss_hip_hier_create(mg, o).  times
 * (optional, 3 doubles): setup seconds (uploads overlapped), seconds of mirror work after the
 * setup returned, of which waiting for the worker.  NULL on failure (mg is set up even then). */
sss_hip_hier *sss_hip_setup_create(SSS_AMG *mg, SSS_MAT *A, SSS_AMG_PARS *pars, const sss_hip_opts *o,
                                   double *times);

/* The setup's Galerkin product A_c = R A P (SSS_blas_mat_rap, SSS_matvec.c:398-534) on the GPU,
 * bit for bit the host product (same entries, same column order, same summation order).  C gets
 * SSS_calloc'd arrays.  Returns 0, or an error code with C untouched (no device, no memory).
 * The setup uses it, when a device is present, for levels with at least SSS_SETUP_GPU_RAP_MIN
 * nonzeros in A (default 10^6) and at most SSS_SETUP_GPU_RAP_MAXROW of them per row on average
 * (default 48); SSS_SETUP_GPU_RAP=0 keeps every product on the host. */
int sss_hip_rap(const SSS_MAT *R, const SSS_MAT *A, const SSS_MAT *P, SSS_MAT *C);

/* Progress hook of the setup (amg_amd/host/sss_setup.c): hook(ctx, mg, done, 0) once levels
 * 0 .. done-1 are final and none of them is the coarsest; hook(ctx, mg, num_levels - 1, 1) at
 * the end. */
typedef void (*sss_setup_hook)(void *ctx, const SSS_AMG *mg, int done, int final);
void sss_amg_setup_hooked(SSS_AMG *mg, SSS_MAT *A, SSS_AMG_PARS *pars, sss_setup_hook hook, void *ctx);

int sss_hip_upload_vec(sss_hip_hier *h, int level, int which, const double *src, int n);
int sss_hip_download_vec(sss_hip_hier *h, int level, int which, double *dst, int n);

/* One V/W-cycle on the device-resident level vectors (asynchronous on the engine stream). */
int sss_hip_cycle(sss_hip_hier *h);
/* wp0 = b0 - A0*x0 and ||wp0||_2, returned to the host (synchronises the stream). */
int sss_hip_residual_norm(sss_hip_hier *h, double *absres);
/* Binary hierarchy file (engine extension; amg_amd/host/sss_hierio.c): what
 * the solve phase reads of a set-up SSS_AMG -- parameters and per level A, P, R, cfmark.  Loading
 * gives a hierarchy field-for-field equal to the one SSS_amg_setup built (free it with
 * SSS_amg_data_destroy).  0 or ERROR_OPEN_FILE / ERROR_WRONG_FILE. */
int SSS_amg_save(const SSS_AMG *mg, const char *path);
int SSS_amg_load(SSS_AMG *mg, const char *path);

/* AMG-preconditioned flexible CG on level 0 (an engine extension -- the
 * reference's Krylov solvers serve only the coarsest level): right-hand side = the level-0 b
 * vector, initial guess / result = the level-0 x vector, one V-cycle per iteration as the
 * preconditioner.  Stops when ||r_k||/||b|| < tol or after maxit iterations; hist (optional)
 * receives the relative residual of each iteration. */
int sss_hip_pcg(sss_hip_hier *h, double tol, int maxit, int *iters, double *relres, double *hist, int hist_cap);
/* The coarsest-level solve alone (on the level vectors of the coarsest level). */
int sss_hip_coarse_solve(sss_hip_hier *h);
/* Pre (post = 0) or post (post = 1) smoothing of one level. */
int sss_hip_smooth(sss_hip_hier *h, int level, int post);
int sss_hip_sync(sss_hip_hier *h);

/* Per-level statistics for reporting: rows, nnz(A), nnz(P), smoother DAG depths; the exact GS
 * engine of the F / C pass (0: one launch per DAG depth, 1: chip-wide dataflow, 2: single CU);
 * whether a one-launch pass ever gave up waiting (gs_stall != 0: results invalid); the storage of
 * A_l in HBM (a_format bits: 1 column-sorted tiles, 2 dictionary tiles (with 1: value
 * dictionaries over the sorted tiles; alone with 64: dictionary ELL rows), 4 free-order rows,
 * 8 merged row groups, 16 wave-per-row;
 * the two-stage inner steps of a C/F-Jacobi level (0: plain C/F-Jacobi). */
typedef struct sss_hip_level_info {
    int rows, nnz, nnz_p, dag_f, dag_c, smoother_kind;
    int gs_engine_f, gs_engine_c, gs_stall, a_format;
    long long a_stream_bytes;   /* bytes of A_l's stored format one tile-path SpMV reads (no vectors) */
    int inner;
    int r_format, p_format;     /* R_l / P_l storage, the a_format bits */
    int pad_;
} sss_hip_level_info;
int sss_hip_level_info_get(sss_hip_hier *h, int level, sss_hip_level_info *out);
int sss_hip_num_levels(sss_hip_hier *h);
/* First level of the V-cycle's single-workgroup tail (sss_tail.hip: the small coarse levels,
 * descent, coarsest solve and ascent in one launch), or -1 when the cycle has none. */
int sss_hip_tail_from(sss_hip_hier *h);
/* Kernel launches of one V-cycle as captured in its hipGraph (host-steered Krylov coarse solves
 * excluded), or -1 before the first captured cycle / without graphs. */
int sss_hip_cycle_launches(sss_hip_hier *h);
/* Stored-format bytes the kernels of one outer iteration read and write (the next sss_hip_cycle and
 * the residual + norm after it; walked into a discarded stream capture, nothing runs): the stored
 * matrix bytes of the rows each launch covers, the x it gathers counted once per covered row, and
 * 8 B per covered row of every row vector it streams.  out[l] for level l, out[nslots - 2] the outer
 * residual + norm, out[nslots - 1] the coarsest solve; nslots >= sss_hip_num_levels(h) + 2. */
int sss_hip_cycle_bytes(sss_hip_hier *h, double *out, int nslots);

/* ---- kernel-level entry points on device memory (tests, bench, roofline) ------------- */
enum {
    SSS_HIP_SPMV_MXY = 0,    /* y = A*x                         (SSS_blas_mv_mxy)      */
    SSS_HIP_SPMV_AMXPY = 1,  /* y += (A*x)*alpha                (SSS_blas_mv_amxpy)    */
    SSS_HIP_SPMV_RESID = 2,  /* y = b + (A*x)*(-1)              (copy + amxpy(-1))     */
    SSS_HIP_SPMV_ACC = 3     /* y += A*x, rows < cap only       (spmv_cuda)            */
};
/* A plan holds the CSR-adaptive row blocking of one matrix (device pointers). */
typedef struct sss_hip_spmv_plan sss_hip_spmv_plan;
sss_hip_spmv_plan *sss_hip_spmv_plan_create(int n, int nnz, const int *d_rp, const int *h_rp);
void sss_hip_spmv_plan_destroy(sss_hip_spmv_plan *p);
int sss_hip_spmv(const sss_hip_spmv_plan *p, int op, double alpha, const int *d_rp, const int *d_ci,
                 const double *d_v, const double *d_x, const double *d_b, double *d_y, int cap,
                 void *stream);

/* Host-memory convenience wrappers (allocate, copy, run, copy back) used by the exported
 * SSS_blas_mv_* / smoother / coarse-solve entry points. */
int sss_hip_host_spmv(int op, double alpha, const SSS_MAT *A, const double *x, const double *b,
                      double *y, int cap);
int sss_hip_host_smooth(const SSS_SMTR *s, int post);
/* The three host-memory entry points keep the device form of their operator (keyed by a content
 * hash of the CSR arrays, the use and the device) in a small cache, so a caller that loops over
 * them with the same matrix uploads it once; this releases the cached device objects. */
void sss_hip_host_cache_clear(void);
int sss_hip_host_coarse_solve(SSS_MAT *A, SSS_VEC *b, SSS_VEC *x, double ctol, int coarse_mode,
                              int row_cap);

/* Engine event timer around `reps` launches of the level-0 residual SpMV on the engine
 * stream: average kernel milliseconds (roofline measurement in bench.py). */
int sss_hip_time_level0_spmv(sss_hip_hier *h, int reps, double *avg_ms);
/* level_ms[l] (nslots >= levels): level l's share of an eager cycle -- pre-smoothing, residual,
 * restriction, zero fill, prolongation, post-smoothing (the coarsest: its solve; a single-workgroup
 * tail: at its first level) -- averaged over reps, events between the steps.  Advances the iterate. */
int sss_hip_time_levels(sss_hip_hier *h, int reps, double *level_ms, int nslots);
/* The same launch from level 0's plain CSR arrays (whatever storage the cycle uses for A_0). */
int sss_hip_time_level0_spmv_csr(sss_hip_hier *h, int reps, double *avg_ms);
/* Average milliseconds of `reps` full iterations (cycle + residual + norm) on the engine
 * stream, timed with HIP events; absres of the last iteration is returned. */
int sss_hip_time_iterations(sss_hip_hier *h, int reps, double *avg_ms, double *absres);

/* ---- row-partitioned multi-GPU solve (one process per GPU) ------------------------- */
/* Every level l < nagg is split into contiguous row ranges: level 0 evenly, level l+1 by
 * ownership of the C points of level l (coarse numbering is monotone in the fine index,
 * SSS_coarsen's cmap).  Each rank keeps its rows (F|C relabeled) plus ghost columns; levels
 * >= nagg (fewer than agg_rows rows, and always the coarsest) are replicated on every rank and
 * cycled redundantly.  Halos move over RCCL (xGMI) or, for tests, over a host transport. */
typedef struct sss_hip_comm sss_hip_comm;
typedef struct sss_hip_dist sss_hip_dist;
typedef struct sss_hip_host_transport {
    void *ctx;
    /* one point-to-point round: send scount[i] doubles (concatenated in sbuf) to rank sdst[i]
     * and receive rcount[i] doubles (concatenated into rbuf) from rank rsrc[i]; 0 = success */
    int (*exchange)(void *ctx, int nsend, const int *sdst, const int *scount, const double *sbuf, int nrecv,
                    const int *rsrc, const int *rcount, double *rbuf);
    int (*allreduce_sum)(void *ctx, double *v, int n);
    /* all[displs[q] .. + counts[q]) <- rank q's `mine` */
    int (*allgatherv)(void *ctx, const double *mine, int count, double *all, const int *counts, const int *displs);
} sss_hip_host_transport;

#define SSS_HIP_RCCL_ID_BYTES 128
/* rank 0 creates the id; the caller broadcasts its bytes (e.g. over torch.distributed) */
int sss_hip_rccl_unique_id(unsigned char *id);
/* device >= 0: hipSetDevice(device) first (the communicator binds the current device) */
sss_hip_comm *sss_hip_comm_rccl(int nranks, int rank, const unsigned char *id, int device);
sss_hip_comm *sss_hip_comm_host(int nranks, int rank, const sss_hip_host_transport *t);
/* Timing only: every collective and halo transfer is skipped, the rest of the rank's cycle (its
 * kernels, halo packs, graph capture) runs as over RCCL -- the per-rank compute floor of a multi-GPU
 * run measured one rank at a time on one GPU (tools/n8_floor.py).  The iterates are meaningless. */
sss_hip_comm *sss_hip_comm_timing(int nranks, int rank);
void sss_hip_comm_destroy(sss_hip_comm *c);

/* mg: the global hierarchy (every rank runs the same host setup).  V-cycles only.
 * agg_rows <= 0: SSS_HIP_AGG_ROWS or 20000. */
sss_hip_dist *sss_hip_dist_create(const SSS_AMG *mg, const sss_hip_opts *o, sss_hip_comm *c, int agg_rows);
/* The same engine from a partition set written by sss_part_save: rank r reads only
 * prefix.r<r> (its rows, ghosts, halo lists) and prefix.tail (the replicated coarse levels), so
 * no rank holds the global hierarchy (the 512^3 8-GPU configuration). */
sss_hip_dist *sss_hip_dist_create_from_files(const char *prefix, const sss_hip_opts *o, sss_hip_comm *c);
void sss_hip_dist_destroy(sss_hip_dist *d);
/* own rows [lo, hi) of level 0 in the original numbering; nagg = number of partitioned levels */
int sss_hip_dist_info(sss_hip_dist *d, int *lo, int *hi, int *nagg, int *nghost0);
/* Own rows, ghosts and nonzeros of this rank's partitioned level l. */
int sss_hip_dist_level_size(sss_hip_dist *d, int l, int *m, int *g, long long *nnz);
/* exact eliminations in force on partitioned level l (agreed over the ranks), a bit mask:
 * 1 zero-first pass, 2 fused C-row residual, 4 dead F-row prolongation, 8 the cycle runs as one
 * captured hipGraph (SSS_HIP_DIST_GRAPH=1 over RCCL with a device-side coarse solve).  <0: bad level. */
int sss_hip_dist_level_flags(sss_hip_dist *d, int l);
/* level-0 vectors, the rank's own rows in the original order (n = hi - lo) */
int sss_hip_dist_upload_vec(sss_hip_dist *d, int which, const double *own, int n);
int sss_hip_dist_download_vec(sss_hip_dist *d, int which, double *own, int n);
int sss_hip_dist_cycle(sss_hip_dist *d);
/* global ||b0 - A0 x0||_2 (one 8-byte allreduce), synchronises */
int sss_hip_dist_residual_norm(sss_hip_dist *d, double *absres);
int sss_hip_dist_sync(sss_hip_dist *d);
/* average ms of `reps` local level-0 residual SpMVs (no exchange): the per-rank roofline */
int sss_hip_dist_time_level0_spmv(sss_hip_dist *d, int reps, double *avg_ms);
/* *cycle_ms: this rank's cycle as it runs (captured graph), averaged over reps; level_ms[l] (l < nagg)
 * one partitioned level's descent + ascent and level_ms[nagg] the replicated tail, from reps eager
 * cycles with events between the steps (nslots >= nagg + 1).  Advances the iterate. */
int sss_hip_dist_time_levels(sss_hip_dist *d, int reps, double *cycle_ms, double *level_ms, int nslots);
/* the replicated tail's per-level times (sss_hip_time_levels on it) */
int sss_hip_dist_time_tail_levels(sss_hip_dist *d, int reps, double *level_ms, int nslots);
/* Per partitioned level: halo exchanges enqueued since the last reset and the doubles this rank sent
 * in them (a captured cycle counts at its capture); the tail all-gather's own / all rows and the
 * number of replicated levels. */
int sss_hip_dist_halo_stats(sss_hip_dist *d, long long *calls, long long *doubles, int nslots, int reset,
                            int *nc_own, int *nc_all, int *tail_levels);

/* Host-only view of the partition (no device needed; used by the CPU multi-process tests).
 * which: 0 = A_l (m x (m+g)), 1 = P_l (m x next-level local), 2 = R_l (own coarse rows x (m+g)).
 * Arrays stay owned by the plan. */
typedef struct sss_part_plan sss_part_plan;
sss_part_plan *sss_part_plan_create(const SSS_AMG *mg, int nranks, int rank, int agg_rows);
/* Partition set of the global hierarchy for nranks ranks: prefix.r0 .. prefix.r<nranks-1> (one
 * rank's plan each, built one at a time) and prefix.tail (levels >= nagg, SSS_amg_save format).
 * Host only.  Returns 0 or an SSS error code. */
int sss_part_save(const SSS_AMG *mg, int nranks, int agg_rows, const char *prefix);
/* One rank's plan read back from its partition file (prefix.r<rank>). */
sss_part_plan *sss_part_plan_load(const char *path);
void sss_part_plan_destroy(sss_part_plan *p);
int sss_part_plan_nagg(const sss_part_plan *p);
/* own range, own count, ghost count of level l (l <= nagg for the range; m/g for l < nagg) */
int sss_part_plan_level(const sss_part_plan *p, int l, int *lo, int *hi, int *m, int *g);
int sss_part_plan_matrix(const sss_part_plan *p, int l, int which, SSS_MAT *out);
/* perm: local id -> global id (m); ghosts: ghost k -> global id (g) */
int sss_part_plan_ids(const sss_part_plan *p, int l, const int **perm, const int **ghosts);
/* halo of level l: nsend/nrecv peers; peer ranks, counts, send local ids (concatenated) */
int sss_part_plan_halo(const sss_part_plan *p, int l, int *nsend, const int **sdst, const int **scount,
                       const int **sidx, int *nrecv, const int **rsrc, const int **rcount);

/* ---- generators (host) -------------------------------------------------------------- */
/* kind 7 or 27; rows of z-planes [z0, z1) of an nx*ny*nz grid, global column indices. */
int sss_gen_stencil(int kind, int nx, int ny, int nz, int z0, int z1, SSS_MAT *A);

#ifdef __cplusplus
}
#endif
#endif
