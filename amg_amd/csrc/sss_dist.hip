// sss_dist.hip — row-partitioned multi-GPU solve phase: one process per GPU, halos and the
// residual-norm reduction over RCCL (xGMI), or over a host transport for tests.
//
// Per partitioned level l < nagg, rank r holds its rows of A_l / P_l / R_l in local numbering
// (sss_part.hpp) and length m + g vectors (own values, then ghosts).  The V-cycle of
// SSS_amg_cycle (Solve/SSS_cycle.cu:848-967) then runs as on one GPU, with a halo exchange in
// front of every kernel that reads off-rank values:
//   smoother   : before every class pass (x), and after each two-stage stage (the stage's
//                iterate, whose lower-rank ghost rows of the pass's class are "lower" entries);
//   residual   : x;   restriction: wp;   prolongation: x_{l+1}.
// Each rank computes every one of its rows exactly as the single-GPU engine does (same entries,
// same order, same inputs), so the iterates are bitwise those of one GPU; only the outer norm is
// summed in a different order.  Level 0 must be smoothed by depth-1 class passes (red-black,
// e.g. 7-point Poisson) or a C/F-Jacobi form; exact GS-CF with intra-class chains is not
// distributed.  Levels >= nagg run replicated on every rank (an ordinary single-GPU hierarchy
// over mg->cg[nagg..]); the restriction into level nagg is all-gathered once per cycle.
#include <rccl/rccl.h>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <vector>

#include "sss_engine.hpp"
#include "sss_part.hpp"

using namespace sss;

struct sss_hip_comm {
    int nranks = 1, rank = 0;
    bool host = false;
    // timing only (sss_hip_comm_timing): every collective and halo transfer is skipped, the rest of
    // the rank's cycle -- its kernels, halo packs, the graph -- runs as over RCCL: the per-rank compute
    // floor of a multi-GPU run, measured one rank at a time on one GPU (its results are meaningless)
    bool timing = false;
    ncclComm_t nccl = nullptr;
    sss_hip_host_transport t{};
};

namespace {

struct Halo {
    std::vector<int> sdst, scount, soff, rsrc, rcount, roff;
    int nsend = 0, nrecv = 0;
    int *d_sidx = nullptr;
    double *d_sbuf = nullptr;
    std::vector<double> h_sbuf, h_rbuf;   // host transport staging
};

struct DLevel {
    int lo = 0, hi = 0, m = 0, g = 0;
    std::vector<int> perm;   // local -> global (own rows)
    DevCSR A, P, R;
    SmootherPlan sm;
    double *b = nullptr, *x = nullptr, *wp = nullptr, *w0 = nullptr, *w1 = nullptr;
    Halo halo;
    // per row block of A, R and P: does the block read a ghost value?  (halo overlap)
    std::vector<char> ghostA, ghostR, ghostP;
};

// Per row block of a local matrix: 1 if any entry reads a column >= own (a ghost).
// the row blocking a DevCSR was uploaded with (first row of each block, nblk + 1 entries)
int device_blocks(const DevCSR &M, std::vector<int> &blk)
{
    blk.assign((size_t)M.nblk + 1, 0);
    if (M.nblk <= 0 || !M.blk) return 0;
    SSS_HIP(hipMemcpy(blk.data(), M.blk, sizeof(int) * blk.size(), hipMemcpyDeviceToHost));
    return 0;
}

std::vector<char> block_ghost_flags(const HostMat &M, int own, const std::vector<int> &blk)
{
    std::vector<char> f(blk.empty() ? 0 : blk.size() - 1, 0);
    for (size_t q = 0; q + 1 < blk.size(); ++q)
        for (int k = M.rp[blk[q]]; k < M.rp[blk[q + 1]] && !f[q]; ++k) f[q] = M.ci[k] >= own;
    return f;
}

__global__ __launch_bounds__(256) void pack_kernel(int n, const int *__restrict__ idx, const double *__restrict__ v,
                                                    double *__restrict__ out)
{
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = v[idx[i]];
}

__global__ __launch_bounds__(256) void gather_kernel(int n, const int *__restrict__ idx, const double *__restrict__ v,
                                                      double *__restrict__ out)
{
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = v[idx[i]];
}

int nccl_fail(ncclResult_t r, const char *what)
{
    fprintf(stderr, "### ERROR: RCCL %s: %s\n", what, ncclGetErrorString(r));
    return ERROR_MISC;
}
#define SSS_NCCL(call)                                  \
    do {                                                \
        ncclResult_t r_ = (call);                       \
        if (r_ != ncclSuccess) return nccl_fail(r_, #call); \
    } while (0)

}  // namespace

struct sss_hip_dist {
    sss_hip_comm *comm = nullptr;
    SSS_AMG_PARS pars{};
    sss_hip_opts opts{};
    hipStream_t stream = nullptr;
    int nagg = 0;
    DLevel L[kMaxLevels];
    sss_hip_hier *tail = nullptr;   // levels >= nagg, replicated
    // restriction into the tail: own coarse rows (global order) -> all-gather -> tail order
    int nc_own = 0, nc_all = 0;
    std::vector<int> counts, displs;
    double *d_cown = nullptr, *d_call = nullptr;
    int *d_tail_perm = nullptr;     // tail level-0 new -> old (null: identity)
    std::vector<double> h_cown, h_call;
    double *partial = nullptr, *d_norm = nullptr, *h_norm = nullptr;   // norm: [0] sum of squares, [1] stall flag
    unsigned *d_err = nullptr;    // stall word of the one-launch GS passes (this rank's levels and tail)
    std::vector<double> stage;
    bool resid_c_ready = false;   // the last cycle's final C pass left r_C and its partials (level 0)
    SSS_AMG tail_host{};          // the tail levels read from a partition set (file-built engines)
    bool own_tail_host = false;
    // halo overlap: RCCL send/recv on a second stream while the engine stream runs interior blocks
    hipStream_t cstream = nullptr;
    hipEvent_t ev_packed = nullptr, ev_halo = nullptr;
    int overlap = 1;   // 0 off, 1 on (RCCL), 2 also split the launches over the host transport (tests)
    // hipGraph of the whole cycle (default over RCCL with a device-side coarse solve; SSS_HIP_DIST_GRAPH=0 off):
    // kernels, halo packs, the grouped RCCL send/recv on the communication stream (joined back by
    // events), the coarse all-gather and the replicated tail, captured once and replayed
    int use_graph = 0;
    hipGraphExec_t cycle_exec = nullptr;
    bool graph_resid_ready = false;   // resid_c_ready as the captured cycle leaves it
    // halo statistics as enqueued (sss_hip_dist_halo_stats): exchanges and doubles sent per level
    long long ex_calls[kMaxLevels] = {}, ex_doubles[kMaxLevels] = {};
    // per-level timing of an eager cycle (sss_hip_dist_time_levels): events after each level's
    // descent, the tail and each level's ascent
    std::vector<hipEvent_t> lev_ev;
};

namespace {

// Halo of level l for vec (own values first, ghosts after): pack the values peers need, send them
// and receive the ghosts.  RCCL: the grouped send/recv runs on the communication stream once the
// pack has run; exchange_end makes the engine stream wait for it, so work enqueued in between (the
// blocks that read no ghost) overlaps the transfer.  Host transport: synchronous, in _begin.
int exchange_begin(sss_hip_dist *d, int l, double *vec)
{
    DLevel &L = d->L[l];
    Halo &H = L.halo;
    sss_hip_comm *c = d->comm;
    const hipStream_t s = d->stream;
    if (H.nsend == 0 && H.nrecv == 0) return 0;
    const int ns = H.soff.empty() ? 0 : H.soff.back();
    d->ex_calls[l]++;
    d->ex_doubles[l] += ns;
    if (ns > 0) {
        hipLaunchKernelGGL(pack_kernel, dim3((ns + 255) / 256), dim3(256), 0, s, ns, H.d_sidx, vec, H.d_sbuf);
        SSS_HIP(hipGetLastError());
    }
    if (c->timing) return 0;
    if (!c->host) {
        SSS_HIP(hipEventRecord(d->ev_packed, s));
        SSS_HIP(hipStreamWaitEvent(d->cstream, d->ev_packed, 0));
        SSS_NCCL(ncclGroupStart());
        ncclResult_t r = ncclSuccess;
        for (int i = 0; i < H.nsend && r == ncclSuccess; ++i)
            r = ncclSend(H.d_sbuf + H.soff[i], (size_t)H.scount[i], ncclDouble, H.sdst[i], c->nccl, d->cstream);
        for (int i = 0; i < H.nrecv && r == ncclSuccess; ++i)
            r = ncclRecv(vec + L.m + H.roff[i], (size_t)H.rcount[i], ncclDouble, H.rsrc[i], c->nccl, d->cstream);
        const ncclResult_t e = ncclGroupEnd();   // always close the group, also after a failed call
        if (r != ncclSuccess) return nccl_fail(r, "ncclSend/ncclRecv (halo)");
        if (e != ncclSuccess) return nccl_fail(e, "ncclGroupEnd (halo)");
        SSS_HIP(hipEventRecord(d->ev_halo, d->cstream));
        return 0;
    }
    H.h_sbuf.resize(std::max(ns, 1));
    H.h_rbuf.resize(std::max(L.g, 1));
    if (ns > 0) SSS_HIP(hipMemcpyAsync(H.h_sbuf.data(), H.d_sbuf, sizeof(double) * ns, hipMemcpyDeviceToHost, s));
    SSS_HIP(hipStreamSynchronize(s));
    if (c->t.exchange(c->t.ctx, H.nsend, H.sdst.data(), H.scount.data(), H.h_sbuf.data(), H.nrecv, H.rsrc.data(),
                      H.rcount.data(), H.h_rbuf.data()))
        return ERROR_MISC;
    if (L.g > 0) SSS_HIP(hipMemcpyAsync(vec + L.m, H.h_rbuf.data(), sizeof(double) * L.g, hipMemcpyHostToDevice, s));
    SSS_HIP(hipStreamSynchronize(s));   // the staging buffer is reused by the next exchange
    return 0;
}

int exchange_end(sss_hip_dist *d, int l)
{
    const Halo &H = d->L[l].halo;
    if (d->comm->host || d->comm->timing || (H.nsend == 0 && H.nrecv == 0)) return 0;
    SSS_HIP(hipStreamWaitEvent(d->stream, d->ev_halo, 0));
    return 0;
}

int exchange(sss_hip_dist *d, int l, double *vec)
{
    int rc = exchange_begin(d, l, vec);
    return rc ? rc : exchange_end(d, l);
}

// launch(b0, b1) over the row blocks [blo, bhi) of a matrix whose per-block ghost flags are
// `ghost`, with vec's halo of level l refreshed in between: the runs of blocks that read no ghost
// go first, overlapping the transfer, the others after it (everything after the exchange when
// there is too little interior work or the transport is synchronous).
int split_launch(sss_hip_dist *d, int l, double *vec, const std::vector<char> &ghost, int blo, int bhi,
                 const std::function<void(int, int)> &launch)
{
    int interior = 0, runs = 0;
    for (int q = blo; q < bhi; ++q) {
        interior += !ghost[q];
        runs += q == blo || ghost[q] != ghost[q - 1];
    }
    const Halo &H = d->L[l].halo;
    const bool halo = H.nsend > 0 || H.nrecv > 0;
    if (!d->overlap || (d->comm->host && d->overlap < 2) || !halo || interior * 4 < (bhi - blo) || runs > 16) {
        int rc = exchange(d, l, vec);
        if (rc) return rc;
        if (bhi > blo) launch(blo, bhi);
        SSS_HIP(hipGetLastError());
        return 0;
    }
    int rc = exchange_begin(d, l, vec);
    if (rc) return rc;
    for (int pass = 0; pass < 2; ++pass) {   // interior runs, then (after the halo) ghost-reading runs
        if (pass == 1 && (rc = exchange_end(d, l))) return rc;
        for (int q = blo; q < bhi;) {
            int e = q + 1;
            while (e < bhi && ghost[e] == ghost[q]) ++e;
            if ((ghost[q] != 0) == (pass == 1)) launch(q, e);
            q = e;
        }
    }
    SSS_HIP(hipGetLastError());
    return 0;
}

// wp = b - A x over this rank's rows of level l (x's halo refreshed, overlapping the interior
// blocks), or over the F rows only when the smoother's last pass already formed the C rows
// (c_done); per-block sums of squares into partial when given.
int residual(sss_hip_dist *d, int l, bool c_done, double *partial)
{
    DLevel &L = d->L[l];
    const int bhi = c_done ? L.A.split_blk : L.A.nblk;
    if (L.A.wave_rows || L.A.vec_rows) {
        int rc = exchange(d, l, L.x);
        return rc ? rc : launch_spmv(L.A, SSS_HIP_SPMV_RESID, -1.0, L.x, L.b, L.wp, 0, partial, d->stream);
    }
    int lrc = 0;
    const int rc = split_launch(d, l, L.x, L.ghostA, 0, bhi, [&](int b0, int b1) {
        lrc = lrc ? lrc : launch_spmv_range(L.A, b0, b1, SSS_HIP_SPMV_RESID, -1.0, L.x, L.b, L.wp, partial, d->stream);
    });
    return rc ? rc : lrc;
}

struct HookCtx {
    sss_hip_dist *d;
    int l;
};
int hook_exchange(void *ctx, double *vec)
{
    auto *h = static_cast<HookCtx *>(ctx);
    return exchange(h->d, h->l, vec);
}

int smooth(sss_hip_dist *d, int l, int post, ResidFuse *rf = nullptr, bool x_zero = false)
{
    DLevel &L = d->L[l];
    HookCtx hc{d, l};
    PassHooks hk;
    hk.ctx = &hc;
    hk.exchange = hook_exchange;
    hk.split = [d, l](double *vec, int blo, int bhi, const std::function<void(int, int)> &launch) {
        return split_launch(d, l, vec, d->L[l].ghostA, blo, bhi, launch);
    };
    hk.w0 = L.w0;
    hk.w1 = L.w1;
    const int sweeps = post ? d->pars.post_iter : d->pars.pre_iter;
    return smoother_run(L.sm, L.A, L.b, L.x, sweeps, d->stream, &hk, rf, nullptr, x_zero);
}

// Sum of n doubles over the ranks, on the host (set-up time only).
int allreduce_host(sss_hip_dist *d, double *v, int n)
{
    sss_hip_comm *c = d->comm;
    if (c->timing) return 0;
    if (c->host) return c->t.allreduce_sum(c->t.ctx, v, n) ? ERROR_MISC : 0;
    double *dv = dev_alloc<double>((size_t)n);
    if (!dv) return ERROR_MISC;
    int rc = 0;
    if (hipMemcpyAsync(dv, v, sizeof(double) * n, hipMemcpyHostToDevice, d->stream) != hipSuccess) rc = ERROR_MISC;
    ncclResult_t r = rc ? ncclSuccess : ncclAllReduce(dv, dv, (size_t)n, ncclDouble, ncclSum, c->nccl, d->stream);
    if (r != ncclSuccess) rc = nccl_fail(r, "ncclAllReduce (set-up)");
    if (!rc && (hipMemcpyAsync(v, dv, sizeof(double) * n, hipMemcpyDeviceToHost, d->stream) != hipSuccess ||
                hipStreamSynchronize(d->stream) != hipSuccess))
        rc = ERROR_MISC;
    dev_free(dv);
    return rc;
}

// The exact eliminations of the single-GPU cycle, made safe across ranks: the fused C-row residual
// needs no C row coupled to a ghost C row (whose new value would arrive only with the next
// exchange), the dead F-row prolongation no F row coupled to a ghost F row (a neighbour would read
// the skipped correction), and the zero-first pass (which also skips its exchange) finite values --
// each agreed over every rank so all ranks run the same exchanges.
int agree_eliminations(sss_hip_dist *d, const PartPlan &plan)
{
    const int nagg = d->nagg;
    std::vector<double> veto((size_t)3 * nagg, 0.0);
    for (int l = 0; l < nagg; ++l) {
        const PartLevel &P = plan.L[l];
        SmootherPlan &sp = d->L[l].sm;
        const int *rp = P.A.rp.data(), *ci = P.A.ci.data();
        bool c_ghost_c = false, f_ghost_f = false;
        for (int c = 0; c < 2; ++c)
            for (int i = sp.pass[c].lo; i < sp.pass[c].hi && sp.pass[c].nrows > 0; ++i)
                for (int k = rp[i]; k < rp[i + 1]; ++k)
                    if (ci[k] >= P.m && P.gclass[ci[k] - P.m] == c) (c ? c_ghost_c : f_ghost_f) = true;
        veto[3 * l + 0] = sp.finite ? 0.0 : 1.0;
        veto[3 * l + 1] = (sp.fuse_resid && !c_ghost_c) ? 0.0 : 1.0;
        veto[3 * l + 2] = (sp.f_overwritten && !f_ghost_f) ? 0.0 : 1.0;
    }
    int rc = allreduce_host(d, veto.data(), (int)veto.size());
    if (rc) return rc;
    for (int l = 0; l < nagg; ++l) {
        SmootherPlan &sp = d->L[l].sm;
        sp.finite = veto[3 * l + 0] == 0.0;
        sp.fuse_resid = veto[3 * l + 1] == 0.0;
        sp.f_overwritten = veto[3 * l + 2] == 0.0;
        sp.pend_ok = false;
    }
    return 0;
}

int allgather_coarse(sss_hip_dist *d)
{
    sss_hip_comm *c = d->comm;
    const hipStream_t s = d->stream;
    if (!c->host) {
        if (c->timing) {   // this rank's own part only
            if (d->nc_own > 0)
                SSS_HIP(hipMemcpyAsync(d->d_call + d->displs[c->rank], d->d_cown, sizeof(double) * d->nc_own,
                                       hipMemcpyDeviceToDevice, s));
            return 0;
        }
        SSS_NCCL(ncclGroupStart());
        for (int q = 0; q < c->nranks; ++q) {
            if (q == c->rank) continue;
            if (d->nc_own > 0) SSS_NCCL(ncclSend(d->d_cown, (size_t)d->nc_own, ncclDouble, q, c->nccl, s));
            if (d->counts[q] > 0)
                SSS_NCCL(ncclRecv(d->d_call + d->displs[q], (size_t)d->counts[q], ncclDouble, q, c->nccl, s));
        }
        SSS_NCCL(ncclGroupEnd());
        if (d->nc_own > 0)
            SSS_HIP(hipMemcpyAsync(d->d_call + d->displs[c->rank], d->d_cown, sizeof(double) * d->nc_own,
                                   hipMemcpyDeviceToDevice, s));
        return 0;
    }
    d->h_cown.resize(std::max(d->nc_own, 1));
    d->h_call.resize(std::max(d->nc_all, 1));
    if (d->nc_own > 0)
        SSS_HIP(hipMemcpyAsync(d->h_cown.data(), d->d_cown, sizeof(double) * d->nc_own, hipMemcpyDeviceToHost, s));
    SSS_HIP(hipStreamSynchronize(s));
    if (c->t.allgatherv(c->t.ctx, d->h_cown.data(), d->nc_own, d->h_call.data(), d->counts.data(), d->displs.data()))
        return ERROR_MISC;
    SSS_HIP(hipMemcpyAsync(d->d_call, d->h_call.data(), sizeof(double) * d->nc_all, hipMemcpyHostToDevice, s));
    SSS_HIP(hipStreamSynchronize(s));
    return 0;
}

// d_norm = {sum of squares, stall flag} -> global sums, on the host: every rank sees a stall on
// any rank and fails with it
int allreduce_norm(sss_hip_dist *d)
{
    sss_hip_comm *c = d->comm;
    if (int rc = launch_err_flag(d->d_err, d->d_norm + 1, d->stream)) return rc;
    if (!c->host && !c->timing) SSS_NCCL(ncclAllReduce(d->d_norm, d->d_norm, 2, ncclDouble, ncclSum, c->nccl, d->stream));
    SSS_HIP(hipMemcpyAsync(d->h_norm, d->d_norm, 2 * sizeof(double), hipMemcpyDeviceToHost, d->stream));
    SSS_HIP(hipStreamSynchronize(d->stream));
    if (c->host && c->t.allreduce_sum(c->t.ctx, d->h_norm, 2)) return ERROR_MISC;
    if (d->h_norm[1] != 0.0) {
        fprintf(stderr, "### ERROR: sss_hip_dist_residual_norm (rank %d): an exact Gauss-Seidel pass stalled on "
                        "the GPU (spin limit reached); the iterate is invalid\n", c->rank);
        return ERROR_MISC;
    }
    return 0;
}

void release(sss_hip_dist *d)
{
    if (!d) return;
    if (d->stream) (void)hipStreamSynchronize(d->stream);
    if (d->cycle_exec) (void)hipGraphExecDestroy(d->cycle_exec);
    for (int l = 0; l < d->nagg; ++l) {
        DLevel &L = d->L[l];
        devcsr_free(L.A);
        devcsr_free(L.P);
        devcsr_free(L.R);
        smoother_free(L.sm);
        dev_free(L.b);
        dev_free(L.x);
        dev_free(L.wp);
        dev_free(L.w0);
        dev_free(L.w1);
        dev_free(L.halo.d_sidx);
        dev_free(L.halo.d_sbuf);
    }
    if (d->tail) sss_hip_hier_destroy(d->tail);
    if (d->own_tail_host) SSS_amg_data_destroy(&d->tail_host);
    dev_free(d->d_cown);
    dev_free(d->d_call);
    dev_free(d->d_tail_perm);
    dev_free(d->partial);
    dev_free(d->d_norm);
    dev_free(d->d_err);
    if (d->h_norm) (void)hipHostFree(d->h_norm);
    for (hipEvent_t e : d->lev_ev) (void)hipEventDestroy(e);
    if (d->stream) (void)hipStreamDestroy(d->stream);
    if (d->cstream) (void)hipStreamDestroy(d->cstream);
    if (d->ev_packed) (void)hipEventDestroy(d->ev_packed);
    if (d->ev_halo) (void)hipEventDestroy(d->ev_halo);
    delete d;
}

int upload_ints(int **dst, const std::vector<int> &src)
{
    *dst = dev_alloc<int>(src.size());
    if (!*dst) return hip_fail(hipErrorOutOfMemory, "hipMalloc", __FILE__, __LINE__);
    if (!src.empty()) SSS_HIP(hipMemcpy(*dst, src.data(), sizeof(int) * src.size(), hipMemcpyHostToDevice));
    return 0;
}

}  // namespace

extern "C" int sss_hip_rccl_unique_id(unsigned char *id)
{
    ncclUniqueId u;
    SSS_NCCL(ncclGetUniqueId(&u));
    std::memcpy(id, u.internal, SSS_HIP_RCCL_ID_BYTES);
    return 0;
}

extern "C" sss_hip_comm *sss_hip_comm_rccl(int nranks, int rank, const unsigned char *id, int device)
{
    if (device >= 0 && hipSetDevice(device) != hipSuccess) return nullptr;
    auto *c = new sss_hip_comm();
    c->nranks = nranks;
    c->rank = rank;
    ncclUniqueId u;
    std::memcpy(u.internal, id, SSS_HIP_RCCL_ID_BYTES);
    ncclResult_t r = ncclCommInitRank(&c->nccl, nranks, u, rank);
    if (r != ncclSuccess) {
        nccl_fail(r, "ncclCommInitRank");
        delete c;
        return nullptr;
    }
    return c;
}

extern "C" sss_hip_comm *sss_hip_comm_host(int nranks, int rank, const sss_hip_host_transport *t)
{
    if (!t || !t->exchange || !t->allreduce_sum || !t->allgatherv) return nullptr;
    auto *c = new sss_hip_comm();
    c->nranks = nranks;
    c->rank = rank;
    c->host = true;
    c->t = *t;
    return c;
}

extern "C" sss_hip_comm *sss_hip_comm_timing(int nranks, int rank)
{
    if (nranks < 1 || rank < 0 || rank >= nranks) return nullptr;
    auto *c = new sss_hip_comm();
    c->nranks = nranks;
    c->rank = rank;
    c->timing = true;
    return c;
}

extern "C" void sss_hip_comm_destroy(sss_hip_comm *c)
{
    if (!c) return;
    if (c->nccl) (void)ncclCommDestroy(c->nccl);
    delete c;
}

// The engine of one rank from its partition `plan` and the replicated tail hierarchy `tailmg`
// (its cg[0] is global level plan.nagg).  Takes ownership of d.  pre_err: a failure this rank met
// before (its partition or tail file unreadable); it still joins the status agreement.
static sss_hip_dist *dist_create_impl(sss_hip_dist *d, PartPlan &plan, const SSS_AMG *tailmg,
                                      const char *pre_err = nullptr)
{
    sss_hip_comm *c = d->comm;
    auto fail = [&](const char *what) {
        fprintf(stderr, "### ERROR: sss_hip_dist_create (rank %d): %s\n", c->rank, what);
        release(d);
        return (sss_hip_dist *)nullptr;
    };
    // Every failure on one rank only (an unreadable or mismatched partition, memory, a level this
    // rank cannot smooth) is recorded, and all ranks agree on the outcome with one collective before
    // the first collective of the set-up, so no rank is left waiting in it.
    const char *err = pre_err;
    if (d->opts.device >= 0 && hipSetDevice(d->opts.device) != hipSuccess && !err) err = "hipSetDevice";
    if (hipStreamCreateWithFlags(&d->stream, hipStreamNonBlocking) != hipSuccess) {
        d->stream = nullptr;   // the agreement then runs on the default stream
        if (!err) err = "stream";
    }
    if (!err && d->pars.cycle_type > 1) err = "only V-cycles are distributed";
    if (!err && (plan.nranks != c->nranks || plan.rank != c->rank)) err = "partition made for another rank layout";
    if (!err && plan.nagg < 1) err = "hierarchy too shallow to partition";
    if (!err && tailmg->num_levels != plan.nl - plan.nagg) err = "tail levels do not match the partition";
    if (!err && (hipStreamCreateWithFlags(&d->cstream, hipStreamNonBlocking) != hipSuccess ||
                 hipEventCreateWithFlags(&d->ev_packed, hipEventDisableTiming) != hipSuccess ||
                 hipEventCreateWithFlags(&d->ev_halo, hipEventDisableTiming) != hipSuccess))
        err = "communication stream";
    if (const char *ov = getenv("SSS_HIP_OVERLAP")) d->overlap = atoi(ov);
    // the cycle is captured into one hipGraph by default over RCCL (SSS_HIP_DIST_GRAPH=0: eager
    // launches); the host transport steers every exchange from the CPU and cannot be captured
    d->use_graph = !c->host;
    if (const char *gz = getenv("SSS_HIP_DIST_GRAPH")) d->use_graph = atoi(gz) != 0 && !c->host;
    if (!err) d->nagg = plan.nagg;

    if (!err) err = [&]() -> const char * {
        // replicated tail first: its level-0 relabeling fixes the column ids of P_{nagg-1}
        sss_hip_opts to = d->opts;
        to.use_graph = 0;
        d->tail = hier_create_impl(tailmg, &to, d->nagg, d->stream);
        if (!d->tail) return "replicated coarse levels";
        const std::vector<int> &tperm = hier_perm(d->tail, 0);
        const int nt = tailmg->cg[0].A.num_rows;
        std::vector<int> tinv;
        if (!tperm.empty()) {
            tinv.resize(nt);
            for (int i = 0; i < nt; ++i) tinv[tperm[i]] = i;
            if (upload_ints(&d->d_tail_perm, tperm)) return "tail perm";
        }
        for (int l = 0; l < d->nagg; ++l) {
            PartLevel &P = plan.L[l];
            DLevel &L = d->L[l];
            L.lo = P.lo;
            L.hi = P.hi;
            L.m = P.m;
            L.g = P.g;
            L.perm = P.perm;
            const int kind = level_kind_of(d->opts, l);
            const int inner = level_inner_of(d->opts, l, plan.cut[l][plan.nranks], plan.gnnz[l]);
            SSS_MAT Av = P.A.view();
            const int enc = level_encoding(d->opts);
            if (devcsr_upload(L.A, Av, P.nF, enc)) return "upload A";
            if (smoother_build(L.sm, Av, P.mark.data(), kind, &L.A, inner, P.gcls.data(), enc)) return "smoother plan";
            for (const auto &ps : L.sm.pass)
                if (ps.nrows > 0 && !ps.range) return "level needs an exact GS-CF chain across ranks (not distributed)";
            if (l + 1 == d->nagg && !tinv.empty())
                for (int &j : P.P.ci) j = tinv[j];
            SSS_MAT Pv = P.P.view(), Rv = P.R.view();
            // (a C-rows-only prolongation keeps the tiles, as hb_level_pr)
            const int tenc = transfer_encoding(d->opts);
            if (devcsr_upload(L.P, Pv, P.nF, L.sm.f_overwritten ? (tenc & ~kEncXell) : tenc) ||
                devcsr_upload(L.R, Rv, -1, restriction_encoding(d->opts)))
                return "upload P/R";
            {   // which row blocks read ghosts (the blockings the uploads made, read back: the
                // column ELL replaces the CSR-adaptive blocking where it is chosen)
                std::vector<int> blk;
                if (device_blocks(L.A, blk)) return "block bounds";
                L.ghostA = block_ghost_flags(P.A, L.m, blk);
                if (device_blocks(L.R, blk)) return "block bounds";
                L.ghostR = block_ghost_flags(P.R, L.m, blk);
                if (device_blocks(L.P, blk)) return "block bounds";
                L.ghostP = block_ghost_flags(P.P, l + 1 < d->nagg ? plan.L[l + 1].m : P.P.cols, blk);
            }
            const size_t nv = (size_t)(L.m + L.g);
            L.b = dev_alloc<double>(nv);
            L.x = dev_alloc<double>(nv);
            L.wp = dev_alloc<double>(nv);
            L.w0 = dev_alloc<double>(nv);
            L.w1 = dev_alloc<double>(nv);
            if (!L.b || !L.x || !L.wp || !L.w0 || !L.w1) return "vectors";
            for (double *v : {L.b, L.x, L.wp, L.w0, L.w1})
                if (hipMemset(v, 0, sizeof(double) * nv) != hipSuccess) return "memset";
            Halo &H = L.halo;
            H.sdst = P.sdst;
            H.scount = P.scount;
            H.rsrc = P.rsrc;
            H.rcount = P.rcount;
            H.nsend = (int)H.sdst.size();
            H.nrecv = (int)H.rsrc.size();
            H.soff.assign(1, 0);
            for (int x : H.scount) H.soff.push_back(H.soff.back() + x);
            H.roff.assign(1, 0);
            for (int x : H.rcount) H.roff.push_back(H.roff.back() + x);
            if (upload_ints(&H.d_sidx, P.sidx)) return "halo";
            H.d_sbuf = dev_alloc<double>(P.sidx.size());
            if (!H.d_sbuf) return "halo buffer";
        }
        // all-gather layout of level nagg
        const auto &cut = plan.cut[d->nagg];
        d->counts.resize(c->nranks);
        d->displs.resize(c->nranks);
        for (int q = 0; q < c->nranks; ++q) {
            d->counts[q] = cut[q + 1] - cut[q];
            d->displs[q] = cut[q];
        }
        d->nc_own = d->counts[c->rank];
        d->nc_all = nt;
        d->d_cown = dev_alloc<double>(d->nc_own);
        d->d_call = dev_alloc<double>(nt);
        d->partial = dev_alloc<double>((size_t)std::max(d->L[0].A.ngrid, 1) + kFinalScratch);
        d->d_norm = dev_alloc<double>(2);
        d->d_err = dev_alloc<unsigned>(1);
        if (!d->d_cown || !d->d_call || !d->partial || !d->d_norm || !d->d_err ||
            hipHostMalloc((void **)&d->h_norm, 2 * sizeof(double)) != hipSuccess ||
            hipMemset(d->d_err, 0, sizeof(unsigned)) != hipSuccess)
            return "buffers";
        // one stall word for every one-launch GS pass of this rank, the replicated tail's included
        for (int l = 0; l < d->nagg; ++l) smoother_set_err(d->L[l].sm, d->d_err);
        hier_set_err_word(d->tail, d->d_err);
        return nullptr;
    }();
    double failed = err ? 1.0 : 0.0;
    if (allreduce_host(d, &failed, 1)) return fail("agreeing the set-up status");
    if (failed > 0.0) return fail(err ? err : "another rank failed its set-up");
    if (agree_eliminations(d, plan)) return fail("agreeing the exact eliminations");
    if (hipStreamSynchronize(d->stream) != hipSuccess) return fail("sync");
    if (!hier_coarse_on_device(d->tail)) d->use_graph = 0;   // a host-steered Krylov coarse solve
    return d;
}

static sss_hip_dist *dist_new(const SSS_AMG_PARS &pars, const sss_hip_opts *o, sss_hip_comm *c)
{
    auto *d = new sss_hip_dist();
    d->comm = c;
    d->pars = pars;
    if (o) d->opts = *o;
    else sss_hip_opts_default(&d->opts);
    return d;
}

extern "C" sss_hip_dist *sss_hip_dist_create(const SSS_AMG *mg, const sss_hip_opts *o, sss_hip_comm *c, int agg_rows)
{
    if (!mg || !c || sss_hip_device_count() <= 0) return nullptr;
    PartPlan plan;
    const char *err = nullptr;
    if (part_plan_build(plan, mg, c->nranks, c->rank, part_agg_rows(agg_rows))) {
        err = "partition";
        plan = PartPlan();
    }
    SSS_AMG sub = *mg;
    sub.cg = mg->cg + plan.nagg;
    sub.num_levels = mg->num_levels - plan.nagg;
    return dist_create_impl(dist_new(mg->pars, o, c), plan, &sub, err);
}

extern "C" sss_hip_dist *sss_hip_dist_create_from_files(const char *prefix, const sss_hip_opts *o, sss_hip_comm *c)
{
    if (!prefix || !c || sss_hip_device_count() <= 0) return nullptr;
    PartPlan plan;
    SSS_AMG_PARS pars;
    std::memset(&pars, 0, sizeof(pars));
    const std::string part = part_file_name(prefix, c->rank), tail = part_tail_name(prefix);
    const char *err = nullptr;
    if (part_plan_read(plan, pars, part.c_str())) {
        fprintf(stderr, "### ERROR: sss_hip_dist_create_from_files (rank %d): cannot read %s\n", c->rank, part.c_str());
        err = "unreadable partition file";
    }
    sss_hip_dist *d = dist_new(pars, o, c);
    if (!err && SSS_amg_load(&d->tail_host, tail.c_str())) {
        fprintf(stderr, "### ERROR: sss_hip_dist_create_from_files (rank %d): cannot read %s\n", c->rank, tail.c_str());
        err = "unreadable tail file";
    } else if (!err) {
        d->own_tail_host = true;
    }
    // a rank that failed here still joins the status agreement of the set-up
    return dist_create_impl(d, plan, &d->tail_host, err);
}

extern "C" void sss_hip_dist_destroy(sss_hip_dist *d) { release(d); }

extern "C" int sss_hip_dist_info(sss_hip_dist *d, int *lo, int *hi, int *nagg, int *nghost0)
{
    if (!d) return ERROR_INPUT_PAR;
    *lo = d->L[0].lo;
    *hi = d->L[0].hi;
    *nagg = d->nagg;
    *nghost0 = d->L[0].g;
    return 0;
}

extern "C" int sss_hip_dist_level_size(sss_hip_dist *d, int l, int *m, int *g, long long *nnz)
{
    if (!d || l < 0 || l >= d->nagg) return ERROR_INPUT_PAR;
    *m = d->L[l].m;
    *g = d->L[l].g;
    *nnz = d->L[l].A.nnz;
    return 0;
}

static double *dist_vec(sss_hip_dist *d, int which)
{
    DLevel &L = d->L[0];
    return which == SSS_HIP_VEC_B ? L.b : which == SSS_HIP_VEC_X ? L.x : which == SSS_HIP_VEC_WP ? L.wp : nullptr;
}

extern "C" int sss_hip_dist_level_flags(sss_hip_dist *d, int l)
{
    if (!d || l < 0 || l >= d->nagg) return ERROR_INPUT_PAR;
    const SmootherPlan &sp = d->L[l].sm;
    return (sp.finite ? 1 : 0) | (sp.fuse_resid ? 2 : 0) | (sp.f_overwritten ? 4 : 0) | (d->cycle_exec ? 8 : 0);
}

extern "C" int sss_hip_dist_upload_vec(sss_hip_dist *d, int which, const double *own, int n)
{
    double *v = dist_vec(d, which);
    DLevel &L = d->L[0];
    if (!v || n != L.m) return ERROR_INPUT_PAR;
    d->resid_c_ready = false;
    d->stage.resize(std::max(n, 1));
    for (int i = 0; i < n; ++i) d->stage[i] = own[L.perm[i] - L.lo];
    SSS_HIP(hipMemcpyAsync(v, d->stage.data(), sizeof(double) * n, hipMemcpyHostToDevice, d->stream));
    SSS_HIP(hipStreamSynchronize(d->stream));
    return 0;
}

extern "C" int sss_hip_dist_download_vec(sss_hip_dist *d, int which, double *own, int n)
{
    double *v = dist_vec(d, which);
    DLevel &L = d->L[0];
    if (!v || n != L.m) return ERROR_INPUT_PAR;
    d->stage.resize(std::max(n, 1));
    SSS_HIP(hipMemcpyAsync(d->stage.data(), v, sizeof(double) * n, hipMemcpyDeviceToHost, d->stream));
    SSS_HIP(hipStreamSynchronize(d->stream));
    for (int i = 0; i < n; ++i) own[L.perm[i] - L.lo] = d->stage[i];
    return 0;
}

static int dist_cycle_enqueue(sss_hip_dist *d);

extern "C" int sss_hip_dist_cycle(sss_hip_dist *d)
{
    d->resid_c_ready = false;
    if (d->use_graph && !d->cycle_exec) {
        // capture once; any failure (a call the capture cannot take) falls back to eager launches
        const hipStream_t s = d->stream;
        SSS_HIP(hipStreamSynchronize(s));
        hipGraph_t g = nullptr;
        int rc = hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal) == hipSuccess ? 0 : ERROR_MISC;
        if (!rc) {
            rc = dist_cycle_enqueue(d);
            d->graph_resid_ready = d->resid_c_ready;
            const hipError_t e = hipStreamEndCapture(s, &g);
            if (!rc && e != hipSuccess) rc = ERROR_MISC;
        }
        hipGraphExec_t ex = nullptr;
        if (!rc && g && hipGraphInstantiate(&ex, g, nullptr, nullptr, 0) != hipSuccess) rc = ERROR_MISC;
        if (g) (void)hipGraphDestroy(g);
        (void)hipGetLastError();
        if (rc || !ex) {
            fprintf(stderr, "[sss_hip] rank %d: the distributed cycle could not be captured; eager launches\n",
                    d->comm->rank);
            d->use_graph = 0;
            return dist_cycle_enqueue(d);
        }
        d->cycle_exec = ex;
    }
    if (d->cycle_exec) {
        SSS_HIP(hipGraphLaunch(d->cycle_exec, d->stream));
        d->resid_c_ready = d->graph_resid_ready;
        return 0;
    }
    return dist_cycle_enqueue(d);
}

static int dist_cycle_enqueue(sss_hip_dist *d)
{
    const hipStream_t s = d->stream;
    const int nagg = d->nagg;
    int rc;
    d->resid_c_ready = false;
    // per-level timing (eager cycles only): event k marks the end of step k -- descent of level
    // 0 .. nagg-1, the replicated tail, ascent of level nagg-1 .. 0
    const bool tev = !d->lev_ev.empty();
    int ek = 0;
    auto mark = [&]() -> int {
        if (tev) SSS_HIP(hipEventRecord(d->lev_ev[(size_t)++ek], s));
        return 0;
    };
    if (tev) SSS_HIP(hipEventRecord(d->lev_ev[0], s));
    for (int l = 0; l < nagg; ++l) {   // descent
        if (l > 0 && (rc = mark())) return rc;
        TraceRange tr("rank %d level %d descent", d->comm->rank, l);
        DLevel &L = d->L[l];
        ResidFuse rf;   // the last C pass may form the residual's C rows (then only F rows remain)
        rf.r = L.wp;
        if ((rc = smooth(d, l, 0, &rf, l > 0))) return rc;   // levels >= 1 were just zeroed
        if ((rc = residual(d, l, rf.done, nullptr))) return rc;
        double *rdst = l + 1 < nagg ? d->L[l + 1].b : d->d_cown;   // restriction wp -> coarse b
        if (!L.R.wave_rows && !L.R.vec_rows) {
            int lrc = 0;
            rc = split_launch(d, l, L.wp, L.ghostR, 0, L.R.nblk, [&](int b0, int b1) {
                lrc = lrc ? lrc : launch_spmv_range(L.R, b0, b1, SSS_HIP_SPMV_MXY, 1.0, L.wp, nullptr, rdst, nullptr, s);
            });
            rc = rc ? rc : lrc;
        } else if (!(rc = exchange(d, l, L.wp))) {
            rc = launch_spmv(L.R, SSS_HIP_SPMV_MXY, 1.0, L.wp, nullptr, rdst, 0, nullptr, s);
        }
        if (rc) return rc;
        if (l + 1 < nagg) {
            DLevel &C = d->L[l + 1];
            SSS_HIP(hipMemsetAsync(C.x, 0, sizeof(double) * (size_t)(C.m + C.g), s));
        } else {
            if ((rc = allgather_coarse(d))) return rc;
            double *tb = hier_vec(d->tail, 0, SSS_HIP_VEC_B), *tx = hier_vec(d->tail, 0, SSS_HIP_VEC_X);
            if (d->d_tail_perm)
                hipLaunchKernelGGL(gather_kernel, dim3((d->nc_all + 255) / 256), dim3(256), 0, s, d->nc_all,
                                   d->d_tail_perm, d->d_call, tb);
            else
                SSS_HIP(hipMemcpyAsync(tb, d->d_call, sizeof(double) * d->nc_all, hipMemcpyDeviceToDevice, s));
            SSS_HIP(hipMemsetAsync(tx, 0, sizeof(double) * (size_t)d->nc_all, s));
        }
    }
    if ((rc = mark())) return rc;
    {
        TraceRange tr("rank %d replicated tail", d->comm->rank);
        if ((rc = sss_hip_cycle(d->tail))) return rc;   // replicated levels, same stream
    }
    if ((rc = mark())) return rc;
    for (int l = nagg - 1; l >= 0; --l) {           // ascent
        if (l < nagg - 1 && (rc = mark())) return rc;
        TraceRange tr("rank %d level %d ascent", d->comm->rank, l);
        DLevel &L = d->L[l];
        double *xc = l + 1 < nagg ? d->L[l + 1].x : hier_vec(d->tail, 0, SSS_HIP_VEC_X);
        // dead F-row correction (see walk_cycle in sss_hier.hip): prolong into the C rows only
        const bool tile = !L.P.wave_rows && !L.P.vec_rows;
        const bool dead_f = L.sm.f_overwritten && d->pars.post_iter > 0 && L.P.split_row == L.sm.pass[0].hi &&
                            L.P.split_row > 0 && tile;
        int lrc = 0;
        auto prolong = [&](int b0, int b1) {
            lrc = lrc ? lrc : launch_spmv_range(L.P, b0, b1, SSS_HIP_SPMV_AMXPY, 1.0, xc, nullptr, L.x, nullptr, s);
        };
        if (l + 1 < nagg && tile) {   // the coarse correction's halo overlaps the interior blocks
            rc = split_launch(d, l + 1, xc, L.ghostP, dead_f ? L.P.split_blk : 0, L.P.nblk, prolong);
        } else {
            if (l + 1 < nagg && (rc = exchange(d, l + 1, xc))) return rc;
            if (dead_f) prolong(L.P.split_blk, L.P.nblk);
            else rc = launch_spmv(L.P, SSS_HIP_SPMV_AMXPY, 1.0, xc, nullptr, L.x, 0, nullptr, s);
        }
        if (rc || (rc = lrc)) return rc;
        if (l == 0 && L.sm.fuse_resid && d->pars.post_iter > 0) {   // outer residual's C rows
            ResidFuse rf;
            rf.r = L.wp;
            rf.partial = d->partial;
            if ((rc = smooth(d, l, 1, &rf))) return rc;
            d->resid_c_ready = rf.done;
        } else if ((rc = smooth(d, l, 1))) {
            return rc;
        }
    }
    return mark();
}

// Timing of this rank's cycle (for the per-rank compute floor with sss_hip_comm_timing): *cycle_ms =
// the cycle as it runs (the captured graph when there is one), averaged over reps; level_ms[l] (l <
// nagg) = level l's descent + ascent and level_ms[nagg] = the replicated tail, from reps eager cycles
// with an event between the steps (launch gaps included).  Advances the iterate.
extern "C" int sss_hip_dist_time_levels(sss_hip_dist *d, int reps, double *cycle_ms, double *level_ms, int nslots)
{
    if (!d || reps < 1 || nslots < d->nagg + 1) return ERROR_INPUT_PAR;
    const int nagg = d->nagg;
    const hipStream_t s = d->stream;
    hipEvent_t e0, e1;
    SSS_HIP(hipEventCreate(&e0));
    SSS_HIP(hipEventCreate(&e1));
    int rc = sss_hip_dist_cycle(d);   // (captures the graph on first use)
    if (!rc && hipStreamSynchronize(s) != hipSuccess) rc = ERROR_MISC;
    if (!rc && hipEventRecord(e0, s) != hipSuccess) rc = ERROR_MISC;
    for (int r = 0; r < reps && !rc; ++r) rc = sss_hip_dist_cycle(d);
    float ms = 0.0f;
    if (!rc && (hipEventRecord(e1, s) != hipSuccess || hipEventSynchronize(e1) != hipSuccess ||
                hipEventElapsedTime(&ms, e0, e1) != hipSuccess))
        rc = ERROR_MISC;
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    if (rc) return rc;
    *cycle_ms = ms / reps;
    d->lev_ev.assign((size_t)2 * nagg + 2, nullptr);
    for (auto &e : d->lev_ev)
        if (hipEventCreate(&e) != hipSuccess) rc = ERROR_MISC;
    std::vector<double> acc((size_t)nagg + 1, 0.0);
    for (int r = 0; r < reps && !rc; ++r) {
        rc = dist_cycle_enqueue(d);
        if (!rc && hipStreamSynchronize(s) != hipSuccess) rc = ERROR_MISC;
        auto seg = [&](int a, int b) {
            float t = 0.0f;
            if (hipEventElapsedTime(&t, d->lev_ev[(size_t)a], d->lev_ev[(size_t)b]) != hipSuccess) rc = ERROR_MISC;
            return (double)t;
        };
        for (int l = 0; l < nagg && !rc; ++l) {
            acc[(size_t)l] += seg(l, l + 1);                                       // descent
            const int k = nagg + 1 + (nagg - 1 - l);                               // ascent of level l
            acc[(size_t)l] += seg(k, k + 1);
        }
        if (!rc) acc[(size_t)nagg] += seg(nagg, nagg + 1);
    }
    for (hipEvent_t e : d->lev_ev)
        if (e) (void)hipEventDestroy(e);
    d->lev_ev.clear();
    if (rc) return rc;
    for (int l = 0; l <= nagg; ++l) level_ms[l] = acc[(size_t)l] / reps;
    return 0;
}

// The replicated tail's own per-level times (sss_hip_time_levels on it; the rank's iterate advances)
extern "C" int sss_hip_dist_time_tail_levels(sss_hip_dist *d, int reps, double *level_ms, int nslots)
{
    if (!d || !d->tail) return ERROR_INPUT_PAR;
    return sss_hip_time_levels(d->tail, reps, level_ms, nslots);
}

// Halo exchanges enqueued per partitioned level since the last reset, and the doubles this rank
// sent in them (a captured cycle counts once, at its capture); nc_own / nc_all: the all-gather
// into the replicated tail (own and all rows of its first level); tail_levels: the replicated levels.
extern "C" int sss_hip_dist_halo_stats(sss_hip_dist *d, long long *calls, long long *doubles, int nslots, int reset,
                                       int *nc_own, int *nc_all, int *tail_levels)
{
    if (!d || nslots < d->nagg) return ERROR_INPUT_PAR;
    for (int l = 0; l < d->nagg; ++l) {
        calls[l] = d->ex_calls[l];
        doubles[l] = d->ex_doubles[l];
        if (reset) d->ex_calls[l] = d->ex_doubles[l] = 0;
    }
    *nc_own = d->nc_own;
    *nc_all = d->nc_all;
    *tail_levels = sss_hip_num_levels(d->tail);
    return 0;
}

extern "C" int sss_hip_dist_residual_norm(sss_hip_dist *d, double *absres)
{
    DLevel &L = d->L[0];
    // C rows and their partials may have come with the cycle's last pass
    int rc = residual(d, 0, d->resid_c_ready, d->partial);
    d->resid_c_ready = false;
    if (rc) return rc;
    if ((rc = launch_final_sum(d->partial, L.A.ngrid, d->d_norm, false, d->stream))) return rc;
    if ((rc = allreduce_norm(d))) return rc;
    *absres = std::sqrt(d->h_norm[0]);
    return 0;
}

extern "C" int sss_hip_dist_time_level0_spmv(sss_hip_dist *d, int reps, double *avg_ms)
{
    DLevel &L = d->L[0];
    hipEvent_t e0, e1;
    SSS_HIP(hipEventCreate(&e0));
    SSS_HIP(hipEventCreate(&e1));
    d->resid_c_ready = false;   // overwrites wp
    SSS_HIP(hipStreamSynchronize(d->stream));
    SSS_HIP(hipEventRecord(e0, d->stream));
    for (int r = 0; r < reps; ++r) {
        int rc = launch_spmv(L.A, SSS_HIP_SPMV_RESID, -1.0, L.x, L.b, L.wp, 0, nullptr, d->stream);
        if (rc) return rc;
    }
    SSS_HIP(hipEventRecord(e1, d->stream));
    SSS_HIP(hipEventSynchronize(e1));
    float ms = 0.f;
    SSS_HIP(hipEventElapsedTime(&ms, e0, e1));
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    *avg_ms = (double)ms / reps;
    return 0;
}

extern "C" int sss_hip_dist_sync(sss_hip_dist *d)
{
    SSS_HIP(hipStreamSynchronize(d->stream));
    return 0;
}
