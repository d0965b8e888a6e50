// sss_tail.hip — the small coarse levels of a V-cycle in ONE single-workgroup launch.
//
// Below a few thousand rows every smoother pass, residual and transfer of SSS_amg_cycle
// (Solve/SSS_cycle.cu:848-967) is a kernel of ~4-5 us whatever its work: a launch, then a chain of
// dependent loads whose data the previous kernel's workgroups left in other XCDs' L2s
// (profiles/r02_circuit_levels.txt: the G3_circuit stand-in's levels 8-9, 1,629 and 209 rows,
// spend 230 us per V-cycle in ~50 such launches).  From the first level small enough (the "tail",
// see tail_build) down to the coarsest and back, one workgroup of 1,024 threads runs every pass
// itself, __syncthreads() between dependent passes, its data in the CU's own caches.
//
// Each pass computes every row exactly as the per-level kernels do -- the same entries in the same
// stored order from the same starting value, the same divisor rules -- so the iterates are bitwise
// those of the per-level launches (tests/test_gpu_tail.py compares SSS_HIP_TAIL=1 and 0):
//   two-stage C/F-Jacobi smoothing (sss_smooth.hip: zero_first_pass, ts_stage0, ts_inner, the
//   no-copy {x, x2} placement of each class), residual / restriction / prolongation (the tile
//   SpMV epilogues of sss_spmv.hip), and the coarsest solve by the explicit inverse (dense_gemv's
//   lane-strided partial sums and xor-butterfly, sss_coarse_direct.hip).
#include "sss_engine.hpp"
#include "sss_tail.hpp"

namespace sss {

namespace {

constexpr int kTailThreads = 1024;

// acc -/+= v[k] x[ci[k]] in stored order, the loads of 8 entries (columns and values, then their x
// values) issued before their products are summed: two dependent round trips per 8 entries
template <bool SUB, class X>
__device__ __forceinline__ double chain_g(double acc, const int *__restrict__ ci, const double *__restrict__ v, int a,
                                          int e, X x)
{
    constexpr int U = 8;
    for (int k0 = a; k0 < e; k0 += U) {
        int c[U];
        double w[U], xv[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            c[u] = k0 + u < e ? ci[k0 + u] : 0;
            w[u] = k0 + u < e ? v[k0 + u] : 0.0;
        }
#pragma unroll
        for (int u = 0; u < U; ++u) xv[u] = k0 + u < e ? x(c[u]) : 0.0;
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (k0 + u < e) {
                if (SUB) acc -= w[u] * xv[u];
                else acc += w[u] * xv[u];
            }
    }
    return acc;
}
__device__ __forceinline__ double chain_sub_g(double acc, const int *__restrict__ ci, const double *__restrict__ v,
                                              int a, int e, const double *x)
{
    return chain_g<true>(acc, ci, v, a, e, [&](int j) { return x[j]; });
}
__device__ __forceinline__ double chain_add_g(double acc, const int *__restrict__ ci, const double *__restrict__ v,
                                              int a, int e, const double *x)
{
    return chain_g<false>(acc, ci, v, a, e, [&](int j) { return x[j]; });
}
// zero_first_pass's sum over a zero iterate (sss_smooth.hip zero_x_sum)
__device__ __forceinline__ double zero_sum(double t, const int *__restrict__ ci, const double *__restrict__ v, int a,
                                           int e)
{
    if (t == 0.0 && signbit(t))
        for (int k = a; k < e; ++k)
            if (signbit(v[k])) return 0.0;
    return t;
}

// One smoothing call (pre: x_zero, the iterate was just zeroed) of a tail level: smoother_run's
// no-copy two-stage path.  cur[c]: where class c's current values live (x or x2).
__device__ void tail_smooth(const TailLevel &L, int sweeps, bool x_zero)
{
    const int tid = threadIdx.x;
    double *cur[2] = {L.x, L.x};
    for (int sw = 0; sw < sweeps; ++sw) {
        for (int c = 0; c < 2; ++c) {
            const TailPass &ps = L.pass[c];
            const int m = ps.hi - ps.lo;
            if (m <= 0) continue;
            const bool zfirst = x_zero && sw == 0 && c == 0 && L.finite;
            double *prev = cur[c] == L.x ? L.x2 : L.x, *next = cur[c];
            // stage 0 into prev (P_q and y_q), or its zero-iterate form
            for (int q = tid; q < m; q += kTailThreads) {
                const int r = ps.lo + q;
                const int a = ps.nrp[q], sp = ps.split[q], e = ps.nrp[q + 1];
                const double d = L.deff[r];
                double Pq, t, y;
                if (zfirst) {
                    Pq = zero_sum(L.b[r], ps.nci, ps.nv, a, sp);
                    t = zero_sum(Pq, ps.nci, ps.nv, sp, e);
                    y = fabs(d) > SMALLFLOAT ? t / d : 0.0;
                } else {
                    const double *c0 = cur[0], *c1 = cur[1];
                    const int cs = L.csplit;
                    auto xs = [&](int j) { return j < cs ? c0[j] : c1[j]; };
                    double acc = chain_g<true>(L.b[r], ps.nci, ps.nv, a, sp, xs);
                    Pq = acc;
                    acc = chain_g<true>(acc, ps.nci, ps.nv, sp, e, xs);
                    y = fabs(d) > SMALLFLOAT ? acc / d : xs(r);
                }
                ps.P[q] = Pq;
                prev[r] = y;
            }
            __syncthreads();
            for (int st = 0; st < L.inner; ++st) {   // Jacobi-Richardson steps on the lower triangle
                for (int q = tid; q < m; q += kTailThreads) {
                    const int r = ps.lo + q;
                    const double d = L.deff[r];
                    const double acc = chain_sub_g(ps.P[q], ps.lci, ps.lv, ps.lrp[q], ps.lrp[q + 1], prev);
                    next[r] = fabs(d) > SMALLFLOAT ? acc / d : prev[r];
                }
                __syncthreads();
                double *t = prev;
                prev = next;
                next = t;
            }
            cur[c] = prev;
        }
    }
    for (int c = 0; c < 2; ++c)   // an odd number of writes to a class: back into x
        if (cur[c] != L.x)
            for (int r = L.pass[c].lo + tid; r < L.pass[c].hi; r += kTailThreads) L.x[r] = cur[c][r];
    __syncthreads();
}

__global__ __launch_bounds__(kTailThreads) void tail_cycle(const TailLevel *__restrict__ lv, int nlev,
                                                           const double *__restrict__ inv, int nc,
                                                           double *__restrict__ cb, double *__restrict__ cx)
{
    const int tid = threadIdx.x;
    // descent
    for (int l = 0; l < nlev; ++l) {
        const TailLevel &L = lv[l];
        tail_smooth(L, L.pre, true);
        for (int r = tid; r < L.n; r += kTailThreads)   // wp = b - A x
            L.wp[r] = L.b[r] + chain_add_g(0.0, L.aci, L.av, L.arp[r], L.arp[r + 1], L.x) * -1.0;
        __syncthreads();
        double *nb = l + 1 < nlev ? lv[l + 1].b : cb, *nx = l + 1 < nlev ? lv[l + 1].x : cx;
        for (int r = tid; r < L.nc; r += kTailThreads) {   // b_{l+1} = R wp, x_{l+1} = 0
            nb[r] = chain_add_g(0.0, L.rci, L.rv, L.rrp[r], L.rrp[r + 1], L.wp);
            nx[r] = 0.0;
        }
        __syncthreads();
    }
    // coarsest: x = inv b (dense_gemv: lane-strided sums, xor butterfly)
    {
        const int wave = tid >> 6, lane = tid & 63;
        for (int row = wave; row < nc; row += kTailThreads / 64) {
            const double *r = inv + (size_t)row * nc;
            double s = 0.0;
            for (int j = lane; j < nc; j += 64) s += r[j] * cb[j];
            for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off, 64);
            if (lane == 0) cx[row] = s;
        }
        __syncthreads();
    }
    // ascent
    for (int l = nlev - 1; l >= 0; --l) {
        const TailLevel &L = lv[l];
        const double *xc = l + 1 < nlev ? lv[l + 1].x : cx;
        for (int r = tid; r < L.n; r += kTailThreads)   // x += P x_{l+1}
            L.x[r] = L.x[r] + chain_add_g(0.0, L.pci, L.pv, L.prp[r], L.prp[r + 1], xc) * 1.0;
        __syncthreads();
        tail_smooth(L, L.post, false);
    }
}

}  // namespace

int tail_launch(const TailPlan &t, hipStream_t s)
{
    ledger_add(t.ledger_bytes);
    hipLaunchKernelGGL(tail_cycle, dim3(1), dim3(kTailThreads), 0, s, t.d_levels, t.nlev, t.inv, t.nc, t.cb, t.cx);
    SSS_HIP(hipGetLastError());
    return 0;
}

int tail_upload(TailPlan &t, const std::vector<TailLevel> &levels)
{
    t.nlev = (int)levels.size();
    t.d_levels = dev_alloc<TailLevel>(levels.size());
    if (!t.d_levels) return hip_fail(hipErrorOutOfMemory, "hipMalloc(tail)", __FILE__, __LINE__);
    SSS_HIP(hipMemcpy(t.d_levels, levels.data(), sizeof(TailLevel) * levels.size(), hipMemcpyHostToDevice));
    return 0;
}

void tail_free(TailPlan &t)
{
    dev_free(t.d_levels);
    t = TailPlan();
}

}  // namespace sss
