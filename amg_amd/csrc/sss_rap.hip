// sss_rap.hip — the Galerkin product A_c = R A P of the setup on the GPU, bit for bit the
// reference's SSS_blas_mat_rap (SSS_matvec.c:398-534; host restatement amg_amd/host/sss_setup.c).
//
// The reference builds coarse row ic by walking, in order, every R entry (q1), every A entry of
// that fine row (q2) and every P entry of the reached fine row (q3), and
//   * the diagonal (ic, ic) is the row's first entry, starting from 0.0 (every product adds),
//   * any other column takes the row's next slot on its first product (assigned), later products
//     of that column add (+=), in walk order,
//   * ra = r * a, rap = ra * p (two roundings, no contraction).
// Its A-marker only skips re-checking columns it has already met, so "first product of a column
// opens a slot, every later one adds" is the whole rule.
//
// Here G lanes walk one coarse row: the (q1, q2) steps go in order, the P row of each step is
// spread over the G lanes (its columns are distinct, so no slot is touched twice in one step and
// every slot still receives its products in walk order).  New columns of a step take consecutive
// slots in q3 order (a ballot prefix).  Columns -> slots live in an LDS hash table per row, values
// and columns in LDS slot arrays; pass 0 counts each row's slots, pass 1 (after the host prefix
// sum) fills the rows.  A row with more slots than its table holds is retried with a larger
// per-row table, and the few left after the largest one are built on the host (the same walk).
#include "sss_engine.hpp"

#include <cstring>
#include <memory>
#include <mutex>
#include <numeric>

namespace sss {

namespace {

constexpr unsigned kEmpty = 0xffffffffu;

__device__ __forceinline__ unsigned rap_hash(unsigned c, int hs) { return (c * 0x9E3779B1u) >> 7 & (unsigned)(hs - 1); }

// One launch: rows list[0 .. nrows) (coarse row ids), G lanes per row, VS slots per row.
// MODE 0: cnt[t] = the row's slot count, or -1 if it needs more than VS slots.
// MODE 1: the row written at C[start[row] ..) (cols, vals).
template <int G, int VS, int RPB, int MODE>
__global__ __launch_bounds__(G * RPB) void rap_rows(int nrows, const int *__restrict__ list, const int *__restrict__ rrp,
                                                const int *__restrict__ rci, const double *__restrict__ rv,
                                                const int *__restrict__ arp, const int *__restrict__ aci,
                                                const double *__restrict__ av, const int *__restrict__ prp,
                                                const int *__restrict__ pci, const double *__restrict__ pv,
                                                int *__restrict__ cnt, const long long *__restrict__ start,
                                                int *__restrict__ cci, double *__restrict__ cval)
{
    constexpr int HS = 2 * VS;
    __shared__ unsigned hkey[RPB][HS];
    __shared__ int hslot[RPB][HS];
    __shared__ int scol[RPB][MODE == 1 ? VS : 1];
    __shared__ double sval[RPB][MODE == 1 ? VS : 1];
    const int lane = threadIdx.x & 63, g = threadIdx.x / G, gl = threadIdx.x % G;
    const int gbase = lane - gl;   // first lane of this row's group within the wave
    const unsigned long long gmask = (G == 64 ? ~0ull : ((1ull << G) - 1)) << gbase;
    const int t = blockIdx.x * RPB + g;
    const bool live = t < nrows;
    const int ic = live ? (list ? list[t] : t) : 0;
    unsigned *hk = hkey[g];
    int *hs = hslot[g];
    for (int k = gl; k < HS; k += G) hk[k] = kEmpty;
    __syncthreads();
    int nslots = 0;
    bool over = false;
    if (live) {
        // the diagonal: slot 0, value 0.0
        if (gl == 0) {
            const unsigned h = rap_hash((unsigned)ic, HS);
            hk[h] = (unsigned)ic;
            hs[h] = 0;
            if (MODE == 1) scol[g][0] = ic, sval[g][0] = 0.0;
        }
        nslots = 1;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        for (int q1 = rrp[ic]; q1 < rrp[ic + 1] && !over; ++q1) {
            const double r = rv[q1];
            const int i1 = rci[q1];
            const int a0 = arp[i1], a1 = arp[i1 + 1];
            for (int ab = a0; ab < a1 && !over; ab += G) {
                // this chunk's A entries and their P row bounds, one per lane
                int i2 = 0, p0 = 0, p1 = 0;
                double a = 0.0;
                if (ab + gl < a1) {
                    i2 = aci[ab + gl];
                    a = av[ab + gl];
                    p0 = prp[i2];
                    p1 = prp[i2 + 1];
                }
                const int ne = min(G, a1 - ab);
                for (int e = 0; e < ne && !over; ++e) {
                    const double ae = __shfl(a, gbase + e, 64);
                    const int e0 = __shfl(p0, gbase + e, 64), e1 = __shfl(p1, gbase + e, 64);
                    const double ra = r * ae;
                    for (int pb = e0; pb < e1; pb += G) {
                        const int q3 = pb + gl;
                        const bool act = q3 < e1;
                        unsigned col = 0;
                        double rap = 0.0;
                        if (act) {
                            col = (unsigned)pci[q3];
                            if (MODE == 1) rap = ra * pv[q3];
                        }
                        // look the column up (read-only in this phase)
                        int slot = -1;
                        unsigned h = rap_hash(col, HS);
                        if (act) {
                            for (;;) {
                                const unsigned k = hk[h];
                                if (k == col) {
                                    slot = hs[h];
                                    break;
                                }
                                if (k == kEmpty) break;
                                h = (h + 1) & (HS - 1);
                            }
                        }
                        const bool fresh = act && slot < 0;
                        const unsigned long long m = __ballot(fresh) & gmask;
                        const int nnew = __popcll(m);
                        if (nslots + nnew > VS) {
                            over = true;
                            break;
                        }
                        __builtin_amdgcn_wave_barrier();
                        if (fresh) {
                            slot = nslots + __popcll(m & ((1ull << lane) - 1));
                            for (;;) {   // claim an empty bucket from h on (keys of one step are distinct)
                                const unsigned old = atomicCAS(&hk[h], kEmpty, col);
                                if (old == kEmpty) break;
                                h = (h + 1) & (HS - 1);
                            }
                            hs[h] = slot;
                            if (MODE == 1) scol[g][slot] = (int)col, sval[g][slot] = rap;
                        } else if (act && MODE == 1) {
                            sval[g][slot] += rap;
                        }
                        nslots += nnew;
                        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                        __builtin_amdgcn_wave_barrier();
                        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                    }
                }
            }
        }
        if (MODE == 0) {
            if (gl == 0) cnt[t] = over ? -1 : nslots;
        } else if (!over) {
            const long long s0 = start[ic];
            for (int k = gl; k < nslots; k += G) {
                cci[s0 + k] = scol[g][k];
                cval[s0 + k] = sval[g][k];
            }
        }
    }
}

struct DevMat {
    int *rp = nullptr, *ci = nullptr;
    double *v = nullptr;
    ~DevMat()
    {
        dev_free(rp);
        dev_free(ci);
        dev_free(v);
    }
    int up(const SSS_MAT &M)
    {
        rp = dev_alloc<int>((size_t)M.num_rows + 1);
        ci = dev_alloc<int>((size_t)std::max(M.num_nnzs, 1));
        v = dev_alloc<double>((size_t)std::max(M.num_nnzs, 1));
        if (!rp || !ci || !v) return hip_fail(hipErrorOutOfMemory, "hipMalloc(RAP operand)", __FILE__, __LINE__);
        if (int rc = h2d(rp, M.row_ptr, sizeof(int) * ((size_t)M.num_rows + 1))) return rc;
        if (M.num_nnzs > 0) {
            if (int rc = h2d(ci, M.col_idx, sizeof(int) * (size_t)M.num_nnzs)) return rc;
            if (int rc = h2d(v, M.val, sizeof(double) * (size_t)M.num_nnzs)) return rc;
        }
        return 0;
    }
};

// the host walk of one coarse row (the reference's, sss_setup.c SSS_blas_mat_rap), for the rows no
// device table holds: count (out == nullptr) or fill at cci/cval.  mark/slot: nc ints, mark[] != ic.
// mk: a marker value no other row walk of this mark array used
int host_row(int ic, int mk, const SSS_MAT &R, const SSS_MAT &A, const SSS_MAT &P, int *mark, int *slot, int *cci,
             double *cval)
{
    int n = 0;
    mark[ic] = mk;
    slot[ic] = 0;
    if (cci) cci[0] = ic, cval[0] = 0.0;
    n = 1;
    for (int q1 = R.row_ptr[ic]; q1 < R.row_ptr[ic + 1]; ++q1) {
        const double r = R.val[q1];
        const int i1 = R.col_idx[q1];
        for (int q2 = A.row_ptr[i1]; q2 < A.row_ptr[i1 + 1]; ++q2) {
            const double ra = r * A.val[q2];
            const int i2 = A.col_idx[q2];
            for (int q3 = P.row_ptr[i2]; q3 < P.row_ptr[i2 + 1]; ++q3) {
                const int i3 = P.col_idx[q3];
                if (mark[i3] != mk) {
                    mark[i3] = mk;
                    slot[i3] = n;
                    if (cci) cci[n] = i3, cval[n] = ra * P.val[q3];
                    ++n;
                } else if (cci) {
                    cval[slot[i3]] += ra * P.val[q3];
                }
            }
        }
    }
    return n;
}

template <int G, int VS, int RPB, int MODE>
void launch_rows(int nrows, const int *list, const DevMat &R, const DevMat &A, const DevMat &P, int *cnt,
                 const long long *start, int *cci, double *cval, hipStream_t st)
{
    if (nrows <= 0) return;
    hipLaunchKernelGGL((rap_rows<G, VS, RPB, MODE>), dim3((nrows + RPB - 1) / RPB), dim3(G * RPB), 0, st, nrows,
                       list, R.rp, R.ci, R.v, A.rp, A.ci, A.v, P.rp, P.ci, P.v, cnt, start, cci, cval);
}
// table configurations, each for the rows the previous one could not hold: lanes per row, slots
// per row (LDS 28 B per slot), rows per workgroup
template <int MODE>
void launch_cfg(int c, int nrows, const int *list, const DevMat &R, const DevMat &A, const DevMat &P, int *cnt,
                const long long *start, int *cci, double *cval, hipStream_t st)
{
    switch (c) {
    case 0: launch_rows<8, 32, 32, MODE>(nrows, list, R, A, P, cnt, start, cci, cval, st); break;
    case 1: launch_rows<16, 128, 16, MODE>(nrows, list, R, A, P, cnt, start, cci, cval, st); break;
    case 2: launch_rows<64, 512, 4, MODE>(nrows, list, R, A, P, cnt, start, cci, cval, st); break;
    default: launch_rows<64, 4096, 1, MODE>(nrows, list, R, A, P, cnt, start, cci, cval, st); break;
    }
}
// copies on the product's own stream (non-blocking: the mirror worker's uploads, which may run
// at the same time on the default stream, neither wait for it nor hold it up)
int copy_sync(void *dst, const void *src, size_t bytes, hipMemcpyKind k, hipStream_t st)
{
    if (bytes == 0) return 0;
    SSS_HIP(hipMemcpyAsync(dst, src, bytes, k, st));
    SSS_HIP(hipStreamSynchronize(st));
    return 0;
}
constexpr int kCfgs = 4;

}  // namespace

}  // namespace sss

using namespace sss;

// A_c = R A P on the current device (see the file header).  C receives SSS_calloc'd arrays (freed
// by SSS_mat_destroy).  Returns 0, or an error code with C untouched (the caller then runs the
// host product).
extern "C" int sss_hip_rap(const SSS_MAT *Rh, const SSS_MAT *Ah, const SSS_MAT *Ph, SSS_MAT *C)
{
    if (sss_hip_device_count() <= 0) return ERROR_MISC;
    const int nc = Rh->num_rows;
    struct Stream {
        hipStream_t s = nullptr;
        ~Stream()
        {
            if (s) (void)hipStreamDestroy(s);
        }
    } stream;
    if (hipStreamCreateWithFlags(&stream.s, hipStreamNonBlocking) != hipSuccess) return ERROR_MISC;
    hipStream_t st = stream.s;
    DevMat R, A, P;
    if (R.up(*Rh) || A.up(*Ah) || P.up(*Ph)) return ERROR_MISC;
    int *cnt = dev_alloc<int>((size_t)std::max(nc, 1));
    int *list = dev_alloc<int>((size_t)std::max(nc, 1));
    if (!cnt || !list) {
        dev_free(cnt);
        dev_free(list);
        return ERROR_MISC;
    }
    // pass 0 over the configurations, each on the rows the previous one could not hold
    std::vector<int> cfg_of((size_t)nc, -1), pending, h_cnt((size_t)std::max(nc, 1));
    std::vector<int> count((size_t)nc, 0);
    int rc = 0;
    const char *ce = getenv("SSS_HIP_RAP_CFGS");   // tests: fewer device tables, more host rows
    const int ncfg = (ce && *ce) ? std::max(0, std::min(kCfgs, atoi(ce))) : kCfgs;
    if (ncfg == 0) pending.resize((size_t)nc), std::iota(pending.begin(), pending.end(), 0);
    for (int c = 0; c < ncfg && !rc; ++c) {
        const int m = c == 0 ? nc : (int)pending.size();
        if (m == 0) break;
        if (c > 0 && copy_sync(list, pending.data(), sizeof(int) * (size_t)m, hipMemcpyHostToDevice, st)) rc = ERROR_MISC;
        launch_cfg<0>(c, m, c == 0 ? nullptr : list, R, A, P, cnt, nullptr, nullptr, nullptr, st);
        if (!rc && (hipGetLastError() != hipSuccess || copy_sync(h_cnt.data(), cnt, sizeof(int) * (size_t)m, hipMemcpyDeviceToHost, st)))
            rc = ERROR_MISC;
        if (rc) break;
        std::vector<int> next;
        for (int t = 0; t < m; ++t) {
            const int ic = c == 0 ? t : pending[t];
            if (h_cnt[t] < 0) next.push_back(ic);
            else cfg_of[ic] = c, count[ic] = h_cnt[t];
        }
        pending.swap(next);
    }
    // rows no table held (wider than 4,096 entries): counted on the host, in parallel chunks
    // (markers: ic while counting, nc + ic while filling)
    std::vector<long long> start((size_t)nc + 1, 0);
    // one (mark, slot) pair of nc-sized arrays per worker, reused over its chunks and both passes
    // (the markers of distinct rows and passes never collide), not one per 64-row chunk
    std::mutex buf_mu;
    std::vector<std::unique_ptr<std::pair<std::vector<int>, std::vector<int>>>> bufs;
    std::vector<std::pair<std::vector<int>, std::vector<int>> *> idle;
    auto host_rows = [&](bool fill) {
        const int np = (int)pending.size();
        parallel_chunks(np, 64, [&](int a, int e) {
            std::pair<std::vector<int>, std::vector<int>> *bf;
            {
                std::lock_guard<std::mutex> lk(buf_mu);
                if (idle.empty()) {
                    bufs.push_back(std::make_unique<std::pair<std::vector<int>, std::vector<int>>>(
                        std::vector<int>((size_t)nc, -1), std::vector<int>((size_t)nc, 0)));
                    idle.push_back(bufs.back().get());
                }
                bf = idle.back();
                idle.pop_back();
            }
            int *mark = bf->first.data(), *slot = bf->second.data();
            for (int t = a; t < e; ++t) {
                const int ic = pending[t];
                if (fill) host_row(ic, nc + ic, *Rh, *Ah, *Ph, mark, slot, C->col_idx + start[ic], C->val + start[ic]);
                else count[ic] = host_row(ic, ic, *Rh, *Ah, *Ph, mark, slot, nullptr, nullptr);
            }
            std::lock_guard<std::mutex> lk(buf_mu);
            idle.push_back(bf);
        });
    };
    if (!rc && !pending.empty()) host_rows(false);
    for (int ic = 0; ic < nc; ++ic) start[ic + 1] = start[ic] + count[ic];
    if (!rc && start[nc] > INT32_MAX) rc = ERROR_MAT_SIZE;
    long long *d_start = nullptr;
    int *d_ci = nullptr;
    double *d_v = nullptr;
    if (!rc) {
        d_start = dev_alloc<long long>((size_t)nc + 1);
        d_ci = dev_alloc<int>((size_t)std::max<long long>(start[nc], 1));
        d_v = dev_alloc<double>((size_t)std::max<long long>(start[nc], 1));
        if (!d_start || !d_ci || !d_v ||
            copy_sync(d_start, start.data(), sizeof(long long) * ((size_t)nc + 1), hipMemcpyHostToDevice, st))
            rc = ERROR_MISC;
    }
    // pass 1 per configuration, on its rows
    for (int c = 0; c < kCfgs && !rc; ++c) {
        std::vector<int> rows;
        for (int ic = 0; ic < nc; ++ic)
            if (cfg_of[ic] == c) rows.push_back(ic);
        if (rows.empty()) continue;
        if (copy_sync(list, rows.data(), sizeof(int) * rows.size(), hipMemcpyHostToDevice, st)) {
            rc = ERROR_MISC;
            break;
        }
        launch_cfg<1>(c, (int)rows.size(), list, R, A, P, nullptr, d_start, d_ci, d_v, st);
        if (hipGetLastError() != hipSuccess) rc = ERROR_MISC;
    }
    if (!rc && hipStreamSynchronize(st) != hipSuccess) rc = ERROR_MISC;
    if (!rc) {
        const int nnz = (int)start[nc];
        C->num_rows = nc;
        C->num_cols = nc;
        C->num_nnzs = nnz;
        C->row_ptr = (int *)SSS_calloc((size_t)nc + 1, sizeof(int));
        C->col_idx = (int *)SSS_calloc((size_t)std::max(nnz, 1), sizeof(int));
        C->val = (double *)SSS_calloc((size_t)std::max(nnz, 1), sizeof(double));
        for (int ic = 0; ic <= nc; ++ic) C->row_ptr[ic] = (int)start[ic];
        if (nnz > 0 && (copy_sync(C->col_idx, d_ci, sizeof(int) * (size_t)nnz, hipMemcpyDeviceToHost, st) ||
                        copy_sync(C->val, d_v, sizeof(double) * (size_t)nnz, hipMemcpyDeviceToHost, st)))
            rc = ERROR_MISC;
        if (!rc && !pending.empty()) host_rows(true);   // the host-built rows
        if (rc) SSS_mat_destroy(C);
    }
    dev_free(cnt);
    dev_free(list);
    dev_free(d_start);
    dev_free(d_ci);
    dev_free(d_v);
    return rc;
}
