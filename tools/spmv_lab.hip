// spmv_lab.hip — standalone variant bench for the level-0 residual SpMV (r = b - A x) on the
// 7-point Poisson operator, natural or red-black (F|C) row order.  Every variant must give
// bitwise the same y as the baseline (sum from 0.0 in CSR order); prints GB/s per variant
// using the algorithmic byte count 12 nnz + 4 (n+1) + 8 n (x) + 8 n (b) + 8 n (y).
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -o tools/spmv_lab tools/spmv_lab.hip
//   tools/spmv_lab 400
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x)                                                                                   \
    do {                                                                                        \
        hipError_t e_ = (x);                                                                    \
        if (e_ != hipSuccess) {                                                                 \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));  \
            exit(1);                                                                            \
        }                                                                                       \
    } while (0)

constexpr int kThreads = 256;
typedef int i2v __attribute__((ext_vector_type(2)));
typedef int i4v __attribute__((ext_vector_type(4)));
typedef double d2v __attribute__((ext_vector_type(2)));

template <int VEC, bool NT, int RPT, bool XCD = false>
__global__ __launch_bounds__(kThreads) void resid(const int *__restrict__ blk, const int *__restrict__ rp,
                                                  const int *__restrict__ ci, const double *__restrict__ v,
                                                  const double *__restrict__ x, const double *__restrict__ b,
                                                  double *__restrict__ y)
{
    constexpr int kTile = 2048 * RPT;
    __shared__ double sm[kTile];
    int bid = blockIdx.x;
    if (XCD) {   // workgroups are dealt round-robin over the 8 XCDs: give each XCD a contiguous run
        const int nb = gridDim.x, per = (nb + 7) / 8, xcd = bid & 7, idx = bid >> 3;
        const int full = nb - 8 * (per - 1);   // XCDs [0, full) own `per` blocks, the rest per-1
        bid = xcd < full ? xcd * per + idx : full * per + (xcd - full) * (per - 1) + idx;
    }
    const int r0 = blk[bid], r1 = blk[bid + 1];
    const int k0 = rp[r0], k1 = rp[r1];
    if (VEC == 9) {   // prefetch the row extent and b before the tile
        const int r = r0 + (int)threadIdx.x;
        int ra = 0, re = 0;
        double br = 0.0;
        if (r < r1) ra = rp[r], re = rp[r + 1], br = b[r];
        for (int kb = k0; kb < k1; kb += 8 * kThreads) {
            int j[8];
            double a[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const int k = kb + u * kThreads + (int)threadIdx.x;
                j[u] = k < k1 ? ci[k] : -1;
                a[u] = k < k1 ? v[k] : 0.0;
            }
            double xv[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) xv[u] = j[u] >= 0 ? x[j[u]] : 0.0;
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const int k = kb + u * kThreads + (int)threadIdx.x;
                if (k < k1) sm[k - k0] = a[u] * xv[u];
            }
        }
        __syncthreads();
        if (r < r1) {
            double s = 0.0;
            for (int k = ra - k0; k < re - k0; ++k) s += sm[k];
            y[r] = br + s * -1.0;
        }
        return;
    }
    if (VEC == 10) {   // no LDS: thread per row, all loads of the row issued first
        const int r = r0 + (int)threadIdx.x;
        if (r >= r1) return;
        const int ra = rp[r], re = rp[r + 1];
        const double br = b[r];
        double s = 0.0;
        for (int kb = ra; kb < re; kb += 8) {
            int j[8];
            double a[8], xv[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                j[u] = kb + u < re ? ci[kb + u] : -1;
                a[u] = kb + u < re ? v[kb + u] : 0.0;
            }
#pragma unroll
            for (int u = 0; u < 8; ++u) xv[u] = j[u] >= 0 ? x[j[u]] : 0.0;
#pragma unroll
            for (int u = 0; u < 8; ++u)
                if (kb + u < re) s += a[u] * xv[u];
        }
        y[r] = br + s * -1.0;
        return;
    }
    if (VEC == 8) {   // all ci/v loads of the thread first, then all x gathers (MLP)
        for (int kb = k0; kb < k1; kb += 8 * kThreads) {
            int j[8];
            double a[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const int k = kb + u * kThreads + (int)threadIdx.x;
                j[u] = k < k1 ? ci[k] : -1;
                a[u] = k < k1 ? v[k] : 0.0;
            }
            double xv[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) xv[u] = j[u] >= 0 ? x[j[u]] : 0.0;
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const int k = kb + u * kThreads + (int)threadIdx.x;
                if (k < k1) sm[k - k0] = a[u] * xv[u];
            }
        }
    } else if (VEC == 1) {
        for (int k = k0 + threadIdx.x; k < k1; k += kThreads) {
            const int j = NT ? __builtin_nontemporal_load(ci + k) : ci[k];
            const double a = NT ? __builtin_nontemporal_load(v + k) : v[k];
            sm[k - k0] = a * x[j];
        }
    } else if (VEC == 2) {
        const int q0 = k0 >> 1, q1 = (k1 + 1) >> 1;
        for (int q = q0 + threadIdx.x; q < q1; q += kThreads) {
            i2v j;
            d2v a;
            if (NT) {
                j = __builtin_nontemporal_load((const i2v *)ci + q);
                a = __builtin_nontemporal_load((const d2v *)v + q);
            } else {
                j = ((const i2v *)ci)[q];
                a = ((const d2v *)v)[q];
            }
            const int k = 2 * q;
            if (k >= k0) sm[k - k0] = a.x * x[j.x];
            if (k + 1 < k1) sm[k + 1 - k0] = a.y * x[j.y];
        }
    } else {
        const int q0 = k0 >> 2, q1 = (k1 + 3) >> 2;
        for (int q = q0 + threadIdx.x; q < q1; q += kThreads) {
            i4v j;
            d2v a, c;
            if (NT) {
                j = __builtin_nontemporal_load((const i4v *)ci + q);
                a = __builtin_nontemporal_load((const d2v *)v + 2 * q);
                c = __builtin_nontemporal_load((const d2v *)v + 2 * q + 1);
            } else {
                j = ((const i4v *)ci)[q];
                a = ((const d2v *)v)[2 * q];
                c = ((const d2v *)v)[2 * q + 1];
            }
            const int k = 4 * q;
            if (k >= k0 && k < k1) sm[k - k0] = a.x * x[j.x];
            if (k + 1 >= k0 && k + 1 < k1) sm[k + 1 - k0] = a.y * x[j.y];
            if (k + 2 >= k0 && k + 2 < k1) sm[k + 2 - k0] = c.x * x[j.z];
            if (k + 3 < k1) sm[k + 3 - k0] = c.y * x[j.w];
        }
    }
    __syncthreads();
#pragma unroll
    for (int t = 0; t < RPT; ++t) {
        const int r = r0 + t * kThreads + (int)threadIdx.x;
        if (r < r1) {
            const int a = rp[r] - k0, e = rp[r + 1] - k0;
            double s = 0.0;
            for (int k = a; k < e; ++k) s += sm[k];
            y[r] = b[r] + s * -1.0;
        }
    }
}

static std::vector<int> blocks(const std::vector<int> &rp, int n, int rows, int tile)
{
    std::vector<int> blk;
    int r = 0;
    while (r < n) {
        blk.push_back(r);
        int e = r + 1;
        while (e < n && e - r < rows && rp[e + 1] - rp[r] <= tile) ++e;
        r = e;
    }
    blk.push_back(n);
    return blk;
}

int main(int argc, char **argv)
{
    const int N = argc > 1 ? atoi(argv[1]) : 400;
    const int reps = argc > 2 ? atoi(argv[2]) : 20;
    const long long n = (long long)N * N * N;
    for (int order = 0; order < 2; ++order) {
        // order 1: red-black (F = odd parity first), i.e. the relabeled level 0
        std::vector<int> newid(n), perm(n);
        if (order == 0)
            for (long long i = 0; i < n; ++i) newid[i] = (int)i, perm[i] = (int)i;
        else {
            long long c = 0;
            for (int par = 1; par >= 0; --par)
                for (long long i = 0; i < n; ++i) {
                    const int ix = i % N, iy = (i / N) % N, iz = i / ((long long)N * N);
                    if (((ix + iy + iz) & 1) == par) newid[i] = (int)c, perm[c++] = (int)i;
                }
        }
        std::vector<int> rp(n + 1), ci;
        std::vector<double> v;
        ci.reserve(7 * n + 8);
        v.reserve(7 * n + 8);
        for (long long r = 0; r < n; ++r) {
            const long long i = perm[r];
            const int ix = i % N, iy = (i / N) % N, iz = i / ((long long)N * N);
            const long long nb[7] = {i - (long long)N * N, i - N, i - 1, i, i + 1, i + N, i + (long long)N * N};
            const bool ok[7] = {iz > 0, iy > 0, ix > 0, true, ix < N - 1, iy < N - 1, iz < N - 1};
            for (int t = 0; t < 7; ++t)
                if (ok[t]) {
                    ci.push_back(newid[nb[t]]);
                    v.push_back(t == 3 ? 6.0 : -1.0);
                }
            rp[r + 1] = (int)ci.size();
        }
        const long long nnz = ci.size();
        for (int p = 0; p < 8; ++p) ci.push_back(0), v.push_back(0.0);   // vector-load padding
        std::vector<double> hx(n), hb(n);
        for (long long i = 0; i < n; ++i) hx[i] = 1.0 + 1e-3 * (double)(i % 977), hb[i] = 1.0;
        int *drp, *dci, *dblk;
        double *dv, *dx, *db, *dy;
        CK(hipMalloc(&drp, sizeof(int) * (n + 1)));
        CK(hipMalloc(&dci, sizeof(int) * ci.size()));
        CK(hipMalloc(&dv, sizeof(double) * v.size()));
        CK(hipMalloc(&dx, sizeof(double) * n));
        CK(hipMalloc(&db, sizeof(double) * n));
        CK(hipMalloc(&dy, sizeof(double) * n));
        CK(hipMemcpy(drp, rp.data(), sizeof(int) * (n + 1), hipMemcpyHostToDevice));
        CK(hipMemcpy(dci, ci.data(), sizeof(int) * ci.size(), hipMemcpyHostToDevice));
        CK(hipMemcpy(dv, v.data(), sizeof(double) * v.size(), hipMemcpyHostToDevice));
        CK(hipMemcpy(dx, hx.data(), sizeof(double) * n, hipMemcpyHostToDevice));
        CK(hipMemcpy(db, hb.data(), sizeof(double) * n, hipMemcpyHostToDevice));
        const double bytes = 12.0 * nnz + 4.0 * (n + 1) + 24.0 * n;
        std::vector<double> yref(n), yv(n);
        hipEvent_t e0, e1;
        CK(hipEventCreate(&e0));
        CK(hipEventCreate(&e1));
        auto run = [&](const char *name, auto kern, int rpt) {
            std::vector<int> blk = blocks(rp, (int)n, kThreads * rpt, 2048 * rpt);
            CK(hipMalloc(&dblk, sizeof(int) * blk.size()));
            CK(hipMemcpy(dblk, blk.data(), sizeof(int) * blk.size(), hipMemcpyHostToDevice));
            const int nb = (int)blk.size() - 1;
            CK(hipMemset(dy, 0, sizeof(double) * n));
            hipLaunchKernelGGL(kern, dim3(nb), dim3(kThreads), 0, 0, dblk, drp, dci, dv, dx, db, dy);
            CK(hipDeviceSynchronize());
            CK(hipEventRecord(e0));
            for (int r = 0; r < reps; ++r)
                hipLaunchKernelGGL(kern, dim3(nb), dim3(kThreads), 0, 0, dblk, drp, dci, dv, dx, db, dy);
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            ms /= reps;
            CK(hipMemcpy(yv.data(), dy, sizeof(double) * n, hipMemcpyDeviceToHost));
            bool same = true;
            if (!strcmp(name, "scalar"))
                yref = yv;
            else
                same = memcmp(yref.data(), yv.data(), sizeof(double) * n) == 0;
            printf("order=%s %-16s blocks=%8d  %.4f ms  %7.1f GB/s  %s\n", order ? "redblack" : "natural ", name, nb,
                   ms, bytes / ms / 1e6, same ? "bitwise-ok" : "MISMATCH");
            fflush(stdout);
            CK(hipFree(dblk));
        };
        run("scalar", resid<1, false, 1>, 1);
        run("scalar-nt", resid<1, true, 1>, 1);
        run("vec2", resid<2, false, 1>, 1);
        run("vec2-nt", resid<2, true, 1>, 1);
        run("vec4", resid<4, false, 1>, 1);
        run("vec4-nt", resid<4, true, 1>, 1);
        run("scalar-xcd", resid<1, false, 1, true>, 1);
        run("vec2-xcd", resid<2, false, 1, true>, 1);
        run("vec4-xcd", resid<4, false, 1, true>, 1);
        run("batch8", resid<8, false, 1>, 1);
        run("batch8-xcd", resid<8, false, 1, true>, 1);
        run("batch8-nt-xcd", resid<8, true, 1, true>, 1);
        run("batch8-pf", resid<9, false, 1>, 1);
        run("batch8-pf-xcd", resid<9, false, 1, true>, 1);
        run("direct", resid<10, false, 1>, 1);
        run("direct-xcd", resid<10, false, 1, true>, 1);
        run("scalar-r2", resid<1, false, 2>, 2);
        run("vec4-r2", resid<4, false, 2>, 2);
        run("vec4-nt-r2", resid<4, true, 2>, 2);
        hipFree(drp), hipFree(dci), hipFree(dv), hipFree(dx), hipFree(db), hipFree(dy);
    }
    return 0;
}
