// runs_lab.hip — merged row groups of a long-row Galerkin level (7-pt 400^3 level 6 shape: ~100K
// rows, ~800 entries per row, the 8 rows of a group sharing ~2.8x their columns) in two layouts
// (lab only, not product code):
//   M: the engine's merged groups -- one 32-bit key  col << 4 | row  and one value per entry,
//      lanes strided over the group's entries, x gathered per entry;
//   R: column runs -- one 32-bit key  col << 8 | row mask  per distinct column of the group, the
//      values of a run contiguous; a wave scan of the runs' popcounts places each lane's values,
//      x gathered once per run.
//   hipcc -O3 --offload-arch=gfx950 -ffp-contract=off tools/runs_lab.hip -o tools/runs_lab
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#define CK(x)                                                                                   \
    do {                                                                                        \
        hipError_t e = (x);                                                                     \
        if (e != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e)); exit(1); } \
    } while (0)

constexpr int G = 8;

// M: one wave per group (W waves per group: a contiguous share each), U entries in flight per lane
template <int W>
__global__ __launch_bounds__(256) void kM(int ng, const int *gp, const unsigned *mk, const double *mv, const double *x,
                                          double *y)
{
    constexpr int U = 8;
    __shared__ double red[4][G];
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, gpb = 4 / W;
    const int g = blockIdx.x * gpb + w / W, part = w % W;
    double s[G];
    for (int u = 0; u < G; ++u) s[u] = 0.0;
    if (g < ng) {
        const int a = gp[g], e = gp[g + 1], len = e - a, per = (len + W - 1) / W;
        const int k0 = a + min(len, part * per), k1 = a + min(len, (part + 1) * per);
        for (int k = k0 + lane; k < k1; k += 64 * U) {
            unsigned q[U];
            double v[U];
#pragma unroll
            for (int t = 0; t < U; ++t) {
                const int kk = k + 64 * t;
                q[t] = kk < k1 ? mk[kk] : 0u;
                v[t] = kk < k1 ? mv[kk] : 0.0;
            }
#pragma unroll
            for (int t = 0; t < U; ++t) {
                if (k + 64 * t >= k1) break;
                const double p = v[t] * x[q[t] >> 4];
#pragma unroll
                for (int u = 0; u < G; ++u) s[u] += (q[t] & 15u) == (unsigned)u ? p : 0.0;
            }
        }
    }
#pragma unroll
    for (int u = 0; u < G; ++u)
        for (int off = 32; off > 0; off >>= 1) s[u] += __shfl_xor(s[u], off, 64);
    if (lane == 0)
        for (int u = 0; u < G; ++u) red[w][u] = s[u];
    __syncthreads();
    const int t = threadIdx.x;
    if (t < gpb * G) {
        const int gi = t / G, u = t % G, gg = blockIdx.x * gpb + gi;
        if (gg < ng) {
            double acc = 0.0;
            for (int v = 0; v < W; ++v) acc += red[gi * W + v][u];
            y[gg * G + u] = acc;
        }
    }
}

// R: one wave per group; per iteration 64 runs (one per lane), an inclusive wave scan of their
// popcounts gives each lane its values' offset
__device__ __forceinline__ int wave_incl_scan(int v)
{
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const int t = __shfl_up(v, off, 64);
        if (lane >= off) v += t;
    }
    return v;
}
template <int U>
__global__ __launch_bounds__(256) void kR(int ng, const int *rg, const int *vg, const unsigned *rk, const double *mv,
                                          const double *x, double *y)
{
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int g = blockIdx.x * 4 + w;
    double s[G];
    for (int u = 0; u < G; ++u) s[u] = 0.0;
    if (g < ng) {
        const int a = rg[g], e = rg[g + 1];
        int vb = vg[g];
        for (int t0 = a; t0 < e; t0 += 64 * U) {
            unsigned key[U];
            double xv[U];
            int cnt[U], off[U];
#pragma unroll
            for (int j = 0; j < U; ++j) {
                const int t = t0 + 64 * j + lane;
                key[j] = t < e ? rk[t] : 0u;
            }
#pragma unroll
            for (int j = 0; j < U; ++j) {
                const int t = t0 + 64 * j + lane;
                xv[j] = t < e ? x[key[j] >> 8] : 0.0;
                cnt[j] = __popc(key[j] & 0xffu);
            }
#pragma unroll
            for (int j = 0; j < U; ++j) {
                const int incl = wave_incl_scan(cnt[j]);
                off[j] = vb + incl - cnt[j];
                vb += __shfl(incl, 63, 64);
            }
#pragma unroll
            for (int j = 0; j < U; ++j) {
                const unsigned m = key[j] & 0xffu;
                int k = off[j];
#pragma unroll
                for (int u = 0; u < G; ++u)
                    if (m & (1u << u)) s[u] += mv[k++] * xv[j];
            }
        }
    }
#pragma unroll
    for (int u = 0; u < G; ++u)
        for (int off = 32; off > 0; off >>= 1) s[u] += __shfl_xor(s[u], off, 64);
    if (lane == 0 && g < ng)
        for (int u = 0; u < G; ++u) y[g * G + u] = s[u];
}

int main(int argc, char **argv)
{
    const int n = argc > 1 ? atoi(argv[1]) : 101911;
    const int per_row = argc > 2 ? atoi(argv[2]) : 822;
    const double share = argc > 3 ? atof(argv[3]) : 2.8;
    const int ng = (n + G - 1) / G;
    const int pool = (int)(per_row * G / share);
    std::mt19937 rng(7);
    std::vector<int> gp(1, 0), rg(1, 0), vg(1, 0);
    std::vector<unsigned> mk, rk;
    std::vector<double> mv, rv;
    std::vector<int> cols(pool);
    for (int g = 0; g < ng; ++g) {
        // the group's column pool: clustered around the group's position
        const int center = g * G;
        cols.assign(pool, 0);
        for (int c = 0; c < pool; ++c) {
            long long v = (long long)center + ((long long)(rng() % (2ull * (unsigned)n)) - (long long)n) / 4;
            cols[c] = (int)((v % n + n) % n);
        }
        std::sort(cols.begin(), cols.end());
        cols.erase(std::unique(cols.begin(), cols.end()), cols.end());
        const double p = std::min(1.0, (double)per_row / cols.size());
        std::uniform_real_distribution<double> U01(0, 1);
        for (int c : cols) {
            unsigned mask = 0;
            for (int r = 0; r < G; ++r)
                if (g * G + r < n && U01(rng) < p) mask |= 1u << r;
            if (!mask) continue;
            rk.push_back((unsigned)c << 8 | mask);
            for (int r = 0; r < G; ++r)
                if (mask & (1u << r)) {
                    const double a = 1.0 + 1e-3 * (rng() % 1000);
                    mk.push_back((unsigned)c << 4 | r);
                    mv.push_back(a);
                }
        }
        gp.push_back((int)mk.size());
        rg.push_back((int)rk.size());
        vg.push_back((int)mv.size());
    }
    printf("rows %d, entries %zu (%.0f per row), runs %zu (%.2f entries per run)\n", n, mv.size(),
           (double)mv.size() / n, rk.size(), (double)mv.size() / rk.size());
    int *d_gp, *d_rg, *d_vg;
    unsigned *d_mk, *d_rk;
    double *d_mv, *x, *y1, *y2;
    CK(hipMalloc(&d_gp, gp.size() * 4));
    CK(hipMalloc(&d_rg, rg.size() * 4));
    CK(hipMalloc(&d_vg, vg.size() * 4));
    CK(hipMalloc(&d_mk, mk.size() * 4));
    CK(hipMalloc(&d_rk, rk.size() * 4));
    CK(hipMalloc(&d_mv, mv.size() * 8));
    CK(hipMalloc(&x, (size_t)n * 8));
    CK(hipMalloc(&y1, (size_t)ng * G * 8));
    CK(hipMalloc(&y2, (size_t)ng * G * 8));
    CK(hipMemcpy(d_gp, gp.data(), gp.size() * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_rg, rg.data(), rg.size() * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_vg, vg.data(), vg.size() * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_mk, mk.data(), mk.size() * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_rk, rk.data(), rk.size() * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_mv, mv.data(), mv.size() * 8, hipMemcpyHostToDevice));
    {
        std::vector<double> h(n);
        for (int i = 0; i < n; ++i) h[i] = 1.0 + 1e-4 * (i % 97);
        CK(hipMemcpy(x, h.data(), (size_t)n * 8, hipMemcpyHostToDevice));
    }
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const double bytesM = 12.0 * mv.size() + 4.0 * gp.size() + 8.0 * n * 2;
    const double bytesR = 8.0 * mv.size() + 4.0 * rk.size() + 8.0 * rg.size() + 8.0 * n * 2;
    auto run = [&](const char *name, double bytes, auto launch) {
        for (int i = 0; i < 3; ++i) launch();
        CK(hipDeviceSynchronize());
        const int reps = 20;
        CK(hipEventRecord(e0));
        for (int i = 0; i < reps; ++i) launch();
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        ms /= reps;
        printf("%-22s %8.1f us  %6.0f GB/s of its bytes (%.2f GB)\n", name, ms * 1e3, bytes / (ms * 1e-3) / 1e9, bytes / 1e9);
    };
    run("M merged W=4", bytesM, [&] { hipLaunchKernelGGL(kM<4>, dim3(ng), dim3(256), 0, 0, ng, d_gp, d_mk, d_mv, x, y1); });
    run("M merged W=2", bytesM, [&] { hipLaunchKernelGGL(kM<2>, dim3((ng + 1) / 2), dim3(256), 0, 0, ng, d_gp, d_mk, d_mv, x, y1); });
    run("M merged W=1", bytesM, [&] { hipLaunchKernelGGL(kM<1>, dim3((ng + 3) / 4), dim3(256), 0, 0, ng, d_gp, d_mk, d_mv, x, y1); });
    run("R runs U=1", bytesR, [&] { hipLaunchKernelGGL(kR<1>, dim3((ng + 3) / 4), dim3(256), 0, 0, ng, d_rg, d_vg, d_rk, d_mv, x, y2); });
    run("R runs U=2", bytesR, [&] { hipLaunchKernelGGL(kR<2>, dim3((ng + 3) / 4), dim3(256), 0, 0, ng, d_rg, d_vg, d_rk, d_mv, x, y2); });
    run("R runs U=4", bytesR, [&] { hipLaunchKernelGGL(kR<4>, dim3((ng + 3) / 4), dim3(256), 0, 0, ng, d_rg, d_vg, d_rk, d_mv, x, y2); });
    std::vector<double> a(ng * G), b(ng * G);
    CK(hipMemcpy(a.data(), y1, a.size() * 8, hipMemcpyDeviceToHost));
    CK(hipMemcpy(b.data(), y2, b.size() * 8, hipMemcpyDeviceToHost));
    double md = 0;
    for (size_t i = 0; i < a.size(); ++i) md = std::max(md, std::abs(a[i] - b[i]) / std::max(1e-300, std::abs(a[i])));
    printf("max rel diff M vs R: %.3g\n", md);
    return 0;
}
