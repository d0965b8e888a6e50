// sss_part.hip — host-side row partition of the hierarchy (see sss_part.hpp) and its C ABI
// (sss_part_plan_*, include/sss_hip.h), which the CPU multi-process tests drive without a GPU.
#include "sss_part.hpp"

#include <algorithm>
#include <thread>

#include "../../include/sss_hip.h"

namespace sss {

namespace {

template <class Fn>
void parallel_for(int n, Fn fn)
{
    const int nt = (int)std::max(1u, std::min(32u, std::thread::hardware_concurrency()));
    if (n < (1 << 15) || nt == 1) {
        fn(0, n);
        return;
    }
    std::vector<std::thread> th;
    const int chunk = (n + nt - 1) / nt;
    for (int t = 0; t < nt; ++t) {
        const int lo = t * chunk, hi = std::min(n, lo + chunk);
        if (lo < hi) th.emplace_back(fn, lo, hi);
    }
    for (auto &t : th) t.join();
}

struct ColMap {   // global id of one level -> local id of this rank
    int lo = 0, hi = 0, m = 0;
    const std::vector<int> *inv = nullptr;      // own: global - lo -> local
    const std::vector<int> *ghosts = nullptr;   // ascending
    int operator()(int j) const
    {
        if (j >= lo && j < hi) return (*inv)[j - lo];
        return m + (int)(std::lower_bound(ghosts->begin(), ghosts->end(), j) - ghosts->begin());
    }
};

// rows taken in order `rows` (global ids of M), columns mapped by `cmap` (identity if null)
template <class Map>
void take_rows(const SSS_MAT &M, const std::vector<int> &rows, int ncols, Map cmap, HostMat &out)
{
    const int nr = (int)rows.size();
    out.rows = nr;
    out.cols = ncols;
    out.rp.assign((size_t)nr + 1, 0);
    for (int i = 0; i < nr; ++i) out.rp[i + 1] = out.rp[i] + (M.row_ptr[rows[i] + 1] - M.row_ptr[rows[i]]);
    out.ci.resize((size_t)out.rp[nr]);
    out.v.resize((size_t)out.rp[nr]);
    parallel_for(nr, [&](int a, int b) {
        for (int i = a; i < b; ++i) {
            int q = out.rp[i];
            for (int k = M.row_ptr[rows[i]]; k < M.row_ptr[rows[i] + 1]; ++k, ++q) {
                out.ci[q] = cmap(M.col_idx[k]);
                out.v[q] = M.val[k];
            }
        }
    });
}

}  // namespace

int part_plan_build(PartPlan &p, const SSS_AMG *mg, int nranks, int rank, int agg_rows)
{
    const int nl = mg->num_levels, N = nranks;
    if (nl < 1 || N < 1 || rank < 0 || rank >= N) return ERROR_INPUT_PAR;
    p.nranks = N;
    p.rank = rank;
    p.nl = nl;
    int nagg = nl - 1;
    for (int l = 1; l < nl - 1; ++l)
        if (mg->cg[l].A.num_rows <= agg_rows) {
            nagg = l;
            break;
        }
    p.nagg = nagg;
    p.cut.assign((size_t)nagg + 1, std::vector<int>((size_t)N + 1, 0));
    const int n0 = mg->cg[0].A.num_rows;
    for (int q = 0; q <= N; ++q) p.cut[0][q] = (int)((long long)q * n0 / N);
    for (int l = 0; l < nagg; ++l) {   // coarse cut = number of C points before the fine cut
        const SSS_AMG_COMP &C = mg->cg[l];
        const int n = C.A.num_rows;
        if (!C.cfmark.d || C.cfmark.n < n) return ERROR_INPUT_PAR;
        std::vector<int> cpre((size_t)n + 1, 0);
        for (int i = 0; i < n; ++i) cpre[i + 1] = cpre[i] + (C.cfmark.d[i] == 1);
        if (cpre[n] != mg->cg[l + 1].A.num_rows) return ERROR_INPUT_PAR;   // coarse numbering is not cmap
        for (int q = 0; q <= N; ++q) p.cut[l + 1][q] = cpre[p.cut[l][q]];
    }
    p.L.assign((size_t)nagg, PartLevel());

    // pass 1: own rows and their F|C relabeling
    std::vector<std::vector<int>> inv((size_t)nagg);
    for (int l = 0; l < nagg; ++l) {
        PartLevel &P = p.L[l];
        const int *mark = mg->cg[l].cfmark.d;
        P.lo = p.cut[l][rank];
        P.hi = p.cut[l][rank + 1];
        P.m = P.hi - P.lo;
        P.perm.reserve(P.m);
        for (int i = P.lo; i < P.hi; ++i)
            if (mark[i] != 1) P.perm.push_back(i);
        P.nF = (int)P.perm.size();
        for (int i = P.lo; i < P.hi; ++i)
            if (mark[i] == 1) P.perm.push_back(i);
        inv[l].resize(P.m);
        P.mark.resize(P.m);
        for (int k = 0; k < P.m; ++k) {
            inv[l][P.perm[k] - P.lo] = k;
            P.mark[k] = mark[P.perm[k]];
        }
    }

    // pass 2: ghost sets of every rank (own rows of A_l, R_l, P_{l-1}) -> ghosts + halo plan
    for (int l = 0; l < nagg; ++l) {
        PartLevel &P = p.L[l];
        const int n = mg->cg[l].A.num_rows;
        std::vector<int> stamp((size_t)n, -1);
        auto ghost_set = [&](int q) {
            std::vector<int> g;
            const int qlo = p.cut[l][q], qhi = p.cut[l][q + 1];
            auto scan = [&](const SSS_MAT &M, int r0, int r1) {
                for (int i = r0; i < r1; ++i)
                    for (int k = M.row_ptr[i]; k < M.row_ptr[i + 1]; ++k) {
                        const int j = M.col_idx[k];
                        if ((j < qlo || j >= qhi) && stamp[j] != q) {
                            stamp[j] = q;
                            g.push_back(j);
                        }
                    }
            };
            scan(mg->cg[l].A, qlo, qhi);
            scan(mg->cg[l].R, p.cut[l + 1][q], p.cut[l + 1][q + 1]);
            if (l > 0) scan(mg->cg[l - 1].P, p.cut[l - 1][q], p.cut[l - 1][q + 1]);
            std::sort(g.begin(), g.end());
            return g;
        };
        for (int q = 0; q < N; ++q) {
            std::vector<int> g = ghost_set(q);
            if (q == rank) {
                P.ghosts = std::move(g);
                continue;
            }
            auto a = std::lower_bound(g.begin(), g.end(), P.lo), b = std::lower_bound(g.begin(), g.end(), P.hi);
            if (a == b) continue;
            P.sdst.push_back(q);
            P.scount.push_back((int)(b - a));
            for (auto it = a; it != b; ++it) P.sidx.push_back(inv[l][*it - P.lo]);
        }
        P.g = (int)P.ghosts.size();
        for (int q = 0; q < N; ++q) {
            if (q == rank) continue;
            auto a = std::lower_bound(P.ghosts.begin(), P.ghosts.end(), p.cut[l][q]);
            auto b = std::lower_bound(P.ghosts.begin(), P.ghosts.end(), p.cut[l][q + 1]);
            if (a == b) continue;
            P.rsrc.push_back(q);
            P.rcount.push_back((int)(b - a));
        }
        const int *mark = mg->cg[l].cfmark.d;
        P.gcls.resize(P.g);
        P.gclass.resize(P.g);
        for (int k = 0; k < P.g; ++k) {
            P.gclass[k] = mark[P.ghosts[k]] == 1;
            P.gcls[k] = P.ghosts[k] < P.lo ? P.gclass[k] : -1;
        }
    }

    // pass 3: local matrices
    for (int l = 0; l < nagg; ++l) {
        PartLevel &P = p.L[l];
        const SSS_AMG_COMP &C = mg->cg[l];
        ColMap cm{P.lo, P.hi, P.m, &inv[l], &P.ghosts};
        take_rows(C.A, P.perm, P.m + P.g, cm, P.A);
        std::vector<int> crow;   // own coarse rows of R_l in the next level's local order
        if (l + 1 < nagg) {
            crow = p.L[l + 1].perm;
            ColMap cn{p.L[l + 1].lo, p.L[l + 1].hi, p.L[l + 1].m, &inv[l + 1], &p.L[l + 1].ghosts};
            take_rows(C.P, P.perm, p.L[l + 1].m + p.L[l + 1].g, cn, P.P);
        } else {
            for (int c = p.cut[l + 1][rank]; c < p.cut[l + 1][rank + 1]; ++c) crow.push_back(c);
            take_rows(C.P, P.perm, C.P.num_cols, [](int j) { return j; }, P.P);
        }
        take_rows(C.R, crow, P.m + P.g, cm, P.R);
    }
    return 0;
}

}  // namespace sss

struct sss_part_plan {
    sss::PartPlan p;
};

extern "C" sss_part_plan *sss_part_plan_create(const SSS_AMG *mg, int nranks, int rank, int agg_rows)
{
    auto *pp = new sss_part_plan();
    if (sss::part_plan_build(pp->p, mg, nranks, rank, agg_rows > 0 ? agg_rows : 20000)) {
        delete pp;
        return nullptr;
    }
    return pp;
}

extern "C" void sss_part_plan_destroy(sss_part_plan *p) { delete p; }

extern "C" int sss_part_plan_nagg(const sss_part_plan *p) { return p ? p->p.nagg : -1; }

extern "C" int sss_part_plan_level(const sss_part_plan *pp, int l, int *lo, int *hi, int *m, int *g)
{
    const auto &p = pp->p;
    if (l < 0 || l > p.nagg) return ERROR_INPUT_PAR;
    *lo = p.cut[l][p.rank];
    *hi = p.cut[l][p.rank + 1];
    *m = *hi - *lo;
    *g = l < p.nagg ? p.L[l].g : 0;
    return 0;
}

extern "C" int sss_part_plan_matrix(const sss_part_plan *pp, int l, int which, SSS_MAT *out)
{
    const auto &p = pp->p;
    if (l < 0 || l >= p.nagg || which < 0 || which > 2) return ERROR_INPUT_PAR;
    const auto &L = p.L[l];
    *out = (which == 0 ? L.A : which == 1 ? L.P : L.R).view();
    return 0;
}

extern "C" int sss_part_plan_ids(const sss_part_plan *pp, int l, const int **perm, const int **ghosts)
{
    const auto &p = pp->p;
    if (l < 0 || l >= p.nagg) return ERROR_INPUT_PAR;
    *perm = p.L[l].perm.data();
    *ghosts = p.L[l].ghosts.data();
    return 0;
}

extern "C" int sss_part_plan_halo(const sss_part_plan *pp, int l, int *nsend, const int **sdst, const int **scount,
                                  const int **sidx, int *nrecv, const int **rsrc, const int **rcount)
{
    const auto &p = pp->p;
    if (l < 0 || l >= p.nagg) return ERROR_INPUT_PAR;
    const auto &L = p.L[l];
    *nsend = (int)L.sdst.size();
    *sdst = L.sdst.data();
    *scount = L.scount.data();
    *sidx = L.sidx.data();
    *nrecv = (int)L.rsrc.size();
    *rsrc = L.rsrc.data();
    *rcount = L.rcount.data();
    return 0;
}
