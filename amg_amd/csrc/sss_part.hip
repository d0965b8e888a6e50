// sss_part.hip — host-side row partition of the hierarchy (see sss_part.hpp) and its C ABI
// (sss_part_plan_*, include/sss_hip.h), which the CPU multi-process tests drive without a GPU.
#include "sss_part.hpp"

#include <algorithm>
#include <atomic>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <string>
#include <thread>

#include "../../include/sss_hip.h"

namespace sss {

constexpr int kMaxPartLevels = max_AMG_LVL;

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

// Partitioned level count and the cuts of every partitioned level (identical for all ranks).
static int part_cuts(const SSS_AMG *mg, int N, int agg_rows, int &nagg, std::vector<std::vector<int>> &cut)
{
    const int nl = mg->num_levels;
    nagg = nl - 1;
    for (int l = 1; l < nl - 1; ++l)
        if (mg->cg[l].A.num_rows <= agg_rows) {
            nagg = l;
            break;
        }
    cut.assign((size_t)nagg + 1, std::vector<int>((size_t)N + 1, 0));
    const int n0 = mg->cg[0].A.num_rows;
    for (int q = 0; q <= N; ++q) cut[0][q] = (int)((long long)q * n0 / N);
    for (int l = 0; l < nagg; ++l) {   // coarse cut = number of C points before the fine cut
        const SSS_AMG_COMP &C = mg->cg[l];
        const int n = C.A.num_rows;
        if (!C.cfmark.d || C.cfmark.n < n) return ERROR_INPUT_PAR;
        std::vector<int> cpre((size_t)n + 1, 0);
        for (int i = 0; i < n; ++i) cpre[i + 1] = cpre[i] + (C.cfmark.d[i] == 1);
        if (cpre[n] != mg->cg[l + 1].A.num_rows) return ERROR_INPUT_PAR;   // coarse numbering is not cmap
        for (int q = 0; q <= N; ++q) cut[l + 1][q] = cpre[cut[l][q]];
    }
    return 0;
}

// Ghost set (ascending global ids) of rank q on level l: the off-rank columns of its own rows of
// A_l, of R_l's coarse rows it owns and of P_{l-1}'s fine rows it owns.
static std::vector<int> ghost_set(const SSS_AMG *mg, const std::vector<std::vector<int>> &cut, int l, int q)
{
    std::vector<int> g;
    const int qlo = cut[l][q], qhi = cut[l][q + 1];
    auto scan = [&](const SSS_MAT &M, int r0, int r1) {
        for (int i = r0; i < r1; ++i)
            for (int k = M.row_ptr[i]; k < M.row_ptr[i + 1]; ++k) {
                const int j = M.col_idx[k];
                if (j < qlo || j >= qhi) g.push_back(j);
            }
    };
    scan(mg->cg[l].A, qlo, qhi);
    scan(mg->cg[l].R, cut[l + 1][q], cut[l + 1][q + 1]);
    if (l > 0) scan(mg->cg[l - 1].P, cut[l - 1][q], cut[l - 1][q + 1]);
    std::sort(g.begin(), g.end());
    g.erase(std::unique(g.begin(), g.end()), g.end());
    return g;
}

// Every rank's ghost sets of every partitioned level, computed once (in parallel over ranks and
// levels) for a partition set: gs[l][q].
using GhostSets = std::vector<std::vector<std::vector<int>>>;
static void all_ghost_sets(const SSS_AMG *mg, const std::vector<std::vector<int>> &cut, int nagg, int N, GhostSets &gs)
{
    gs.assign((size_t)nagg, std::vector<std::vector<int>>((size_t)N));
    const int jobs = nagg * N;
    const int nt = (int)std::max(1u, std::min(32u, std::thread::hardware_concurrency()));
    std::atomic<int> next{0};
    auto work = [&]() {
        for (int t; (t = next.fetch_add(1)) < jobs;) gs[(size_t)(t % nagg)][(size_t)(t / nagg)] = ghost_set(mg, cut, t % nagg, t / nagg);
    };
    std::vector<std::thread> th;
    for (int t = 1; t < std::min(nt, jobs); ++t) th.emplace_back(work);
    work();
    for (auto &t : th) t.join();
}

static int part_plan_build_impl(PartPlan &p, const SSS_AMG *mg, int nranks, int rank, int agg_rows,
                                const GhostSets *pre)
{
    const int nl = mg->num_levels, N = nranks;
    if (nl < 1 || N < 1 || rank < 0 || rank >= N) return ERROR_INPUT_PAR;
    p.nranks = N;
    p.rank = rank;
    p.nl = nl;
    int nagg = 0;
    if (int rc = part_cuts(mg, N, agg_rows, nagg, p.cut)) return rc;
    p.nagg = nagg;
    p.L.assign((size_t)nagg, PartLevel());
    p.gnnz.resize((size_t)nagg);
    for (int l = 0; l < nagg; ++l) p.gnnz[l] = mg->cg[l].A.num_nnzs;

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
        for (int q = 0; q < N; ++q) {
            std::vector<int> g = pre ? (*pre)[(size_t)l][(size_t)q] : ghost_set(mg, p.cut, l, q);
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

int part_agg_rows(int agg_rows)
{
    if (agg_rows > 0) return agg_rows;
    const char *e = getenv("SSS_HIP_AGG_ROWS");
    const int v = (e && *e) ? atoi(e) : 0;
    return v > 0 ? v : kAggRowsDefault;
}

int part_plan_build(PartPlan &p, const SSS_AMG *mg, int nranks, int rank, int agg_rows)
{
    return part_plan_build_impl(p, mg, nranks, rank, agg_rows, nullptr);
}

// The partition files of every rank (one plan in memory at a time), the ghost sets computed once.
int part_save_all(const SSS_AMG *mg, int nranks, int agg_rows, const char *prefix, int &nagg)
{
    std::vector<std::vector<int>> cut;
    if (int rc = part_cuts(mg, nranks, agg_rows, nagg, cut)) return rc;
    if (nagg < 1) return ERROR_INPUT_PAR;
    GhostSets gs;
    all_ghost_sets(mg, cut, nagg, nranks, gs);
    for (int r = 0; r < nranks; ++r) {
        PartPlan plan;
        if (int rc = part_plan_build_impl(plan, mg, nranks, r, agg_rows, &gs)) return rc;
        if (int rc = part_plan_write(plan, mg->pars, part_file_name(prefix, r).c_str())) return rc;
    }
    return 0;
}

}  // namespace sss

namespace sss {

// ---- partition files -------------------------------------------------------------------------
// Layout (little-endian, native LP64):  "SSSPART1"  int32 version=2  int32 sizeof(SSS_AMG_PARS)
//   SSS_AMG_PARS  int32 nranks, rank, nl, nagg;  nagg+1 cut vectors;  int64 vector gnnz;  per level l < nagg:
//   int32 lo, hi, m, g, nF;  int vectors perm, ghosts, mark, gcls, gclass;  matrices A, P, R;
//   int vectors sdst, scount, sidx, rsrc, rcount.   vector := int64 count + data;
//   matrix := int32 rows, cols + int vectors rp, ci + double vector v.
namespace {
const char kPartMagic[8] = {'S', 'S', 'S', 'P', 'A', 'R', 'T', '1'};
constexpr int kPartVersion = 2;

struct Out {
    FILE *f;
    bool bad = false;
    void raw(const void *p, size_t n)
    {
        if (!bad && n && fwrite(p, 1, n, f) != n) bad = true;
    }
    void i32(int v)
    {
        const int32_t x = v;
        raw(&x, sizeof(x));
    }
    template <class T>
    void vec(const std::vector<T> &v)
    {
        const int64_t n = (int64_t)v.size();
        raw(&n, sizeof(n));
        raw(v.data(), sizeof(T) * v.size());
    }
    void mat(const HostMat &m)
    {
        i32(m.rows);
        i32(m.cols);
        vec(m.rp);
        vec(m.ci);
        vec(m.v);
    }
};
struct In {
    FILE *f;
    bool bad = false;
    void raw(void *p, size_t n)
    {
        if (!bad && n && fread(p, 1, n, f) != n) bad = true;
    }
    int i32()
    {
        int32_t x = 0;
        raw(&x, sizeof(x));
        return x;
    }
    template <class T>
    void vec(std::vector<T> &v)
    {
        int64_t n = 0;
        raw(&n, sizeof(n));
        if (bad || n < 0 || n > ((int64_t)1 << 40)) {
            bad = true;
            return;
        }
        v.resize((size_t)n);
        raw(v.data(), sizeof(T) * (size_t)n);
    }
    // a CSR block read back: dimensions, monotone row pointers from 0 and columns in range, so a
    // corrupt or mismatched file is ERROR_WRONG_FILE instead of out-of-bounds device reads
    void mat(HostMat &m)
    {
        m.rows = i32();
        m.cols = i32();
        if (bad || m.rows < 0 || m.cols < 0) {
            bad = true;
            return;
        }
        vec(m.rp);
        vec(m.ci);
        vec(m.v);
        if (bad || m.rp.size() != (size_t)m.rows + 1 || m.ci.size() != m.v.size() || m.rp[0] != 0 ||
            (size_t)m.rp.back() != m.ci.size()) {
            bad = true;
            return;
        }
        for (int i = 0; i < m.rows && !bad; ++i) bad = m.rp[i + 1] < m.rp[i];
        for (size_t k = 0; k < m.ci.size() && !bad; ++k) bad = m.ci[k] < 0 || m.ci[k] >= m.cols;
    }
};
}  // namespace

int part_plan_write(const PartPlan &p, const SSS_AMG_PARS &pars, const char *path)
{
    FILE *f = fopen(path, "wb");
    if (!f) return ERROR_OPEN_FILE;
    Out o{f};
    o.raw(kPartMagic, sizeof(kPartMagic));
    o.i32(kPartVersion);
    o.i32((int)sizeof(SSS_AMG_PARS));
    o.raw(&pars, sizeof(pars));
    o.i32(p.nranks);
    o.i32(p.rank);
    o.i32(p.nl);
    o.i32(p.nagg);
    for (const auto &c : p.cut) o.vec(c);
    o.vec(p.gnnz);
    for (const auto &L : p.L) {
        o.i32(L.lo), o.i32(L.hi), o.i32(L.m), o.i32(L.g), o.i32(L.nF);
        o.vec(L.perm), o.vec(L.ghosts), o.vec(L.mark), o.vec(L.gcls), o.vec(L.gclass);
        o.mat(L.A), o.mat(L.P), o.mat(L.R);
        o.vec(L.sdst), o.vec(L.scount), o.vec(L.sidx), o.vec(L.rsrc), o.vec(L.rcount);
    }
    const bool bad = o.bad;
    return (fclose(f) != 0 || bad) ? ERROR_OPEN_FILE : 0;
}

// The cross-field invariants of one level read back from a file (the halo lists index the level's
// own values and ghosts, the local matrices have the level's local shapes).
static bool part_level_consistent(const PartLevel &L, int nranks)
{
    if (L.m != L.hi - L.lo || L.m < 0 || L.g < 0 || L.nF < 0 || L.nF > L.m) return false;
    if (L.gcls.size() != (size_t)L.g || L.gclass.size() != (size_t)L.g) return false;
    for (int v : L.perm)
        if (v < L.lo || v >= L.hi) return false;
    if (L.A.rows != L.m || L.A.cols != L.m + L.g || L.R.cols != L.m + L.g || L.P.rows != L.m) return false;
    if (L.scount.size() != L.sdst.size() || L.rcount.size() != L.rsrc.size()) return false;
    long long ns = 0, nr = 0;
    for (size_t i = 0; i < L.sdst.size(); ++i) {
        if (L.sdst[i] < 0 || L.sdst[i] >= nranks || L.scount[i] < 0) return false;
        ns += L.scount[i];
    }
    for (size_t i = 0; i < L.rsrc.size(); ++i) {
        if (L.rsrc[i] < 0 || L.rsrc[i] >= nranks || L.rcount[i] < 0) return false;
        nr += L.rcount[i];
    }
    if (ns != (long long)L.sidx.size() || nr != L.g) return false;
    for (int v : L.sidx)
        if (v < 0 || v >= L.m) return false;
    return true;
}

int part_plan_read(PartPlan &p, SSS_AMG_PARS &pars, const char *path)
{
    FILE *f = fopen(path, "rb");
    if (!f) return ERROR_OPEN_FILE;
    In in{f};
    char magic[8];
    in.raw(magic, sizeof(magic));
    if (in.bad || memcmp(magic, kPartMagic, sizeof(magic)) || in.i32() != kPartVersion ||
        in.i32() != (int)sizeof(SSS_AMG_PARS)) {
        fclose(f);
        return ERROR_WRONG_FILE;
    }
    in.raw(&pars, sizeof(pars));
    p = PartPlan();
    p.nranks = in.i32();
    p.rank = in.i32();
    p.nl = in.i32();
    p.nagg = in.i32();
    if (in.bad || p.nranks < 1 || p.rank < 0 || p.rank >= p.nranks || p.nagg < 1 || p.nagg >= p.nl ||
        p.nl > kMaxPartLevels) {
        fclose(f);
        return ERROR_WRONG_FILE;
    }
    p.cut.resize((size_t)p.nagg + 1);
    for (auto &c : p.cut) {
        in.vec(c);
        if (c.size() != (size_t)p.nranks + 1) in.bad = true;
    }
    in.vec(p.gnnz);
    if (p.gnnz.size() != (size_t)p.nagg) in.bad = true;
    p.L.resize((size_t)p.nagg);
    for (auto &L : p.L) {
        L.lo = in.i32(), L.hi = in.i32(), L.m = in.i32(), L.g = in.i32(), L.nF = in.i32();
        in.vec(L.perm), in.vec(L.ghosts), in.vec(L.mark), in.vec(L.gcls), in.vec(L.gclass);
        in.mat(L.A), in.mat(L.P), in.mat(L.R);
        in.vec(L.sdst), in.vec(L.scount), in.vec(L.sidx), in.vec(L.rsrc), in.vec(L.rcount);
        if (!in.bad && (L.perm.size() != (size_t)L.m || L.ghosts.size() != (size_t)L.g || L.mark.size() != (size_t)L.m))
            in.bad = true;
        if (!in.bad) in.bad = !part_level_consistent(L, p.nranks);
    }
    const bool bad = in.bad;
    fclose(f);
    return bad ? ERROR_WRONG_FILE : 0;
}

std::string part_file_name(const char *prefix, int rank) { return std::string(prefix) + ".r" + std::to_string(rank); }
std::string part_tail_name(const char *prefix) { return std::string(prefix) + ".tail"; }

}  // namespace sss

struct sss_part_plan {
    sss::PartPlan p;
};

extern "C" int sss_part_save(const SSS_AMG *mg, int nranks, int agg_rows, const char *prefix)
{
    if (!mg || nranks < 1 || !prefix) return ERROR_INPUT_PAR;
    agg_rows = sss::part_agg_rows(agg_rows);
    int nagg = -1;
    if (int rc = sss::part_save_all(mg, nranks, agg_rows, prefix, nagg)) return rc;
    SSS_AMG tail = *mg;   // the replicated levels, as their own hierarchy
    tail.cg = mg->cg + nagg;
    tail.num_levels = mg->num_levels - nagg;
    return SSS_amg_save(&tail, sss::part_tail_name(prefix).c_str());
}

extern "C" sss_part_plan *sss_part_plan_load(const char *path)
{
    auto *pp = new sss_part_plan();
    SSS_AMG_PARS pars;
    if (sss::part_plan_read(pp->p, pars, path)) {
        delete pp;
        return nullptr;
    }
    return pp;
}

extern "C" sss_part_plan *sss_part_plan_create(const SSS_AMG *mg, int nranks, int rank, int agg_rows)
{
    auto *pp = new sss_part_plan();
    if (sss::part_plan_build(pp->p, mg, nranks, rank, sss::part_agg_rows(agg_rows))) {
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
