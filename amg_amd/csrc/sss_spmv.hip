// sss_spmv.hip — CSR SpMV family for every level (gfx950, wave64, fp64, no contraction).
//
// Replaces SSS_blas_mv_amxpy / SSS_blas_mv_mxy (SSS_utils.c:161-201) and the coarse-grid
// spmv_kernel / alpha_spmv_kernel (Solve/SSS_cuda.cu:77-118, which launch <<<64,64>>> and
// re-upload the whole CSR per call).  Here the CSR lives in HBM for the whole solve.
//
// Kernel: CSR-adaptive.  At upload each matrix is cut into row blocks of <= 256 rows holding
// <= kTileEntries nonzeros.  A workgroup stages its block's val/col slice into LDS with
// coalesced loads (the slice is contiguous in CSR), then each thread walks ONE row from LDS
// and accumulates in stored CSR order starting from 0.0 — the reference's exact summation
// order, so results are bitwise identical to the host reference.  A row longer than the
// tile forms a block on its own: the workgroup computes the products a_k*x_{c_k} in parallel
// (identically rounded), stages them in LDS and one lane adds them in order (bitwise again).
//
// Roofline: HBM-bound, 12 B/nnz (fp64 value + int32 column) + 4 B/row (row_ptr) + 8 B/row
// per vector stream (x compulsory, y, b); no MFMA (≈0.13 flop/byte).
#include "sss_engine.hpp"

#include <cstdlib>
#include "sss_spmv_dev.hpp"

#include <algorithm>
#include <type_traits>
#include <condition_variable>
#include <cstring>
#include <mutex>
#include <sched.h>
#include <sys/resource.h>
#include <sys/syscall.h>
#include <unistd.h>

namespace sss {

int hip_fail(hipError_t e, const char *what, const char *file, int line)
{
    fprintf(stderr, "### ERROR: HIP call %s failed at %s:%d: %s\n", what, file, line, hipGetErrorString(e));
    return ERROR_MISC;
}

// Host -> device copy of a large host array through a ring of pinned staging buffers: host threads
// copy chunk k + 1 into one buffer while the DMA engine moves chunk k out of another (a pageable
// hipMemcpy of the 400^3 hierarchy's ~60 GB ran at ~3 GB/s).  Small copies go straight through.
// ---- host worker pool (sss_engine.hpp) ----------------------------------------------------------
// Threads: SSS_HOST_THREADS, else the usable CPUs (affinity mask, capped by a cgroup v2 cpu.max
// quota), at most 32.
static int usable_cpus()
{
    const char *e = getenv("SSS_HOST_THREADS");
    if (e && *e) return std::max(1, atoi(e));
    int n = (int)std::max(1u, std::thread::hardware_concurrency());
    cpu_set_t set;
    if (sched_getaffinity(0, sizeof(set), &set) == 0) n = std::max(1, CPU_COUNT(&set));
    if (FILE *f = fopen("/sys/fs/cgroup/cpu.max", "r")) {
        char q[32] = {0};
        long long period = 0;
        if (fscanf(f, "%31s %lld", q, &period) == 2 && strcmp(q, "max") != 0 && period > 0)
            n = std::min(n, (int)std::max(1LL, (atoll(q) + period - 1) / period));
        fclose(f);
    }
    return std::min(n, 32);
}

// Upload helpers run at a lower CPU priority (nice SSS_HOST_NICE, default 10): when the mirror is
// built while the setup runs (sss_hip_setup_create), the setup's serial RS pass and its OpenMP
// regions keep their cores and the upload takes what they leave idle.
void host_thread_background()
{
    const char *e = getenv("SSS_HOST_NICE");
    const int nice = (e && *e) ? atoi(e) : 10;
    if (nice > 0) (void)setpriority(PRIO_PROCESS, (id_t)syscall(SYS_gettid), nice);
}

namespace {
// Several callers may hold jobs at once (the mirror's level tasks run side by side after the setup):
// each job is a loop body that returns once its shared chunk counter is exhausted; an idle worker
// joins any open job, and a job closes for newcomers as soon as one of its threads has returned.
struct HostPool {
    struct Job {
        const std::function<void()> *work = nullptr;
        int inside = 0;
        bool open = false;
    };
    static constexpr int kJobs = 8;
    std::mutex mu;
    std::condition_variable cv, done_cv;
    Job jobs[kJobs];
    int nt = 1, rr = 0;
    static thread_local bool in_worker;
    HostPool()
    {
        nt = usable_cpus();
        for (int t = 1; t < nt; ++t) std::thread([this] { loop(); }).detach();   // lives as long as the process
    }
    int open_job() const
    {
        for (int k = 0; k < kJobs; ++k)
            if (jobs[(rr + k) % kJobs].open) return (rr + k) % kJobs;
        return -1;
    }
    void loop()
    {
        in_worker = true;
        host_thread_background();
        for (;;) {
            int j;
            {
                std::unique_lock<std::mutex> lk(mu);
                cv.wait(lk, [&] { return open_job() >= 0; });
                j = open_job();
                rr = (j + 1) % kJobs;
                ++jobs[j].inside;
            }
            (*jobs[j].work)();
            std::lock_guard<std::mutex> lk(mu);
            jobs[j].open = false;   // its counter is exhausted: nothing left to join
            if (--jobs[j].inside == 0) done_cv.notify_all();
        }
    }
    bool run(const std::function<void()> &work)
    {
        if (in_worker) return false;
        int j = -1;
        {
            std::lock_guard<std::mutex> lk(mu);
            for (int k = 0; k < kJobs && j < 0; ++k)
                if (!jobs[k].work) j = k;
            if (j < 0) return false;
            jobs[j].work = &work;
            jobs[j].inside = 0;
            jobs[j].open = true;
        }
        cv.notify_all();
        work();
        {
            std::unique_lock<std::mutex> lk(mu);
            jobs[j].open = false;
            done_cv.wait(lk, [&] { return jobs[j].inside == 0; });
            jobs[j].work = nullptr;
        }
        return true;
    }
};
thread_local bool HostPool::in_worker = false;

HostPool &host_pool()
{
    static HostPool *p = new HostPool();   // never destroyed: detached workers outlive static teardown
    return *p;
}
}   // namespace

int host_pool_threads() { return host_pool().nt; }
bool host_pool_run(const std::function<void()> &work) { return host_pool().run(work); }

int h2d(void *dst, const void *src, size_t bytes)
{
    constexpr size_t kChunk = (size_t)32 << 20;
    constexpr int kSlots = 4;
    if (bytes < ((size_t)4 << 20)) {
        if (bytes) SSS_HIP(hipMemcpy(dst, src, bytes, hipMemcpyHostToDevice));
        return 0;
    }
    static std::mutex mu;
    static char *buf[kSlots];
    static hipEvent_t ev[kSlots];
    static hipStream_t st = nullptr;
    std::lock_guard<std::mutex> guard(mu);
    if (!st) {
        for (int k = 0; k < kSlots; ++k) {
            SSS_HIP(hipHostMalloc((void **)&buf[k], kChunk));
            SSS_HIP(hipEventCreateWithFlags(&ev[k], hipEventDisableTiming));
        }
        SSS_HIP(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    }
    const char *s = static_cast<const char *>(src);
    char *d = static_cast<char *>(dst);
    int slot = 0;
    for (size_t off = 0; off < bytes; off += kChunk, slot = (slot + 1) % kSlots) {
        const size_t n = std::min(kChunk, bytes - off);
        SSS_HIP(hipEventSynchronize(ev[slot]));   // the slot's previous DMA has finished
        const int parts = 8;
        const size_t per = (n + parts - 1) / parts;
        parallel_chunks(parts, 1, [&](int a, int e) {
            for (int t = a; t < e; ++t) {
                const size_t lo = (size_t)t * per, hi = std::min(n, lo + per);
                if (lo < hi) std::memcpy(buf[slot] + lo, s + off + lo, hi - lo);
            }
        });
        SSS_HIP(hipMemcpyAsync(d + off, buf[slot], n, hipMemcpyHostToDevice, st));
        SSS_HIP(hipEventRecord(ev[slot], st));
    }
    SSS_HIP(hipStreamSynchronize(st));
    return 0;
}

// Average entries per row from which a matrix takes the wave-per-row kernels (kWaveRowMin;
// SSS_HIP_WAVE_MIN overrides it at upload time, which the tests use to cover both paths).
int wave_row_min()
{
    const char *e = getenv("SSS_HIP_WAVE_MIN");
    return (e && *e) ? atoi(e) : kWaveRowMin;
}

// Free-order threshold (kFreeRowMin; SSS_HIP_FREE_MIN overrides it at upload time).
int free_row_min()
{
    const char *e = getenv("SSS_HIP_FREE_MIN");
    return (e && *e) ? atoi(e) : kFreeRowMin;
}

// Rows per merged group for a free-order matrix of n rows (0: wave-per-row kernels).  Measured on
// 7-pt 400^3 (tools/lab_rows.hip, residual, one wave per group): G = 8 from ~100K rows (level 6:
// 204 vs 311 us), G = 4 below (levels 7-9: 1.1-1.4x).  With one workgroup per group (4 waves split
// the entries) small matrices gain too: from 2,000 rows the V-cycle's levels 9-10 took 0.97 ms
// against 1.09 ms with 12,000 (tools/gpu/prof.sh).  SSS_HIP_MERGE_G / _MIN_ROWS override (tests).
static int merge_group_size(int n)
{
    const char *g = getenv("SSS_HIP_MERGE_G"), *m = getenv("SSS_HIP_MERGE_MIN_ROWS");
    const int min_rows = (m && *m) ? atoi(m) : 2000;
    if (n < min_rows) return 0;
    if (g && *g) return atoi(g) <= 0 ? 0 : atoi(g) >= 8 ? 8 : 4;   // kernel instances: 4 and 8
    return n >= 80000 ? 8 : 4;
}

// {first row, first entry} of every block, so a block's bounds are one independent load.
int upload_block_bounds(int2 **dst, const std::vector<int> &blk, const int *h_rp, const int2 **host)
{
    std::vector<int2> bk(blk.size());
    for (size_t q = 0; q < blk.size(); ++q) bk[q] = make_int2(blk[q], h_rp[blk[q]]);
    *dst = dev_alloc<int2>(bk.size());
    if (!*dst) return hip_fail(hipErrorOutOfMemory, "hipMalloc(bk)", __FILE__, __LINE__);
    if (host) {
        delete[] *host;
        int2 *c = new int2[bk.size()];
        std::copy(bk.begin(), bk.end(), c);
        *host = c;
    }
    return h2d(*dst, bk.data(), sizeof(int2) * bk.size());
}

thread_local ByteLedger *g_ledger = nullptr;

double matrix_bytes(const DevCSR &A, int blo, int bhi)
{
    if (bhi <= blo || A.n == 0) return 0.0;
    if (!A.h_bk || A.nblk == 0 || (blo == 0 && bhi >= A.nblk)) return (double)A.stream_bytes;
    const bool by_rows = A.dv_ell || A.dv_xell || A.nnz == 0;
    const double part = by_rows ? (double)(A.h_bk[bhi].x - A.h_bk[blo].x) / A.n
                                : (double)(A.h_bk[bhi].y - A.h_bk[blo].y) / A.nnz;
    return part * (double)A.stream_bytes;
}

double matrix_bytes_rows(const DevCSR &A, int lo, int hi)
{
    if (hi <= lo || A.n == 0) return 0.0;
    if (!A.h_bk || A.nblk == 0) return (double)A.stream_bytes * (hi - lo) / A.n;
    auto blk_of = [&](int r) {   // first block starting at or after row r
        int a = 0, b = A.nblk;
        while (a < b) {
            const int m = (a + b) / 2;
            if (A.h_bk[m].x < r) a = m + 1;
            else b = m;
        }
        return a;
    };
    return matrix_bytes(A, blk_of(lo), blk_of(hi));
}

int build_row_blocks(const int *h_rp, int n, std::vector<int> &blk, int split)
{
    blk.clear();
    int r = 0;
    while (r < n) {
        blk.push_back(r);
        const int base = h_rp[r];
        const int lim = (split > r && split < n) ? split : n;   // never straddle the class split
        int e = r + 1;
        if (h_rp[e] - base <= kTileEntries) {
            while (e < lim && e - r < kBlock && h_rp[e + 1] - base <= kTileEntries) ++e;
        }
        r = e;
    }
    blk.push_back(n);
    return (int)blk.size() - 1;
}

// Distinct 64-bit patterns of one block (at most 256), collected by open addressing; rank(id)
// is the pattern's position in ascending order -- what sort + unique + lower_bound gives, at a
// hash probe per entry instead of a sort of the whole block.
struct SmallDict {
    static constexpr int kSlots = 1024;
    unsigned long long key[kSlots];
    short slot[kSlots];                 // -1: empty; else local id
    unsigned long long val[256];        // local id -> pattern (insertion order)
    unsigned char rk[256];              // local id -> rank
    int n = 0;
    void clear()
    {
        std::memset(slot, 0xff, sizeof(slot));
        n = 0;
    }
    int insert(unsigned long long u, int cap)   // local id, or -1 past cap distinct patterns
    {
        unsigned h = (unsigned)((u * 0x9E3779B97F4A7C15ull) >> 54);
        for (;; h = (h + 1) & (kSlots - 1)) {
            if (slot[h] < 0) {
                if (n >= cap) return -1;
                slot[h] = (short)n;
                key[h] = u;
                val[n] = u;
                return n++;
            }
            if (key[h] == u) return slot[h];
        }
    }
    template <class T>
    void finish(std::vector<T> &sorted)   // ranks + the patterns in ascending order
    {
        int ord[256];
        for (int t = 0; t < n; ++t) ord[t] = t;
        std::sort(ord, ord + n, [&](int a, int b) { return (T)val[a] < (T)val[b]; });
        sorted.resize((size_t)n);
        for (int t = 0; t < n; ++t) rk[ord[t]] = (unsigned char)t, sorted[t] = (T)val[ord[t]];
    }
};
static inline unsigned long long bits_of(double d)
{
    unsigned long long u;
    std::memcpy(&u, &d, sizeof(u));
    return u;
}
static inline double double_of(unsigned long long u)
{
    double d;
    std::memcpy(&d, &u, sizeof(d));
    return d;
}

// Sorted tile segments of a blocking: a block's entries, or kTileEntries chunks of a long row
// (exactly the segments the tile kernels stage, sss_spmv_dev.hpp csr_block_rows).  Per block the
// columns are cut into two clusters at their widest gap; returns false when a cluster spans
// 2^kTileColBits columns or more (the matrix then keeps stored-order staging).  One sort of
// (column << 32 | position) keys per segment gives both the column order and, on ties, the
// stored order (a stable sort by column).
static bool build_sorted_tiles(const SSS_MAT &h, const std::vector<int> &blk, HostBuf<unsigned> &pk,
                               HostBuf<double> &pv, std::vector<int2> &pb)
{
    const int *rp = h.row_ptr, *ci = h.col_idx;
    const int nb = (int)blk.size() - 1;
    constexpr long long kSpan = kTileDiagMark;   // larger offsets mark diagonal entries
    pk.resize((size_t)h.num_nnzs);
    pv.resize((size_t)h.num_nnzs);
    pb.resize((size_t)std::max(nb, 1));
    std::atomic<int> ok{1};
    parallel_chunks(nb, 512, [&](int qlo, int qhi) {
        std::vector<unsigned long long> key, seg;
        std::vector<int> rowof;
        for (int q = qlo; q < qhi && ok; ++q) {
            const int a0 = rp[blk[q]], e0 = rp[blk[q + 1]];
            if (a0 == e0) {
                pb[q] = make_int2(0, 0);
                continue;
            }
            rowof.resize((size_t)(e0 - a0));   // entry position -> its row (one pass over the block)
            for (int r = blk[q]; r < blk[q + 1]; ++r)
                for (int k = rp[r]; k < rp[r + 1]; ++k) rowof[(size_t)(k - a0)] = r;
            key.resize((size_t)(e0 - a0));
            for (int k = a0; k < e0; ++k) key[(size_t)(k - a0)] = (unsigned long long)(unsigned)ci[k] << 32 | (unsigned)(k - a0);
            std::sort(key.begin(), key.end());
            auto col = [&](size_t t) { return (int)(key[t] >> 32); };
            const size_t m = key.size();
            size_t gap = 0;   // cut after col(gap)
            for (size_t t = 1; t < m; ++t)
                if (col(t) - col(t - 1) > col(gap + 1) - col(gap)) gap = t - 1;
            const int b0 = col(0), b1 = m > 1 ? col(gap + 1) : col(0);
            const int cut = b1;   // columns >= cut go to cluster 1
            if (m > 1 && ((long long)col(gap) - b0 >= kSpan || (long long)col(m - 1) - b1 >= kSpan)) {
                ok = 0;
                return;
            }
            pb[q] = make_int2(b0, b1);
            const int r0 = blk[q];
            for (int a = a0; a < e0; a += kTileEntries) {
                const int e = std::min(e0, a + kTileEntries);
                const unsigned long long *sk = key.data();
                if (e - a != e0 - a0) {   // a long row's chunk: its own column order
                    seg.resize((size_t)(e - a));
                    for (int k = a; k < e; ++k) seg[(size_t)(k - a)] = (unsigned long long)(unsigned)ci[k] << 32 | (unsigned)(k - a0);
                    std::sort(seg.begin(), seg.end());
                    sk = seg.data();
                }
                for (int t = 0; t < e - a; ++t) {
                    const int k = a0 + (int)(unsigned)sk[t], c = ci[k];
                    const int r = rowof[(size_t)(k - a0)];   // the entry's row
                    const unsigned cl = (m > 1 && c >= cut) ? 1u : 0u;
                    const unsigned off = c == r ? kTileDiagMark + (unsigned)(r - r0) : (unsigned)(c - (cl ? b1 : b0));
                    pk[(size_t)a + t] = (cl << 31) | (off << kTileShift) | (unsigned)(k - a);
                    pv[(size_t)a + t] = h.val[k];
                }
            }
        }
    });
    return ok != 0;
}

// Rows of a free-order (tree-summed) matrix, stored column-sorted within each segment.
static void sort_row_segments(const SSS_MAT &h, const int *seg, HostBuf<int> &ci, HostBuf<double> &v)
{
    const int n = h.num_rows;
    const int *rp = h.row_ptr;
    ci.resize((size_t)h.num_nnzs);
    v.resize((size_t)h.num_nnzs);
    parallel_chunks(n, 256, [&](int rlo, int rhi) {
        std::vector<unsigned long long> key;   // column << 32 | position: a stable sort by column
        for (int r = rlo; r < rhi; ++r) {
            const int cut[3] = {rp[r], seg ? seg[r] : rp[r + 1], rp[r + 1]};
            for (int part = 0; part < 2; ++part) {
                const int a = cut[part], e = cut[part + 1];
                key.resize((size_t)std::max(0, e - a));
                for (int t = 0; t < e - a; ++t) key[t] = (unsigned long long)(unsigned)h.col_idx[a + t] << 32 | (unsigned)t;
                std::sort(key.begin(), key.end());
                for (int t = 0; t < e - a; ++t) {
                    const int k = a + (int)(unsigned)key[t];
                    ci[(size_t)a + t] = h.col_idx[k], v[(size_t)a + t] = h.val[k];
                }
            }
        }
    });
}

// Merged row groups of a free-order matrix: group g = rows [gG, gG + G); its entries keep their CSR
// span [rp[gG], rp[gG + G]), sorted by (column, segment, row); segment 1 = [seg[r], rp[r+1]) of a
// two-segment row.
static void build_merged(const SSS_MAT &h, const int *seg, int G, std::vector<int> &gp, HostBuf<unsigned> &mk,
                         HostBuf<double> &mv)
{
    const int n = h.num_rows, ng = (n + G - 1) / G;
    const int *rp = h.row_ptr, *ci = h.col_idx;
    gp.resize((size_t)ng + 1);
    mk.resize((size_t)h.num_nnzs);
    mv.resize((size_t)h.num_nnzs);
    parallel_chunks(ng, 64, [&](int glo, int ghi) {
        std::vector<std::pair<unsigned long long, int>> ent;   // ((col << 4 | seg << 3 | row), position)
        std::vector<unsigned long long> key;   // the same order as one integer: merged key << 24 | position
        for (int g = glo; g < ghi; ++g) {
            const int r0 = g * G, r1 = std::min(n, r0 + G);
            const int base = rp[r0], cnt = rp[r1] - base;
            if (cnt < (1 << 24)) {
                key.resize((size_t)cnt);
                for (int r = r0; r < r1; ++r)
                    for (int k = rp[r]; k < rp[r + 1]; ++k) {
                        const unsigned long long sg = (seg && k >= seg[r]) ? 1u : 0u;
                        key[(size_t)(k - base)] =
                            ((((unsigned long long)ci[k] << kMergeShift) | (sg << 3) | (unsigned)(r - r0)) << 24) |
                            (unsigned)(k - base);
                    }
                std::sort(key.begin(), key.end());
                gp[g] = base;
                for (int t = 0; t < cnt; ++t) {
                    mk[(size_t)base + t] = (unsigned)(key[t] >> 24);
                    mv[(size_t)base + t] = h.val[base + (int)(key[t] & 0xffffff)];
                }
                continue;
            }
            ent.clear();
            for (int r = r0; r < r1; ++r)
                for (int k = rp[r]; k < rp[r + 1]; ++k) {
                    const unsigned sg = (seg && k >= seg[r]) ? 1u : 0u;
                    ent.emplace_back(((unsigned long long)ci[k] << kMergeShift) | (sg << 3) | (unsigned)(r - r0), k);
                }
            std::sort(ent.begin(), ent.end());
            int pos = rp[r0];
            gp[g] = pos;
            for (const auto &e : ent) {
                mk[pos] = (unsigned)e.first;
                mv[pos] = h.val[e.second];
                ++pos;
            }
        }
    });
    gp[ng] = rp[n];
}

DevDict devdict(const DevCSR &A, int blo)
{
    DevDict t;
    t.tree_long = A.tree_long ? 1 : 0;
    if (!has_dict(A)) return t;
    t.code = A.dv_code;
    t.ell = A.dv_ell;
    t.ellb = A.dv_ell_base;
    t.ellw = A.ell_w;
    t.xell = A.dv_xell;
    t.xshift = A.xell_shift;
    t.pd = A.dv_pd + blo;
    t.dd = A.dv_dd;
    t.vd = A.dv_vd;
    if (A.dv_vi) {
        t.pk = A.pk;
        t.vi = A.dv_vi;
        t.pb = A.pb + blo;
    }
    return t;
}

// Dictionary tiles of a square matrix (DevCSR::dv_*): per block, the distinct column offsets
// col - row and the distinct value bit patterns, each at most 256 (false when a block has more);
// the codes of each staging segment (the block, or a kTileEntries chunk of a longer row) in
// column order.
static bool build_dict_tiles(const SSS_MAT &h, const std::vector<int> &blk, HostBuf<unsigned> &code,
                             std::vector<int4> &pd, std::vector<int> &dd, std::vector<double> &vd)
{
    const int *rp = h.row_ptr, *ci = h.col_idx;
    const double *v = h.val;
    const int nb = (int)blk.size() - 1;
    if (h.num_rows != h.num_cols || nb <= 0) return false;
    std::vector<std::vector<int>> bd(nb);
    std::vector<std::vector<unsigned long long>> bv(nb);
    code.resize((size_t)h.num_nnzs);
    std::atomic<int> ok{1};
    parallel_chunks(nb, 256, [&](int qlo, int qhi) {
        std::unique_ptr<SmallDict> Dd(new SmallDict()), Vd(new SmallDict());
        std::vector<unsigned long long> key;
        std::vector<int> rowof;
        std::vector<unsigned char> did, vid;   // entry -> local dictionary ids
        for (int q = qlo; q < qhi && ok; ++q) {
            const int a0 = rp[blk[q]], e0 = rp[blk[q + 1]];
            rowof.resize((size_t)(e0 - a0));
            did.resize((size_t)(e0 - a0));
            vid.resize((size_t)(e0 - a0));
            Dd->clear();
            Vd->clear();
            for (int r = blk[q]; r < blk[q + 1]; ++r)
                for (int k = rp[r]; k < rp[r + 1]; ++k) {
                    rowof[(size_t)(k - a0)] = r;
                    const int di = Dd->insert((unsigned long long)(long long)(ci[k] - r), 256);
                    const int vi = Vd->insert(bits_of(v[k]), 256);
                    if (di < 0 || vi < 0) {
                        ok = 0;
                        return;
                    }
                    did[(size_t)(k - a0)] = (unsigned char)di;
                    vid[(size_t)(k - a0)] = (unsigned char)vi;
                }
            std::vector<long long> ds;
            Dd->finish(ds);
            Vd->finish(bv[q]);
            bd[q].assign(ds.begin(), ds.end());
            for (int a = a0; a < e0; a += kTileEntries) {   // staging segments, column-sorted
                const int e = std::min(e0, a + kTileEntries);
                key.resize((size_t)(e - a));
                for (int k = a; k < e; ++k) key[(size_t)(k - a)] = (unsigned long long)(unsigned)ci[k] << 32 | (unsigned)(k - a);
                std::sort(key.begin(), key.end());
                for (int t = 0; t < e - a; ++t) {
                    const int k = a + (int)(unsigned)key[t];
                    const unsigned dix = Dd->rk[did[(size_t)(k - a0)]], vix = Vd->rk[vid[(size_t)(k - a0)]];
                    code[(size_t)a + t] = vix << (kTileShift + 8) | dix << kTileShift | (unsigned)(k - a);
                }
            }
        }
    });
    if (!ok) return false;
    pd.resize((size_t)nb);
    size_t nd = 0, nv = 0;
    for (int q = 0; q < nb; ++q) {
        pd[q] = make_int4((int)nd, (int)bd[q].size(), (int)nv, (int)bv[q].size());
        nd += bd[q].size();
        nv += bv[q].size();
    }
    dd.resize(std::max<size_t>(nd, 1));
    vd.resize(std::max<size_t>(nv, 1));
    for (int q = 0; q < nb; ++q) {
        std::copy(bd[q].begin(), bd[q].end(), dd.begin() + pd[q].x);
        for (size_t t = 0; t < bv[q].size(); ++t) vd[(size_t)pd[q].z + t] = double_of(bv[q][t]);
    }
    return true;
}

// Value dictionaries over the sorted tiles' values pv (slot order): per block at most 256 distinct
// bit patterns (false when a block has more), vi = each slot's index; pd[block] = {0, 0, base, count}.
static bool build_value_dict(const std::vector<int> &blk, const int *rp, const HostBuf<double> &pv,
                             HostBuf<unsigned char> &vi, std::vector<int4> &pd, std::vector<double> &vd)
{
    const int nb = (int)blk.size() - 1;
    if (nb <= 0) return false;
    std::vector<std::vector<unsigned long long>> bv(nb);
    vi.resize(pv.size());
    std::atomic<int> ok{1};
    parallel_chunks(nb, 256, [&](int qlo, int qhi) {
        std::unique_ptr<SmallDict> Vd(new SmallDict());
        for (int q = qlo; q < qhi && ok; ++q) {
            const int a0 = rp[blk[q]], e0 = rp[blk[q + 1]];
            Vd->clear();
            for (int k = a0; k < e0; ++k) {
                const int id = Vd->insert(bits_of(pv[(size_t)k]), 256);
                if (id < 0) {
                    ok = 0;
                    return;
                }
                vi[(size_t)k] = (unsigned char)id;
            }
            Vd->finish(bv[q]);
            for (int k = a0; k < e0; ++k) vi[(size_t)k] = Vd->rk[vi[(size_t)k]];
        }
    });
    if (!ok) return false;
    pd.resize((size_t)nb);
    size_t nv = 0;
    for (int q = 0; q < nb; ++q) {
        pd[q] = make_int4(0, 0, (int)nv, (int)bv[q].size());
        nv += bv[q].size();
    }
    vd.resize(std::max<size_t>(nv, 1));
    for (int q = 0; q < nb; ++q)
        for (size_t t = 0; t < bv[q].size(); ++t) vd[(size_t)pd[q].z + t] = double_of(bv[q][t]);
    return true;
}

// Dictionary ELL of a square matrix (DevCSR::dv_ell): every row at most 32 entries, every block at
// most 31 distinct column offsets and 8 distinct value bit patterns (false otherwise); width W =
// 8, 16 or 32 bytes per row, codes in stored order, 0xFF pads.
static bool build_ell(const SSS_MAT &h, const std::vector<int> &blk, HostBuf<unsigned char> &ell, int &W,
                      std::vector<int4> &pd, std::vector<int> &dd, std::vector<double> &vd, const int *base = nullptr)
{
    const int *rp = h.row_ptr, *ci = h.col_idx;
    const double *v = h.val;
    const int n = h.num_rows, nb = (int)blk.size() - 1;
    // rectangular matrices (a restriction) too: offsets col - row, no diagonal meaning
    if (nb <= 0 || n <= 0) return false;
    std::atomic<int> Lmax{0};
    parallel_chunks(n, 1 << 16, [&](int lo, int hi) {
        int L = 0;
        for (int r = lo; r < hi; ++r) L = std::max(L, rp[r + 1] - rp[r]);
        int cur = Lmax.load();
        while (L > cur && !Lmax.compare_exchange_weak(cur, L)) {}
    });
    const int L = Lmax.load();
    if (L > 32) return false;
    W = L <= 8 ? 8 : L <= 16 ? 16 : 32;
    // per block at most 31 offsets and 8 values: fixed slots, compacted afterwards
    std::vector<int> bdf((size_t)nb * 31), nd_of(nb), nv_of(nb);
    std::vector<double> bvf((size_t)nb * 8);
    ell.resize((size_t)n * W);
    std::atomic<int> ok{1};
    parallel_chunks(nb, 256, [&](int qlo, int qhi) {
        std::unique_ptr<SmallDict> Dd(new SmallDict()), Vd(new SmallDict());
        std::vector<long long> ds;
        std::vector<unsigned long long> vs;
        for (int q = qlo; q < qhi && ok; ++q) {
            Dd->clear();
            Vd->clear();
            unsigned char *row0 = ell.data() + (size_t)blk[q] * W;
            std::memset(row0, 0xff, (size_t)(blk[q + 1] - blk[q]) * W);
            for (int r = blk[q]; r < blk[q + 1]; ++r)
                for (int k = rp[r]; k < rp[r + 1]; ++k) {
                    const int di = Dd->insert((unsigned long long)(long long)(ci[k] - (base ? base[r] : r)), 31);
                    const int vi = Vd->insert(bits_of(v[k]), 8);
                    if (di < 0 || vi < 0) {
                        ok = 0;
                        return;
                    }
                    ell[(size_t)r * W + (k - rp[r])] = (unsigned char)(vi << 5 | di);
                }
            Dd->finish(ds);
            Vd->finish(vs);
            nd_of[q] = (int)ds.size();
            nv_of[q] = (int)vs.size();
            std::copy(ds.begin(), ds.end(), bdf.begin() + (size_t)q * 31);
            for (size_t t = 0; t < vs.size(); ++t) bvf[(size_t)q * 8 + t] = double_of(vs[t]);
            for (int r = blk[q]; r < blk[q + 1]; ++r)
                for (int k = 0; k < rp[r + 1] - rp[r]; ++k) {
                    unsigned char &c = ell[(size_t)r * W + k];
                    c = (unsigned char)(Vd->rk[c >> 5] << 5 | Dd->rk[c & 31]);
                }
        }
    });
    if (!ok) return false;
    pd.resize((size_t)nb);
    size_t nd = 0, nv = 0;
    for (int q = 0; q < nb; ++q) {
        pd[q] = make_int4((int)nd, nd_of[q], (int)nv, nv_of[q]);
        nd += nd_of[q];
        nv += nv_of[q];
    }
    dd.resize(std::max<size_t>(nd, 1));
    vd.resize(std::max<size_t>(nv, 1));
    parallel_chunks(nb, 4096, [&](int qlo, int qhi) {
        for (int q = qlo; q < qhi; ++q) {
            std::copy(bdf.begin() + (size_t)q * 31, bdf.begin() + (size_t)q * 31 + nd_of[q], dd.begin() + pd[q].x);
            std::copy(bvf.begin() + (size_t)q * 8, bvf.begin() + (size_t)q * 8 + nv_of[q], vd.begin() + pd[q].z);
        }
    });
    return true;
}

// Column ELL of a square matrix (DevCSR::dv_xell) over blocks of 256 rows: W 32-bit codes per row
// (stored order, 0xFFFFFFFF pads), each block's distinct values (<= 128, ascending) in vd at
// pd[q].z / .w (false when a block has more).  W = the longest row rounded up to 16, 20, 24 or 32.
static int xell_width(int L) { return L <= 8 ? 8 : L <= 16 ? 16 : L <= 20 ? 20 : L <= 24 ? 24 : L <= 32 ? 32 : L <= 40 ? 40 : 0; }
// column bits of a code: the smallest S >= 23 with ncols < 2^S (so the all-ones pad is never a
// column), 0 past 28 (fewer than 16 value slots)
static int xell_shift_for(int ncols)
{
    for (int S = 23; S <= 28; ++S)
        if ((long long)ncols < (1LL << S)) return S;
    return 0;
}
// 256-row blocks (cut at the class split): the column ELL's blocking
static int build_rows_blocks(int n, std::vector<int> &blk, int split)
{
    blk.clear();
    for (int r = 0; r < n;) {
        blk.push_back(r);
        const int lim = (split > r && split < n) ? split : n;
        r = std::min(lim, r + kBlock);
    }
    blk.push_back(n);
    return (int)blk.size() - 1;
}
// Distinct 64-bit values of a row range (up to kXellValues), open addressing; ranks = ascending order.
struct XellValues {
    static constexpr int kSlots = 4 * kXellValues;
    unsigned long long key[kSlots];
    short slot[kSlots];
    unsigned long long val[kXellValues];
    unsigned short rk[kXellValues];
    int n = 0;
    void clear()
    {
        std::memset(slot, 0xff, sizeof(slot));
        n = 0;
    }
    int insert(unsigned long long u, int cap)   // local id, or -1 past cap distinct values
    {
        for (unsigned h = (unsigned)((u * 0x9E3779B97F4A7C15ull) >> 53) & (kSlots - 1);; h = (h + 1) & (kSlots - 1)) {
            if (slot[h] < 0) {
                if (n >= cap) return -1;
                slot[h] = (short)n;
                key[h] = u;
                val[n] = u;
                return n++;
            }
            if (key[h] == u) return slot[h];
        }
    }
    void finish(std::vector<double> &sorted)
    {
        int ord[kXellValues];
        for (int t = 0; t < n; ++t) ord[t] = t;
        std::sort(ord, ord + n, [&](int a, int b) { return val[a] < val[b]; });
        sorted.resize((size_t)n);
        for (int t = 0; t < n; ++t) rk[ord[t]] = (unsigned short)t, sorted[t] = double_of(val[ord[t]]);
    }
};
// Column ELL codes and blocking: the rows in chunks of 256 (cut at the class split); a chunk whose
// rows hold more distinct values than a code can index (2^(32 - S), at most kXellValues) is halved
// until its parts fit (false below 16 rows).  Blocks, their value dictionaries (ascending) and every
// row's W codes in stored order.
static bool build_xell(const SSS_MAT &h, int split, int W, int S, std::vector<int> &blk, HostBuf<unsigned> &codes,
                       std::vector<int4> &pd, std::vector<double> &vd)
{
    const int vcap = std::min(kXellValues, 1 << (32 - S));
    const int *rp = h.row_ptr, *ci = h.col_idx;
    const double *v = h.val;
    std::vector<int> chunks;
    const int nc = build_rows_blocks(h.num_rows, chunks, split);
    codes.resize((size_t)h.num_rows * W);
    struct Part {
        int r0;
        std::vector<double> vals;
    };
    std::vector<std::vector<Part>> parts((size_t)nc);
    std::atomic<int> ok{1};
    parallel_chunks(nc, 64, [&](int clo, int chi) {
        std::unique_ptr<XellValues> D(new XellValues());
        // rows [r0, r1) as one block if their values fit, else halved
        std::function<bool(int, int, std::vector<Part> &)> fit = [&](int r0, int r1, std::vector<Part> &out) -> bool {
            D->clear();
            bool fits = true;
            for (int k = rp[r0]; k < rp[r1] && fits; ++k) fits = D->insert(bits_of(v[k]), vcap) >= 0;
            if (!fits) {
                if (r1 - r0 <= 16) return false;
                const int mid = r0 + (r1 - r0) / 2;
                return fit(r0, mid, out) && fit(mid, r1, out);
            }
            Part p;
            p.r0 = r0;
            D->finish(p.vals);
            for (int r = r0; r < r1; ++r) {
                unsigned *row = codes.data() + (size_t)r * W;
                int s = 0;
                for (int k = rp[r]; k < rp[r + 1]; ++k, ++s)
                    row[s] = (unsigned)D->rk[D->insert(bits_of(v[k]), vcap)] << S | (unsigned)ci[k];
                for (; s < W; ++s) row[s] = 0xffffffffu;
            }
            out.push_back(std::move(p));
            return true;
        };
        for (int c = clo; c < chi && ok; ++c)
            if (!fit(chunks[c], chunks[c + 1], parts[c])) ok = 0;
    });
    if (!ok) return false;
    blk.clear();
    pd.clear();
    vd.clear();
    for (int c = 0; c < nc; ++c)
        for (const Part &p : parts[c]) {
            blk.push_back(p.r0);
            pd.push_back(make_int4(0, 0, (int)vd.size(), (int)p.vals.size()));
            vd.insert(vd.end(), p.vals.begin(), p.vals.end());
        }
    blk.push_back(h.num_rows);
    if (vd.empty()) vd.push_back(0.0);
    return true;
}
static bool xell_on()
{
    const char *e = getenv("SSS_HIP_XELL");   // 0: no column ELL (read per upload: tests compare both ways)
    return !(e && *e == '0');
}

int devcsr_upload(DevCSR &d, const SSS_MAT &h, int split, int enc, const int *seg)
{
    PhaseTimer pt("devcsr");
    d.n = h.num_rows;
    d.ncols = h.num_cols;
    d.nnz = h.num_nnzs;
    d.wave_rows = d.n > 0 && (long long)d.nnz >= (long long)wave_row_min() * d.n;
    d.vec_rows = d.n > 0 && (enc & kEncFreeOrder) && (long long)d.nnz >= (long long)free_row_min() * d.n;
    d.tree_long = (enc & kEncFreeOrder) && !d.vec_rows;
    if (d.vec_rows && (unsigned long long)std::max(d.ncols, 1) < (1ull << (32 - kMergeShift))) {
        d.mg_G = merge_group_size(d.n);
        if (seg && d.mg_G > 4) d.mg_G = 4;   // two segments: 2G accumulators per lane
    }
    d.rp = dev_alloc<int>((size_t)d.n + 1);
    d.ci = dev_alloc<int>((size_t)d.nnz);
    d.v = dev_alloc<double>((size_t)d.nnz);
    if (!d.rp || !d.ci || !d.v) return hip_fail(hipErrorOutOfMemory, "hipMalloc(CSR)", __FILE__, __LINE__);
    pt.mark("alloc");
    if (int rc = h2d(d.rp, h.row_ptr, sizeof(int) * ((size_t)d.n + 1))) return rc;
    if (d.nnz > 0) {
        // free-order rows are read column-sorted by the wave-tree kernels; a two-stage split copy
        // with a merged copy (kEncMergedOnly) is read only through that (launch_ts_*): stored order
        if (d.vec_rows && !((enc & kEncMergedOnly) && d.mg_G > 0) && !device_builders_on()) {
            HostBuf<int> sci;
            HostBuf<double> sv;
            sort_row_segments(h, seg, sci, sv);
            if (int rc = h2d(d.ci, sci.data(), sizeof(int) * (size_t)d.nnz)) return rc;
            if (int rc = h2d(d.v, sv.data(), sizeof(double) * (size_t)d.nnz)) return rc;
            d.rows_sorted = true;
        } else {
            if (int rc = h2d(d.ci, h.col_idx, sizeof(int) * (size_t)d.nnz)) return rc;
            if (int rc = h2d(d.v, h.val, sizeof(double) * (size_t)d.nnz)) return rc;
        }
    }
    pt.mark("csr");
    std::vector<int> blk;
    d.nblk = build_row_blocks(h.row_ptr, d.n, blk, split);
    d.split_blk = d.nblk;
    d.split_row = split;
    if (split >= 0)
        for (int q = 0; q <= d.nblk; ++q)
            if (blk[q] >= split) { d.split_blk = q; break; }
    d.blk = dev_alloc<int>(blk.size());
    if (!d.blk) return hip_fail(hipErrorOutOfMemory, "hipMalloc(blk)", __FILE__, __LINE__);
    if (int rc = h2d(d.blk, blk.data(), sizeof(int) * blk.size())) return rc;
    if (int rc = upload_block_bounds(&d.bk, blk, h.row_ptr, &d.h_bk)) return rc;
    d.ngrid = (d.wave_rows || d.vec_rows) ? (d.n + 3) / 4 : d.nblk;
    pt.mark("blocks");
    if (d.mg_G > 0 && device_builders_on()) {   // from the stored-order CSR just uploaded
        d.mg_two = seg != nullptr;
        const char *wz = getenv("SSS_HIP_MERGE_W");
        d.mg_W = (wz && *wz) ? atoi(wz) : 4;
        d.mg_W = d.mg_W >= 4 ? 4 : d.mg_W >= 2 ? 2 : 1;
        if (int rc = merged_build_device(d, seg)) return rc;
        d.ngrid = (d.mg_ng + 4 / d.mg_W - 1) / (4 / d.mg_W);
    } else if (d.mg_G > 0) {
        std::vector<int> gp;
        HostBuf<unsigned> mk;
        HostBuf<double> mv;
        build_merged(h, seg, d.mg_G, gp, mk, mv);
        d.mg_two = seg != nullptr;
        d.mg_ng = (int)gp.size() - 1;
        // waves per group: 4 (fewer -- longer waves over shorter groups -- measured no better on
        // 7-pt 400^3: levels 5-10 6.6 ms per V-cycle with W = 1/2 by group size, 6.5 ms with 4)
        const char *wz = getenv("SSS_HIP_MERGE_W");
        d.mg_W = (wz && *wz) ? atoi(wz) : 4;
        d.mg_W = d.mg_W >= 4 ? 4 : d.mg_W >= 2 ? 2 : 1;
        d.ngrid = (d.mg_ng + 4 / d.mg_W - 1) / (4 / d.mg_W);
        d.mg_gp = dev_alloc<int>(gp.size());
        d.mg_k = dev_alloc<unsigned>(mk.size());
        d.mg_v = dev_alloc<double>(mv.size());
        if (!d.mg_gp || !d.mg_k || !d.mg_v) return hip_fail(hipErrorOutOfMemory, "hipMalloc(merged)", __FILE__, __LINE__);
        if (int rc = h2d(d.mg_gp, gp.data(), sizeof(int) * gp.size())) return rc;
        if (int rc = h2d(d.mg_k, mk.data(), sizeof(unsigned) * mk.size())) return rc;
        if (int rc = h2d(d.mg_v, mv.data(), sizeof(double) * mv.size())) return rc;
    }
    if (d.vec_rows && !((enc & kEncMergedOnly) && d.mg_G > 0) && device_builders_on() && d.nnz > 0)
        if (int rc = sort_rows_device(d, seg)) return rc;   // after the merged build (stored order)
    pt.mark("merged");
    // dictionary ELL first (one thread per row), else dictionary tiles (the tile kernels then stage
    // from them instead of the sorted copy)
    const char *dz = getenv("SSS_HIP_DICT");   // 0: never (tests compare both ways)
    const char *ez = getenv("SSS_HIP_ELL");    // 0: no ELL (dictionary tiles where they qualify)
    const bool based = (enc & kEncEllBase) && d.n != d.ncols;
    if ((enc & (kEncDict | kEncEll | kEncEllBase)) && !(dz && *dz == '0') && !(ez && *ez == '0') && !d.wave_rows &&
        !d.vec_rows && d.nnz > 0 && ((enc & kEncEll) || based || d.n == d.ncols)) {
        HostBuf<unsigned char> ell;
        std::vector<int4> pd;
        std::vector<int> dd;
        std::vector<double> vd;
        std::vector<int> base;
        if (based) {   // each row's first column (0 for an empty row)
            base.resize((size_t)d.n);
            parallel_chunks(d.n, 1 << 16, [&](int lo, int hi) {
                for (int r = lo; r < hi; ++r) base[r] = h.row_ptr[r] < h.row_ptr[r + 1] ? h.col_idx[h.row_ptr[r]] : 0;
            });
        }
        int W = 0;
        if (build_ell(h, blk, ell, W, pd, dd, vd, based ? base.data() : nullptr)) {
            if (based) {
                d.dv_ell_base = dev_alloc<int>(base.size());
                if (!d.dv_ell_base) return hip_fail(hipErrorOutOfMemory, "hipMalloc(ELL bases)", __FILE__, __LINE__);
                if (int rc = h2d(d.dv_ell_base, base.data(), sizeof(int) * base.size())) return rc;
            }
            d.ell_w = W;
            d.dv_ell = dev_alloc<unsigned char>(ell.size());
            d.dv_pd = dev_alloc<int4>(pd.size());
            d.dv_dd = dev_alloc<int>(dd.size());
            d.dv_vd = dev_alloc<double>(vd.size());
            if (!d.dv_ell || !d.dv_pd || !d.dv_dd || !d.dv_vd)
                return hip_fail(hipErrorOutOfMemory, "hipMalloc(dictionary ELL)", __FILE__, __LINE__);
            if (int rc = h2d(d.dv_ell, ell.data(), ell.size())) return rc;
            if (int rc = h2d(d.dv_pd, pd.data(), sizeof(int4) * pd.size())) return rc;
            if (int rc = h2d(d.dv_dd, dd.data(), sizeof(int) * dd.size())) return rc;
            if (int rc = h2d(d.dv_vd, vd.data(), sizeof(double) * vd.size())) return rc;
        }
    }
    pt.mark("ell");
    // column ELL where the 1-byte dictionary did not fit: its own 256-row blocking replaces the
    // CSR-adaptive one (no tile staging, so no entry limit per block)
    const int xshift = xell_shift_for(d.ncols);
    if ((enc & kEncXell) && !(dz && *dz == '0') && xell_on() && !d.dv_ell && !d.wave_rows && !d.vec_rows &&
        d.nnz > 0 && xshift > 0) {
        std::atomic<int> Lmax{0};
        parallel_chunks(d.n, 1 << 16, [&](int lo, int hi) {
            int L = 0;
            for (int r = lo; r < hi; ++r) L = std::max(L, h.row_ptr[r + 1] - h.row_ptr[r]);
            int cur = Lmax.load();
            while (L > cur && !Lmax.compare_exchange_weak(cur, L)) {}
        });
        // rows padded to W: not where that makes the codes larger than the CSR entries (4 W bytes
        // per row against 12 per entry: at least W / 3 entries per row on average; 7-pt level-1
        // prolongation, 3.2 entries in 8 slots: 362 -> 294 us per V-cycle)
        int W = xell_width(Lmax.load());
        if ((long long)d.nnz * 3 < (long long)W * d.n) W = 0;
        // 40-slot rows only where no range relaxation reads them (two-stage levels' matrices and split
        // copies): the relaxation kernels spill at that width
        if (W == 40 && !(enc & kEncMergedOnly)) W = 0;
        std::vector<int> xb;
        HostBuf<unsigned> codes;
        std::vector<int4> pd;
        std::vector<double> vd;
        if (W > 0 && build_xell(h, split, W, xshift, xb, codes, pd, vd)) {
            dev_free(d.blk);
            dev_free(d.bk);
            d.blk = nullptr;
            d.bk = nullptr;
            blk.swap(xb);
            d.nblk = (int)blk.size() - 1;
            d.split_blk = d.nblk;
            if (split >= 0)
                for (int q = 0; q <= d.nblk; ++q)
                    if (blk[q] >= split) { d.split_blk = q; break; }
            d.ngrid = d.nblk;
            d.blk = dev_alloc<int>(blk.size());
            if (!d.blk) return hip_fail(hipErrorOutOfMemory, "hipMalloc(blk)", __FILE__, __LINE__);
            if (int rc = h2d(d.blk, blk.data(), sizeof(int) * blk.size())) return rc;
            if (int rc = upload_block_bounds(&d.bk, blk, h.row_ptr, &d.h_bk)) return rc;
            d.xell_w = W;
            d.xell_shift = xshift;
            d.dv_xell = dev_alloc<unsigned>(codes.size());
            d.dv_pd = dev_alloc<int4>(pd.size());
            d.dv_vd = dev_alloc<double>(vd.size());
            if (!d.dv_xell || !d.dv_pd || !d.dv_vd)
                return hip_fail(hipErrorOutOfMemory, "hipMalloc(column ELL)", __FILE__, __LINE__);
            if (int rc = h2d(d.dv_xell, codes.data(), sizeof(unsigned) * codes.size())) return rc;
            if (int rc = h2d(d.dv_pd, pd.data(), sizeof(int4) * pd.size())) return rc;
            if (int rc = h2d(d.dv_vd, vd.data(), sizeof(double) * vd.size())) return rc;
        }
    }
    pt.mark("xell");
    if ((enc & kEncDict) && !(dz && *dz == '0') && !d.dv_ell && !d.dv_xell && !d.wave_rows && !d.vec_rows && d.nnz > 0) {
        HostBuf<unsigned> code;
        std::vector<int4> pd;
        std::vector<int> dd;
        std::vector<double> vd;
        if (build_dict_tiles(h, blk, code, pd, dd, vd)) {
            d.dv_code = dev_alloc<unsigned>(code.size());
            d.dv_pd = dev_alloc<int4>(pd.size());
            d.dv_dd = dev_alloc<int>(dd.size());
            d.dv_vd = dev_alloc<double>(vd.size());
            if (!d.dv_code || !d.dv_pd || !d.dv_dd || !d.dv_vd)
                return hip_fail(hipErrorOutOfMemory, "hipMalloc(dictionary tiles)", __FILE__, __LINE__);
            if (int rc = h2d(d.dv_code, code.data(), sizeof(unsigned) * code.size())) return rc;
            if (int rc = h2d(d.dv_pd, pd.data(), sizeof(int4) * pd.size())) return rc;
            if (int rc = h2d(d.dv_dd, dd.data(), sizeof(int) * dd.size())) return rc;
            if (int rc = h2d(d.dv_vd, vd.data(), sizeof(double) * vd.size())) return rc;
        }
    }
    pt.mark("dict");
    // the tile kernels of a wave-path matrix never run on the hierarchy; no sorted copy for them
    HostBuf<unsigned> pk;
    HostBuf<double> pv;
    std::vector<int2> pb;
    if ((enc & kEncSortedTiles) && !d.dv_code && !d.dv_ell && !d.dv_xell && !d.wave_rows && !d.vec_rows && d.nnz > 0 &&
        build_sorted_tiles(h, blk, pk, pv, pb)) {
        d.pk = dev_alloc<unsigned>((size_t)d.nnz);
        d.pb = dev_alloc<int2>(pb.size());
        if (!d.pk || !d.pb) return hip_fail(hipErrorOutOfMemory, "hipMalloc(sorted tiles)", __FILE__, __LINE__);
        if (int rc = h2d(d.pk, pk.data(), sizeof(unsigned) * (size_t)d.nnz)) return rc;
        if (int rc = h2d(d.pb, pb.data(), sizeof(int2) * pb.size())) return rc;
        pt.mark("sorted");
        HostBuf<unsigned char> vi;
        std::vector<int4> pd;
        std::vector<double> vd;
        if ((enc & kEncDict) && !(dz && *dz == '0') && build_value_dict(blk, h.row_ptr, pv, vi, pd, vd)) {
            d.dv_vi = dev_alloc<unsigned char>(vi.size());
            d.dv_pd = dev_alloc<int4>(pd.size());
            d.dv_vd = dev_alloc<double>(vd.size());
            if (!d.dv_vi || !d.dv_pd || !d.dv_vd)
                return hip_fail(hipErrorOutOfMemory, "hipMalloc(value dictionaries)", __FILE__, __LINE__);
            if (int rc = h2d(d.dv_vi, vi.data(), vi.size())) return rc;
            if (int rc = h2d(d.dv_pd, pd.data(), sizeof(int4) * pd.size())) return rc;
            if (int rc = h2d(d.dv_vd, vd.data(), sizeof(double) * vd.size())) return rc;
        } else {
            d.pv = dev_alloc<double>((size_t)d.nnz);
            if (!d.pv) return hip_fail(hipErrorOutOfMemory, "hipMalloc(sorted tiles)", __FILE__, __LINE__);
            if (int rc = h2d(d.pv, pv.data(), sizeof(double) * (size_t)d.nnz)) return rc;
        }
    }
    pt.mark("tiles");
    // what one SpMV over the stored format reads besides the vectors (reported for the roofline)
    const long long nnz = d.nnz, nb = d.nblk, rows = d.n;
    if (has_dict(d)) {
        long long dict = 0;
        std::vector<int4> pd((size_t)nb);
        if (nb > 0) SSS_HIP(hipMemcpy(pd.data(), d.dv_pd, sizeof(int4) * (size_t)nb, hipMemcpyDeviceToHost));
        for (const auto &p : pd) dict += 4LL * p.y + 8LL * p.w;
        d.stream_bytes = d.dv_xell ? 4LL * d.xell_w * rows + 8 * (nb + 1) + 16 * nb + dict
                         : d.dv_ell ? (long long)(d.ell_w + (d.dv_ell_base ? 4 : 0)) * rows + 8 * (nb + 1) + 16 * nb + dict
                                  : (d.dv_vi ? 5 * nnz + 8 * nb : 4 * nnz) + 4 * (rows + 1) + 8 * (nb + 1) + 16 * nb + dict;
    } else if (d.pk) {
        d.stream_bytes = 12 * nnz + 4 * (rows + 1) + 8 * (nb + 1) + 8 * nb;
    } else {
        d.stream_bytes = 12 * nnz + 4 * (rows + 1) + 8 * (nb + 1);
    }
    return 0;
}

int devcsr_sort_rows(DevCSR &d, const SSS_MAT &h, const int *seg)
{
    if (!d.vec_rows || d.rows_sorted || d.nnz == 0) return 0;
    if (device_builders_on()) return sort_rows_device(d, seg);
    HostBuf<int> sci;
    HostBuf<double> sv;
    sort_row_segments(h, seg, sci, sv);
    if (int rc = h2d(d.ci, sci.data(), sizeof(int) * (size_t)d.nnz)) return rc;
    if (int rc = h2d(d.v, sv.data(), sizeof(double) * (size_t)d.nnz)) return rc;
    d.rows_sorted = true;
    return 0;
}

void devcsr_free(DevCSR &d)
{
    dev_free(d.rp);
    dev_free(d.ci);
    dev_free(d.v);
    dev_free(d.blk);
    dev_free(d.bk);
    dev_free(d.pk);
    dev_free(d.pv);
    dev_free(d.pb);
    dev_free(d.mg_gp);
    dev_free(d.mg_k);
    dev_free(d.mg_v);
    dev_free(d.dv_code);
    dev_free(d.dv_ell);
    dev_free(d.dv_ell_base);
    dev_free(d.dv_xell);
    dev_free(d.dv_vi);
    dev_free(d.dv_pd);
    dev_free(d.dv_dd);
    dev_free(d.dv_vd);
    delete[] d.h_bk;
    d = DevCSR();
}

// ---- kernel -------------------------------------------------------------------------------
template <int OP, bool NORM, int DICT = 0>   // DICT: with_tile_kind (8/16/32: dictionary ELL, that width)
__global__ __launch_bounds__(kBlock) void spmv_adaptive(const int2 *__restrict__ blk, const int *__restrict__ rp,
                                                        const int *__restrict__ ci, const double *__restrict__ v,
                                                        const double *__restrict__ x, const double *__restrict__ b,
                                                        double *__restrict__ y, double alpha, int cap,
                                                        double *__restrict__ partial, const unsigned *__restrict__ pk,
                                                        const double *__restrict__ pv, const int2 *__restrict__ pb,
                                                        DevDict dt = DevDict())
{
    auto epi = [&](int r, double s) -> double {
        double out;
        if constexpr (OP == SSS_HIP_SPMV_MXY) out = s;
        else if constexpr (OP == SSS_HIP_SPMV_AMXPY) out = y[r] + s * alpha;
        else if constexpr (OP == SSS_HIP_SPMV_RESID) out = b[r] + s * alpha;
        else {
            if (cap > 0 && r >= cap) return 0.0;   // as-shipped <<<64,64>>> row cap
            out = y[r] + s;
        }
        y[r] = out;
        return NORM ? out * out : 0.0;
    };
    if constexpr (DICT >= kXell) {   // column ELL rows of width DICT - kXell: one thread per row
        constexpr int W = DICT - kXell;
        __shared__ XellSmem es;
        const int bid = blockIdx.x;
        unsigned w[W];
        double br = 0.0;
        int r = 0;
        bool live = false;
        const bool valid = bid < dt.bend;
#pragma unroll
        for (int t = 0; t < W; ++t) w[t] = 0xffffffffu;
        if (valid) {   // codes (and b) in flight across the dictionary's barrier
            const int2 ba = blk[bid], be = blk[bid + 1];
            r = ba.x + (int)threadIdx.x;
            live = r < be.x;
            if (live) {
                xell_codes<W>(dt.xell, r, w);
                if constexpr (OP == SSS_HIP_SPMV_RESID) br = b[r];
            }
            xell_load_dict_nosync(dt, bid, es);
        }
        __syncthreads();
        double sq = 0.0;
        if (live) {
            double xv[W];
            int ds;
            const int len = xell_gather<W>(w, r, dt.xshift, [&](int c) -> double { return x[c]; }, xv, ds);
            const double sum = xell_add(0.0, w, xv, es, dt.xshift, 0, len);
            if constexpr (OP == SSS_HIP_SPMV_RESID) {
                const double out = br + sum * alpha;
                y[r] = out;
                sq = NORM ? out * out : 0.0;
            } else {
                sq = epi(r, sum);
            }
        }
        if (NORM && valid) {
            const double t = block_sum(sq, es.red);
            if (threadIdx.x == 0) partial[bid] = t;
        }
    } else if constexpr (DICT >= 8) {   // dictionary ELL rows of width DICT: one thread per row, its sum
        constexpr int W = DICT;   // from 0.0 in stored order; kEllRpt row blocks per workgroup
        constexpr int RPT = kEllRpt;
        __shared__ EllSmem es[RPT];
        const int g = (int)blockIdx.x;
        unsigned w[RPT][W / 4];
        double br[RPT];
        int r[RPT], rb[RPT];   // rb: the row's offset base (its own index, or dt.ellb[r])
        bool live[RPT], valid[RPT];
#pragma unroll
        for (int j = 0; j < RPT; ++j) {   // codes (and b) in flight across the dictionaries' barrier
            const int bid = g * RPT + j;
            valid[j] = bid < dt.bend;
            live[j] = false;
            br[j] = 0.0;
            r[j] = rb[j] = 0;
#pragma unroll
            for (int t = 0; t < W / 4; ++t) w[j][t] = 0u;
            if (valid[j]) {
                const int2 ba = blk[bid], be = blk[bid + 1];
                r[j] = ba.x + (int)threadIdx.x;
                live[j] = r[j] < be.x;
                if (live[j]) {
                    ell_codes<W>(dt.ell, r[j], w[j]);
                    rb[j] = dt.ellb ? dt.ellb[r[j]] : r[j];
                    if constexpr (OP == SSS_HIP_SPMV_RESID) br[j] = b[r[j]];
                }
                ell_load_dicts_nosync(dt, bid, es[j]);
            }
        }
        __syncthreads();
#pragma unroll
        for (int j = 0; j < RPT; ++j) {
            double sq = 0.0;
            if (live[j]) {
                double p[W];
                int ds;
                double dv;
                const int len = ell_decode<W>(w[j], rb[j], es[j], [&](int c) -> double { return x[c]; }, p, ds, dv);
                if constexpr (OP == SSS_HIP_SPMV_RESID) {
                    const double out = br[j] + ell_add(0.0, p, 0, len) * alpha;
                    y[r[j]] = out;
                    sq = NORM ? out * out : 0.0;
                } else {
                    sq = epi(r[j], ell_add(0.0, p, 0, len));
                }
            }
            if (NORM && valid[j]) {
                const double t = block_sum(sq, es[j].red);
                if (threadIdx.x == 0) partial[g * RPT + j] = t;
            }
        }
    } else {
        __shared__ SpmvSmem sm;
        __shared__ std::conditional_t<DICT != 0, DictSmem, char> dsm;
        DictSmem *ds = nullptr;
        if constexpr (DICT != 0) ds = &dsm;
        const double sq = csr_block_rows(blk, rp, ci, v, x, sm, epi, pk, pv, pb, &dt, ds);
        if (NORM) {
            const double t = block_sum(sq, sm.red);
            if (threadIdx.x == 0) partial[xcd_bid()] = t;
        }
    }
}

// Long rows: one wave per row.  TREE = false: lane 0 chains the products in stored order
// (bitwise); TREE = true: free-order tree sum (DevCSR::vec_rows).
template <int OP, bool NORM, bool TREE>
__global__ __launch_bounds__(kBlock) void spmv_wave(int n, const int *__restrict__ rp, const int *__restrict__ ci,
                                                    const double *__restrict__ v, const double *__restrict__ x,
                                                    const double *__restrict__ b, double *__restrict__ y, double alpha,
                                                    int cap, double *__restrict__ partial)
{
    __shared__ __attribute__((aligned(16))) double strips[TREE ? 1 : 4][TREE ? 1 : kWaveStage];
    __shared__ double red[kBlock / 64];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int r = xcd_bid() * 4 + wave;
    double sq = 0.0;
    if (r < n) {
        auto prod = [&](int c, double a) { return a * x[c]; };
        const double s = TREE ? wave_row_sum(rp[r], rp[r + 1], ci, v, prod)
                              : wave_row_chain<false>(rp[r], rp[r + 1], ci, v, prod, 0.0, strips[TREE ? 0 : wave]);
        if (lane == 0) {
            bool write = true;
            double out;
            if constexpr (OP == SSS_HIP_SPMV_MXY) out = s;
            else if constexpr (OP == SSS_HIP_SPMV_AMXPY) out = y[r] + s * alpha;
            else if constexpr (OP == SSS_HIP_SPMV_RESID) out = b[r] + s * alpha;
            else {
                write = !(cap > 0 && r >= cap);
                out = write ? y[r] + s : 0.0;
            }
            if (write) y[r] = out;
            if (NORM) sq = out * out;
        }
    }
    if (NORM) {
        const double t = block_sum(sq, red);
        if (threadIdx.x == 0) partial[xcd_bid()] = t;
    }
}

// Free order, merged row groups (DevCSR::mg_*): W waves per group of G rows (merged_block).
template <int OP, bool NORM, int G>
__global__ __launch_bounds__(kBlock) void spmv_merged(int n, int ng, int W, const int *__restrict__ gp,
                                                      const unsigned *__restrict__ mk, const double *__restrict__ mv,
                                                      const double *__restrict__ x, const double *__restrict__ b,
                                                      double *__restrict__ y, double alpha, int cap,
                                                      double *__restrict__ partial)
{
    __shared__ double red[8 * G];
    __shared__ double nred[kBlock / 64];
    int g = 0, u = 0;
    double sr = 0.0, unused = 0.0, sq = 0.0;
    if (merged_block<G, 1>(gp, ng, W, mk, mv, [&](int c) -> double { return x[c]; }, red, g, u, sr, unused)) {
        const int r = g * G + u;
        if (r < n) {
            bool write = true;
            double out;
            if constexpr (OP == SSS_HIP_SPMV_MXY) out = sr;
            else if constexpr (OP == SSS_HIP_SPMV_AMXPY) out = y[r] + sr * alpha;
            else if constexpr (OP == SSS_HIP_SPMV_RESID) out = b[r] + sr * alpha;
            else {
                write = !(cap > 0 && r >= cap);
                out = write ? y[r] + sr : 0.0;
            }
            if (write) y[r] = out;
            if (NORM) sq = out * out;
        }
    }
    if (NORM) {
        const double t = block_sum(sq, nred);
        if (threadIdx.x == 0) partial[xcd_bid()] = t;
    }
}

template <int OP, bool NORM>
static void launch_op(const DevCSR &A, double alpha, const double *x, const double *b, double *y, int cap,
                      double *partial, hipStream_t s)
{
    if (A.mg_G == 8)
        hipLaunchKernelGGL((spmv_merged<OP, NORM, 8>), dim3(A.ngrid), dim3(kBlock), 0, s, A.n, A.mg_ng, A.mg_W,
                           A.mg_gp, A.mg_k, A.mg_v, x, b, y, alpha, cap, partial);
    else if (A.mg_G == 4)
        hipLaunchKernelGGL((spmv_merged<OP, NORM, 4>), dim3(A.ngrid), dim3(kBlock), 0, s, A.n, A.mg_ng, A.mg_W,
                           A.mg_gp, A.mg_k, A.mg_v, x, b, y, alpha, cap, partial);
    else if (A.vec_rows)
        hipLaunchKernelGGL((spmv_wave<OP, NORM, true>), dim3(A.ngrid), dim3(kBlock), 0, s, A.n, A.rp, A.ci, A.v, x,
                           b, y, alpha, cap, partial);
    else if (A.wave_rows)
        hipLaunchKernelGGL((spmv_wave<OP, NORM, false>), dim3(A.ngrid), dim3(kBlock), 0, s, A.n, A.rp, A.ci, A.v, x,
                           b, y, alpha, cap, partial);
    else
        with_tile_kind(A, [&](auto K) {
            constexpr int KK = decltype(K)::value;
            DevDict dt = devdict(A, 0);
            dt.bend = A.nblk;
            const int grid = (A.nblk + rows_per_wg(KK) - 1) / rows_per_wg(KK);
            hipLaunchKernelGGL((spmv_adaptive<OP, NORM, KK>), dim3(grid), dim3(kBlock), 0, s, A.bk, A.rp, A.ci, A.v, x,
                               b, y, alpha, cap, partial, A.pk, A.pv, A.pb, dt);
        });
}

// ledger: row vectors an SpMV op streams besides the gathered x (MXY writes y; the others read b or y
// and write y)
static double spmv_row_bytes(int op) { return op == SSS_HIP_SPMV_MXY ? 8.0 : 16.0; }

int launch_spmv(const DevCSR &A, int op, double alpha, const double *x, const double *b, double *y, int cap,
                double *partial, hipStream_t stream)
{
    if (A.n == 0 || A.nblk == 0) return 0;
    if (ledger_on()) ledger_add(matrix_bytes(A, 0, A.nblk) + xgather_bytes(A, A.n) + spmv_row_bytes(op) * A.n);
    switch (op) {
    case SSS_HIP_SPMV_MXY: launch_op<SSS_HIP_SPMV_MXY, false>(A, alpha, x, b, y, cap, nullptr, stream); break;
    case SSS_HIP_SPMV_AMXPY: launch_op<SSS_HIP_SPMV_AMXPY, false>(A, alpha, x, b, y, cap, nullptr, stream); break;
    case SSS_HIP_SPMV_RESID:
        if (partial) launch_op<SSS_HIP_SPMV_RESID, true>(A, alpha, x, b, y, cap, partial, stream);
        else launch_op<SSS_HIP_SPMV_RESID, false>(A, alpha, x, b, y, cap, nullptr, stream);
        break;
    case SSS_HIP_SPMV_ACC: launch_op<SSS_HIP_SPMV_ACC, false>(A, alpha, x, b, y, cap, nullptr, stream); break;
    default: return ERROR_INPUT_PAR;
    }
    SSS_HIP(hipGetLastError());
    return 0;
}

// x_r += P e over C rows whose prolongation row is one stored 1.0 (the injection of the C point's
// coarse value; sss_hier.hip hb_level_pr finds them): the tile AMXPY epilogue's arithmetic --
// s = 0.0 + 1.0 * e_c from the stored-order chain, out = x_r + s * 1.0 -- without the CSR arrays,
// their row blocks or the LDS staging.
__global__ __launch_bounds__(kBlock) void prolong_inject(int m, int lo, const int *__restrict__ col,
                                                         const double *__restrict__ e, double *__restrict__ x)
{
    const int q = blockIdx.x * kBlock + (int)threadIdx.x;
    if (q < m) {
        const double s = 0.0 + 1.0 * e[col[q]];
        x[lo + q] = x[lo + q] + s * 1.0;
    }
}

int launch_prolong_inject(int m, int lo, const int *col, const double *e, double *x, hipStream_t s)
{
    if (m <= 0) return 0;
    ledger_add(28.0 * m);   // col, the gathered e, x read and written
    hipLaunchKernelGGL(prolong_inject, dim3((m + kBlock - 1) / kBlock), dim3(kBlock), 0, s, m, lo, col, e, x);
    SSS_HIP(hipGetLastError());
    return 0;
}

int launch_spmv_range(const DevCSR &A, int blo, int bhi, int op, double alpha, const double *x, const double *b,
                      double *y, double *partial, hipStream_t s)
{
    if (A.wave_rows || A.vec_rows || blo < 0 || bhi > A.nblk) return ERROR_INPUT_PAR;
    if (op != SSS_HIP_SPMV_RESID && op != SSS_HIP_SPMV_AMXPY && op != SSS_HIP_SPMV_MXY) return ERROR_INPUT_PAR;
    const int nb = bhi - blo;
    if (nb <= 0) return 0;
    if (ledger_on()) {
        const double rows = A.h_bk ? A.h_bk[bhi].x - A.h_bk[blo].x : (double)A.n * nb / A.nblk;
        ledger_add(matrix_bytes(A, blo, bhi) + xgather_bytes(A, rows) + spmv_row_bytes(op) * rows);
    }
    // the kernel indexes blocks from 0: shift the block-indexed arrays
    const int2 *pb = A.pb ? A.pb + blo : nullptr;
    double *pp = partial ? partial + blo : nullptr;
    DevDict dt = devdict(A, blo);
    dt.bend = nb;   // the kernel sees blocks [0, nb)
    auto go = [&](auto op_c, auto norm_c) {
        constexpr int O = decltype(op_c)::value;
        constexpr bool NM = decltype(norm_c)::value;
        with_tile_kind(A, [&](auto K) {
            constexpr int KK = decltype(K)::value;
            const int grid = (nb + rows_per_wg(KK) - 1) / rows_per_wg(KK);
            hipLaunchKernelGGL((spmv_adaptive<O, NM, KK>), dim3(grid), dim3(kBlock), 0, s, A.bk + blo, A.rp, A.ci, A.v,
                               x, b, y, alpha, 0, pp, A.pk, A.pv, pb, dt);
        });
    };
    using T = std::true_type;
    using F = std::false_type;
    if (op == SSS_HIP_SPMV_AMXPY) go(std::integral_constant<int, SSS_HIP_SPMV_AMXPY>(), F());
    else if (op == SSS_HIP_SPMV_MXY) go(std::integral_constant<int, SSS_HIP_SPMV_MXY>(), F());
    else if (partial) go(std::integral_constant<int, SSS_HIP_SPMV_RESID>(), T());
    else go(std::integral_constant<int, SSS_HIP_SPMV_RESID>(), F());
    SSS_HIP(hipGetLastError());
    return 0;
}

// ---- deterministic final reduction ----------------------------------------------------------
// Two fixed-order stages: kFinalChunks workgroups each reduce one contiguous chunk of the partials
// (lane-strided sums + xor tree + waves in order) into scratch[b]; one workgroup then sums those.
// A single workgroup streaming all 250,000 level-0 partials took ~100 us; two stages take ~10 us.
constexpr int kFinalChunks = kFinalScratch;

__device__ __forceinline__ double block_sum_1024(double v, double *red)
{
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
    __syncthreads();
    double t = 0.0;
    if (threadIdx.x == 0)
        for (int w = 0; w < 1024 / 64; ++w) t += red[w];
    return t;
}

__global__ __launch_bounds__(1024) void final_sum_chunks(const double *__restrict__ partials, int n, int chunk,
                                                         double *__restrict__ scratch)
{
    __shared__ double red[1024 / 64];
    const int a = blockIdx.x * chunk, e = min(n, a + chunk);
    double v = 0.0;
    for (int i = a + (int)threadIdx.x; i < e; i += 1024) v += partials[i];
    const double t = block_sum_1024(v, red);
    if (threadIdx.x == 0) scratch[blockIdx.x] = t;
}

__global__ __launch_bounds__(1024) void final_sum_kernel(const double *__restrict__ partials, int n,
                                                         double *__restrict__ out, int take_sqrt)
{
    __shared__ double red[1024 / 64];
    double v = 0.0;
    for (int i = threadIdx.x; i < n; i += 1024) v += partials[i];
    const double t = block_sum_1024(v, red);
    if (threadIdx.x == 0) *out = take_sqrt ? sqrt(t) : t;
}

// partials must have room for n + kFinalChunks doubles (the tail is the first stage's scratch)
int launch_final_sum(double *partials, int n, double *out, bool take_sqrt, hipStream_t s)
{
    ledger_add(8.0 * n);
    if (n > 4 * 1024) {
        const int chunk = (n + kFinalChunks - 1) / kFinalChunks, nb = (n + chunk - 1) / chunk;
        hipLaunchKernelGGL(final_sum_chunks, dim3(nb), dim3(1024), 0, s, partials, n, chunk, partials + n);
        hipLaunchKernelGGL(final_sum_kernel, dim3(1), dim3(1024), 0, s, partials + n, nb, out, take_sqrt ? 1 : 0);
    } else {
        hipLaunchKernelGGL(final_sum_kernel, dim3(1), dim3(1024), 0, s, partials, n, out, take_sqrt ? 1 : 0);
    }
    SSS_HIP(hipGetLastError());
    return 0;
}

}  // namespace sss

// ---- C ABI: plans over caller-owned device CSR ----------------------------------------------
struct sss_hip_spmv_plan {
    sss::DevCSR csr;   // rp/ci/v borrowed from the caller (not owned); blk owned
};

extern "C" sss_hip_spmv_plan *sss_hip_spmv_plan_create(int n, int nnz, const int *d_rp, const int *h_rp)
{
    auto *p = new sss_hip_spmv_plan();
    std::vector<int> blk;
    p->csr.n = n;
    p->csr.nnz = nnz;
    p->csr.rp = const_cast<int *>(d_rp);
    p->csr.nblk = sss::build_row_blocks(h_rp, n, blk);
    p->csr.wave_rows = n > 0 && (long long)nnz >= (long long)sss::wave_row_min() * n;
    p->csr.ngrid = p->csr.wave_rows ? (n + 3) / 4 : p->csr.nblk;
    p->csr.blk = sss::dev_alloc<int>(blk.size());
    if (!p->csr.blk || hipMemcpy(p->csr.blk, blk.data(), sizeof(int) * blk.size(), hipMemcpyHostToDevice) != hipSuccess ||
        sss::upload_block_bounds(&p->csr.bk, blk, h_rp)) {
        sss::dev_free(p->csr.blk);
        sss::dev_free(p->csr.bk);
        delete p;
        return nullptr;
    }
    return p;
}

extern "C" void sss_hip_spmv_plan_destroy(sss_hip_spmv_plan *p)
{
    if (!p) return;
    sss::dev_free(p->csr.blk);
    sss::dev_free(p->csr.bk);
    delete p;
}

extern "C" int sss_hip_spmv(const sss_hip_spmv_plan *p, int op, double alpha, const int *d_rp, const int *d_ci,
                            const double *d_v, const double *d_x, const double *d_b, double *d_y, int cap,
                            void *stream)
{
    sss::DevCSR A = p->csr;
    A.rp = const_cast<int *>(d_rp);
    A.ci = const_cast<int *>(d_ci);
    A.v = const_cast<double *>(d_v);
    return sss::launch_spmv(A, op, alpha, d_x, d_b, d_y, cap, nullptr, (hipStream_t)stream);
}
