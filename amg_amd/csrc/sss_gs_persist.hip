// sss_gs_persist.hip — exact GS-CF class passes with intra-class couplings as ONE launch per pass
// (replaces the one-launch-per-DAG-depth schedule of sss_smooth.hip for SSS_amg_smoother_gs_cf,
// Solve/SSS_smooth.c:4-87; results bitwise identical: every row forms
//     t = b_i - sum_{k: j_k != i} a_k x_{j_k}    in stored order from b_i, then x_i = t / d
// with exactly the x values the sequential reference reads).
//
// Two engines, chosen per pass at plan time by a cost estimate (SSS_HIP_GS_ENGINE overrides):
//
//  * "cu"   — the whole pass in ONE workgroup of 16 waves (one CU).  Rows are taken in depth order
//             from an LDS ticket; a row of depth d waits until every row of depth d-1 has finished
//             (per-depth completion counters in LDS, workgroup-scope release/acquire), so the
//             hand-off between dependent rows costs an LDS round trip, not a cross-CU hop.  Kept
//             for comparison (SSS_HIP_GS_ENGINE=cu): measured slower than flow on every level of
//             7-pt 256^3 -- one CU streams too slowly, and a dependent step is dominated by the
//             row's own in-order chain either way.
//  * "flow" — dataflow over the whole chip (the default): waves dequeue chunks (64 / G rows of one
//             depth, G lanes per row) in depth order from an agent-scope ticket, stage every product
//             they can form before waiting, and finish as soon as the rows they read are done.  A finished row publishes its value as two self-validating
//             8-byte granules {epoch, half of x_i} (sc1 stores; MI355X_MICROARCH.md Valid forms, R2:
//             the data is the flag); a reader of a same-class lower neighbour re-reads its granules
//             (sc1 loads) until both tags carry this launch's epoch.  Old values (same class, j > i)
//             and the other class's values are read from x with plain loads: they do not change
//             during the pass, because a same-class upper neighbour j of i reads x_i and therefore
//             waits for i (the pass requires a structurally symmetric same-class coupling, checked
//             at plan time).  Made for the wide levels (thousands of short rows per depth).
//
// Both engines need the pass's rows to be a contiguous range [lo, hi) (relabeled levels) and make
// progress without any residency assumption (tickets are handed out in depth order, a wave only
// waits for rows whose tickets were handed out earlier).  Every spin is bounded: a pass that
// stalls for ~0.5 s gives up and sets an error word (the engine reports it; results are then
// garbage, but no wave spins forever).  The error word is the hierarchy's (GsPersist::err): the
// engine reads it back with the residual norm and fails loudly (sss_hier.hip).  SSS_HIP_GS_SPIN
// sets the spin limit (test hook: a negative limit reports a stall from every launch).
#include "sss_engine.hpp"
#include "sss_spmv_dev.hpp"

#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <map>
#include <string>
#include <type_traits>

namespace sss {

constexpr int kCuWaves = 16;               // waves of the single-CU engine (1024 threads)
constexpr int kCuMaxDepth = 7168;          // LDS completion counters (28 KiB)
constexpr int kSpinLimit = 1 << 22;        // LDS polls before a cu wave gives up (~0.5 s with s_sleep)
constexpr int kFlowSpinLimit = 1 << 18;    // granule polls before a flow wave gives up (~0.5 s)

// control words of a flow pass: [0] epoch of the last completed launch, [1] ticket, [2] waves that
// have exited, [3] error (stall) flag; from word kCtlShard0 the fused engine's ticket shards, one per
// 128-byte line
constexpr int kTicketShards = 8, kCtlShardStride = 32;
enum { kCtlEpoch = 0, kCtlTicket = 1, kCtlExit = 2, kCtlErr = 3, kCtlShard0 = 32,
       kCtlWords = kCtlShard0 + kTicketShards * kCtlShardStride };

#define RLX_AGENT __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT

__device__ __forceinline__ double x_own(double *x, int i)   // a row's own value, never via the scalar cache
{
    return __longlong_as_double(
        (long long)__hip_atomic_load(reinterpret_cast<unsigned long long *>(x + i), RLX_AGENT));
}

// ---- flow engine -------------------------------------------------------------------------------
__device__ __forceinline__ bool granule_get(const unsigned long long *g, unsigned epoch, double &val)
{
    const unsigned long long a = __hip_atomic_load(const_cast<unsigned long long *>(g), RLX_AGENT);
    const unsigned long long c = __hip_atomic_load(const_cast<unsigned long long *>(g + 1), RLX_AGENT);
    if ((unsigned)(a >> 32) != epoch || (unsigned)(c >> 32) != epoch) return false;
    val = __longlong_as_double((long long)((c << 32) | (a & 0xffffffffull)));
    return true;
}
__device__ __forceinline__ void granule_put(unsigned long long *g, unsigned epoch, double v)
{
    const unsigned long long u = (unsigned long long)__double_as_longlong(v);
    __hip_atomic_store(g, ((unsigned long long)epoch << 32) | (u & 0xffffffffull), RLX_AGENT);
    __hip_atomic_store(g + 1, ((unsigned long long)epoch << 32) | (u >> 32), RLX_AGENT);
}
// x_j of a same-class lower neighbour: spin on its granules (bounded by `spin` polls)
__device__ __forceinline__ double granule_wait(const unsigned long long *g, unsigned epoch, unsigned *err, int spin)
{
    double v = 0.0;
    for (int s = 0; !granule_get(g, epoch, v); ++s) {
        // give up after the limit, or at once when another wave already did (checked every 64 polls)
        if (s >= spin || ((s & 63) == 63 && __hip_atomic_load(err, RLX_AGENT))) {
            __hip_atomic_store(err, 1u, RLX_AGENT);
            return 0.0;
        }
        if (s < 16) __builtin_amdgcn_s_sleep(1);   // back off: polls load the memory system
        else __builtin_amdgcn_s_sleep(8);
    }
    return v;
}

__device__ __forceinline__ void flow_exit(unsigned *ctl, unsigned epoch, unsigned *err, int spin)
{
    if (spin < 0 && (threadIdx.x & 63) == 0) __hip_atomic_store(err, 1u, RLX_AGENT);   // test hook
    // the last wave out resets the ticket and the exit count and publishes the epoch for the next
    // launch (visible to it across the kernel boundary)
    const unsigned total = gridDim.x * (blockDim.x >> 6);
    if ((threadIdx.x & 63) == 0 && __hip_atomic_fetch_add(&ctl[kCtlExit], 1u, RLX_AGENT) == total - 1) {
        __hip_atomic_store(&ctl[kCtlTicket], 0u, RLX_AGENT);
        for (int c = 0; c < kTicketShards; ++c) __hip_atomic_store(&ctl[kCtlShard0 + c * kCtlShardStride], 0u, RLX_AGENT);
        __hip_atomic_store(&ctl[kCtlExit], 0u, RLX_AGENT);
        __hip_atomic_store(&ctl[kCtlEpoch], epoch, RLX_AGENT);
    }
}

// Next ticket for the whole wave.  Every lane takes part in the atomic (lane 0 adds 1, the others
// 0) and the result is read from the first lane into a scalar register: the loop around it then
// has a uniform exit, so the compiler keeps the wave converged (a lane-0-only atomic followed by a
// __shfl lets the structurizer split the loop and broadcast from an inactive lane).
__device__ __forceinline__ int flow_ticket(unsigned *ctl)
{
    const unsigned inc = (threadIdx.x & 63) == 0 ? 1u : 0u;
    return __builtin_amdgcn_readfirstlane((int)__hip_atomic_fetch_add(&ctl[kCtlTicket], inc, RLX_AGENT));
}

// Next local ticket of a shard counter: one lane's atomic (the others add nothing and issue
// nothing), its result read back from lane 0 -- the wave is converged at every call site (a loop head
// whose exit depends on this uniform value only).
__device__ __forceinline__ int flow_ticket_at(unsigned *w)
{
    unsigned t = 0;
    if ((threadIdx.x & 63) == 0) t = __hip_atomic_fetch_add(w, 1u, RLX_AGENT);
    return __builtin_amdgcn_readfirstlane((int)t);
}

// s - p[a] - p[a+1] - ... - p[e-1] in order (chain_fixed: 16-byte pair reads a group of 16 ahead,
// each group's 16 dependent fp64 subtractions in one asm block; reads up to 16 products past e,
// inside the workgroup's LDS row buffers or past the allocation's end, values unused)
__device__ __forceinline__ double chain_sub_pipe(double s, const double *p, int a, int e)
{
    if ((a & 1) && a < e) s -= p[a++];   // 16-byte alignment of the pair reads
    return a < e ? chain_fixed<true, 16>(s, p + a, e - a) : s;
}

constexpr int kGroupBuf = 2048;   // staged products per wave (16 KiB; 64 KiB per workgroup)

// R = 64 / G rows of one depth per ticket, G lanes per row.  Per row and per round of up to
// 32 G entries: (A) the G lanes load the entries and form every product whose x is final --
// the other class, same-class upper neighbours (old values) and lower neighbours whose granules
// are already published -- into the wave's LDS row buffer, keeping a bit per still-pending entry;
// (B) they wait for the pending granules and fill those products; (C) the row's first lane runs
// the stored-order chain over the buffer.  A row never waits before all its own loads are issued.
template <int G, bool NAT, bool DESC>
__global__ __launch_bounds__(kBlock) void gs_flow_group(int nchunks, const int *__restrict__ ck,
                                                        const int *__restrict__ rows, const int *__restrict__ rp,
                                                        const int *__restrict__ ci, const double *__restrict__ v,
                                                        const double *__restrict__ b, double *x,
                                                        const double *__restrict__ deff, unsigned long long *gran,
                                                        int lo, int hi, unsigned *ctl, unsigned *err, int spin, int ovl,
                                                        unsigned long long *trace)
{
    // U: a lane's entries per staging group (8; 4 and 16 measured no faster at 400^3)
    constexpr int R = 64 / G, CAP = kGroupBuf / R, U = 8;
    // a same-pass row this row reads the NEW value of (published by its granules)
    auto dynamic = [&](int c, int i) { return DESC ? (c > i && c < hi) : (c >= lo && c < i); };
    static_assert(CAP / G == 32, "one pending bit per staged entry of a lane");
    __shared__ __attribute__((aligned(16))) double buf[kBlock / 64][kGroupBuf];
    const int lane = threadIdx.x & 63, grp = lane / G, gl = lane % G;
    double *mine = buf[threadIdx.x >> 6] + grp * CAP;
    const unsigned epoch = __hip_atomic_load(&ctl[kCtlEpoch], RLX_AGENT) + 1u;
    for (;;) {
        const int q = flow_ticket(ctl);
        // diagnostic builds (SSS_GS_TRACE): per row, 100 MHz stamps at the ticket, after staging, at the publish
        const unsigned long long t_ticket = trace ? __builtin_amdgcn_s_memrealtime() : 0ull;
        unsigned long long t_staged = 0ull;
        if (q >= nchunks) break;
        const int p = ck[q] + grp;
        const bool active = p < ck[q + 1];
        int i = -1, k0 = 0, len = 0;
        double acc = 0.0, dr = 0.0;
        if (active) {
            i = rows[p];
            k0 = rp[i];
            len = rp[i + 1] - k0;
            acc = b[i];
            dr = deff[i];   // loaded now: after the chain it would be a round trip on the critical path
        }
        int maxlen = len;
        for (int off = 32; off > 0; off >>= 1) maxlen = max(maxlen, __shfl_xor(maxlen, off, 64));
        maxlen = __builtin_amdgcn_readfirstlane(maxlen);
        for (int base = 0; base < maxlen; base += CAP) {
            const int m = active ? min(CAP, len - base) : 0;
            const int nj = m > gl ? (m - gl + G - 1) / G : 0;   // this lane's entries t = gl + G j
            const int kb = k0 + base;
            unsigned pend = 0;
            for (int j0 = 0; j0 < nj; j0 += U) {   // (A)
                int c[U];
                double a[U], xv[U];
                // every load of the group unconditional (slots past the row re-read its entry gl,
                // then read as the diagonal): loads under a condition were issued one round trip
                // at a time; the x value of a same-pass entry is fetched too and left unused
#pragma unroll
                for (int u = 0; u < U; ++u) c[u] = ci[kb + (j0 + u < nj ? gl + G * (j0 + u) : gl)];
#pragma unroll
                for (int u = 0; u < U; ++u) a[u] = v[kb + (j0 + u < nj ? gl + G * (j0 + u) : gl)];
#pragma unroll
                for (int u = 0; u < U; ++u) xv[u] = x[c[u]];
#pragma unroll
                for (int u = 0; u < U; ++u) c[u] = j0 + u < nj ? c[u] : i;
                // the group's granule polls issued together, read after the loop (a poll read
                // inside its own condition waited for its round trip before the next was issued)
                unsigned long long ga[U], gc[U];
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    ga[u] = gc[u] = 0ull;
                    if (dynamic(c[u], i)) {
                        const unsigned long long *gg = gran + 2 * (size_t)(c[u] - lo);
                        ga[u] = __hip_atomic_load(const_cast<unsigned long long *>(gg), RLX_AGENT);
                        gc[u] = __hip_atomic_load(const_cast<unsigned long long *>(gg + 1), RLX_AGENT);
                    }
                }
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    if (j0 + u >= nj) continue;
                    const int t = gl + G * (j0 + u);
                    double val = 0.0;   // the diagonal: subtracting +0.0 is the identity
                    if (dynamic(c[u], i)) {
                        if ((unsigned)(ga[u] >> 32) == epoch && (unsigned)(gc[u] >> 32) == epoch)
                            val = a[u] * __longlong_as_double((long long)((gc[u] << 32) | (ga[u] & 0xffffffffull)));
                        else {
                            pend |= 1u << (j0 + u);
                            if (ovl) val = __longlong_as_double((long long)c[u]);   // its column, until resolved
                        }
                    } else if (c[u] != i) {
                        val = a[u] * xv[u];
                    }
                    mine[t] = val;
                }
            }
            if (!ovl) {
                while (pend) {   // (B)
                    const int j = __builtin_ctz(pend);
                    pend &= pend - 1;
                    const int t = gl + G * j;
                    const int c = ci[kb + t];
                    mine[t] = v[kb + t] * granule_wait(gran + 2 * (size_t)(c - lo), epoch, err, spin);
                }
                wave_sync();
                if (gl == 0 && m > 0) acc = chain_sub_pipe(acc, mine, 0, m);   // (C)
                wave_sync();
                continue;
            }
            if (trace && base == 0) t_staged = __builtin_amdgcn_s_memrealtime();
            // (B) and (C) interleaved: the row's first lane chains over the prefix of entries whose
            // products are staged while the pending granules are polled, the poll loads issued
            // before each chain segment and read after it.  The chain still adds every product in
            // stored order from b_i; it only stops at the first entry still pending.
            wave_sync();
            int k = 0, idle = 0;
            for (;;) {
                // the row group's first pending entry: the chain may run up to it
                int first = pend ? gl + G * __builtin_ctz(pend) : CAP;
#pragma unroll
                for (int off = G / 2; off > 0; off >>= 1) first = min(first, __shfl_xor(first, off, 64));
                const int lim = min(first, m);
                // issue this lane's two lowest pending polls (column from LDS, granule halves, value)
                constexpr int NP = 2;
                int tp[NP];
                unsigned long long ga[NP], gc[NP];
                double ap[NP];
                {
                    unsigned q = pend;
#pragma unroll
                    for (int h = 0; h < NP; ++h) {
                        tp[h] = -1;
                        ga[h] = gc[h] = 0;
                        ap[h] = 0.0;
                        if (q) {
                            tp[h] = gl + G * __builtin_ctz(q);
                            q &= q - 1;
                            const int cp = (int)__double_as_longlong(mine[tp[h]]);
                            const unsigned long long *gg = gran + 2 * (size_t)(cp - lo);
                            ga[h] = __hip_atomic_load(const_cast<unsigned long long *>(gg), RLX_AGENT);
                            gc[h] = __hip_atomic_load(const_cast<unsigned long long *>(gg + 1), RLX_AGENT);
                            ap[h] = v[kb + tp[h]];
                        }
                    }
                }
                const bool advance = gl == 0 && k < lim;
                if (advance) acc = chain_sub_pipe(acc, mine, k, lim);   // (C), overlapping the polls
                if (gl == 0) k = max(k, lim);
                bool got = false;
#pragma unroll
                for (int h = 0; h < NP; ++h)
                    if (tp[h] >= 0 && (unsigned)(ga[h] >> 32) == epoch && (unsigned)(gc[h] >> 32) == epoch) {
                        mine[tp[h]] = ap[h] * __longlong_as_double((long long)((gc[h] << 32) | (ga[h] & 0xffffffffull)));
                        pend &= ~(1u << ((tp[h] - gl) / G));
                        got = true;
                    }
                const bool rowdone = gl != 0 || k >= m;
                if (__all(rowdone && !pend)) break;
                wave_sync();   // resolved products visible to the chain lane (LDS, same wave)
                if (__any(got || advance)) {
                    idle = 0;
                } else {
                    // give up after the limit (as granule_wait), or at once when another wave did
                    if (++idle >= spin || ((idle & 63) == 63 && __hip_atomic_load(err, RLX_AGENT))) {
                        if (gl == 0) __hip_atomic_store(err, 1u, RLX_AGENT);
                        while (pend) {   // garbage results, but every wave reaches the exit
                            mine[gl + G * __builtin_ctz(pend)] = 0.0;
                            pend &= pend - 1;
                        }
                        wave_sync();
                        if (gl == 0 && k < m) acc = chain_sub_pipe(acc, mine, k, m);
                        if (gl == 0) k = m;
                        break;
                    }
                    if (idle < 16) __builtin_amdgcn_s_sleep(1);
                    else __builtin_amdgcn_s_sleep(8);
                }
            }
            wave_sync();
        }
        if (active && gl == 0) {
            const double d = dr;
            // natural order (Solve/SSS_smooth.c:112): x_i = t * d, d the carried reciprocal
            const double xn = NAT ? acc * d : fabs(d) > SMALLFLOAT ? acc / d : x_own(x, i);
            // the granules first: this pass's readers of x_i wait on them, x itself is read later
            granule_put(gran + 2 * (size_t)(i - lo), epoch, xn);
            if (trace) {
                unsigned long long *tr = trace + 4 * (size_t)p;
                tr[0] = t_ticket, tr[1] = t_staged, tr[2] = __builtin_amdgcn_s_memrealtime(), tr[3] = (unsigned)len;
            }
            x[i] = xn;
        }
    }
    flow_exit(ctl, epoch, err, spin);
}

// ---- fused engine: all passes of a smoother call in one launch ---------------------------------
// Node (i, s) is row i's update in sweep s; it produces version s + 1 of x_i (version 0: x before
// the call).  Per sweep the F pass runs before the C pass (Solve/SSS_smooth.c:4-87, both smoother
// directions), so the version of a neighbour j that node (i, s) reads is
//     same class: j < i -> s + 1, j > i -> s;     j in F, i in C: s + 1;     j in C, i in F: s.
// Version 0 is read from x (no node writes x before the last sweep); later versions from j's
// granules, tagged epoch << 4 | version.  On a structurally symmetric level a granule holds every
// version long enough: each reader of version v of x_j is read by j's next update (at a version
// the reader produces), so version v + 1 cannot be published before all readers of v are done,
// and tickets in fused-DAG depth order (every dependency one depth lower) are a topological order
// -- the same progress argument as the per-pass flow engine.  Versions s of row i and every
// neighbour's versions are therefore ordered before node (i, s) publishes, which overlaps the
// tail of each pass with the head of the next (the per-pass launches wait for a whole pass).
__device__ __forceinline__ int fused_need(int c, int i, int s, int split)
{
    const bool cc = c >= split, ic = i >= split;
    return cc == ic ? (c < i ? s + 1 : s) : (cc ? s : s + 1);
}

template <int G>
__global__ __launch_bounds__(kBlock) void gs_fused_group(int nchunks, const int *__restrict__ ck,
                                                         const int *__restrict__ nodes, int n, int split, int last,
                                                         const int *__restrict__ rp, const int *__restrict__ ci,
                                                         const double *__restrict__ v, const double *__restrict__ b,
                                                         double *x, const double *__restrict__ d_first,
                                                         const double *__restrict__ d_later, unsigned long long *gran,
                                                         unsigned *ctl, unsigned *err, int spin, int ovl,
                                                         const int *__restrict__ rp0, const int *__restrict__ ci0,
                                                         const double *__restrict__ v0, int shards)
{
    constexpr int R = 64 / G, CAP = kGroupBuf / R, U = 8;
    // tickets from `nt` counters: shard c hands out chunks c, c + nt, c + 2 nt, ... in order, each
    // to the waves of the workgroups blockIdx = c mod nt.  Every shard's sequence is a subsequence of
    // the topological order and every shard has waves, so the lowest unfinished chunk is always held
    // by a wave whose inputs are final (or is next in its shard, whose waves then hold only finished
    // chunks): no deadlock, as with one counter, at up to nt times its atomic throughput.
    const int nt = min(shards, (int)gridDim.x), shard = (int)blockIdx.x % nt;
    unsigned *tick = ctl + kCtlShard0 + shard * kCtlShardStride;
    static_assert(CAP / G == 32, "one pending bit per staged entry of a lane");
    __shared__ __attribute__((aligned(16))) double buf[kBlock / 64][kGroupBuf];
    const int lane = threadIdx.x & 63, grp = lane / G, gl = lane % G;
    double *mine = buf[threadIdx.x >> 6] + grp * CAP;
    const unsigned epoch = __hip_atomic_load(&ctl[kCtlEpoch], RLX_AGENT) + 1u;
    auto tag = [&](int ver) { return (epoch << 4) | (unsigned)ver; };
    for (;;) {
        const int q = flow_ticket_at(tick) * nt + shard;
        if (q >= nchunks) break;
        const int p = ck[q] + grp;
        const bool active = p < ck[q + 1];
        int i = -1, s = 0, k0 = 0, len = 0;
        double acc = 0.0, dr = 0.0;
        const int *cr = ci;        // this row's stored entries: all of them, or (rp0 set: the sweep-0
        const double *vr = v;      // call on a zero iterate) those read at a later version
        if (active) {
            const int node = nodes[p];
            s = node / n;
            i = node - s * n;
            acc = b[i];
            dr = (s == 0 ? d_first : d_later)[i];
            if (rp0 && s == 0 && __double_as_longlong(acc) != (long long)0x8000000000000000ull) {
                k0 = rp0[i];
                len = rp0[i + 1] - k0;
                cr = ci0, vr = v0;
            } else {
                k0 = rp[i];
                len = rp[i + 1] - k0;
            }
        }
        bool linked = false;   // an off-diagonal entry: some neighbour orders version s of x_i first
        int maxlen = len;
        for (int off = 32; off > 0; off >>= 1) maxlen = max(maxlen, __shfl_xor(maxlen, off, 64));
        maxlen = __builtin_amdgcn_readfirstlane(maxlen);
        for (int base = 0; base < maxlen; base += CAP) {
            const int m = active ? min(CAP, len - base) : 0;
            const int nj = m > gl ? (m - gl + G - 1) / G : 0;
            const int kb = k0 + base;
            unsigned pend = 0;
            for (int j0 = 0; j0 < nj; j0 += U) {   // (A) stage every product whose version exists
                int c[U], nd[U];
                double a[U], xv[U];
                unsigned long long ga[U], gc[U];
#pragma unroll
                for (int u = 0; u < U; ++u) c[u] = cr[kb + (j0 + u < nj ? gl + G * (j0 + u) : gl)];
#pragma unroll
                for (int u = 0; u < U; ++u) a[u] = vr[kb + (j0 + u < nj ? gl + G * (j0 + u) : gl)];
#pragma unroll
                for (int u = 0; u < U; ++u) nd[u] = (j0 + u < nj && c[u] != i) ? fused_need(c[u], i, s, split) : -1;
                // the group's loads issued together and read after the loop
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    xv[u] = 0.0;
                    ga[u] = gc[u] = 0ull;
                    if (nd[u] == 0) {
                        xv[u] = x[c[u]];
                    } else if (nd[u] > 0) {
                        const unsigned long long *gg = gran + 2 * (size_t)c[u];
                        ga[u] = __hip_atomic_load(const_cast<unsigned long long *>(gg), RLX_AGENT);
                        gc[u] = __hip_atomic_load(const_cast<unsigned long long *>(gg + 1), RLX_AGENT);
                    }
                }
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    if (j0 + u >= nj) continue;
                    double val = 0.0;   // the diagonal: subtracting +0.0 is the identity
                    if (nd[u] == 0) {
                        val = a[u] * xv[u];
                    } else if (nd[u] > 0) {
                        linked = true;
                        const unsigned want = tag(nd[u]);
                        if ((unsigned)(ga[u] >> 32) == want && (unsigned)(gc[u] >> 32) == want)
                            val = a[u] * __longlong_as_double((long long)((gc[u] << 32) | (ga[u] & 0xffffffffull)));
                        else {
                            pend |= 1u << (j0 + u);
                            if (ovl) val = __longlong_as_double((long long)c[u]);   // its column, until resolved
                        }
                    }
                    mine[gl + G * (j0 + u)] = val;
                }
            }
            if (!ovl) {
                while (pend) {   // (B)
                    const int j = __builtin_ctz(pend);
                    pend &= pend - 1;
                    const int t = gl + G * j;
                    const int c = cr[kb + t];
                    mine[t] = vr[kb + t] * granule_wait(gran + 2 * (size_t)c, tag(fused_need(c, i, s, split)), err, spin);
                }
                wave_sync();
                if (gl == 0 && m > 0) acc = chain_sub_pipe(acc, mine, 0, m);   // (C)
                wave_sync();
                continue;
            }
            // (B) and (C) interleaved as in gs_flow_group: the chain runs up to the first pending entry
            wave_sync();
            int k = 0, idle = 0;
            for (;;) {
                int first = pend ? gl + G * __builtin_ctz(pend) : CAP;
#pragma unroll
                for (int off = G / 2; off > 0; off >>= 1) first = min(first, __shfl_xor(first, off, 64));
                const int lim = min(first, m);
                constexpr int NP = 2;
                int tp[NP];
                unsigned want[NP];
                unsigned long long ga[NP], gc[NP];
                double ap[NP];
                {
                    unsigned qq = pend;
#pragma unroll
                    for (int h = 0; h < NP; ++h) {
                        tp[h] = -1;
                        want[h] = 0;
                        ga[h] = gc[h] = 0;
                        ap[h] = 0.0;
                        if (qq) {
                            tp[h] = gl + G * __builtin_ctz(qq);
                            qq &= qq - 1;
                            const int cp = (int)__double_as_longlong(mine[tp[h]]);
                            want[h] = tag(fused_need(cp, i, s, split));
                            const unsigned long long *gg = gran + 2 * (size_t)cp;
                            ga[h] = __hip_atomic_load(const_cast<unsigned long long *>(gg), RLX_AGENT);
                            gc[h] = __hip_atomic_load(const_cast<unsigned long long *>(gg + 1), RLX_AGENT);
                            ap[h] = vr[kb + tp[h]];
                        }
                    }
                }
                const bool advance = gl == 0 && k < lim;
                if (advance) acc = chain_sub_pipe(acc, mine, k, lim);
                if (gl == 0) k = max(k, lim);
                bool got = false;
#pragma unroll
                for (int h = 0; h < NP; ++h)
                    if (tp[h] >= 0 && (unsigned)(ga[h] >> 32) == want[h] && (unsigned)(gc[h] >> 32) == want[h]) {
                        mine[tp[h]] = ap[h] * __longlong_as_double((long long)((gc[h] << 32) | (ga[h] & 0xffffffffull)));
                        pend &= ~(1u << ((tp[h] - gl) / G));
                        got = true;
                    }
                const bool rowdone = gl != 0 || k >= m;
                if (__all(rowdone && !pend)) break;
                wave_sync();
                if (__any(got || advance)) {
                    idle = 0;
                } else {
                    if (++idle >= spin || ((idle & 63) == 63 && __hip_atomic_load(err, RLX_AGENT))) {
                        if (gl == 0) __hip_atomic_store(err, 1u, RLX_AGENT);
                        while (pend) {
                            mine[gl + G * __builtin_ctz(pend)] = 0.0;
                            pend &= pend - 1;
                        }
                        wave_sync();
                        if (gl == 0 && k < m) acc = chain_sub_pipe(acc, mine, k, m);
                        if (gl == 0) k = m;
                        break;
                    }
                    if (idle < 16) __builtin_amdgcn_s_sleep(1);
                    else __builtin_amdgcn_s_sleep(8);
                }
            }
            wave_sync();
        }
        // any lane of the row group staged an off-diagonal entry
#pragma unroll
        for (int off = G / 2; off > 0; off >>= 1) linked = linked || __shfl_xor((int)linked, off, 64);
        if (active && gl == 0) {
            unsigned long long *own = gran + 2 * (size_t)i;
            double xn;
            if (fabs(dr) > SMALLFLOAT) xn = acc / dr;
            else xn = s == 0 ? x_own(x, i) : granule_wait(own, tag(s), err, spin);   // unchanged
            // a row without neighbours is ordered after its previous update only here
            if (s > 0 && !linked) (void)granule_wait(own, tag(s), err, spin);
            granule_put(own, tag(s + 1), xn);
            if (s == last) x[i] = xn;   // x holds version 0 until the last sweep
        }
    }
    flow_exit(ctl, epoch, err, spin);
}

// ---- single-CU engine --------------------------------------------------------------------------
// One workgroup of kCuWaves waves.  h_off[d] .. h_off[d+1]: positions of depth d in `rows`.
__global__ __launch_bounds__(64 * kCuWaves) void gs_cu(int nrows, int ndepth, const int *__restrict__ rows,
                                                       const int *__restrict__ h_off, const int *__restrict__ rp,
                                                       const int *__restrict__ ci, const double *__restrict__ v,
                                                       const double *__restrict__ b, double *x,
                                                       const double *__restrict__ deff, unsigned *err, int spin)
{
    __shared__ int done[kCuMaxDepth];
    __shared__ int ticket, abort_flag;
    __shared__ __attribute__((aligned(16))) double strips[kCuWaves][kWaveStage];
    for (int t = threadIdx.x; t < ndepth; t += blockDim.x) done[t] = 0;
    if (threadIdx.x == 0) ticket = 0, abort_flag = 0;
    __syncthreads();
    const int lane = threadIdx.x & 63;
    double *strip = strips[threadIdx.x >> 6];
    constexpr int U = kWaveStage / 64;
    int d = 0;
    for (;;) {
        const int p = __builtin_amdgcn_readfirstlane(
            __hip_atomic_fetch_add(&ticket, lane == 0 ? 1 : 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP));
        if (p >= nrows) break;
        while (p >= h_off[d + 1]) ++d;   // tickets rise, so each wave's depth only moves forward
        const int i = rows[p];
        const int k0 = rp[i], k1 = rp[i + 1];
        // the first strip's entries do not depend on the pass: load them before waiting
        int c[U];
        double a[U];
        {
            const int m = min(kWaveStage, k1 - k0);
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int q = lane + 64 * u;
                c[u] = q < m ? ci[k0 + q] : 0;
                a[u] = q < m ? v[k0 + q] : 0.0;
            }
        }
        if (d > 0) {
            const int need = h_off[d] - h_off[d - 1];
            for (int s = 0; __hip_atomic_load(&done[d - 1], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) < need; ++s) {
                // give up after the limit, or at once when another wave of the pass already did
                if (s >= spin || __hip_atomic_load(&abort_flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) {
                    if (lane == 0) {
                        __hip_atomic_store(err, 1u, RLX_AGENT);
                        __hip_atomic_store(&abort_flag, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                    }
                    break;
                }
                __builtin_amdgcn_s_sleep(1);
            }
        }
        double acc = b[i];
        for (int base = k0; base < k1; base += kWaveStage) {
            const int m = min(kWaveStage, k1 - base);
            if (base != k0) {
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    const int q = lane + 64 * u;
                    c[u] = q < m ? ci[base + q] : 0;
                    a[u] = q < m ? v[base + q] : 0.0;
                }
            }
            double xv[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int q = lane + 64 * u;
                xv[u] = (q < m && c[u] != i) ? x[c[u]] : 0.0;
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int q = lane + 64 * u;
                if (q < m) strip[q] = c[u] == i ? 0.0 : a[u] * xv[u];
            }
            wave_sync();
            if (lane == 0) acc = chain_sub(acc, strip, 0, m);
            wave_sync();
        }
        if (lane == 0) {
            const double dd = deff[i];
            if (fabs(dd) > SMALLFLOAT) x[i] = acc / dd;
            // release: the x store above is visible to every wave of the workgroup that acquires
            // this counter
            __hip_atomic_fetch_add(&done[d], 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
    }
    if (spin < 0 && threadIdx.x == 0) __hip_atomic_store(err, 1u, RLX_AGENT);   // test hook
}

// ---- planning ----------------------------------------------------------------------------------
// Structural symmetry of the entries (i, j), i in [r0, r1), j != i, that keep(i, j) selects: every
// such (i, j) has its (j, i).  One streaming pass (no per-row sort, no lookups in other rows): the
// sums over entries of sign(j - i) * H(min(i, j), max(i, j)) for two independent 64-bit mixes H
// vanish (mod 2^64) for a symmetric pattern and, for an unsymmetric one, only by a collision of
// probability ~2^-128.  Even then nothing is silent: the one-launch engines rely on the symmetry
// for progress, and a pass that waits for a value never published gives up and reports a stall.
static inline unsigned long long mix64(unsigned long long z)
{
    z += 0x9e3779b97f4a7c15ull;
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
}
template <class Keep>
static bool pattern_symmetric(const int *rp, const int *ci, int r0, int r1, Keep keep)
{
    std::atomic<unsigned long long> h1{0}, h2{0};
    parallel_chunks(r1 - r0, 1 << 14, [&](int a, int e) {
        unsigned long long s1 = 0, s2 = 0;
        for (int i = r0 + a; i < r0 + e; ++i)
            for (int k = rp[i]; k < rp[i + 1]; ++k) {
                const int j = ci[k];
                if (j == i || !keep(i, j)) continue;
                const unsigned long long key = ((unsigned long long)(unsigned)std::min(i, j) << 32) | (unsigned)std::max(i, j);
                const unsigned long long u1 = mix64(key), u2 = mix64(key ^ 0x5851f42d4c957f2dull);
                if (j > i) s1 += u1, s2 += u2;
                else s1 -= u1, s2 -= u2;
            }
        h1 += s1;
        h2 += s2;
    });
    return h1.load() == 0 && h2.load() == 0;
}

static const char *gs_engine_env()
{
    const char *e = getenv("SSS_HIP_GS_ENGINE");
    return e ? e : "auto";
}

// Rows of the pass are ps.h_off-ordered by depth; A is the level matrix (host), [lo, hi) the pass's
// contiguous row range.  Chooses the engine and builds its device data.
int gs_persist_build(PassSchedule &ps, const SSS_MAT &A, int lo, int hi, bool long_rows, bool natural, bool desc)
{
    GsPersist &g = ps.gp;
    g = GsPersist();
    g.natural = natural;
    g.desc = desc;
    std::string want = gs_engine_env();
    if ((natural || desc) && want == "cu") want = "flow";   // the single-CU engine runs GS-CF passes only
    if (want == "launch" || ps.depth <= 1 || ps.nrows == 0) return 0;
    const int *rp = A.row_ptr, *ci = A.col_idx;
    long long nnz = 0;
    for (int i = lo; i < hi; ++i) nnz += rp[i + 1] - rp[i];
    const double avg = (double)nnz / std::max(1, hi - lo);
    // Engine choice.  Measured on MI355X (7-pt 256^3, 2-sweep pre-smoother per level, tools/
    // gs_level_times.py): flow beats one launch per depth on every level (level 1:
    // 23 vs 68 ms, level 4: 18 vs 42, level 8: 107 vs 216), the single-CU engine loses to flow
    // everywhere (one CU streams too slowly and the chain of a long row is the same either way),
    // so "auto" is flow, and cu only on request.
    int engine = want == "cu" ? 2 : 1;
    if (engine == 2 && ps.depth > kCuMaxDepth) engine = 1;
    if (engine == 1) {
        // the flow engine needs every same-class coupling in both directions (see the header)
        const bool sym = pattern_symmetric(rp, ci, lo, hi, [&](int, int j) { return j >= lo && j < hi; });
        if (!sym) {
            // the single-CU engine divides by the stale GS-CF divisor; a natural-order pass
            // multiplies by the carried reciprocal (Solve/SSS_smooth.c:112), so it keeps the
            // per-depth launches
            if (ps.depth <= kCuMaxDepth && !natural && !desc) engine = 2;
            else return 0;
        }
    }
    g.engine = engine;
    g.lo = lo;
    g.hi = hi;
    g.spin = engine == 2 ? kSpinLimit : kFlowSpinLimit;
    if (const char *sp = getenv("SSS_HIP_GS_SPIN")) g.spin = atoi(sp);
    if (engine == 2) {
        std::vector<int> off(ps.h_off.begin(), ps.h_off.end());
        g.h_off = dev_alloc<int>(off.size());
        g.ctl = dev_alloc<unsigned>(kCtlWords);
        if (!g.h_off || !g.ctl) return hip_fail(hipErrorOutOfMemory, "hipMalloc(gs cu)", __FILE__, __LINE__);
        SSS_HIP(hipMemcpy(g.h_off, off.data(), sizeof(int) * off.size(), hipMemcpyHostToDevice));
        SSS_HIP(hipMemset(g.ctl, 0, sizeof(unsigned) * kCtlWords));
        g.err = g.ctl + kCtlErr;
        return 0;
    }
    // lanes per row from the average row length: about 8 entries per lane and round
    g.G = avg <= 24 ? 4 : avg <= 48 ? 8 : avg <= 96 ? 16 : avg <= 192 ? 32 : 64;
    // the row's chain overlapping the polls of its pending granules: measured at 7-pt 256^3
    // (tools/gpu/gs_overlap.sh, pre-smoother per call) 19 % faster on the levels of 700-1400
    // entries per row (level 7: 106 -> 86 ms, level 8: 108 -> 87), 5 % on level 5 (407), but
    // 9-12 % slower on levels 3-4 (64 and 198), where the chain is short against the loop's polls
    g.overlap = avg >= 300;
    (void)long_rows;
    g.gran = dev_alloc<unsigned long long>(2 * (size_t)(hi - lo));
    g.ctl = dev_alloc<unsigned>(kCtlWords);
    if (!g.gran || !g.ctl) return hip_fail(hipErrorOutOfMemory, "hipMalloc(gs flow)", __FILE__, __LINE__);
    SSS_HIP(hipMemset(g.gran, 0, sizeof(unsigned long long) * 2 * (size_t)(hi - lo)));
    SSS_HIP(hipMemset(g.ctl, 0, sizeof(unsigned) * kCtlWords));
    g.err = g.ctl + kCtlErr;
    {   // chunks: up to 64 / G rows of one depth
        const int R = 64 / g.G;
        std::vector<int> ck;
        for (int l = 0; l < ps.depth; ++l)
            for (int s0 = ps.h_off[l]; s0 < ps.h_off[l + 1]; s0 += R) ck.push_back(s0);
        ck.push_back(ps.nrows);
        g.nchunks = (int)ck.size() - 1;
        g.ck = dev_alloc<int>(ck.size());
        if (!g.ck) return hip_fail(hipErrorOutOfMemory, "hipMalloc(gs chunks)", __FILE__, __LINE__);
        SSS_HIP(hipMemcpy(g.ck, ck.data(), sizeof(int) * ck.size(), hipMemcpyHostToDevice));
    }
    int cus = 256;
    {
        int dev = 0;
        hipDeviceProp_t prop;
        if (hipGetDevice(&dev) == hipSuccess && hipGetDeviceProperties(&prop, dev) == hipSuccess)
            cus = prop.multiProcessorCount;
    }
    // waves in flight: a few per ticket of one depth (more only spin on rows of later depths, and
    // their polls load the memory system), capped by the tickets and by 8 per CU
    const double per_depth = (double)g.nchunks / std::max(1, ps.depth);
    int waves = (int)std::min<double>(1024.0, std::max(32.0, 4.0 * per_depth));
    waves = std::min(waves, std::min(g.nchunks, cus * 8));
    g.grid = std::max(1, (waves + 3) / 4);
    return 0;
}

void gs_persist_free(PassSchedule &ps)
{
    GsPersist &g = ps.gp;
    dev_free(g.h_off);
    dev_free(g.ctl);
    dev_free(g.gran);
    dev_free(g.ck);
    g = GsPersist();
}

// Fused depth of the nodes of one pass-depth group (rows of one class, one depth of its own pass:
// independent of each other): fd(i, s) = 1 + max(fd(i, s - 1), fd of each version node (i, s) reads).
// G lanes per row.
template <int G>
__global__ __launch_bounds__(kBlock) void fused_depth_group(int cnt, const int *__restrict__ grows,
                                                            const int *__restrict__ rp, const int *__restrict__ ci,
                                                            int n, int split, int s, int *fd)
{
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    const int r = t / G, gl = t % G;
    int dep = 0, i = -1;
    if (r < cnt) {
        i = grows[r];
        if (gl == 0 && s > 0) dep = fd[(size_t)(s - 1) * n + i];
        for (int k = rp[i] + gl; k < rp[i + 1]; k += G) {
            const int j = ci[k];
            if (j == i) continue;
            const int need = fused_need(j, i, s, split);
            if (need > 0) dep = max(dep, fd[(size_t)(need - 1) * n + j]);
        }
    }
#pragma unroll
    for (int off = G / 2; off > 0; off >>= 1) dep = max(dep, __shfl_xor(dep, off, 64));
    if (r < cnt && gl == 0) fd[(size_t)s * n + i] = dep + 1;
}

// Fused plan.  Requires F rows [0, split) and C rows [split, n) (relabeled level) and a structurally
// symmetric level (checked here; otherwise no plan and the per-pass engines run).  Fused depth:
// fd(i, s) = 1 + max(fd(i, s - 1), fd of the version of every neighbour that node (i, s) reads),
// on the GPU pass by pass over each pass's own depth groups (rows of one group are independent,
// the uploaded level dA and the passes' depth-ordered rows), or on the host in one serial pass.
int gs_fused_build(GsFused &f, const SSS_MAT &A, const DevCSR *dA, const PassSchedule *pass, const int *cls,
                   int sweeps)
{
    f = GsFused();
    const int n = A.num_rows;
    const int *rp = A.row_ptr, *ci = A.col_idx;
    if (n <= 0 || sweeps < 1 || sweeps > 14 || A.num_cols != n || (long long)n * sweeps >= (1ll << 31)) return 0;
    int split = 0;
    while (split < n && cls[split] == 0) ++split;
    for (int i = split; i < n; ++i)
        if (cls[i] != 1) return 0;
    if (!pattern_symmetric(rp, ci, 0, n, [&](int, int j) { return j >= 0 && j < n; })) return 0;
    const long long nnz = rp[n];
    const double avg = (double)nnz / n;
    f.G = avg <= 24 ? 4 : avg <= 48 ? 8 : avg <= 96 ? 16 : avg <= 192 ? 32 : 64;
    std::vector<int> fd((size_t)n * sweeps, 0);   // fd[s * n + i]
    // on the GPU, one launch per depth group of each pass (~40 us each with the plan's other host
    // work around), or on the host, one serial pass (~2.5 ns per entry and sweep): whichever is
    // cheaper (400^3: level 1, 32M rows, GPU; levels 5-10, thousands of groups, host)
    const double gpu_s = 40e-6 * sweeps * (double)(pass[0].depth + pass[1].depth);
    const double host_s = 2.5e-9 * sweeps * (double)nnz;
    const char *fde = getenv("SSS_HIP_FUSED_DEPTH");   // gpu | host: force one form (tests)
    const bool on_gpu = fde && *fde ? std::string(fde) == "gpu" : gpu_s < host_s;
    if (dA && dA->rp && dA->ci && dA->n == n && pass[0].rows && pass[1].rows && on_gpu) {
        int *d_fd = dev_alloc<int>(fd.size());
        if (!d_fd) return hip_fail(hipErrorOutOfMemory, "hipMalloc(fused depth)", __FILE__, __LINE__);
        auto go = [&](auto kern, int cnt, const int *grows, int sw) {
            const long long threads = (long long)cnt * f.G;
            hipLaunchKernelGGL(kern, dim3((unsigned)((threads + kBlock - 1) / kBlock)), dim3(kBlock), 0, nullptr, cnt,
                               grows, dA->rp, dA->ci, n, split, sw, d_fd);
        };
        for (int sw = 0; sw < sweeps; ++sw)
            for (int c = 0; c < 2; ++c)
                for (int d = 0; d < pass[c].depth; ++d) {
                    const int cnt = pass[c].h_off[d + 1] - pass[c].h_off[d];
                    const int *grows = pass[c].rows + pass[c].h_off[d];
                    if (cnt <= 0) continue;
                    switch (f.G) {
                    case 4: go(fused_depth_group<4>, cnt, grows, sw); break;
                    case 8: go(fused_depth_group<8>, cnt, grows, sw); break;
                    case 16: go(fused_depth_group<16>, cnt, grows, sw); break;
                    case 32: go(fused_depth_group<32>, cnt, grows, sw); break;
                    default: go(fused_depth_group<64>, cnt, grows, sw); break;
                    }
                }
        const hipError_t e1 = hipGetLastError();
        const hipError_t e2 = hipMemcpy(fd.data(), d_fd, sizeof(int) * fd.size(), hipMemcpyDeviceToHost);
        dev_free(d_fd);
        if (e1 != hipSuccess) return hip_fail(e1, "fused_depth_group", __FILE__, __LINE__);
        if (e2 != hipSuccess) return hip_fail(e2, "hipMemcpy(fused depth)", __FILE__, __LINE__);
    } else {
        // one serial pass in the sequential smoother's own order (every dependency of a node comes
        // earlier in it), the rows streamed in order
        for (int sw = 0; sw < sweeps; ++sw)
            for (int c = 0; c < 2; ++c)
                for (int i = c ? split : 0; i < (c ? n : split); ++i) {
                    int dep = sw > 0 ? fd[(size_t)(sw - 1) * n + i] : 0;
                    for (int k = rp[i]; k < rp[i + 1]; ++k) {
                        const int j = ci[k];
                        if (j == i) continue;
                        const int need = (cls[j] == c) ? (j < i ? sw + 1 : sw) : (cls[j] ? sw : sw + 1);
                        if (need > 0) dep = std::max(dep, fd[(size_t)(need - 1) * n + j]);
                    }
                    fd[(size_t)sw * n + i] = dep + 1;
                }
    }
    int depth = 0;
    for (int x : fd) depth = std::max(depth, x);
    std::vector<int> doff((size_t)depth + 2, 0);
    for (int x : fd) doff[(size_t)x]++;
    for (int d = 0; d <= depth; ++d) doff[(size_t)d + 1] += doff[(size_t)d];
    std::vector<int> order(fd.size());
    {
        std::vector<int> fill(doff.begin(), doff.end() - 1);
        for (size_t t = 0; t < fd.size(); ++t) order[(size_t)fill[(size_t)fd[t] - 1]++] = (int)t;
    }
    f.overlap = avg >= 300;
    // Lanes per row G: the cheapest by a latency model fitted to 2-sweep calls on 7-pt 256^3 and
    // the circuit stand-in at G = 2 ... 64 (tools/gpu/r05_g_sweep.sh, profiles/r05_gs_fused/):
    //  * each fused depth step costs the larger of its tickets -- the eight ticket shards hand out
    //    chunks of 64 / G rows at ~4.5 ns each (one device-wide counter: ~13 ns; re-fitted at 400^3,
    //    profiles/r05_shards/), so npd * G / 64 * 4.5 ns for npd nodes per depth --
    //    and a node's latency, ~2 us + 1 us per group of 8 loads a lane issues for an average row
    //    + 20 ns per entry a lane stages;
    //  * hub rows (longer than 4x the average and than one staging round of 32 G entries) add
    //    ~2 us per further round, each sweep.
    // 7-pt level 1 (19 entries, ~14K nodes per depth): G = 2 (9.4 ms; 13.3 at 4, 24.7 at 8); level
    // 2 (35 entries, ~2K): 8 (5.7; 9.0 at 16); level 3 (64, ~280): 32 (4.3; 19.2 at 2); the long-row
    // levels 64; the circuit stand-in's level 1 (7 entries, hub rows up to 11K): 8-16 (8.9 / 8.3
    // ms against 13.3 at 4 and 20.8 at 64).
    int maxlen = 0;
    for (int i = 0; i < n; ++i) maxlen = std::max(maxlen, rp[i + 1] - rp[i]);
    {
        const double npd = (double)n * sweeps / std::max(1, depth);
        double best = 0.0;
        for (int g = 2; g <= 64; g *= 2) {
            const double tick = npd * g / 64.0 * 4.5e-9;
            const double lat = 2e-6 + std::ceil(std::min(avg, 32.0 * g) / (8.0 * g)) * 1e-6 + avg / g * 20e-9;
            double hub = 0.0;
            const double hub_min = std::max(4.0 * avg, 32.0 * g);
            if (maxlen > hub_min)
                for (int i = 0; i < n; ++i) {
                    const int len = rp[i + 1] - rp[i];
                    if (len > hub_min) hub += std::ceil(len / (32.0 * g)) - 1.0;
                }
            const double est = depth * std::max(tick, lat) + sweeps * hub * 2e-6;
            if (g == 2 || est < best) best = est, f.G = g;
        }
    }
    if (const char *e = getenv("SSS_HIP_FUSED_G")) {   // test hook: lanes per row 2 ... 64
        const int g = atoi(e);
        if (g == 2 || g == 4 || g == 8 || g == 16 || g == 32 || g == 64) f.G = g;
    }
    f.shards = kTicketShards;
    if (const char *e = getenv("SSS_HIP_FUSED_SHARDS")) f.shards = std::min(kTicketShards, std::max(1, atoi(e)));
    if (getenv("SSS_HIP_TIMING"))
        fprintf(stderr, "[sss_hip]   fused GS-CF plan n=%d: depth %d (%.0f nodes per depth), rows %.1f avg / %d max, G = %d\n",
                n, depth, (double)n * sweeps / std::max(1, depth), avg, maxlen, f.G);
    const int R = 64 / f.G;
    std::vector<int> ck;
    for (int d = 0; d < depth; ++d)
        for (int s0 = doff[(size_t)d]; s0 < doff[(size_t)d + 1]; s0 += R) ck.push_back(s0);
    ck.push_back((int)order.size());
    f.nchunks = (int)ck.size() - 1;
    f.depth = depth;
    f.sweeps = sweeps;
    f.n = n;
    f.split = split;
    f.spin = kFlowSpinLimit;
    if (const char *sp = getenv("SSS_HIP_GS_SPIN")) f.spin = atoi(sp);
    f.ck = dev_alloc<int>(ck.size());
    f.nodes = dev_alloc<int>(order.size());
    f.gran = dev_alloc<unsigned long long>(2 * (size_t)n);
    f.ctl = dev_alloc<unsigned>(kCtlWords);
    if (!f.ck || !f.nodes || !f.gran || !f.ctl) {
        gs_fused_free(f);
        return hip_fail(hipErrorOutOfMemory, "hipMalloc(gs fused)", __FILE__, __LINE__);
    }
    // an upload failure frees what this plan holds (as the allocation failures do)
#define SSS_FUSED_HIP(call)                                          \
    do {                                                             \
        hipError_t e_ = (call);                                      \
        if (e_ != hipSuccess) {                                      \
            gs_fused_free(f);                                        \
            return hip_fail(e_, #call, __FILE__, __LINE__);          \
        }                                                            \
    } while (0)
    SSS_FUSED_HIP(hipMemcpy(f.ck, ck.data(), sizeof(int) * ck.size(), hipMemcpyHostToDevice));
    SSS_FUSED_HIP(hipMemcpy(f.nodes, order.data(), sizeof(int) * order.size(), hipMemcpyHostToDevice));
    SSS_FUSED_HIP(hipMemset(f.gran, 0, sizeof(unsigned long long) * 2 * (size_t)n));
    SSS_FUSED_HIP(hipMemset(f.ctl, 0, sizeof(unsigned) * kCtlWords));
    {   // sweep-0 rows on a zero iterate (finite values only): the entries read at version 1
        const double *av = A.val;
        std::atomic<bool> fin{true};
        parallel_chunks(n, 1 << 16, [&](int a, int e) {
            for (long long k = rp[a]; k < rp[e] && fin; ++k)
                if (!std::isfinite(av[k])) fin = false;
        });
        if (fin) {
            std::vector<int> r0((size_t)n + 1, 0);
            auto keep = [&](int i, int j) { return j != i && ((cls[j] == cls[i]) ? j < i : cls[j] == 0); };
            parallel_chunks(n, 4096, [&](int a, int e) {
                for (int i = a; i < e; ++i) {
                    int c = 0;
                    for (int k = rp[i]; k < rp[i + 1]; ++k) c += keep(i, ci[k]);
                    r0[(size_t)i + 1] = c;
                }
            });
            for (int i = 0; i < n; ++i) r0[(size_t)i + 1] += r0[(size_t)i];
            HostBuf<int> c0;
            HostBuf<double> w0;
            c0.resize((size_t)std::max(r0[(size_t)n], 1)), w0.resize((size_t)std::max(r0[(size_t)n], 1));
            parallel_chunks(n, 4096, [&](int a, int e) {
                for (int i = a; i < e; ++i) {
                    int o = r0[(size_t)i];
                    for (int k = rp[i]; k < rp[i + 1]; ++k)
                        if (keep(i, ci[k])) c0[(size_t)o] = ci[k], w0[(size_t)o] = av[k], ++o;
                }
            });
            f.rp0 = dev_alloc<int>(r0.size());
            f.ci0 = dev_alloc<int>(c0.size());
            f.v0 = dev_alloc<double>(w0.size());
            if (!f.rp0 || !f.ci0 || !f.v0) {
                gs_fused_free(f);
                return hip_fail(hipErrorOutOfMemory, "hipMalloc(gs fused rows)", __FILE__, __LINE__);
            }
            SSS_FUSED_HIP(hipMemcpy(f.rp0, r0.data(), sizeof(int) * r0.size(), hipMemcpyHostToDevice));
            SSS_FUSED_HIP(hipMemcpy(f.ci0, c0.data(), sizeof(int) * c0.size(), hipMemcpyHostToDevice));
            SSS_FUSED_HIP(hipMemcpy(f.v0, w0.data(), sizeof(double) * w0.size(), hipMemcpyHostToDevice));
        }
    }
#undef SSS_FUSED_HIP
    f.err = f.ctl + kCtlErr;
    int cus = 256;
    {
        int dev = 0;
        hipDeviceProp_t prop;
        if (hipGetDevice(&dev) == hipSuccess && hipGetDeviceProperties(&prop, dev) == hipSuccess)
            cus = prop.multiProcessorCount;
    }
    // Progress needs every workgroup that takes tickets to be resident (a waiting wave spins until its
    // producers finish), and with sharded tickets at least one resident workgroup per shard: cap the
    // grid at what the occupancy API says can be co-resident on the device (the kernel takes
    // min(shards, grid) counters, so every shard then has a resident workgroup).
    int per_cu = 0;
    {
        auto occ = [&](auto kern) {
            if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, kBlock, 0) != hipSuccess) per_cu = 0;
        };
        switch (f.G) {
        case 2: occ(gs_fused_group<2>); break;
        case 4: occ(gs_fused_group<4>); break;
        case 8: occ(gs_fused_group<8>); break;
        case 16: occ(gs_fused_group<16>); break;
        case 32: occ(gs_fused_group<32>); break;
        default: occ(gs_fused_group<64>); break;
        }
    }
    const int resident = per_cu > 0 ? per_cu * cus : 2 * cus;
    const double per_depth = (double)f.nchunks / std::max(1, depth);
    // waves in flight: at least 512 (1,024 on the long-row levels), so that nodes several fused
    // depths ahead are staged before their dependencies finish (7-pt 400^3, 2-sweep calls,
    // profiles/r05_gs_fused/: levels 5 / 6 / 8 31.3 / 60.8 / 128.1 ms with the former minimum of 32
    // waves, 28.9 / 56.1 / 120.6 with 1,024; 2,048 slower everywhere)
    int waves = (int)std::min<double>(1024.0, std::max(f.overlap ? 1024.0 : 512.0, 4.0 * per_depth));
    if (const char *e = getenv("SSS_HIP_FUSED_WAVES")) waves = std::max(4, atoi(e));   // lab hook
    waves = std::min(waves, std::min(f.nchunks, cus * 8));
    f.grid = std::max(1, std::min((waves + 3) / 4, resident));
    f.engine = 1;
    return 0;
}

void gs_fused_free(GsFused &f)
{
    dev_free(f.rp0);
    dev_free(f.ci0);
    dev_free(f.v0);
    dev_free(f.ck);
    dev_free(f.nodes);
    dev_free(f.gran);
    dev_free(f.ctl);
    f = GsFused();
}

int gs_fused_run(const GsFused &f, const DevCSR &A, const double *b, double *x, const double *d_first,
                 const double *d_later, bool x_zero, hipStream_t s)
{
    if (!f.engine) return ERROR_INPUT_PAR;
    auto go = [&](auto kern) {
        hipLaunchKernelGGL(kern, dim3(f.grid), dim3(kBlock), 0, s, f.nchunks, f.ck, f.nodes, f.n, f.split,
                           f.sweeps - 1, A.rp, A.ci, A.v, b, x, d_first, d_later, f.gran, f.ctl, f.err, f.spin,
                           f.overlap ? 1 : 0, x_zero ? f.rp0 : (const int *)nullptr, f.ci0, f.v0, f.shards);
    };
    switch (f.G) {   // (every G the planner can choose; the chunk table holds 64 / G rows per ticket)
    case 2: go(gs_fused_group<2>); break;
    case 4: go(gs_fused_group<4>); break;
    case 8: go(gs_fused_group<8>); break;
    case 16: go(gs_fused_group<16>); break;
    case 32: go(gs_fused_group<32>); break;
    case 64: go(gs_fused_group<64>); break;
    default: return ERROR_INPUT_PAR;
    }
    SSS_HIP(hipGetLastError());
    return 0;
}


// Diagnostic builds only (make EXTRA=-DSSS_GS_TRACE): each flow pass writes its rows' stamps to a
// buffer that gs_trace_dump appends, with the pass's depth offsets, to $SSS_GS_TRACE_FILE.
#ifdef SSS_GS_TRACE
static std::map<const PassSchedule *, unsigned long long *> &gs_traces()
{
    static std::map<const PassSchedule *, unsigned long long *> m;
    return m;
}
static unsigned long long *gs_trace_buf(const PassSchedule &ps)
{
    auto &m = gs_traces();
    auto it = m.find(&ps);
    if (it != m.end()) return it->second;
    unsigned long long *d = dev_alloc<unsigned long long>(4 * (size_t)std::max(ps.nrows, 1));
    m[&ps] = d;
    return d;
}
static void gs_trace_dump(const PassSchedule &ps, hipStream_t s)
{
    const char *f = getenv("SSS_GS_TRACE_FILE");
    if (!f || hipStreamSynchronize(s) != hipSuccess) return;
    std::vector<unsigned long long> h(4 * (size_t)ps.nrows);
    if (hipMemcpy(h.data(), gs_trace_buf(ps), sizeof(unsigned long long) * h.size(), hipMemcpyDeviceToHost) != hipSuccess)
        return;
    FILE *fp = fopen(f, "ab");
    if (!fp) return;
    const int hdr[2] = {ps.nrows, ps.depth};
    fwrite(hdr, sizeof hdr, 1, fp);
    fwrite(ps.h_off.data(), sizeof(int), (size_t)ps.depth + 1, fp);
    fwrite(h.data(), sizeof(unsigned long long), h.size(), fp);
    fclose(fp);
}
#else
static unsigned long long *gs_trace_buf(const PassSchedule &) { return nullptr; }
static void gs_trace_dump(const PassSchedule &, hipStream_t) {}
#endif

int gs_persist_run(const PassSchedule &ps, const DevCSR &A, const double *b, double *x, const double *deff,
                   hipStream_t s)
{
    const GsPersist &g = ps.gp;
    if (g.engine == 2) {
        hipLaunchKernelGGL(gs_cu, dim3(1), dim3(64 * kCuWaves), 0, s, ps.nrows, ps.depth, ps.rows, g.h_off, A.rp, A.ci,
                           A.v, b, x, deff, g.err, g.spin);
    } else if (g.engine == 1) {
        auto go = [&](auto kern) {
            hipLaunchKernelGGL(kern, dim3(g.grid), dim3(kBlock), 0, s, g.nchunks, g.ck, ps.rows, A.rp, A.ci, A.v, b, x,
                               deff, g.gran, g.lo, g.hi, g.ctl, g.err, g.spin, g.overlap ? 1 : 0,
                               gs_trace_buf(ps));
        };
        auto by_g = [&](auto nat, auto desc) {
            constexpr bool N = decltype(nat)::value, D = decltype(desc)::value;
            switch (g.G) {
            case 4: go(gs_flow_group<4, N, D>); break;
            case 8: go(gs_flow_group<8, N, D>); break;
            case 16: go(gs_flow_group<16, N, D>); break;
            case 32: go(gs_flow_group<32, N, D>); break;
            default: go(gs_flow_group<64, N, D>); break;
            }
        };
        using T = std::true_type;
        using F = std::false_type;
        if (g.natural && g.desc) by_g(T(), T());
        else if (g.natural) by_g(T(), F());
        else by_g(F(), F());
        gs_trace_dump(ps, s);
    } else {
        return ERROR_INPUT_PAR;
    }
    SSS_HIP(hipGetLastError());
    return 0;
}

int gs_persist_error(const PassSchedule &ps, unsigned *out)
{
    *out = 0;
    if (!ps.gp.err) return 0;
    unsigned e = 0;
    SSS_HIP(hipMemcpy(&e, ps.gp.err, sizeof(unsigned), hipMemcpyDeviceToHost));
    *out = e;
    return 0;
}

int gs_fused_error(const GsFused &f, unsigned *out, bool clear)
{
    *out = 0;
    if (!f.engine || !f.err) return 0;
    unsigned e = 0;
    SSS_HIP(hipMemcpy(&e, f.err, sizeof(unsigned), hipMemcpyDeviceToHost));
    *out = e;
    if (e && clear) SSS_HIP(hipMemset(f.err, 0, sizeof(unsigned)));
    return 0;
}

void smoother_set_err(SmootherPlan &sp, unsigned *err)
{
    for (auto &ps : sp.pass)
        if (ps.gp.engine && err) ps.gp.err = err;
    if (sp.fz.engine && err) sp.fz.err = err;
}

// the error word as a double (1.0 if any pass of the hierarchy stalled since the last read, else
// 0.0) into *out, and the word cleared: one thread
__global__ void err_flag_kernel(unsigned *err, double *out)
{
    const unsigned e = __hip_atomic_exchange(err, 0u, RLX_AGENT);
    *out = e ? 1.0 : 0.0;
}

int launch_err_flag(unsigned *err, double *out, hipStream_t s)
{
    hipLaunchKernelGGL(err_flag_kernel, dim3(1), dim3(1), 0, s, err, out);
    SSS_HIP(hipGetLastError());
    return 0;
}

}  // namespace sss
