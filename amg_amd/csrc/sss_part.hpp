// sss_part.hpp — host-side row partition of an SSS_AMG hierarchy for the multi-GPU engine.
//
// Rank r owns rows [lo_r, hi_r) of every partitioned level l < nagg (original numbering).
// Level 0 is cut evenly; level l+1 inherits the cut through the C points of level l: coarse
// point c is the c-th C point of level l in fine order (SSS_coarsen cmap, amg_amd/host/
// sss_setup.c coarse renumbering), so it belongs to the owner of that fine row and every
// rank's coarse points form a contiguous range again.
//
// Local numbering of a level: own rows relabeled F-first / C-second (ascending inside each
// class, as the single-GPU engine does), then ghosts in ascending global order.  A level's
// ghost set is the union of the off-rank columns of its own A_l rows, of R_l's own coarse rows
// and of P_{l-1}'s own fine rows, so one halo plan serves every vector of the level.
#pragma once

#include <string>
#include <vector>

#include "../../include/sss_amg.h"

namespace sss {

struct HostMat {   // CSR owned by vectors
    int rows = 0, cols = 0;
    std::vector<int> rp, ci;
    std::vector<double> v;
    SSS_MAT view() const
    {
        SSS_MAT m;
        m.num_rows = rows;
        m.num_cols = cols;
        m.num_nnzs = (int)ci.size();
        m.row_ptr = const_cast<int *>(rp.data());
        m.col_idx = const_cast<int *>(ci.data());
        m.val = const_cast<double *>(v.data());
        return m;
    }
};

struct PartLevel {
    int lo = 0, hi = 0, m = 0, g = 0, nF = 0;
    std::vector<int> perm;     // local id -> global id (own rows)
    std::vector<int> ghosts;   // ghost k (local id m + k) -> global id, ascending
    std::vector<int> mark;     // cfmark in local order
    std::vector<int> gcls;     // per ghost: class (0 F, 1 C) if owned by a lower rank, else -1
    std::vector<int> gclass;   // per ghost: class (0 F, 1 C), whoever owns it
    HostMat A;                 // m x (m + g)
    HostMat P;                 // m x (next level local ids), or global coarse ids when l + 1 == nagg
    HostMat R;                 // own coarse rows (next level local order, or global order at nagg) x (m + g)
    // halo: peers this rank sends to / receives from, in ascending rank order
    std::vector<int> sdst, scount, sidx;   // sidx: local ids, concatenated per peer
    std::vector<int> rsrc, rcount;         // ghosts from rsrc[i] are contiguous, in peer order
};

struct PartPlan {
    int nranks = 1, rank = 0, nl = 0, nagg = 0;
    std::vector<std::vector<int>> cut;   // cut[l][q] = first row of rank q on level l (l <= nagg), size nranks + 1
    std::vector<long long> gnnz;         // nnz of the whole level l (l < nagg): per-level choices every rank makes alike
    std::vector<PartLevel> L;            // l < nagg
};

// agg_rows: the first level l >= 1 with at most agg_rows rows, and every level below it, is
// replicated (the coarsest always is).  Returns 0 or an SSS error code.
constexpr int kAggRowsDefault = 20000;
// agg_rows if > 0, else SSS_HIP_AGG_ROWS, else kAggRowsDefault
int part_agg_rows(int agg_rows);
int part_plan_build(PartPlan &p, const SSS_AMG *mg, int nranks, int rank, int agg_rows);

// Partition file of one rank (sss_part_save): its PartPlan plus the solve parameters (format 2:
// with the levels' global nnz).  The
// replicated tail levels (cg[nagg..]) live in a separate hierarchy file (SSS_amg_save format)
// that every rank loads.  Returns 0 or ERROR_OPEN_FILE / ERROR_WRONG_FILE.
int part_plan_write(const PartPlan &p, const SSS_AMG_PARS &pars, const char *path);
int part_plan_read(PartPlan &p, SSS_AMG_PARS &pars, const char *path);
std::string part_file_name(const char *prefix, int rank);   // prefix.r<rank>
std::string part_tail_name(const char *prefix);             // prefix.tail

}  // namespace sss
