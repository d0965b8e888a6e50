// sss_tail.hpp — the single-workgroup tail of the V-cycle (sss_tail.hip): device descriptors of
// the small coarse levels it runs, built by the hierarchy mirror (sss_hier.hip tail_build).
#pragma once

#include <vector>

#include <hip/hip_runtime.h>

namespace sss {

struct TailPass {                  // one class pass of the two-stage C/F-Jacobi smoother
    int lo = 0, hi = 0;            // the class's rows
    const int *nrp = nullptr, *nci = nullptr, *split = nullptr;   // [N_i | L_i] rows (split absolute)
    const double *nv = nullptr;
    const int *lrp = nullptr, *lci = nullptr;                      // L_i rows
    const double *lv = nullptr;
    double *P = nullptr;           // P_q of the current pass
};
struct TailLevel {
    int n = 0, nc = 0;             // rows, rows of the next level
    double *b = nullptr, *x = nullptr, *x2 = nullptr, *wp = nullptr;
    const double *deff = nullptr;  // the rows' divisors (their diagonals)
    int csplit = 0, inner = 0, pre = 0, post = 0, finite = 0;
    TailPass pass[2];
    const int *arp = nullptr, *aci = nullptr, *rrp = nullptr, *rci = nullptr, *prp = nullptr, *pci = nullptr;
    const double *av = nullptr, *rv = nullptr, *pv = nullptr;
};
struct TailPlan {
    int from = -1;                 // first tail level (-1: no tail)
    int nlev = 0;
    TailLevel *d_levels = nullptr; // device copy of the descriptors
    const double *inv = nullptr;   // the coarsest level's explicit inverse (row-major nc x nc)
    int nc = 0;
    double *cb = nullptr, *cx = nullptr;   // the coarsest level's b and x
    double ledger_bytes = 0.0;     // stored bytes one tail launch streams (sss_engine.hpp ByteLedger)
};

int tail_upload(TailPlan &t, const std::vector<TailLevel> &levels);
int tail_launch(const TailPlan &t, hipStream_t s);
void tail_free(TailPlan &t);

}  // namespace sss
