// sss_build.hip — device-side builders of the free-order storage formats (upload time).
//
// The long-row levels of a throughput-mode hierarchy (levels 5-10 of 7-pt 400^3) are read through
//   * merged row groups (DevCSR::mg_*): the entries of G consecutive rows, sorted by the unique
//     key  col << 4 | segment << 3 | row-in-group  (sss_engine.hpp), and
//   * column-sorted row segments (DevCSR::rows_sorted): each row -- or each of its two segments
//     [rp, seg) / [seg, rp + 1) -- sorted by column.
// The host builders (sss_spmv.hip build_merged / sort_row_segments) sort these on the CPU, 3-4 ns
// per entry on the 16-core box, which was most of the mirror construction left after an
// overlapped setup (profiles/r03_host_phases_seq_400.txt: 0.5-0.8 s per coarse level).  Here the
// stored-order CSR already resident in HBM is sorted in place on the GPU by a segmented radix sort.
// Every key is unique inside its segment (a row's columns are distinct, and the segment / row bits
// separate the rows of a group), so the result does not depend on the sort's stability: it is the
// host builder's output bit for bit (tests/test_gpu_setup_pipeline.py compares whole solves).
#include <hipcub/hipcub.hpp>

#include "sss_engine.hpp"

namespace sss {

namespace {

// key[k] of every entry of row r: col << kMergeShift | segment << 3 | (r mod G)
__global__ __launch_bounds__(kBlock) void merged_keys(int n, int G, const int *__restrict__ rp,
                                                      const int *__restrict__ ci, const int *__restrict__ seg,
                                                      unsigned *__restrict__ key)
{
    const int r = blockIdx.x * kBlock + threadIdx.x;
    if (r >= n) return;
    const unsigned rig = (unsigned)(r % G);
    const int s = seg ? seg[r] : rp[r + 1];
    for (int k = rp[r]; k < rp[r + 1]; ++k)
        key[k] = ((unsigned)ci[k] << kMergeShift) | ((k >= s ? 1u : 0u) << 3) | rig;
}

// gp[g] = rp[g G] (g < ng), gp[ng] = rp[n]
__global__ __launch_bounds__(kBlock) void group_bounds(int n, int G, int ng, const int *__restrict__ rp,
                                                       int *__restrict__ gp)
{
    const int g = blockIdx.x * kBlock + threadIdx.x;
    if (g < ng) gp[g] = rp[g * G];
    else if (g == ng) gp[g] = rp[n];
}

// segment offsets of two-segment rows: off[2r] = rp[r], off[2r + 1] = seg[r], off[2n] = rp[n]
__global__ __launch_bounds__(kBlock) void segment_offsets(int n, const int *__restrict__ rp, const int *__restrict__ seg,
                                                          int *__restrict__ off)
{
    const int r = blockIdx.x * kBlock + threadIdx.x;
    if (r < n) {
        off[2 * r] = rp[r];
        off[2 * r + 1] = seg[r];
    } else if (r == n) {
        off[2 * n] = rp[n];
    }
}

// out = in sorted within each segment [off[s], off[s + 1]) by the 32-bit key (keys unique per
// segment), values carried along
int segmented_sort(const unsigned *kin, unsigned *kout, const double *vin, double *vout, int nnz, int nseg,
                   const int *off, hipStream_t s)
{
    if (nnz == 0 || nseg == 0) return 0;
    size_t tb = 0;
    SSS_HIP(hipcub::DeviceSegmentedRadixSort::SortPairs(nullptr, tb, kin, kout, vin, vout, nnz, nseg, off, off + 1, 0,
                                                        32, s));
    void *tmp = nullptr;
    SSS_HIP(hipMalloc(&tmp, std::max<size_t>(tb, 1)));
    const hipError_t e = hipcub::DeviceSegmentedRadixSort::SortPairs(tmp, tb, kin, kout, vin, vout, nnz, nseg, off,
                                                                     off + 1, 0, 32, s);
    const hipError_t e2 = hipStreamSynchronize(s);
    (void)hipFree(tmp);
    SSS_HIP(e);
    SSS_HIP(e2);
    return 0;
}

int upload_seg(const int *h_seg, int n, int **d_seg)
{
    *d_seg = nullptr;
    if (!h_seg) return 0;
    *d_seg = dev_alloc<int>((size_t)n);
    if (!*d_seg) return hip_fail(hipErrorOutOfMemory, "hipMalloc(seg)", __FILE__, __LINE__);
    return h2d(*d_seg, h_seg, sizeof(int) * (size_t)n);
}

}  // namespace

bool device_builders_on()
{
    const char *e = getenv("SSS_HIP_GPU_BUILD");   // 0: the host builders (tests compare both)
    return !(e && *e == '0');
}

// d: rp / ci / v resident in stored order, d.mg_G > 0.  Fills mg_gp, mg_k, mg_v, mg_ng.
int merged_build_device(DevCSR &d, const int *h_seg)
{
    const int n = d.n, G = d.mg_G, ng = (n + G - 1) / G;
    d.mg_ng = ng;
    d.mg_gp = dev_alloc<int>((size_t)ng + 1);
    d.mg_k = dev_alloc<unsigned>((size_t)d.nnz);
    d.mg_v = dev_alloc<double>((size_t)d.nnz);
    unsigned *key = dev_alloc<unsigned>((size_t)d.nnz);
    int *dseg = nullptr;
    int rc = (!d.mg_gp || !d.mg_k || !d.mg_v || !key) ? hip_fail(hipErrorOutOfMemory, "hipMalloc(merged)", __FILE__, __LINE__)
                                                        : upload_seg(h_seg, n, &dseg);
    if (!rc) {
        hipLaunchKernelGGL(group_bounds, dim3((ng + kBlock) / kBlock), dim3(kBlock), 0, nullptr, n, G, ng, d.rp, d.mg_gp);
        if (n > 0)
            hipLaunchKernelGGL(merged_keys, dim3((n + kBlock - 1) / kBlock), dim3(kBlock), 0, nullptr, n, G, d.rp, d.ci,
                               dseg, key);
        const hipError_t e = hipGetLastError();
        if (e != hipSuccess) rc = hip_fail(e, "merged_keys", __FILE__, __LINE__);
    }
    if (!rc) rc = segmented_sort(key, d.mg_k, d.v, d.mg_v, d.nnz, ng, d.mg_gp, nullptr);
    dev_free(key);
    dev_free(dseg);
    return rc;
}

// d.ci / d.v (stored order) sorted by column within each row, or each row segment when h_seg is
// given; sets d.rows_sorted.
int sort_rows_device(DevCSR &d, const int *h_seg)
{
    const int n = d.n;
    unsigned *kin = dev_alloc<unsigned>((size_t)d.nnz);
    double *vin = dev_alloc<double>((size_t)d.nnz);
    int *dseg = nullptr, *off = nullptr;
    int rc = (!kin || !vin) ? hip_fail(hipErrorOutOfMemory, "hipMalloc(row sort)", __FILE__, __LINE__) : 0;
    if (!rc && h_seg) {
        rc = upload_seg(h_seg, n, &dseg);
        off = rc ? nullptr : dev_alloc<int>(2 * (size_t)n + 1);
        if (!rc && !off) rc = hip_fail(hipErrorOutOfMemory, "hipMalloc(row sort)", __FILE__, __LINE__);
        if (!rc) hipLaunchKernelGGL(segment_offsets, dim3((n + kBlock) / kBlock), dim3(kBlock), 0, nullptr, n, d.rp, dseg, off);
    }
    if (!rc && hipMemcpy(kin, d.ci, sizeof(int) * (size_t)d.nnz, hipMemcpyDeviceToDevice) != hipSuccess) rc = ERROR_MISC;
    if (!rc && hipMemcpy(vin, d.v, sizeof(double) * (size_t)d.nnz, hipMemcpyDeviceToDevice) != hipSuccess) rc = ERROR_MISC;
    if (!rc)   // columns are non-negative, so their unsigned order is the column order
        rc = segmented_sort(kin, reinterpret_cast<unsigned *>(d.ci), vin, d.v, d.nnz, h_seg ? 2 * n : n,
                            h_seg ? off : d.rp, nullptr);
    if (!rc) d.rows_sorted = true;
    dev_free(kin);
    dev_free(vin);
    dev_free(dseg);
    dev_free(off);
    return rc;
}

}  // namespace sss
