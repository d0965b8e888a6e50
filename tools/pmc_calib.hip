// pmc_calib.hip — FETCH_SIZE calibration on gfx950 for the access widths the engine uses.
// Each kernel streams exactly `bytes` bytes of a fresh 2 GiB buffer once (coalesced), with 4, 8
// or 16 bytes per lane; compare rocprofv3 --pmc FETCH_SIZE (KiB) with the byte count.
//   hipcc --offload-arch=gfx950 -O3 -o tools/pmc_calib tools/pmc_calib.hip
#include <hip/hip_runtime.h>

#include <cstdio>

template <class T>
__global__ void stream_read(const T *__restrict__ a, size_t n, double *out)
{
    double s = 0.0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const T v = a[i];
        s += (double)(((const int *)&v)[0]);
    }
    if (s == 12345.678) out[0] = s;   // keep the loads
}

int main()
{
    const size_t bytes = size_t(2) << 30;
    char *buf;
    double *out;
    if (hipMalloc(&buf, bytes) != hipSuccess || hipMalloc(&out, 8) != hipSuccess) return 1;
    hipMemset(buf, 1, bytes);
    hipDeviceSynchronize();
    for (int rep = 0; rep < 2; ++rep) {
        hipLaunchKernelGGL(stream_read<int>, dim3(8192), dim3(256), 0, 0, (const int *)buf, bytes / 4, out);
        hipLaunchKernelGGL(stream_read<double>, dim3(8192), dim3(256), 0, 0, (const double *)buf, bytes / 8, out);
        hipLaunchKernelGGL(stream_read<int4>, dim3(8192), dim3(256), 0, 0, (const int4 *)buf, bytes / 16, out);
    }
    hipDeviceSynchronize();
    printf("calibration: %zu bytes per kernel\n", bytes);
    return 0;
}
