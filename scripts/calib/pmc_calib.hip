// FETCH_SIZE calibration for the access widths the cascade uses (MI355X_MICROARCH.md, HBM:
// "calibrate on a known byte count in your own access pattern").  Streams a 2 GiB buffer once
// with 8 B/lane (global_load_dwordx2, the cascade's alpha column loads) and once with
// 16 B/lane loads; rocprofv3 --pmc FETCH_SIZE on this binary gives KB counted per byte read.
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void k_stream_b64(const double* __restrict__ a, size_t n, double* __restrict__ out)
{
    double s = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) s += a[i];
    if (s == 12345.0) out[0] = s;   // keep the loads
}
__global__ void k_stream_b128(const double2* __restrict__ a, size_t n, double* __restrict__ out)
{
    double s = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const double2 v = a[i];
        s += v.x + v.y;
    }
    if (s == 12345.0) out[0] = s;
}

int main()
{
    const size_t bytes = (size_t)2 << 30;
    double *a, *out;
    if (hipMalloc(&a, bytes) != hipSuccess || hipMalloc(&out, 64) != hipSuccess) return 1;
    if (hipMemset(a, 0, bytes) != hipSuccess) return 1;
    hipLaunchKernelGGL(k_stream_b64, dim3(4096), dim3(256), 0, 0, a, bytes / 8, out);
    hipLaunchKernelGGL(k_stream_b128, dim3(4096), dim3(256), 0, 0, (const double2*)a, bytes / 16, out);
    if (hipDeviceSynchronize() != hipSuccess) return 1;
    printf("{\"calib_bytes\": %zu}\n", bytes);
    (void)hipFree(a);
    (void)hipFree(out);
    return 0;
}
