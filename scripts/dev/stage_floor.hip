// Stage-latency floor of a barrier-separated wavefront kernel on gfx950 (diagnostic, not product code).
// One workgroup per CU-slot runs `iters` stages; per stage the "chain" wave does the work of mode m, the other
// waves only hit the barrier.  Prints s_memtime cycles per stage (median of workgroup 0's waves' view).
//   hipcc --offload-arch=gfx950 -O3 -o scripts/dev/stage_floor scripts/dev/stage_floor.hip
//   ./scripts/dev/stage_floor
// modes: 0 barrier only; 1 + one LDS write->barrier->read round trip on the chain wave; 2 + a 16-deep dependent
// fp64 chain on it; 3 + 16 LDS loads issued together (the records); 4 = 3 + 2 VALU-heavy waves (120 fp64 ops each)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

__global__ __launch_bounds__(1024) void k_floor(int mode, int iters, unsigned long long* out, double* sink)
{
    __shared__ double lds[16 * 64 + 64];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
    double x = lane * 1e-3 + 1.0, acc = 0.0;
    for (int i = threadIdx.x; i < 16 * 64 + 64; i += blockDim.x) lds[i] = 1.0 + i * 1e-6;
    __syncthreads();
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < iters; ++it) {
        if (wave == nw - 1 && mode >= 1) {
            double v = lds[16 * 64 + lane];
            if (mode >= 3) {
                double r = 0.0;
#pragma unroll
                for (int f = 0; f < 16; ++f) r += lds[f * 64 + lane];
                v += r;
            }
            if (mode >= 2) {
#pragma unroll
                for (int d = 0; d < 16; ++d) v = fma(v, 0.999999, 1e-9);
            }
            lds[16 * 64 + lane] = v;
        } else if (mode >= 4 && wave >= nw - 3) {
            double a = x, b = x * 0.5;
#pragma unroll
            for (int d = 0; d < 60; ++d) { a = fma(a, 0.9999, b); b = fma(b, 1.0001, a); }
            acc += a + b;
        }
        __syncthreads();
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if (lane == 0) out[blockIdx.x * 16 + wave] = t1 - t0;
    if (acc == 12345.0) sink[threadIdx.x] = acc + lds[lane];
}

int main()
{
    int ncu = 0;
    hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
    unsigned long long* d;
    double* sink;
    const int iters = 2000;
    hipMalloc(&d, sizeof(unsigned long long) * 16 * 4096);
    hipMalloc(&sink, sizeof(double) * 1024);
    for (int waves : {8, 14, 16})
        for (int per_cu : {1, 2})
            for (int mode = 0; mode <= 4; ++mode) {
                if (waves * per_cu > 16) continue;
                const int nb = ncu * per_cu;
                hipLaunchKernelGGL(k_floor, dim3(nb), dim3(64 * waves), 0, 0, mode, iters, d, sink);
                hipDeviceSynchronize();
                hipEvent_t e0, e1;
                hipEventCreate(&e0);
                hipEventCreate(&e1);
                hipEventRecord(e0);
                hipLaunchKernelGGL(k_floor, dim3(nb), dim3(64 * waves), 0, 0, mode, iters, d, sink);
                hipEventRecord(e1);
                hipEventSynchronize(e1);
                float ms = 0;
                hipEventElapsedTime(&ms, e0, e1);
                std::vector<unsigned long long> h(16 * nb);
                hipMemcpy(h.data(), d, sizeof(unsigned long long) * 16 * nb, hipMemcpyDeviceToHost);
                std::vector<double> c;
                for (int b = 0; b < nb; ++b) c.push_back((double)h[b * 16] / iters);
                std::sort(c.begin(), c.end());
                printf("waves %2d  wg/cu %d  mode %d : %7.1f cycles/stage (median s_memtime), %6.3f us/stage (events)\n",
                       waves, per_cu, mode, c[c.size() / 2], ms * 1e3 / iters);
            }
    return 0;
}
