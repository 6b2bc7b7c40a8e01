// Issue rate and dependent latency of fp64 VALU instructions for ONE wave per SIMD (the
// association kernel's regime): cycles per v_fma_f64 with 8 independent chains and with 1 chain,
// the same for fp32, and per ds_read_b128 round trip. Probe only (scripts/probe, not the library).
// build: hipcc --offload-arch=gfx950 -O3 valu_f64_rate.hip -o valu_f64_rate
#include <hip/hip_runtime.h>
#include <cstdio>

template <typename F, int CH>
__global__ void chain(F* out, long long* cyc, int iters)
{
    F a[CH];
    for (int c = 0; c < CH; c++) a[c] = (F)(threadIdx.x + c) * (F)1e-3;
    const F m = (F)0.999999, k = (F)1e-7;
    __syncthreads();
    const long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < iters; i++) {
#pragma unroll
        for (int r = 0; r < 16; r++)
#pragma unroll
            for (int c = 0; c < CH; c++) a[c] = __builtin_fma(a[c], m, k);
    }
    const long long t1 = __builtin_amdgcn_s_memtime();
    F s = 0;
    for (int c = 0; c < CH; c++) s += a[c];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

__global__ void lds_rt(double* out, long long* cyc, int iters)
{
    __shared__ double4 buf[256];
    buf[threadIdx.x] = make_double4(threadIdx.x, 1, 2, 3);
    __syncthreads();
    int idx = threadIdx.x;
    double s = 0;
    const long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < iters; i++) {
        const double4 v = buf[idx & 255];
        idx = (int)v.x + 1;   // dependent chain of LDS reads
        s += v.y;
    }
    const long long t1 = __builtin_amdgcn_s_memtime();
    out[blockIdx.x * blockDim.x + threadIdx.x] = s + idx;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <typename F>
static double run(void (*kern)(F*, long long*, int), int iters, double per)
{
    F* out; long long* cyc;
    (void)hipMalloc(&out, 256 * 64 * 8); (void)hipMalloc(&cyc, 256 * 8);
    hipLaunchKernelGGL(kern, dim3(256), dim3(64), 0, 0, out, cyc, iters);
    (void)hipDeviceSynchronize();
    long long h[256];
    (void)hipMemcpy(h, cyc, sizeof(h), hipMemcpyDeviceToHost);
    long long mn = h[0];
    for (int i = 0; i < 256; i++) mn = h[i] < mn ? h[i] : mn;
    (void)hipFree(out); (void)hipFree(cyc);
    return (double)mn / per;
}

int main()
{
    const int it = 2000;
    // warm
    run(chain<double, 8>, it, 1);
    printf("{\"f64_fma_indep8_cyc\": %.2f, ", run(chain<double, 8>, it, 16.0 * 8 * it));
    printf("\"f64_fma_dep1_cyc\": %.2f, ", run(chain<double, 1>, it, 16.0 * it));
    printf("\"f32_fma_indep8_cyc\": %.2f, ", run(chain<float, 8>, it, 16.0 * 8 * it));
    printf("\"f32_fma_dep1_cyc\": %.2f, ", run(chain<float, 1>, it, 16.0 * it));
    printf("\"lds_b128_dependent_roundtrip_cyc\": %.1f}\n", run(lds_rt, it, (double)it));
    return 0;
}
