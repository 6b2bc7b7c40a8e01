// Probe: sustained rate of v_mfma_f64_16x16x4_f64 on the whole chip (no memory traffic), with C
// independent accumulator chains per wave and W waves per SIMD (the fp64 flush's instruction).
//   hipcc --offload-arch=gfx950 -O3 -o mfma_f64_rate scripts/probe/mfma_f64_rate.hip
#include <hip/hip_runtime.h>

#include <stdio.h>

typedef double f64x4 __attribute__((ext_vector_type(4)));

template <int C>
__global__ __launch_bounds__(256) void mfma_loop(double* out, int iters, double a, double b)
{
    f64x4 acc[C];
#pragma unroll
    for (int c = 0; c < C; c++) acc[c] = f64x4{0.0, 0.0, 0.0, 0.0};
    double av = a + threadIdx.x * 1e-7, bv = b;
    for (int i = 0; i < iters; i++) {
#pragma unroll
        for (int s = 0; s < 8; s++)
#pragma unroll
            for (int c = 0; c < C; c++) acc[c] = __builtin_amdgcn_mfma_f64_16x16x4f64(av, bv, acc[c], 0, 0, 0);
    }
    double t = 0.0;
#pragma unroll
    for (int c = 0; c < C; c++) t += acc[c][0] + acc[c][1] + acc[c][2] + acc[c][3];
    if (t == 12345.0) out[0] = t;
}

template <int C>
void run(int blocks_per_cu, int ncu)
{
    double* out;
    (void)hipMalloc(&out, 8);
    const int iters = 1000;
    const int grid = ncu * blocks_per_cu;
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    for (int rep = 0; rep < 3; rep++) {
        (void)hipEventRecord(e0);
        hipLaunchKernelGGL(mfma_loop<C>, dim3(grid), dim3(256), 0, 0, out, iters, 1.0, 1e-9);
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        float ms = 0;
        (void)hipEventElapsedTime(&ms, e0, e1);
        const double n_mfma = (double)grid * 4 * iters * 8 * C;   // per SIMD: grid*4/(4*ncu)
        const double flops = n_mfma * 16 * 16 * 4 * 2;
        const double per_simd = n_mfma / (ncu * 4.0);
        if (rep == 2)
            printf("chains %d, waves/SIMD %d: %.3f ms, %.1f TF/s, %.1f ns per MFMA per SIMD\n", C, blocks_per_cu, ms,
                   flops / ms / 1e9, ms * 1e6 / per_simd);
    }
    (void)hipFree(out);
}

int main()
{
    hipDeviceProp_t prop;
    (void)hipGetDeviceProperties(&prop, 0);
    const int ncu = prop.multiProcessorCount;
    printf("CUs %d, clock %d kHz\n", ncu, prop.clockRate);
    run<1>(1, ncu);
    run<2>(1, ncu);
    run<4>(1, ncu);
    run<8>(1, ncu);
    run<8>(2, ncu);
    run<16>(1, ncu);
    return 0;
}
