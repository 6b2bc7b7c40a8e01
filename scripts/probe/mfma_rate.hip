// Probe: sustained rate of v_mfma_f32_32x32x2_f32 on the whole chip (no memory traffic), with
// C independent accumulator chains per wave and W waves per SIMD. Build:
//   hipcc --offload-arch=gfx950 -O3 -o mfma_rate scripts/probe/mfma_rate.hip
#include <hip/hip_runtime.h>

#include <stdio.h>

typedef float f32x16 __attribute__((ext_vector_type(16)));

template <int C>
__global__ __launch_bounds__(256) void mfma_loop(float* out, int iters, float a, float b)
{
    f32x16 acc[C];
#pragma unroll
    for (int c = 0; c < C; c++)
        for (int k = 0; k < 16; k++) acc[c][k] = 0.f;
    float av = a + threadIdx.x * 1e-7f, bv = b;
    for (int i = 0; i < iters; i++) {
#pragma unroll
        for (int s = 0; s < 8; s++)
#pragma unroll
            for (int c = 0; c < C; c++) acc[c] = __builtin_amdgcn_mfma_f32_32x32x2f32(av, bv, acc[c], 0, 0, 0);
    }
    float t = 0.f;
#pragma unroll
    for (int c = 0; c < C; c++)
        for (int k = 0; k < 16; k++) t += acc[c][k];
    if (t == 12345.f) out[0] = t;
}

template <int C>
void run(int blocks_per_cu, int ncu)
{
    float* out;
    (void)hipMalloc(&out, 4);
    const int iters = 2000;
    const int grid = ncu * blocks_per_cu;
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    for (int rep = 0; rep < 3; rep++) {
        (void)hipEventRecord(e0);
        hipLaunchKernelGGL(mfma_loop<C>, dim3(grid), dim3(256), 0, 0, out, iters, 1.0f, 1e-9f);
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        float ms = 0;
        (void)hipEventElapsedTime(&ms, e0, e1);
        const double flops = (double)grid * 4 * iters * 8 * C * 32 * 32 * 2 * 2;
        if (rep == 2)
            printf("chains %d, waves/SIMD %d: %.3f ms, %.1f TF/s\n", C, blocks_per_cu, ms, flops / ms / 1e9);
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
    run<4>(2, ncu);
    run<8>(1, ncu);
    run<8>(2, ncu);
    return 0;
}
