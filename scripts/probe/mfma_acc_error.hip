// Probe: the rounding of the fp32 accumulation inside the split arithmetics' MFMAs.
// For v_mfma_f32_32x32x16_f16 / _bf16 (the split flushes) and v_mfma_f32_32x32x2_f32 (EXACT):
// D = C + Σ_k A_k·B_k against the exact sum (double; the products of 16-bit inputs are exact), in
// units of ulp(exact): mean (bias) and RMS, and how often D is the correctly rounded sum.
// Cases: C of the size of the products (cancellation) and C 2^8 .. 2^16 above them (a small
// correction added to a large accumulator: the split products' lo terms onto −2^(2σ)·P).
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef __bf16 b8 __attribute__((ext_vector_type(8)));
typedef float f16v __attribute__((ext_vector_type(16)));

// A[32][K], B[32][K] row-major; C, D 32×32 row-major. MODE 0 f16 (K 16), 1 bf16 (K 16), 2 f32 (K 2)
template <int MODE>
__global__ void probe(const float* A, const float* B, const float* C, float* D)
{
    constexpr int K = MODE == 2 ? 2 : 16;
    const int lane = threadIdx.x;
    f16v acc;
    for (int k = 0; k < 16; k++) acc[k] = C[((k & 3) + 8 * (k >> 2) + 4 * (lane >> 5)) * 32 + (lane & 31)];
    if constexpr (MODE == 0) {
        h8 a, b;
        for (int t = 0; t < 8; t++) {
            a[t] = (_Float16)A[(lane & 31) * K + 8 * (lane >> 5) + t];
            b[t] = (_Float16)B[(lane & 31) * K + 8 * (lane >> 5) + t];
        }
        acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, acc, 0, 0, 0);
    } else if constexpr (MODE == 1) {
        b8 a, b;
        for (int t = 0; t < 8; t++) {
            a[t] = (__bf16)A[(lane & 31) * K + 8 * (lane >> 5) + t];
            b[t] = (__bf16)B[(lane & 31) * K + 8 * (lane >> 5) + t];
        }
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc, 0, 0, 0);
    } else {
        const float a = A[(lane & 31) * K + (lane >> 5)];
        const float b = B[(lane & 31) * K + (lane >> 5)];
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc, 0, 0, 0);
    }
    for (int k = 0; k < 16; k++) D[((k & 3) + 8 * (k >> 2) + 4 * (lane >> 5)) * 32 + (lane & 31)] = acc[k];
}

static float q16(float x, int mode)   // the value the MFMA sees
{
    if (mode == 0) return (float)(_Float16)x;
    if (mode == 1) {
        unsigned u;
        memcpy(&u, &x, 4);
        u &= 0xffff0000u;   // exact bf16 values only (the planes are truncations)
        memcpy(&x, &u, 4);
        return x;
    }
    return x;
}

template <int MODE>
void run(const char* name, int cscale_log2, int trials)
{
    constexpr int K = MODE == 2 ? 2 : 16;
    std::vector<float> A(32 * K), B(32 * K), C(1024), D(1024);
    float *dA, *dB, *dC, *dD;
    hipMalloc(&dA, A.size() * 4); hipMalloc(&dB, B.size() * 4);
    hipMalloc(&dC, 4096); hipMalloc(&dD, 4096);
    std::mt19937 rng(1234 + MODE * 7 + cscale_log2);
    std::uniform_real_distribution<float> u(-1.f, 1.f);
    double sum = 0, sum2 = 0, n = 0, rne = 0, worst = 0;
    for (int tr = 0; tr < trials; tr++) {
        for (auto& x : A) x = q16(u(rng), MODE);
        for (auto& x : B) x = q16(u(rng), MODE);
        for (auto& x : C) x = u(rng) * ldexpf(1.f, cscale_log2);
        hipMemcpy(dA, A.data(), A.size() * 4, hipMemcpyHostToDevice);
        hipMemcpy(dB, B.data(), B.size() * 4, hipMemcpyHostToDevice);
        hipMemcpy(dC, C.data(), 4096, hipMemcpyHostToDevice);
        hipLaunchKernelGGL(probe<MODE>, dim3(1), dim3(64), 0, 0, dA, dB, dC, dD);
        hipMemcpy(D.data(), dD, 4096, hipMemcpyDeviceToHost);
        for (int r = 0; r < 32; r++)
            for (int c = 0; c < 32; c++) {
                double ex = C[r * 32 + c];
                for (int k = 0; k < K; k++) ex += (double)A[r * K + k] * (double)B[c * K + k];
                const double ulp = ldexp(1.0, ilogb(ex) - 23);
                const double e = ((double)D[r * 32 + c] - ex) / ulp;
                sum += e; sum2 += e * e; n += 1;
                rne += D[r * 32 + c] == (float)ex;
                worst = fmax(worst, fabs(e));
            }
    }
    printf("%-6s C~2^%-3d n=%.0f  mean %+.4f ulp  rms %.4f ulp  worst %.3f ulp  correctly rounded %.4f\n",
           name, cscale_log2, n, sum / n, sqrt(sum2 / n), worst, rne / n);
    hipFree(dA); hipFree(dB); hipFree(dC); hipFree(dD);
}

int main()
{
    for (int cs : {0, 4, 8, 12, 16}) {
        run<0>("f16", cs, 200);
        run<1>("bf16", cs, 200);
        run<2>("f32", cs, 200);
    }
    return 0;
}
