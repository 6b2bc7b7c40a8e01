// Probe: is v_mfma_f32_32x32x16_f16 / 32x32x8_f16 bit-identical to an ordered fp32 fmaf chain
// over its K products (products of fp16 are exact in fp32)? Prints mismatch counts for several
// CPU emulations over random inputs.
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef _Float16 h4 __attribute__((ext_vector_type(4)));
typedef float f16v __attribute__((ext_vector_type(16)));

// A[32][K], B[32][K] (row-major, k fastest), C[32][32] in; D out. K = 16 or 8.
template <int K>
__global__ void probe(const _Float16* A, const _Float16* B, const float* C, float* D)
{
    const int lane = threadIdx.x;
    f16v acc;
    // 32x32 accumulator layout: element k of lane: row = (k&3) + 8*(k>>2) + 4*(lane>>5), col = lane&31
    for (int k = 0; k < 16; k++) acc[k] = C[((k & 3) + 8 * (k >> 2) + 4 * (lane >> 5)) * 32 + (lane & 31)];
    if constexpr (K == 16) {
        // operand: lane holds row (lane&31), k = 8*(lane>>5) .. +7
        h8 a, b;
        for (int t = 0; t < 8; t++) {
            a[t] = A[(lane & 31) * K + 8 * (lane >> 5) + t];
            b[t] = B[(lane & 31) * K + 8 * (lane >> 5) + t];
        }
        acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, acc, 0, 0, 0);
    } else {
        h4 a, b;
        for (int t = 0; t < 4; t++) {
            a[t] = A[(lane & 31) * K + 4 * (lane >> 5) + t];
            b[t] = B[(lane & 31) * K + 4 * (lane >> 5) + t];
        }
        acc = __builtin_amdgcn_mfma_f32_32x32x8f16(a, b, acc, 0, 0, 0);
    }
    for (int k = 0; k < 16; k++) D[((k & 3) + 8 * (k >> 2) + 4 * (lane >> 5)) * 32 + (lane & 31)] = acc[k];
}

template <int K>
void run(int trials)
{
    std::vector<_Float16> A(32 * K), B(32 * K);
    std::vector<float> C(1024), D(1024);
    _Float16 *dA, *dB;
    float *dC, *dD;
    hipMalloc(&dA, A.size() * 2); hipMalloc(&dB, B.size() * 2);
    hipMalloc(&dC, 4096); hipMalloc(&dD, 4096);
    long mis_chain = 0, mis_chain_rev = 0, mis_exact = 0, mis_pair = 0, total = 0;
    srand(1234);
    for (int tr = 0; tr < trials; tr++) {
        for (auto& x : A) x = (_Float16)((rand() / (float)RAND_MAX - 0.5f) * (float)(1 << (rand() % 6)));
        for (auto& x : B) x = (_Float16)((rand() / (float)RAND_MAX - 0.5f) * (float)(1 << (rand() % 6)));
        for (auto& x : C) x = (rand() / (float)RAND_MAX - 0.5f) * 100.f;
        hipMemcpy(dA, A.data(), A.size() * 2, hipMemcpyHostToDevice);
        hipMemcpy(dB, B.data(), B.size() * 2, hipMemcpyHostToDevice);
        hipMemcpy(dC, C.data(), 4096, hipMemcpyHostToDevice);
        hipLaunchKernelGGL(probe<K>, dim3(1), dim3(64), 0, 0, dA, dB, dC, dD);
        hipMemcpy(D.data(), dD, 4096, hipMemcpyDeviceToHost);
        for (int r = 0; r < 32; r++)
            for (int c = 0; c < 32; c++) {
                float p[K];
                for (int k = 0; k < K; k++) p[k] = (float)A[r * K + k] * (float)B[c * K + k];  // exact
                float chain = C[r * 32 + c];
                for (int k = 0; k < K; k++) chain = chain + p[k];
                float chainr = C[r * 32 + c];
                for (int k = K - 1; k >= 0; k--) chainr = chainr + p[k];
                double ex = C[r * 32 + c];
                for (int k = 0; k < K; k++) ex += (double)p[k];
                float exf = (float)ex;
                // pairwise: sum products in a tree (fp32), then add C
                float t[K];
                for (int k = 0; k < K; k++) t[k] = p[k];
                for (int w = K; w > 1; w /= 2)
                    for (int k = 0; k < w / 2; k++) t[k] = t[2 * k] + t[2 * k + 1];
                float pair = C[r * 32 + c] + t[0];
                const float g = D[r * 32 + c];
                mis_chain += g != chain;
                mis_chain_rev += g != chainr;
                mis_exact += g != exf;
                mis_pair += g != pair;
                total++;
            }
    }
    printf("K=%d: %ld elements; mismatches: chain %ld, reverse chain %ld, exact-sum-one-rounding %ld, pairwise %ld\n",
           K, total, mis_chain, mis_chain_rev, mis_exact, mis_pair);
}

int main()
{
    run<16>(50);
    run<8>(50);
    return 0;
}
