// Probe for a split-bf16 flush: is v_mfma_f32_32x32x16_bf16 deterministic and
// position-independent (the same A row, B column and C value give the same output bits wherever
// they sit in the 32×32 tile and whatever the other rows/columns hold)? If so, an association
// kernel could replay a split-bf16 flush bit for bit with the same instruction. Prints mismatch
// counts; no product code depends on it.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef __bf16 bf8 __attribute__((ext_vector_type(8)));
typedef float f16v __attribute__((ext_vector_type(16)));

// A[32][16], B[32][16] (row-major, k fastest), C[32][32]; D = C + A·Bᵀ
__global__ void probe(const __bf16* A, const __bf16* B, const float* C, float* D)
{
    const int lane = threadIdx.x;
    f16v acc;
    for (int k = 0; k < 16; k++) acc[k] = C[((k & 3) + 8 * (k >> 2) + 4 * (lane >> 5)) * 32 + (lane & 31)];
    bf8 a, b;
    for (int t = 0; t < 8; t++) {
        a[t] = A[(lane & 31) * 16 + 8 * (lane >> 5) + t];
        b[t] = B[(lane & 31) * 16 + 8 * (lane >> 5) + t];
    }
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc, 0, 0, 0);
    for (int k = 0; k < 16; k++) D[((k & 3) + 8 * (k >> 2) + 4 * (lane >> 5)) * 32 + (lane & 31)] = acc[k];
}

static __bf16 rnd_bf16(int e) { return (__bf16)((rand() / (float)RAND_MAX - 0.5f) * (float)(1 << (rand() % e))); }

int main()
{
    std::vector<__bf16> A(512), B(512), A2(512), B2(512);
    std::vector<float> C(1024), C2(1024), D(1024), D2(1024), D3(1024);
    __bf16 *dA, *dB;
    float *dC, *dD;
    hipMalloc(&dA, 1024); hipMalloc(&dB, 1024); hipMalloc(&dC, 4096); hipMalloc(&dD, 4096);
    long mis_pos = 0, mis_rep = 0, mis_exact = 0, total = 0;
    srand(7);
    for (int tr = 0; tr < 2000; tr++) {
        for (auto& x : A) x = rnd_bf16(12);
        for (auto& x : B) x = rnd_bf16(12);
        for (auto& x : C) x = (rand() / (float)RAND_MAX - 0.5f) * 1000.f;
        hipMemcpy(dA, A.data(), 1024, hipMemcpyHostToDevice);
        hipMemcpy(dB, B.data(), 1024, hipMemcpyHostToDevice);
        hipMemcpy(dC, C.data(), 4096, hipMemcpyHostToDevice);
        hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, dA, dB, dC, dD);
        hipMemcpy(D.data(), dD, 4096, hipMemcpyDeviceToHost);
        hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, dA, dB, dC, dD);   // repeat
        hipMemcpy(D3.data(), dD, 4096, hipMemcpyDeviceToHost);
        // permute rows of A (and of C) and columns of B (and of C): the same (row, col) pairs at
        // other positions, with other neighbours
        int pr[32], pc[32];
        for (int i = 0; i < 32; i++) pr[i] = pc[i] = i;
        for (int i = 31; i > 0; i--) { int j = rand() % (i + 1); int t = pr[i]; pr[i] = pr[j]; pr[j] = t; }
        for (int i = 31; i > 0; i--) { int j = rand() % (i + 1); int t = pc[i]; pc[i] = pc[j]; pc[j] = t; }
        for (int r = 0; r < 32; r++)
            for (int k = 0; k < 16; k++) { A2[pr[r] * 16 + k] = A[r * 16 + k]; B2[pc[r] * 16 + k] = B[r * 16 + k]; }
        for (int r = 0; r < 32; r++)
            for (int c = 0; c < 32; c++) C2[pr[r] * 32 + pc[c]] = C[r * 32 + c];
        hipMemcpy(dA, A2.data(), 1024, hipMemcpyHostToDevice);
        hipMemcpy(dB, B2.data(), 1024, hipMemcpyHostToDevice);
        hipMemcpy(dC, C2.data(), 4096, hipMemcpyHostToDevice);
        hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, dA, dB, dC, dD);
        hipMemcpy(D2.data(), dD, 4096, hipMemcpyDeviceToHost);
        for (int r = 0; r < 32; r++)
            for (int c = 0; c < 32; c++) {
                const float g = D[r * 32 + c];
                mis_pos += g != D2[pr[r] * 32 + pc[c]];
                mis_rep += g != D3[r * 32 + c];
                double ex = C[r * 32 + c];
                for (int k = 0; k < 16; k++) ex += (double)(float)A[r * 16 + k] * (double)(float)B[c * 16 + k];
                mis_exact += g != (float)ex;
                total++;
            }
    }
    printf("{\"elements\": %ld, \"repeat_mismatch\": %ld, \"position_mismatch\": %ld, \"vs_exact_sum_rounded_once\": %ld}\n",
           total, mis_rep, mis_pos, mis_exact);
    return 0;
}
