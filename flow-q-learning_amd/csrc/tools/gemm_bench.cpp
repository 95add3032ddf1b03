// Stand-alone micro-benchmark of fq::launch_gemm over the launch shapes of
// one population step (developer tool, not part of libfqlpop's C ABI).
// For each shape and tile variant: checks the result against a naive fp32
// GPU GEMM, then times `iters` back-to-back launches between HIP events.
//   ./gemm_bench [members=16] [iters=50]
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../kernels.h"

using namespace fq;

#define CK(x)                                                                               \
    do {                                                                                    \
        hipError_t e = (x);                                                                 \
        if (e != hipSuccess) {                                                              \
            std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e)); \
            std::exit(1);                                                                   \
        }                                                                                   \
    } while (0)

// naive reference: one thread per C element, same (i, j, r) indexing as fq::GemmArgs
__global__ void ref_gemm(const float* A, const float* B, float* C, int M, int N, int K, int lda, int ldb, int ldc,
                         bool arc, bool brc, long long sA, long long sB, long long sC) {
    const int z = blockIdx.z;
    const int i = blockIdx.y * 16 + threadIdx.y, j = blockIdx.x * 16 + threadIdx.x;
    if (i >= M || j >= N) return;
    A += z * sA; B += z * sB; C += z * sC;
    float s = 0.f;
    for (int r = 0; r < K; ++r) {
        const float a = arc ? A[(long long)i * lda + r] : A[(long long)r * lda + i];
        const float b = brc ? B[(long long)j * ldb + r] : B[(long long)r * ldb + j];
        s = fmaf(a, b, s);
    }
    C[(long long)i * ldc + j] = s;
}

__global__ void fill(float* p, long long n, unsigned seed) {
    const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    unsigned x = (unsigned)i * 2654435761u ^ seed;
    x ^= x >> 13; x *= 0x5bd1e995u; x ^= x >> 15;
    p[i] = ((x & 0xFFFFFF) / 16777216.0f - 0.5f);
}

// pure MFMA issue loop: registers only, random operands, NACC independent chains
template <int NACC>
__global__ __launch_bounds__(256) void mfma_peak(float* out, int iters, float seed) {
    typedef float f16v __attribute__((ext_vector_type(16)));
    f16v acc[NACC];
    for (int c = 0; c < NACC; ++c)
        for (int r = 0; r < 16; ++r) acc[c][r] = 0.f;
    float a = seed * (threadIdx.x + 1) * 1e-3f, b = seed * (blockIdx.x + 3) * 1e-3f;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int c = 0; c < NACC; ++c) acc[c] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc[c], 0, 0, 0);
        a += 1e-7f;
    }
    float s = 0.f;
    for (int c = 0; c < NACC; ++c)
        for (int r = 0; r < 16; ++r) s += acc[c][r];
    out[blockIdx.x * 256 + threadIdx.x] = s;
}

struct Shape {
    const char* name;
    int layout, M, N, K, ny;
};

int main(int argc, char** argv) {
    const int nz = argc > 1 ? std::atoi(argv[1]) : 16;
    const int iters = argc > 2 ? std::atoi(argv[2]) : 50;
    const int H = 512;
    // (i, j, r) of every GEMM family in the step (B = 256)
    const Shape shapes[] = {
        {"euler fwd  512x256x512", LAYOUT_FWD, H, 256, H, 1},
        {"bc fwd     512x512x512", LAYOUT_FWD, H, 512, H, 1},
        {"os fwd     512x768x512", LAYOUT_FWD, H, 768, H, 1},
        {"critic fwd 512x512x512 e2", LAYOUT_FWD, H, 512, H, 2},
        {"target fwd 512x256x512 e2", LAYOUT_FWD, H, 256, H, 2},
        {"first fwd  512x256x34", LAYOUT_FWD, H, 256, 34, 1},
        {"actor dX   512x256x512", LAYOUT_DX, H, 256, H, 1},
        {"critic dX  512x512x512 e2", LAYOUT_DX, H, 512, H, 2},
        {"actor dW   512x512x256", LAYOUT_DW, H, H, 256, 1},
        {"critic dW  512x512x256 e2", LAYOUT_DW, H, H, 256, 2},
        {"first dW   34x512x256", LAYOUT_DW, 34, H, 256, 1},
    };
    hipStream_t s;
    CK(hipStreamCreate(&s));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    std::vector<int> hs(nz);
    for (int i = 0; i < nz; ++i) hs[i] = i;
    int* slots;
    CK(hipMalloc(&slots, sizeof(int) * nz));
    CK(hipMemcpy(slots, hs.data(), sizeof(int) * nz, hipMemcpyHostToDevice));

    {
        float* o;
        CK(hipMalloc(&o, sizeof(float) * 256 * 4096));
        for (int wgs : {256, 512, 1024}) {
            const int it = 4000;
            hipLaunchKernelGGL(mfma_peak<2>, dim3(wgs), dim3(256), 0, s, o, it, 0.37f);
            CK(hipEventRecord(e0, s));
            hipLaunchKernelGGL(mfma_peak<2>, dim3(wgs), dim3(256), 0, s, o, it, 0.37f);
            CK(hipEventRecord(e1, s));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            const double fl = 2.0 * 32 * 32 * 2 * 2.0 * it * 4 * wgs;
            std::printf("mfma_f32_32x32x2 peak loop: %d WGs x 4 waves x 2 chains: %.1f TFLOP/s (%.2f ms)\n", wgs,
                        fl / (ms * 1e-3) / 1e12, ms);
        }
        CK(hipFree(o));
    }
    std::printf("%-28s %5s %10s %10s %9s\n", "shape", "t/var", "us", "TFLOP/s", "maxerr");
    for (const Shape& sh : shapes) {
        const bool arc = sh.layout != LAYOUT_FWD, brc = sh.layout == LAYOUT_DW;
        // operand extents: A is (i x r) or (r x i) etc; allocate generously
        const long long szA = (long long)std::max(sh.M, sh.K) * std::max(sh.M, sh.K) + 1024;
        const long long szB = (long long)std::max(sh.N, sh.K) * std::max(sh.N, sh.K) + 1024;
        const long long szC = (long long)sh.M * sh.N + 1024;
        const int lda = arc ? sh.K : sh.M, ldb = brc ? sh.K : sh.N, ldc = sh.N;
        float *A, *B, *C, *R, *bias;
        const long long nb = (long long)nz * sh.ny;
        CK(hipMalloc(&A, sizeof(float) * szA * nb));
        CK(hipMalloc(&B, sizeof(float) * szB * nb));
        CK(hipMalloc(&C, sizeof(float) * szC * nb));
        CK(hipMalloc(&R, sizeof(float) * szC * nb));
        CK(hipMalloc(&bias, sizeof(float) * 4096 * nb));
        hipLaunchKernelGGL(fill, dim3((unsigned)((szA * nb + 255) / 256)), dim3(256), 0, s, A, szA * nb, 1u);
        hipLaunchKernelGGL(fill, dim3((unsigned)((szB * nb + 255) / 256)), dim3(256), 0, s, B, szB * nb, 2u);
        CK(hipMemset(bias, 0, sizeof(float) * 4096 * nb));
        hipLaunchKernelGGL(ref_gemm, dim3((sh.N + 15) / 16, (sh.M + 15) / 16, (unsigned)nb), dim3(16, 16), 0, s, A, B,
                           R, sh.M, sh.N, sh.K, lda, ldb, ldc, arc, brc, szA, szB, szC);
        CK(hipStreamSynchronize(s));
        std::vector<float> hr((size_t)szC * nb), hc((size_t)szC * nb);
        CK(hipMemcpy(hr.data(), R, sizeof(float) * szC * nb, hipMemcpyDeviceToHost));
        const int tvs[][2] = {{0, 0}, {1, 0}, {2, 0}, {3, 0}, {0, 4}, {1, 4}, {2, 4}, {0, 5}};
        for (const auto& tv : tvs) {
            const int tile = tv[0], variant = tv[1];
            if (variant >= 4 && sh.layout != LAYOUT_FWD) continue;
            GemmArgs g{};
            g.A = tref(A, szA * sh.ny, szA);
            g.B = tref(B, szB * sh.ny, szB);
            g.C = tref(C, szC * sh.ny, szC);
            g.bias = tref(bias, 4096LL * sh.ny, 4096);
            g.M = sh.M; g.N = sh.N; g.K = sh.K; g.lda = lda; g.ldb = ldb; g.ldc = ldc;
            g.ny = sh.ny; g.nz = nz; g.slots = slots;
            const int epi = sh.layout == LAYOUT_FWD ? EPI_BIAS : EPI_STORE;
            CK(hipMemset(C, 0, sizeof(float) * szC * nb));
            launch_gemm_variant(sh.layout, epi, tile, variant, g, s);
            CK(hipStreamSynchronize(s));
            CK(hipMemcpy(hc.data(), C, sizeof(float) * szC * nb, hipMemcpyDeviceToHost));
            double maxerr = 0;
            for (long long b = 0; b < nb; ++b)
                for (int i = 0; i < sh.M; ++i)
                    for (int j = 0; j < sh.N; ++j) {
                        const long long o = b * szC + (long long)i * ldc + j;
                        maxerr = std::max(maxerr, (double)std::fabs(hc[o] - hr[o]));
                    }
            CK(hipEventRecord(e0, s));
            for (int it = 0; it < iters; ++it) launch_gemm_variant(sh.layout, epi, tile, variant, g, s);
            CK(hipEventRecord(e1, s));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            const double us = 1000.0 * ms / iters;
            const double fl = 2.0 * sh.M * sh.N * (double)sh.K * nb;
            std::printf("%-28s %3d/%d %10.2f %10.2f %9.2e\n", sh.name, tile, variant, us, fl / us / 1e6, maxerr);
        }
        CK(hipFree(A)); CK(hipFree(B)); CK(hipFree(C)); CK(hipFree(R)); CK(hipFree(bias));
    }
    return 0;
}
