// Developer micro-benchmark: the column-resident, weight-streamed MLP chain of
// stream_mlp_bench.hip with fp32 products emulated on bf16 matrix cores
// ("bf16x6"): every fp32 operand x is split into three bf16 terms
// x = x0 + x1 + x2 (round-to-nearest, each the rounding of the remainder), and
// W^T x is accumulated in fp32 from the six products w0x0 + w0x1 + w1x0 + w0x2 +
// w1x1 + w2x0 (the dropped w1x2, w2x1, w2x2 are below 2^-26 relative), each a
// v_mfma_f32_16x16x32_bf16.  The weights are pre-split into a fragment-major
// image (one 1 KiB wave load per (out tile, k block, term)); the activations
// live in LDS as three bf16 planes [term][column][feature].
//   ./split_mlp_bench [members=16] [ncols=256] [iters=20]
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x)                                                                                       \
    do {                                                                                            \
        hipError_t e = (x);                                                                         \
        if (e != hipSuccess) {                                                                      \
            std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e)); \
            std::exit(1);                                                                           \
        }                                                                                           \
    } while (0)

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __amdgpu_buffer_rsrc_t rsrc_t;

constexpr int H = 512, LAYERS = 3, NKB = H / 32, NOT = H / 16;
constexpr int RS = H + 8;  // LDS row stride (bf16): +16 B per column row against bank conflicts

__device__ __forceinline__ rsrc_t make_rsrc(const void* p, long long bytes) {
    return __builtin_amdgcn_make_buffer_rsrc((void*)p, (short)0, (int)bytes, 0x00020000);
}
__device__ __forceinline__ bf16x8 bload(rsrc_t r, int byte_off) {
    return __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(r, byte_off, 0, 0));
}
__device__ __forceinline__ float gelu_fast(float x) {
    const float y = 0.7978845608028654f * (x + 0.044715f * x * x * x);
    return x / (1.0f + __expf(-2.0f * y));
}
// x = h + m + l, each term the bf16 rounding of what the previous ones leave
__device__ __forceinline__ void split3(float x, __bf16& h, __bf16& m, __bf16& l) {
    h = (__bf16)x;
    const float r1 = x - (float)h;
    m = (__bf16)r1;
    l = (__bf16)(r1 - (float)m);
}

// CG column groups of 16 (NC = 16 CG columns per block), 8 waves, wave w owns
// output tiles 4w..4w+3 (64 features).  One slab: the epilogue overwrites the
// layer input after a barrier.  PF k-blocks of weight fragments in flight.
template <int CG, int PF, int MODE>
__global__ __launch_bounds__(512, 1) void split_chain(const bf16x8* __restrict__ Wsp, const float* __restrict__ bias,
                                                     const float* __restrict__ X, float* __restrict__ Y, int ncols) {
    constexpr int NC = 16 * CG;
    __shared__ __attribute__((aligned(16))) __bf16 slab[3][NC][RS];
    const int tiles = ncols / NC;
    const int total = gridDim.x, q = total >> 3, rr = total & 7, xcd = blockIdx.x & 7, loc = blockIdx.x >> 3;
    const int bid = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + loc;
    const int m = bid / tiles, c0 = (bid % tiles) * NC;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int li = lane & 15, lk = lane >> 4;
    for (int e = tid; e < H * NC; e += 512) {
        const int f = e / NC, j = e % NC;
        __bf16 a, b, c;
        split3(X[((long long)m * H + f) * ncols + c0 + j], a, b, c);
        slab[0][j][f] = a; slab[1][j][f] = b; slab[2][j][f] = c;
    }
    // fragment (l, ot, kb, p) of this lane: byte offset ((((l*NOT + ot)*NKB + kb)*3 + p)*64 + lane)*16
    const long long wbytes = (long long)LAYERS * NOT * NKB * 3 * 64 * 16;
    const rsrc_t rW = make_rsrc(reinterpret_cast<const char*>(Wsp) + (MODE == 2 ? 0LL : (long long)m) * wbytes, wbytes);
    auto foff = [&](int l, int t, int kb, int p) { return ((((l * NOT + 4 * w + t) * NKB + kb) * 3 + p) * 64 + lane) * 16; };
    bf16x8 ring[PF][4][3];
#pragma unroll
    for (int pf = 0; pf < PF; ++pf)
#pragma unroll
        for (int t = 0; t < 4; ++t)
#pragma unroll
            for (int p = 0; p < 3; ++p) ring[pf][t][p] = bload(rW, foff(0, t, pf, p));
    __syncthreads();
    for (int l = 0; l < LAYERS; ++l) {
        f32x4 acc[4][CG];
#pragma unroll
        for (int t = 0; t < 4; ++t)
#pragma unroll
            for (int g = 0; g < CG; ++g) acc[t][g] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int kb = 0; kb < NKB; ++kb) {
            const int slot = kb % PF;
            bf16x8 b[CG][3];
#pragma unroll
            for (int g = 0; g < CG; ++g)
#pragma unroll
                for (int p = 0; p < 3; ++p)
                    b[g][p] = *reinterpret_cast<const bf16x8*>(&slab[p][16 * g + li][32 * kb + 8 * lk]);
            // small terms first; (term, tile, group) order keeps 4 CG independent chains in flight
#pragma unroll
            for (int tm = 0; tm < 6; ++tm) {
                const int pa = tm == 0 ? 2 : tm == 1 ? 1 : tm == 2 ? 0 : tm == 3 ? 1 : tm == 4 ? 0 : 0;
                const int pb = tm == 0 ? 0 : tm == 1 ? 1 : tm == 2 ? 2 : tm == 3 ? 0 : tm == 4 ? 1 : 0;
#pragma unroll
                for (int t = 0; t < 4; ++t)
#pragma unroll
                    for (int g = 0; g < CG; ++g)
                        acc[t][g] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ring[slot][t][pa], b[g][pb], acc[t][g], 0, 0, 0);
            }
            // refill: k block kb + PF of this layer, or of the next one
            const int nk = kb + PF, nl = l + (nk >= NKB ? 1 : 0);
            if (nl < LAYERS && MODE != 1) {
#pragma unroll
                for (int t = 0; t < 4; ++t)
#pragma unroll
                    for (int p = 0; p < 3; ++p) ring[slot][t][p] = bload(rW, foff(nl, t, nk % NKB, p));
            }
        }
        __syncthreads();  // every wave has read the layer input
        // tile t, group g, reg r: feature 64 w + 16 t + 4 lk + r, column 16 g + li
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            const int f0 = 64 * w + 16 * t + 4 * lk;
            const float4 bv = *reinterpret_cast<const float4*>(bias + ((long long)m * LAYERS + l) * H + f0);
#pragma unroll
            for (int g = 0; g < CG; ++g) {
                float v[4] = {gelu_fast(acc[t][g][0] + bv.x), gelu_fast(acc[t][g][1] + bv.y),
                              gelu_fast(acc[t][g][2] + bv.z), gelu_fast(acc[t][g][3] + bv.w)};
                if (l == LAYERS - 1) {
#pragma unroll
                    for (int r = 0; r < 4; ++r) Y[((long long)m * H + f0 + r) * ncols + c0 + 16 * g + li] = v[r];
                } else {
                    bf16x4 hv, mv, lv;
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        __bf16 a, bb, c;
                        split3(v[r], a, bb, c);
                        hv[r] = a; mv[r] = bb; lv[r] = c;
                    }
                    *reinterpret_cast<bf16x4*>(&slab[0][16 * g + li][f0]) = hv;
                    *reinterpret_cast<bf16x4*>(&slab[1][16 * g + li][f0]) = mv;
                    *reinterpret_cast<bf16x4*>(&slab[2][16 * g + li][f0]) = lv;
                }
            }
        }
        __syncthreads();
    }
}

static uint16_t bf16_bits(float x) {  // round to nearest even
    uint32_t u;
    std::memcpy(&u, &x, 4);
    return (uint16_t)((u + 0x7FFFu + ((u >> 16) & 1u)) >> 16);
}
static float bf16_val(uint16_t b) {
    uint32_t u = (uint32_t)b << 16;
    float f;
    std::memcpy(&f, &u, 4);
    return f;
}

template <int CG, int PF, int MODE>
static double run(const bf16x8* dW, const float* db, const float* dX, float* dY, int members, int ncols, int iters) {
    const int blocks = members * ncols / (16 * CG);
    hipLaunchKernelGGL((split_chain<CG, PF, MODE>), dim3(blocks), dim3(512), 0, 0, dW, db, dX, dY, ncols);
    CK(hipDeviceSynchronize());
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    CK(hipEventRecord(e0));
    for (int i = 0; i < iters; ++i)
        hipLaunchKernelGGL((split_chain<CG, PF, MODE>), dim3(blocks), dim3(512), 0, 0, dW, db, dX, dY, ncols);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    return ms * 1e3 / iters;
}

int main(int argc, char** argv) {
    const int members = argc > 1 ? std::atoi(argv[1]) : 16;
    const int ncols = argc > 2 ? std::atoi(argv[2]) : 256;
    const int iters = argc > 3 ? std::atoi(argv[3]) : 20;
    std::vector<float> W((size_t)members * LAYERS * H * H), bias((size_t)members * LAYERS * H), X((size_t)members * H * ncols);
    uint64_t s = 12345;
    auto rnd = [&]() { s = s * 6364136223846793005ull + 1442695040888963407ull; return ((s >> 11) * (1.0 / 9007199254740992.0)) * 2 - 1; };
    const float lim = std::sqrt(6.0f / (2 * H));
    for (auto& v : W) v = (float)(rnd() * lim);  // W[m][l][in][out]
    for (auto& v : bias) v = (float)(rnd() * 0.1);
    for (auto& v : X) v = (float)(rnd() * 1.5);
    // fragment image: lane (li, lk) of (l, ot, kb, p) holds W^T[out = 16 ot + li][in = 32 kb + 8 lk + j], term p
    std::vector<uint16_t> Wsp((size_t)members * LAYERS * H * H * 3);
    for (int m = 0; m < members; ++m)
        for (int l = 0; l < LAYERS; ++l)
            for (int ot = 0; ot < NOT; ++ot)
                for (int kb = 0; kb < NKB; ++kb)
                    for (int lane = 0; lane < 64; ++lane)
                        for (int j = 0; j < 8; ++j) {
                            const int o = 16 * ot + (lane & 15), i = 32 * kb + 8 * (lane >> 4) + j;
                            float r = W[(((size_t)m * LAYERS + l) * H + i) * H + o];
                            for (int p = 0; p < 3; ++p) {
                                const uint16_t b = bf16_bits(r);
                                r -= bf16_val(b);
                                const size_t fr = ((((size_t)m * LAYERS + l) * NOT + ot) * NKB + kb) * 3 + p;
                                Wsp[(fr * 64 + lane) * 8 + j] = b;
                            }
                        }
    bf16x8* dW;
    float *db, *dX, *dY;
    CK(hipMalloc(&dW, Wsp.size() * 2));
    CK(hipMalloc(&db, bias.size() * 4));
    CK(hipMalloc(&dX, X.size() * 4));
    CK(hipMalloc(&dY, X.size() * 4));
    CK(hipMemcpy(dW, Wsp.data(), Wsp.size() * 2, hipMemcpyHostToDevice));
    CK(hipMemcpy(db, bias.data(), bias.size() * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(dX, X.data(), X.size() * 4, hipMemcpyHostToDevice));
    const double flops = 2.0 * members * ncols * LAYERS * (double)H * H;
    auto check = [&](const char* name) {
        std::vector<float> Yh(X.size());
        CK(hipMemcpy(Yh.data(), dY, Yh.size() * 4, hipMemcpyDeviceToHost));
        double worst = 0;
        const int m = members - 1;
        for (int c = 0; c < ncols; c += 37) {
            std::vector<double> x(H), y(H);
            for (int f = 0; f < H; ++f) x[f] = X[((size_t)m * H + f) * ncols + c];
            for (int l = 0; l < LAYERS; ++l) {
                for (int o = 0; o < H; ++o) {
                    double a = bias[((size_t)m * LAYERS + l) * H + o];
                    for (int i = 0; i < H; ++i) a += (double)W[(((size_t)m * LAYERS + l) * H + i) * H + o] * x[i];
                    const double yy = 0.7978845608028654 * (a + 0.044715 * a * a * a);
                    y[o] = 0.5 * a * (1 + std::tanh(yy));
                }
                x = y;
            }
            for (int f = 0; f < H; ++f) {
                const double d = std::fabs(Yh[((size_t)m * H + f) * ncols + c] - x[f]) / (std::fabs(x[f]) + 1e-2);
                if (d > worst) worst = d;
            }
        }
        std::printf("  %s check: worst rel err %.3e\n", name, worst);
    };
#define RUN(CG, PF, MODE)                                                                                    \
    {                                                                                                        \
        const double us = run<CG, PF, MODE>(dW, db, dX, dY, members, ncols, iters);                          \
        std::printf("CG=%d PF=%d MODE=%d NC=%d blocks=%d: %.1f us  %.1f TF/s (fp32-equivalent)\n", CG, PF, MODE, 16 * CG, \
                    members * ncols / (16 * CG), us, flops / us * 1e-6);                                     \
        check("split");                                                                                      \
    }
    RUN(1, 2, 0);
    RUN(1, 2, 1);
    RUN(1, 2, 2);
    RUN(2, 2, 0);
    RUN(2, 2, 1);
    RUN(2, 2, 2);
    return 0;
}
