// Developer micro-benchmark: a "column-resident, weight-streamed" MLP chain.
// A block owns NC=16 columns of one member for ALL H=512 features, keeps the
// activation slab x'[H][16] in LDS across layers and streams the weights
// W[k][i] straight from global memory into MFMA A fragments (16x16x4 f32),
// with a PF-deep register prefetch ring.  Measures TFLOP/s of 3 chained
// 512x512 hidden layers (gelu epilogue) for 16 members x 256 columns, and
// checks against a naive GPU reference.
//   ./stream_mlp_bench [members=16] [iters=20]
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                                       \
    do {                                                                                            \
        hipError_t e = (x);                                                                         \
        if (e != hipSuccess) {                                                                      \
            std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e)); \
            std::exit(1);                                                                           \
        }                                                                                           \
    } while (0)

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __amdgpu_buffer_rsrc_t rsrc_t;
__device__ __forceinline__ rsrc_t make_rsrc(const float* p, long long n_elems) {
    return __builtin_amdgcn_make_buffer_rsrc((void*)p, (short)0, (int)(n_elems * 4), 0x00020000);
}
__device__ __forceinline__ float4 bload4(rsrc_t r, int elem_off) {
    return __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(r, elem_off * 4, 0, 0));
}
constexpr int H = 512, NC = 16, LAYERS = 3;

__device__ __forceinline__ float gelu_f(float x) {
    const float y = 0.7978845608028654f * (x + 0.044715f * x * x * x);
    return 0.5f * x * (1.0f + tanhf(y));
}
// tanh(y) = 1 - 2 / (1 + e^{2y}) on v_exp_f32 (no libm branches)
__device__ __forceinline__ float gelu_fast(float x) {
    const float y = 0.7978845608028654f * (x + 0.044715f * x * x * x);
    const float t = 1.0f - 2.0f / (1.0f + __expf(2.0f * y));
    return 0.5f * x * (1.0f + t);
}

// W: [member][layer][k=H][i=H] ; bias [member][layer][H] ; X: [member][H][ncols] (feature-major)
// NW waves split the H output features (FW = H/NW each, TQ = FW/64 float4 W loads
// per lane per k-step); the W ring runs across layer boundaries (the refill of
// the last PF k-steps of layer l fetches the first ones of layer l+1).
template <int PF, int NW, bool ROT>
__global__ __launch_bounds__(64 * NW, 1) void mlp_stream16(const float* __restrict__ W, const float* __restrict__ bias,
                                                           const float* __restrict__ X, float* __restrict__ Y,
                                                           int ncols) {
    constexpr int NT = 64 * NW, FW = H / NW, TQ = FW / 64, NTL = 4 * TQ;
    __shared__ __attribute__((aligned(16))) float slab[2][H * NC];
    __shared__ float bs[LAYERS][H];
    const int tiles = ncols / NC;
    // XCD-aware: the 8 XCDs take blocks round-robin; give each XCD a contiguous
    // range of logical blocks so one member's column tiles share an L2
    const int total = gridDim.x, q = total >> 3, rr = total & 7, x = blockIdx.x & 7, loc = blockIdx.x >> 3;
    const int bid = (x < rr ? x * (q + 1) : rr * (q + 1) + (x - rr) * q) + loc;
    const int m = bid / tiles, c0 = (bid % tiles) * NC;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int li = lane & 15, lk = lane >> 4;
    for (int e = tid; e < H * NC; e += NT) {
        const int f = e / NC, j = e % NC;
        slab[0][e] = X[((long long)m * H + f) * ncols + c0 + j];
    }
    for (int e = tid; e < LAYERS * H; e += NT) bs[e / H][e % H] = bias[(long long)m * LAYERS * H + e];
    const rsrc_t rW = make_rsrc(W + (long long)m * LAYERS * H * H, (long long)LAYERS * H * H);
    const int lo = lk * H + FW * w + 4 * li;  // + 4 s H (+ 64 q)
    constexpr int NS = H / 4;                 // k-steps per layer
    // ROT: each column tile walks K from its own starting step, so the 16 tiles
    // of a member do not hammer the same L2 channels in lockstep
    const int s_rot = ROT ? ((bid % tiles) * (NS / tiles)) & (NS - 1) : 0;
    float4 ring[PF][TQ];
#pragma unroll
    for (int p = 0; p < PF; ++p)
#pragma unroll
        for (int t = 0; t < TQ; ++t) ring[p][t] = bload4(rW, lo + 4 * ((s_rot + p) & (NS - 1)) * H + 64 * t);
    __syncthreads();
    int cur = 0;
    for (int l = 0; l < LAYERS; ++l) {
        f32x4 acc[NTL];
#pragma unroll
        for (int t = 0; t < NTL; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
        const float* xs = slab[cur];
        const int lbase = lo + l * H * H;
        float bnext = xs[(4 * s_rot + lk) * NC + li];
        for (int s0 = 0; s0 < NS; s0 += PF) {
#pragma unroll
            for (int p = 0; p < PF; ++p) {
                const int s = s0 + p;
                const float b = bnext;
                bnext = xs[(4 * ((s_rot + s + 1) & (NS - 1)) + lk) * NC + li];  // one step ahead
                __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (int t = 0; t < TQ; ++t) {
                    const float4 a = ring[p][t];
                    acc[4 * t + 0] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.x, b, acc[4 * t + 0], 0, 0, 0);
                    acc[4 * t + 1] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.y, b, acc[4 * t + 1], 0, 0, 0);
                    acc[4 * t + 2] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.z, b, acc[4 * t + 2], 0, 0, 0);
                    acc[4 * t + 3] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.w, b, acc[4 * t + 3], 0, 0, 0);
                }
                __builtin_amdgcn_sched_barrier(0);
                {
                    const int j = s + PF;  // ring refill: k-step j of this layer or j - NS of the next
                    const int off = lbase + (j >= NS ? H * H : 0) + 4 * ((s_rot + j) & (NS - 1)) * H;
#pragma unroll
                    for (int t = 0; t < TQ; ++t) ring[p][t] = bload4(rW, off + 64 * t);
                }
                __builtin_amdgcn_sched_barrier(0);
            }
        }
        // epilogue: tile 4t + c, reg r, lane (lk, li): feature FW w + 64 t + 4 (4 lk + r) + c, column li
        float* xo = slab[cur ^ 1];
#pragma unroll
        for (int tt = 0; tt < NTL; ++tt)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int f = FW * w + 64 * (tt >> 2) + 4 * (4 * lk + r) + (tt & 3);
                xo[f * NC + li] = gelu_fast(acc[tt][r] + bs[l][f]);
            }
        __syncthreads();
        cur ^= 1;
    }
    for (int e = tid; e < H * NC; e += NT) {
        const int f = e / NC, j = e % NC;
        Y[((long long)m * H + f) * ncols + c0 + j] = slab[cur][e];
    }
}

// CG column groups of 16 per block (NC = 16 CG): one W fragment feeds CG MFMA
// sets, halving W traffic per FLOP at CG = 2.  8 waves, single slab (the
// epilogue overwrites the input after a barrier).
template <int PF, int CG, int MODE>
__global__ __launch_bounds__(512, 1) void mlp_stream_cg(const float* __restrict__ W, const float* __restrict__ bias,
                                                        const float* __restrict__ X, float* __restrict__ Y,
                                                        int ncols) {
    constexpr int NCT = 16 * CG, NT = 512;
    __shared__ __attribute__((aligned(16))) float slab[H * NCT + 64];
    const int tiles = ncols / NCT;
    const int total = gridDim.x, q = total >> 3, rr = total & 7, x = blockIdx.x & 7, loc = blockIdx.x >> 3;
    const int bid = (x < rr ? x * (q + 1) : rr * (q + 1) + (x - rr) * q) + loc;
    const int m = bid / tiles, c0 = (bid % tiles) * NCT;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int li = lane & 15, lk = lane >> 4;
    for (int e = tid; e < H * NCT; e += NT) {
        const int f = e / NCT, j = e % NCT;
        slab[e] = X[((long long)m * H + f) * ncols + c0 + j];
    }
    if (MODE == 7 && (blockIdx.x & 1)) {  // stagger: odd blocks start ~half a layer late
        for (int i = 0; i < 2; ++i) __builtin_amdgcn_s_sleep(127);
    }
    const rsrc_t rW = make_rsrc(W + (MODE == 5 ? 0LL : (long long)m) * LAYERS * H * H, (long long)LAYERS * H * H);
    const int lo = lk * H + 64 * w + 4 * li;
    constexpr int NS = H / 4;
    float4 ring[PF];
#pragma unroll
    for (int p = 0; p < PF; ++p) ring[p] = bload4(rW, lo + 4 * p * H);
    __syncthreads();
    for (int l = 0; l < LAYERS; ++l) {
        f32x4 acc[CG][4];
#pragma unroll
        for (int g = 0; g < CG; ++g)
#pragma unroll
            for (int t = 0; t < 4; ++t) acc[g][t] = f32x4{0.f, 0.f, 0.f, 0.f};
        float4 bias4[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) bias4[r] = *reinterpret_cast<const float4*>(bias + ((long long)m * LAYERS + l) * H + 64 * w + 16 * lk + 4 * r);
        const int lbase = lo + l * H * H;
        float bnext[CG];
#pragma unroll
        for (int g = 0; g < CG; ++g) bnext[g] = slab[lk * NCT + 16 * g + li];
        for (int s0 = 0; s0 < NS; s0 += PF) {
#pragma unroll
            for (int p = 0; p < PF; ++p) {
                const int s = s0 + p;
                float b[CG];
#pragma unroll
                for (int g = 0; g < CG; ++g) {
                    b[g] = bnext[g];
                    // MODE 3: no LDS reads either (MFMA issue ceiling of the structure)
                    if (MODE == 3 || MODE == 4) bnext[g] += 1e-9f;
                    else bnext[g] = slab[(4 * (s + 1) + lk) * NCT + 16 * g + li];
                }
                __builtin_amdgcn_sched_barrier(0);
                const float4 a = ring[p];
#pragma unroll
                for (int g = 0; g < CG; ++g) {
                    if (MODE == 2) { acc[g][0][0] += a.x * b[g] + a.y + a.z + a.w; continue; }
                    acc[g][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.x, b[g], acc[g][0], 0, 0, 0);
                    acc[g][1] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.y, b[g], acc[g][1], 0, 0, 0);
                    acc[g][2] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.z, b[g], acc[g][2], 0, 0, 0);
                    acc[g][3] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.w, b[g], acc[g][3], 0, 0, 0);
                }
                __builtin_amdgcn_sched_barrier(0);
                // MODE 1: no weight loads (MFMA + LDS ceiling); MODE 2: loads only
                if (MODE != 1 && MODE != 3 && MODE != 4) ring[p] = bload4(rW, lbase + 4 * (s + PF) * H);
                else ring[p].x += 1e-9f;
                __builtin_amdgcn_sched_barrier(0);
            }
        }
        if (MODE == 4) {  // no epilogue, no barriers (timing only)
            if (l == LAYERS - 1)
#pragma unroll
                for (int g = 0; g < CG; ++g) slab[(64 * w + 16 * lk) * NCT + 16 * g + li] = acc[g][0][0] + acc[g][1][1] + acc[g][2][2] + acc[g][3][3];
            continue;
        }
        __syncthreads();
#pragma unroll
        for (int g = 0; g < CG; ++g)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const float bb[4] = {bias4[r].x, bias4[r].y, bias4[r].z, bias4[r].w};
#pragma unroll
                for (int c = 0; c < 4; ++c) {
                    const int f = 64 * w + 16 * lk + 4 * r + c;
                    slab[f * NCT + 16 * g + li] = MODE == 6 ? acc[g][c][r] + bb[c] : gelu_fast(acc[g][c][r] + bb[c]);
                }
            }
        __syncthreads();
    }
    for (int e = tid; e < H * NCT; e += NT) {
        const int f = e / NCT, j = e % NCT;
        Y[((long long)m * H + f) * ncols + c0 + j] = slab[e];
    }
}

// Barrier-free variant of mlp_stream_cg<8, 1, 0>: double-buffered slab, wave w
// walks each layer's K from its own 64 rows (k-step 16 w) and waits on an LDS
// progress counter (all 8 waves published the layer input) before reading the
// others' rows.  SLEEP: s_sleep in the spin (else a plain spin).
template <int SLEEP>
__global__ __launch_bounds__(512, 1) void mlp_stream_rot(const float* __restrict__ W, const float* __restrict__ bias,
                                                         const float* __restrict__ X, float* __restrict__ Y,
                                                         int ncols) {
    constexpr int NC = 16, NT = 512, PF = 8, NS = H / 4;
    __shared__ __attribute__((aligned(16))) float slab[2][H * NC + 64];
    __shared__ int prog;
    const int tiles = ncols / NC;
    const int total = gridDim.x, q = total >> 3, rr = total & 7, x = blockIdx.x & 7, loc = blockIdx.x >> 3;
    const int bid = (x < rr ? x * (q + 1) : rr * (q + 1) + (x - rr) * q) + loc;
    const int m = bid / tiles, c0 = (bid % tiles) * NC;
    const int tid = threadIdx.x, lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int li = lane & 15, lk = lane >> 4;
    for (int e = tid; e < H * NC; e += NT) {
        const int f = e / NC, j = e % NC;
        slab[0][e] = X[((long long)m * H + f) * ncols + c0 + j];
    }
    if (tid == 0) prog = 0;
    const rsrc_t rW = make_rsrc(W + (long long)m * LAYERS * H * H, (long long)LAYERS * H * H);
    const int lo = lk * H + 64 * w + 4 * li;
    const int r0 = 16 * w;
    float4 ring[PF];
#pragma unroll
    for (int p = 0; p < PF; ++p) ring[p] = bload4(rW, lo + 4 * ((r0 + p) & (NS - 1)) * H);
    __syncthreads();
    for (int l = 0; l < LAYERS; ++l) {
        const float* xs = slab[l & 1];
        float* xo = slab[(l + 1) & 1];
        f32x4 acc[4];
#pragma unroll
        for (int t = 0; t < 4; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
        float4 bias4[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) bias4[r] = *reinterpret_cast<const float4*>(bias + ((long long)m * LAYERS + l) * H + 64 * w + 16 * lk + 4 * r);
        const int lbase = lo + l * H * H;
        float bnext = xs[(4 * r0 + lk) * NC + li];
        for (int s0 = 0; s0 < NS; s0 += PF) {
            const int nb = s0 + PF < NS ? lbase + 4 * ((r0 + s0 + PF) & (NS - 1)) * H : lbase + H * H + 4 * r0 * H;
#pragma unroll
            for (int p = 0; p < PF; ++p) {
                const int s = s0 + p;
                const float b = bnext;
                if (l > 0 && p == PF - 1 && s0 == 16 - PF) {
                    __atomic_signal_fence(__ATOMIC_SEQ_CST);
                    while (__builtin_amdgcn_readfirstlane(__hip_atomic_load(&prog, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) < 8 * l)
                        if (SLEEP) __builtin_amdgcn_s_sleep(1);
                    __atomic_signal_fence(__ATOMIC_SEQ_CST);
                }
                bnext = xs[(4 * ((r0 + s + 1) & (NS - 1)) + lk) * NC + li];
                __builtin_amdgcn_sched_barrier(0);
                const float4 a = ring[p];
                acc[0] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.x, b, acc[0], 0, 0, 0);
                acc[1] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.y, b, acc[1], 0, 0, 0);
                acc[2] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.z, b, acc[2], 0, 0, 0);
                acc[3] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.w, b, acc[3], 0, 0, 0);
                __builtin_amdgcn_sched_barrier(0);
                ring[p] = bload4(rW, nb + 4 * p * H);
                __builtin_amdgcn_sched_barrier(0);
            }
        }
        // layer 0's first k-loop read slab[0] only after the initial barrier; layer l>=1 waited above.
        // xo = slab[(l+1)&1] held layer l-1's input: every wave is past reading it (it published l-1
        // after its own k-loop l-1, and we passed the wait of this layer).
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const float bb[4] = {bias4[r].x, bias4[r].y, bias4[r].z, bias4[r].w};
#pragma unroll
            for (int c = 0; c < 4; ++c) {
                const int f = 64 * w + 16 * lk + 4 * r + c;
                xo[f * NC + li] = gelu_fast(acc[c][r] + bb[c]);
            }
        }
        __atomic_signal_fence(__ATOMIC_SEQ_CST);
        __builtin_amdgcn_s_waitcnt(0xC07F);
        if (lane == 0) __hip_atomic_fetch_add(&prog, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        __atomic_signal_fence(__ATOMIC_SEQ_CST);
    }
    __syncthreads();
    for (int e = tid; e < H * NC; e += NT) {
        const int f = e / NC, j = e % NC;
        Y[((long long)m * H + f) * ncols + c0 + j] = slab[LAYERS & 1][e];
    }
}

template <int SLEEP>
void run_rot(int nm, int iters, const float* W, const float* b, const float* X, float* Y,
             const std::vector<float>& ref, int ncols, hipStream_t s) {
    const dim3 grid(nm * (ncols / 16));
    hipLaunchKernelGGL((mlp_stream_rot<SLEEP>), grid, dim3(512), 0, s, W, b, X, Y, ncols);
    CK(hipStreamSynchronize(s));
    std::vector<float> got(ref.size());
    CK(hipMemcpy(got.data(), Y, sizeof(float) * got.size(), hipMemcpyDeviceToHost));
    double err = 0;
    for (size_t i = 0; i < got.size(); ++i) err = std::max(err, (double)std::fabs(got[i] - ref[i]));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    CK(hipEventRecord(e0, s));
    for (int i = 0; i < iters; ++i) hipLaunchKernelGGL((mlp_stream_rot<SLEEP>), grid, dim3(512), 0, s, W, b, X, Y, ncols);
    CK(hipEventRecord(e1, s));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    const double us = 1000.0 * ms / iters;
    const double fl = 2.0 * H * H * (double)ncols * nm * LAYERS;
    std::printf("stream_rot SLEEP=%d members %d cols %d: %8.2f us per 3 layers  %7.2f TFLOP/s  maxerr %.2e\n", SLEEP,
                nm, ncols, us, fl / us / 1e6, err);
}

// Transposed-access (dX) streaming: Y[k][m] = sum_i W[k][i] X[i][m] (W row-major
// [k][i], the flax kernel read along its output index i = the reduction).
// Wave w owns output rows 64w .. 64w+63 as 4 tiles of 16; a k-step covers 16
// reduction indices: lane (li, lk) loads float4 W[64w + 16t + li][16s + 4lk ..],
// component c is MFMA c's reduction index 16s + 4lk + c, B = X[16s + 4lk + c][li].
template <int PF>
__global__ __launch_bounds__(512, 1) void dx_stream(const float* __restrict__ W, const float* __restrict__ bias,
                                                    const float* __restrict__ X, float* __restrict__ Y, int ncols) {
    constexpr int NC = 16, NT = 512;
    __shared__ __attribute__((aligned(16))) float slab[H * NC + 256];
    const int tiles = ncols / NC;
    const int total = gridDim.x, q = total >> 3, rr = total & 7, x = blockIdx.x & 7, loc = blockIdx.x >> 3;
    const int bid = (x < rr ? x * (q + 1) : rr * (q + 1) + (x - rr) * q) + loc;
    const int m = bid / tiles, c0 = (bid % tiles) * NC;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int li = lane & 15, lk = lane >> 4;
    for (int e = tid; e < H * NC; e += NT) {
        const int f = e / NC, j = e % NC;
        slab[e] = X[((long long)m * H + f) * ncols + c0 + j];
    }
    const rsrc_t rW = make_rsrc(W + (long long)m * LAYERS * H * H, (long long)LAYERS * H * H);
    constexpr int NS = H / 16;
    float4 ring[PF][4];
    const int lo = (64 * w + li) * H + 4 * lk;  // + 16 t H + 16 s
#pragma unroll
    for (int p = 0; p < PF; ++p)
#pragma unroll
        for (int t = 0; t < 4; ++t) ring[p][t] = bload4(rW, lo + 16 * t * H + 16 * p);
    __syncthreads();
    for (int l = 0; l < LAYERS; ++l) {
        f32x4 acc[4];
#pragma unroll
        for (int t = 0; t < 4; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
        const int lbase = lo + l * H * H;
        float bn[4];
#pragma unroll
        for (int c = 0; c < 4; ++c) bn[c] = slab[(4 * lk + c) * NC + li];
        for (int s0 = 0; s0 < NS; s0 += PF) {
#pragma unroll
            for (int p = 0; p < PF; ++p) {
                const int s = s0 + p;
                float b[4];
#pragma unroll
                for (int c = 0; c < 4; ++c) {
                    b[c] = bn[c];
                    bn[c] = slab[(16 * (s + 1) + 4 * lk + c) * NC + li];
                }
                __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (int t = 0; t < 4; ++t) {
                    const float4 a = ring[p][t];
                    acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.x, b[0], acc[t], 0, 0, 0);
                    acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.y, b[1], acc[t], 0, 0, 0);
                    acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.z, b[2], acc[t], 0, 0, 0);
                    acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.w, b[3], acc[t], 0, 0, 0);
                }
                __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (int t = 0; t < 4; ++t) ring[p][t] = bload4(rW, lbase + 16 * t * H + 16 * (s + PF));
                __builtin_amdgcn_sched_barrier(0);
            }
        }
        __syncthreads();
        // tile t, reg r, lane (lk, li): row 64w + 16t + 4lk + r, column li
#pragma unroll
        for (int t = 0; t < 4; ++t)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int f = 64 * w + 16 * t + 4 * lk + r;
                slab[f * NC + li] = gelu_fast(acc[t][r] + bias[((long long)m * LAYERS + l) * H + f]);
            }
        __syncthreads();
    }
    for (int e = tid; e < H * NC; e += NT) {
        const int f = e / NC, j = e % NC;
        Y[((long long)m * H + f) * ncols + c0 + j] = slab[e];
    }
}

__global__ void ref_layer_t(const float* W, const float* bias, const float* X, float* Y, int ncols, int l) {
    const int m = blockIdx.z, k = blockIdx.y, j = blockIdx.x * 64 + threadIdx.x;
    if (j >= ncols) return;
    const float* Wl = W + ((long long)m * LAYERS + l) * H * H;
    float s = 0.f;
    for (int i = 0; i < H; ++i) s = fmaf(Wl[(long long)k * H + i], X[((long long)m * H + i) * ncols + j], s);
    Y[((long long)m * H + k) * ncols + j] = gelu_f(s + bias[((long long)m * LAYERS + l) * H + k]);
}

template <int PF>
void run_dx(int nm, int iters, const float* W, const float* b, const float* X, float* Y, float* T0, float* T1,
            int ncols, hipStream_t s) {
    const long long nX = (long long)nm * H * ncols;
    const float* in = X;
    float* outs[2] = {T0, T1};
    for (int l = 0; l < LAYERS; ++l) {
        hipLaunchKernelGGL(ref_layer_t, dim3(ncols / 64, H, nm), dim3(64), 0, s, W, b, in, outs[l & 1], ncols, l);
        in = outs[l & 1];
    }
    CK(hipStreamSynchronize(s));
    std::vector<float> ref(nX), got(nX);
    CK(hipMemcpy(ref.data(), in, 4 * nX, hipMemcpyDeviceToHost));
    const dim3 grid(nm * (ncols / 16));
    hipLaunchKernelGGL((dx_stream<PF>), grid, dim3(512), 0, s, W, b, X, Y, ncols);
    CK(hipStreamSynchronize(s));
    CK(hipMemcpy(got.data(), Y, 4 * nX, hipMemcpyDeviceToHost));
    double err = 0;
    for (long long i = 0; i < nX; ++i) err = std::max(err, (double)std::fabs(got[i] - ref[i]));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    CK(hipEventRecord(e0, s));
    for (int i = 0; i < iters; ++i) hipLaunchKernelGGL((dx_stream<PF>), grid, dim3(512), 0, s, W, b, X, Y, ncols);
    CK(hipEventRecord(e1, s));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    const double us = 1000.0 * ms / iters;
    const double fl = 2.0 * H * H * (double)ncols * nm * LAYERS;
    std::printf("dx_stream PF=%d members %d cols %d: %8.2f us per 3 layers  %7.2f TFLOP/s  maxerr %.2e\n", PF, nm,
                ncols, us, fl / us / 1e6, err);
}

template <int PF, int CG, int MODE>
void run_cg(int nm, int iters, const float* W, const float* b, const float* X, float* Y,
            const std::vector<float>& ref, int ncols, hipStream_t s) {
    const dim3 grid(nm * (ncols / (16 * CG)));
    hipLaunchKernelGGL((mlp_stream_cg<PF, CG, MODE>), grid, dim3(512), 0, s, W, b, X, Y, ncols);
    CK(hipStreamSynchronize(s));
    std::vector<float> got(ref.size());
    CK(hipMemcpy(got.data(), Y, sizeof(float) * got.size(), hipMemcpyDeviceToHost));
    double err = 0;
    for (size_t i = 0; i < got.size(); ++i) err = std::max(err, (double)std::fabs(got[i] - ref[i]));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    CK(hipEventRecord(e0, s));
    for (int i = 0; i < iters; ++i) hipLaunchKernelGGL((mlp_stream_cg<PF, CG, MODE>), grid, dim3(512), 0, s, W, b, X, Y, ncols);
    CK(hipEventRecord(e1, s));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    const double us = 1000.0 * ms / iters;
    const double fl = 2.0 * H * H * (double)ncols * nm * LAYERS;
    std::printf("stream_cg MODE=%d CG=%d PF=%d members %d cols %d: %8.2f us per 3 layers  %7.2f TFLOP/s  maxerr %.2e\n", MODE, CG,
                PF, nm, ncols, us, fl / us / 1e6, err);
}

__global__ void ref_layer(const float* W, const float* bias, const float* X, float* Y, int ncols, int l) {
    const int m = blockIdx.z, i = blockIdx.y, j = blockIdx.x * 64 + threadIdx.x;
    if (j >= ncols) return;
    const float* Wl = W + ((long long)m * LAYERS + l) * H * H;
    float s = 0.f;
    for (int k = 0; k < H; ++k) s = fmaf(Wl[(long long)k * H + i], X[((long long)m * H + k) * ncols + j], s);
    Y[((long long)m * H + i) * ncols + j] = gelu_f(s + bias[((long long)m * LAYERS + l) * H + i]);
}

__global__ void fill(float* p, long long n, unsigned seed, float scale) {
    const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    unsigned x = (unsigned)i * 2654435761u ^ seed;
    x ^= x >> 13; x *= 0x5bd1e995u; x ^= x >> 15;
    p[i] = ((x & 0xFFFFFF) / 16777216.0f - 0.5f) * scale;
}

template <int PF, int NW, bool ROT>
void run(int nm, int iters, const float* W, const float* b, const float* X, float* Y, const std::vector<float>& ref,
         int ncols, hipStream_t s) {
    const dim3 grid(nm * (ncols / NC));
    hipLaunchKernelGGL((mlp_stream16<PF, NW, ROT>), grid, dim3(64 * NW), 0, s, W, b, X, Y, ncols);
    CK(hipStreamSynchronize(s));
    std::vector<float> got(ref.size());
    CK(hipMemcpy(got.data(), Y, sizeof(float) * got.size(), hipMemcpyDeviceToHost));
    double err = 0;
    for (size_t i = 0; i < got.size(); ++i) err = std::max(err, (double)std::fabs(got[i] - ref[i]));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    CK(hipEventRecord(e0, s));
    for (int i = 0; i < iters; ++i) hipLaunchKernelGGL((mlp_stream16<PF, NW, ROT>), grid, dim3(64 * NW), 0, s, W, b, X, Y, ncols);
    CK(hipEventRecord(e1, s));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    const double us = 1000.0 * ms / iters;
    const double fl = 2.0 * H * H * (double)ncols * nm * LAYERS;
    std::printf("stream16 ROT=%d NW=%d PF=%d  members %d cols %d: %8.2f us per 3 layers  %7.2f TFLOP/s  maxerr %.2e\n", (int)ROT, NW, PF, nm,
                ncols, us, fl / us / 1e6, err);
}

int main(int argc, char** argv) {
    const int nm = argc > 1 ? std::atoi(argv[1]) : 16;
    const int iters = argc > 2 ? std::atoi(argv[2]) : 20;
    const int ncols = argc > 3 ? std::atoi(argv[3]) : 256;
    const long long nW = (long long)nm * LAYERS * H * H, nb = (long long)nm * LAYERS * H,
                    nX = (long long)nm * H * ncols;
    float *W, *b, *X, *Y, *T0, *T1;
    CK(hipMalloc(&W, 4 * nW));
    CK(hipMalloc(&b, 4 * nb));
    CK(hipMalloc(&X, 4 * nX));
    CK(hipMalloc(&Y, 4 * nX));
    CK(hipMalloc(&T0, 4 * nX));
    CK(hipMalloc(&T1, 4 * nX));
    hipStream_t s;
    CK(hipStreamCreate(&s));
    hipLaunchKernelGGL(fill, dim3((unsigned)((nW + 255) / 256)), dim3(256), 0, s, W, nW, 1u, 0.15f);
    hipLaunchKernelGGL(fill, dim3((unsigned)((nb + 255) / 256)), dim3(256), 0, s, b, nb, 2u, 0.2f);
    hipLaunchKernelGGL(fill, dim3((unsigned)((nX + 255) / 256)), dim3(256), 0, s, X, nX, 3u, 2.0f);
    // reference chain
    const float* in = X;
    float* outs[2] = {T0, T1};
    for (int l = 0; l < LAYERS; ++l) {
        hipLaunchKernelGGL(ref_layer, dim3(ncols / 64, H, nm), dim3(64), 0, s, W, b, in, outs[l & 1], ncols, l);
        in = outs[l & 1];
    }
    CK(hipStreamSynchronize(s));
    std::vector<float> ref(nX);
    CK(hipMemcpy(ref.data(), in, 4 * nX, hipMemcpyDeviceToHost));
    run_cg<8, 1, 0>(nm, iters, W, b, X, Y, ref, ncols, s);

    run_cg<8, 1, 6>(nm, iters, W, b, X, Y, ref, ncols, s);
    run_rot<1>(nm, iters, W, b, X, Y, ref, ncols, s);
    run_rot<0>(nm, iters, W, b, X, Y, ref, ncols, s);

    return 0;
}
