// HIP / CDNA4 (gfx950) kernels of the FQL population update.
//
// One launch of every kernel covers ALL active population members
// (blockIdx -> (tile, ensemble member y, member z); z -> slot via `slots`).
// Activations are feature-major x'[feature][row]; see kernels.h.
//
// Reference semantics ([EXT] upstream fql, restated in SURVEY.md App. A and
// oracle/fql_oracle.py):
//   MLP  (fql/utils/networks.py)      -> gemm_kernel + ln_gelu_fwd_kernel + head_fwd_kernel
//   critic_loss / actor_loss (fql/agents/fql.py) -> loss_* kernels
//   jax.grad                           -> bwd_* kernels + gemm_kernel (dX, dW layouts)
//   optax.adam + target_update         -> adam_kernel ; apply_loss_fn grad stats -> finalize_kernel
//
// The production step (H = 512) runs the fused forms: stream_fwd_kernel (whole-network
// forwards), euler_flow_kernel (Euler steps 1..9 in one persistent launch),
// stream_bwd_kernel (whole dX chains), gemm_group_kernel_o4<..., EPI_ADAM> (every dW of a net
// with optax.adam / the target EMA / W^T copies / grad stats in the epilogue); the per-layer
// kernels above remain the path for other widths (engine options select either).
//
// Sections: GEMM and the fused optimiser epilogue | persistent Euler flow | column
// reductions | LayerNorm | head | streamed forward | backward | streamed backward | RNG |
// sampling | losses | optimiser | init | world-model rollout.
#include "kernels.h"

#include <hip/hip_runtime.h>
#include <math.h>

#include <type_traits>

// The explicit waits (__builtin_amdgcn_s_waitcnt with vmcnt / lgkmcnt immediates, e.g. 0x0F74)
// use the gfx9 simm16 field layout, which gfx10+ encodes differently; the v_permlane*_swap
// inline asm exists on gfx950 only.  Device code is built for gfx950 alone (Makefile ARCH).
#if defined(__HIP_DEVICE_COMPILE__) && !defined(__gfx950__)
#error "fqlpop kernels target gfx950 (MI355X) only: the s_waitcnt immediates use the gfx9 encoding"
#endif


namespace fq {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

#define DEV __device__ __forceinline__

DEV float* at(TRef t, int slot, int y = 0) {
    return t.p + (long long)slot * t.ss + (long long)y * t.sy;
}

constexpr float kSqrt2OverPi = 0.7978845608028654f;

DEV float gelu_f(float x) {
    const float y = kSqrt2OverPi * (x + 0.044715f * x * x * x);
    return 0.5f * x * (1.0f + tanhf(y));
}

DEV float gelu_grad_f(float x) {
    const float t = tanhf(kSqrt2OverPi * (x + 0.044715f * x * x * x));
    return 0.5f * (1.0f + t) +
           0.5f * x * (1.0f - t * t) * kSqrt2OverPi * (1.0f + 3.0f * 0.044715f * x * x);
}

DEV float clip1(float x) { return fminf(fmaxf(x, -1.0f), 1.0f); }

DEV float wave_sum(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}
DEV float wave_max(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
    return v;
}
DEV float wave_min(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fminf(v, __shfl_xor(v, o, 64));
    return v;
}

// the lane id (0..63) from v_mbcnt, in volatile asm: recomputed where it is used, never
// hoisted (and so never spilled) by the compiler
DEV int lane_id_asm() {
    int l;
    asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(l));
    return l;
}

// Sum over the 4 lanes l, l^16, l^32, l^48 (the lk index of the streamed kernels' lane
// layout), every lane getting the sum: v_permlane16_swap / v_permlane32_swap (VALU, no
// LDS traffic and no per-lane ds_bpermute address to keep live; __shfl_xor's addresses
// were the spilled registers of the LN backward).  The same additions as
// v += shfl_xor(v, 16); v += shfl_xor(v, 32) (fp add is commutative): bit-identical.
// Inline asm: this compiler folds the two results of __builtin_amdgcn_permlane16_swap
// into one when both inputs are the same value.  The s_nop covers the VALU-write ->
// permlane-read hazard.
DEV float lk_sum(float v) {
    float a = v, b = v;
    asm volatile("s_nop 1\n\tv_permlane16_swap_b32 %0, %1" : "+v"(a), "+v"(b));
    float s = a + b, c = s;
    asm volatile("s_nop 1\n\tv_permlane32_swap_b32 %0, %1" : "+v"(s), "+v"(c));
    return s + c;
}

// N block-wide reductions over the first 4 waves (256 threads) in ONE pair of barriers:
// each value's wave reduction (butterfly), then the 4 wave results combined left to right
// (red[0] + red[1] + red[2] + red[3]; max / min pairwise), the order of the round-5
// one-value-per-barrier-pair reductions, so the results are bit-identical to those.
// kind[i]: 0 sum, 1 max, 2 min; red: 8 N floats.  In a 512-thread block the other waves
// only join the barriers (their values are ignored), so the result is the 256-thread one.
template <int N>
DEV void block_reduce_n(float (&v)[N], const int (&kind)[N], float* red) {
#pragma unroll
    for (int i = 0; i < N; ++i) v[i] = kind[i] == 1 ? wave_max(v[i]) : kind[i] == 2 ? wave_min(v[i]) : wave_sum(v[i]);
    const int w = threadIdx.x >> 6;
    __syncthreads();
    if ((threadIdx.x & 63) == 0) {
#pragma unroll
        for (int i = 0; i < N; ++i) red[i * 8 + w] = v[i];
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < N; ++i) {
        const float* r = red + i * 8;
        v[i] = kind[i] == 1   ? fmaxf(fmaxf(r[0], r[1]), fmaxf(r[2], r[3]))
               : kind[i] == 2 ? fminf(fminf(r[0], r[1]), fminf(r[2], r[3]))
                              : r[0] + r[1] + r[2] + r[3];
    }
}

// Block-uniform values through readfirstlane (SGPRs): see gemm_body
DEV int uni(int v) { return __builtin_amdgcn_readfirstlane(v); }
DEV long long uni64(long long v) {
    const int lo = __builtin_amdgcn_readfirstlane((int)(v & 0xffffffffLL));
    const int hi = __builtin_amdgcn_readfirstlane((int)(v >> 32));
    return ((long long)hi << 32) | (unsigned int)lo;
}
template <class T>
DEV T* uniptr(T* p) {
    return reinterpret_cast<T*>(uni64(reinterpret_cast<long long>(p)));
}

// Bijective XCD-aware remap: blocks b and b+8 share an XCD under round-robin
// dispatch, so give each XCD a contiguous range of logical work ids (members'
// tiles then share that XCD's L2 for their weight panel).  Speed only.
DEV int xcd_remap(int bid, int total) {
    const int q = total >> 3, r = total & 7, x = bid & 7, loc = bid >> 3;
    return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + loc;
}

// optax.adam moments and the target EMA of one element, every rounding step explicit (fp
// contraction off, fmaf where a fused multiply-add is meant): the kernels that run the
// optimiser (adam_chunk, the fused dW epilogue, the wave-specialised launch) then give
// bit-identical results whatever the surrounding code lets the compiler fuse.
DEV void adam_moments(float g, float& m, float& v) {
#pragma clang fp contract(off)
    m = fmaf(0.1f, g, 0.9f * m);
    v = fmaf(0.001f, g * g, 0.999f * v);
}
DEV float ema_target(float p, float t, float tau) {
#pragma clang fp contract(off)
    return fmaf(tau, p, (1.0f - tau) * t);
}
// the fused epilogues' step: bias corrections by reciprocal, the step by v_sqrt + v_rcp
// (<= 2 ulp from optax's IEEE divisions)
DEV float adam_step_fast(float p, float m, float v, float rbc1, float rbc2, float lr) {
#pragma clang fp contract(off)
    const float mh = m * rbc1, vh = v * rbc2;
    return fmaf(-lr, mh * __builtin_amdgcn_rcpf(__builtin_amdgcn_sqrtf(vh) + 1e-8f), p);
}
// adam_chunk's step: IEEE divisions, as optax
DEV float adam_step_ieee(float p, float m, float v, float bc1, float bc2, float lr) {
#pragma clang fp contract(off)
    const float mh = m / bc1, vh = v / bc2;
    return fmaf(-lr, mh / (sqrtf(vh) + 1e-8f), p);
}

// optax.adam (b1 .9, b2 .999, eps 1e-8 outside the sqrt, bias correction with
// count+1) + target EMA from the pre-update critic + per-chunk grad stats, one
// chunk of one member per block (adam_kernel; and the small-leaf blocks of the fused dW
// launch).  NT-thread blocks: threads 0..255 do the work, the others only join the
// barriers (the wave-specialised launch has 512), so the results do not depend on NT.
template <int NT>
DEV void adam_chunk_t(const AdamArgs& a, int bx, int z) {
    const int ci = a.ids ? a.ids[bx] : a.chunk_base + bx;
    const int slot = a.slots[z];
    const Chunk ck = a.chunks[ci];
    const long long base = (long long)slot * a.P + a.net_off + ck.off;
    const float t = (float)(a.count[slot] + 1);
    const float bc1 = 1.0f - powf(0.9f, t), bc2 = 1.0f - powf(0.999f, t);
    float mx = -INFINITY, mn = INFINITY, ss = 0.f;
    const float lr = a.lr, tau = a.tau;
    const bool hasT = a.target != nullptr;
    if (NT == 256 || threadIdx.x < 256) {
        const float* __restrict__ Pin = a.p_in + base;
        float* __restrict__ P = a.p_out + base;
        const float* __restrict__ G = a.g + base;
        float* __restrict__ Mm = a.m + base;
        float* __restrict__ V = a.v + base;
        float* __restrict__ T = hasT ? a.target + (long long)slot * a.PT + ck.off : nullptr;
        auto one = [&](float g, float& p, float& m, float& v, float& tp) {
            adam_moments(g, m, v);
            if (hasT) tp = ema_target(p, tp, tau);
            p = adam_step_ieee(p, m, v, bc1, bc2, lr);
            mx = fmaxf(mx, g);
            mn = fminf(mn, g);
            ss = fmaf(g, g, ss);
        };
        if ((ck.len & 3) == 0) {
            for (int i = threadIdx.x * 4; i < ck.len; i += 1024) {
                const float4 g4 = *reinterpret_cast<const float4*>(G + i);
                float4 p4 = *reinterpret_cast<const float4*>(Pin + i);
                float4 m4 = *reinterpret_cast<float4*>(Mm + i);
                float4 v4 = *reinterpret_cast<float4*>(V + i);
                float4 t4 = make_float4(0.f, 0.f, 0.f, 0.f);
                if (hasT) t4 = *reinterpret_cast<float4*>(T + i);
                one(g4.x, p4.x, m4.x, v4.x, t4.x);
                one(g4.y, p4.y, m4.y, v4.y, t4.y);
                one(g4.z, p4.z, m4.z, v4.z, t4.z);
                one(g4.w, p4.w, m4.w, v4.w, t4.w);
                *reinterpret_cast<float4*>(P + i) = p4;
                *reinterpret_cast<float4*>(Mm + i) = m4;
                *reinterpret_cast<float4*>(V + i) = v4;
                if (hasT) *reinterpret_cast<float4*>(T + i) = t4;
            }
        } else {
            for (int i = threadIdx.x; i < ck.len; i += 256) {
                const float gv = G[i];
                float p = Pin[i], m = Mm[i], v = V[i], tv = hasT ? T[i] : 0.f;
                one(gv, p, m, v, tv);
                P[i] = p;
                Mm[i] = m;
                V[i] = v;
                if (hasT) T[i] = tv;
            }
        }
    }
    __shared__ float red[3 * 8];
    float st3[3] = {mx, mn, ss};
    block_reduce_n<3>(st3, {1, 2, 0}, red);
    mx = st3[0];
    mn = st3[1];
    ss = st3[2];
    if (threadIdx.x == 0) {
        float* st = a.stats + ((long long)slot * a.n_total_chunks + ci) * 3;
        st[0] = mx;
        st[1] = mn;
        st[2] = ss;
    }
}
DEV void adam_chunk(const AdamArgs& a, int bx, int z) { adam_chunk_t<256>(a, bx, z); }


// =============================================================== GEMM ======
// C[i][j] = sum_r A(i,r) B(r,j) over one (member, ensemble) pair per block
// tile.  256 threads = 4 waves in a 2x2 grid; each wave owns (BM/2)x(BN/2)
// built from 32x32 v_mfma_f32_32x32x2_f32 tiles (exact fp32 fma chain).
// K staged through LDS in BK=32 slices, register double-buffered: the global
// loads of slice k+1 are in flight while slice k feeds the MFMAs.
// LDS images: i-contiguous operands are stored [r][i] (lanes 0..31 read 32
// consecutive floats: conflict-free ds_read_b32); r-contiguous operands are
// stored [i][r] with row pitch BK+1 (bank = (i + r) mod 32: conflict-free).

// Buffer resources: a raw buffer load past `num_records` bytes returns 0, so
// the K tail of the first layer (K = 33/34) and the 33/34-row dW of the
// first layer need no per-element guard (a guarded load compiles to a
// branch + s_waitcnt vmcnt(0) per load, which serialises the pipeline).
typedef __amdgpu_buffer_rsrc_t rsrc_t;
DEV rsrc_t make_rsrc(const float* p, long long n_elems) {
    return __builtin_amdgcn_make_buffer_rsrc((void*)p, (short)0, (int)(n_elems * 4), 0x00020000);
}
DEV float4 bload4(rsrc_t r, int elem_off) {
    return __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(r, elem_off * 4, 0, 0));
}
// dword buffer load / store with a per-lane byte offset and a wave-uniform
// (SGPR) byte offset: strided per-lane accesses without 64-bit address VGPRs
DEV float bload1(rsrc_t r, int voff_b, int soff_b) {
    return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, voff_b, soff_b, 0));
}
DEV void bstore1(rsrc_t r, float v, int voff_b, int soff_b) {
    __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(int, v), r, voff_b, soff_b, 0);
}

// Block prologue of the streamed kernels: in0[e] (e < EF_K0MAX*16 + 64) = rows [0, K0) of a
// [K0][ld] input at columns c0 .. c0+15, zero below.  Unguarded buffer loads (rows >= K0
// fall past the range and read 0), all issued before the first wait: a guarded load
// compiles to a branch + vmcnt(0) each, which serialised this loop.
template <int NT>
DEV void load_in0(float* in0, const float* x, int K0, int ld, int c0) {
    constexpr int N = 64 * 16 + 64, IT = (N + NT - 1) / NT;
    static_assert(N >= 16, "");
    const rsrc_t rX = make_rsrc(x, (long long)K0 * ld);
    float v[IT];
#pragma unroll
    for (int q = 0; q < IT; ++q) {
        const int e = min((int)threadIdx.x + q * NT, N - 1), r = e >> 4, j = e & 15;
        v[q] = bload1(rX, (r * ld + c0 + j) * 4, 0);
    }
#pragma unroll
    for (int q = 0; q < IT; ++q) {
        const int e = (int)threadIdx.x + q * NT;
        if (e < N) in0[e] = v[q];
    }
}

// Global -> register staging of one operand slice.  An "IC" (i-contiguous)
// operand slice is BK rows (r) x TILE cols (i); an "RC" slice is TILE rows (i)
// x BK cols (r).  Element p of the thread's float4 list.
template <int TILE, int BK, bool RC>
DEV float4 stage_load(rsrc_t X, int ld, int p, int i0, int k0) {
    const int idx = threadIdx.x + 256 * p;
    if constexpr (RC) {
        const int row = idx / (BK / 4), c = (idx % (BK / 4)) * 4;
        return bload4(X, (i0 + row) * ld + k0 + c);
    } else {
        const int row = idx / (TILE / 4), c = (idx % (TILE / 4)) * 4;
        return bload4(X, (k0 + row) * ld + i0 + c);
    }
}

// r-contiguous LDS image pitch: BK + 1 (conflict-free ds_read_b32 fragments), or BK + 4 with
// the "k-blocked" fragment order (KB): lane half lh of a 32x32x2 MFMA reads k = 8 lh + kk
// instead of 2 kk + lh, so its 8 k-values of a 16-wide slice are contiguous (two
// ds_read_b128 instead of eight ds_read_b32) and the staging writes are float4 too; a
// pitch of 20 floats keeps 16 consecutive lanes' b128 reads on distinct banks
template <int BK, bool KB>
constexpr int rc_pitch() { return KB ? BK + 4 : BK + 1; }
template <int BM, int BN, int BK, bool ARC, bool BRC, int EPI>
constexpr bool gemm_kb() { return ARC && BRC && BK == 16 && EPI == EPI_ADAM; }

template <int TILE, int BK, bool RC, int PITCH = BK + 1>
DEV void stage_store(float* __restrict__ S, int p, float4 v) {
    const int idx = threadIdx.x + 256 * p;
    if constexpr (RC) {
        const int row = idx / (BK / 4), c = (idx % (BK / 4)) * 4;
        float* d = S + row * PITCH + c;
        if constexpr (PITCH % 4 == 0) {
            *reinterpret_cast<float4*>(d) = v;
        } else {
            d[0] = v.x; d[1] = v.y; d[2] = v.z; d[3] = v.w;
        }
    } else {
        const int row = idx / (TILE / 4), c = (idx % (TILE / 4)) * 4;
        *reinterpret_cast<float4*>(S + row * TILE + c) = v;
    }
}

template <int BM, int BN, int BK, bool ARC, bool BRC, bool KB = false>
constexpr int gemm_smem_floats() {
    constexpr int P = rc_pitch<BK, KB>();
    return 2 * ((ARC ? BM * P : BK * BM) + (BRC ? BN * P : BK * BN)) + BM;
}

// Fused optimiser epilogue of a dW tile (AdamEpi in kernels.h).  The gradient
// tile goes from the accumulators to LDS (the operand buffers are free after
// the k-loop), then the block walks it in row order with float4 accesses:
// optax.adam (b1 .9, b2 .999, eps 1e-8 outside the sqrt, bias correction with
// count+1) reading p from the current buffer and writing the other one, the
// target EMA from the pre-update p (critic), grad stats.  The new p goes back
// into the LDS tile, and a second pass writes W^T rows (float4 along i).
// float4 global access, optionally non-temporal (a streamed optimiser operand read or
// written once per step need not displace the weights the streamed kernels re-read)
typedef float f32v4 __attribute__((ext_vector_type(4)));
DEV float4 ld4(const float* p, int nt) {
    if (nt) {
        const f32v4 v = __builtin_nontemporal_load(reinterpret_cast<const f32v4*>(p));
        return float4{v.x, v.y, v.z, v.w};
    }
    return *reinterpret_cast<const float4*>(p);
}
DEV void st4(float* p, float4 v, int nt) {
    if (nt) __builtin_nontemporal_store(f32v4{v.x, v.y, v.z, v.w}, reinterpret_cast<f32v4*>(p));
    else *reinterpret_cast<float4*>(p) = v;
}

// float4 buffer load / store with a cache policy: nt = non-temporal (a streamed optimiser
// operand read and written once per step need not displace the weights the streamed
// kernels re-read from L2 / MALL)
constexpr int BUF_AUX_NT = 2;
DEV float4 bload4_aux(rsrc_t r, int off_b, int nt) {
    return __builtin_bit_cast(float4, nt ? __builtin_amdgcn_raw_buffer_load_b128(r, off_b, 0, BUF_AUX_NT)
                                         : __builtin_amdgcn_raw_buffer_load_b128(r, off_b, 0, 0));
}
DEV void bstore4_aux(rsrc_t r, float4 v, int off_b, int nt) {
    const auto w = __builtin_bit_cast(__attribute__((ext_vector_type(4))) int, v);
    if (nt) __builtin_amdgcn_raw_buffer_store_b128(w, r, off_b, 0, BUF_AUX_NT);
    else __builtin_amdgcn_raw_buffer_store_b128(w, r, off_b, 0, 0);
}

// The epilogue's first batch of p, m, v (and target) rows, issued by the k-loop's last slice
// (their loads do not depend on the gradient): their latency then runs under the last
// slice's MFMAs and the gradient tile's staging instead of after it.  Same loads, same
// registers' contents as the epilogue's own issue: bit-identical.
constexpr int ADAM_U = 2;
struct AdamPre {
    float4 p[ADAM_U], m[ADAM_U], v[ADAM_U], t[ADAM_U];
};
template <int BM, int BN>
DEV void adam_issue0(const AdamEpi& e, int gi, const GemmArgs& g, int slot, int y, int i0, int j0, AdamPre& pre) {
    constexpr int TPR = BN / 4, RPI = 256 / TPR;
    const int gM = uni(g.M), ldc = uni(g.ldc), tid = threadIdx.x;
    const long long pb = uni64((long long)slot * e.P + e.w_off[gi] + (long long)y * e.ens);
    const long long nleaf = (long long)gM * ldc;
    const rsrc_t rP = make_rsrc(e.p_in + pb, nleaf);
    const rsrc_t rM = make_rsrc(e.m + pb, nleaf), rV = make_rsrc(e.v + pb, nleaf);
    const bool hasT = e.target != nullptr;
    const rsrc_t rT = make_rsrc(uniptr(hasT ? e.target + (long long)slot * e.PT + e.w_off[gi] + (long long)y * e.ens
                                            : e.m + pb), nleaf);
    const int cj = (tid % TPR) * 4, ri = tid / TPR;
#pragma unroll
    for (int u = 0; u < ADAM_U; ++u) {
        const int off = ((i0 + u * RPI + ri) * ldc + j0 + cj) * 4;
        pre.p[u] = bload4_aux(rP, off, 0);
        pre.m[u] = bload4_aux(rM, off, 1);
        pre.v[u] = bload4_aux(rV, off, 1);
        pre.t[u] = hasT ? bload4_aux(rT, off, 1) : float4{0.f, 0.f, 0.f, 0.f};
    }
}

template <int BM, int BN, bool DUAL, bool PRE>
DEV void adam_epilogue(const AdamEpi& e, int gi, const GemmArgs& g, f32x16 (&acc)[BM / 64][BN / 64],
                       f32x16 (&acc2)[BM / 64][BN / 64], int slot, int y, int tile, int per, int i0, int j0,
                       int wi, int wj, int l32, int lh, float* smem, const AdamPre& pre) {
    constexpr int TM = BM / 64, TN = BN / 64;
    constexpr int PT = BN + 1;  // LDS row pitch (odd: the transposed read of pass 2 spreads over banks)
    // (the launching kernel sizes smem for the gradient tile: group_smem_floats)
    const int gM = uni(g.M), ldc = uni(g.ldc), tid = threadIdx.x;
    const long long pb = uni64((long long)slot * e.P + e.w_off[gi] + (long long)y * e.ens);
    // the leaf as buffer resources: rows past M (the first layer's last tile) read 0 and
    // their stores drop, so no access needs a row guard (a guarded load is a branch + a
    // vmcnt(0) wait)
    const long long nleaf = (long long)gM * ldc;
    const rsrc_t rP = make_rsrc(e.p_in + pb, nleaf), rPo = make_rsrc(e.p_out + pb, nleaf);
    const rsrc_t rM = make_rsrc(e.m + pb, nleaf), rV = make_rsrc(e.v + pb, nleaf);
    // the target arena mirrors the critic block, which sits at arena offset 0
    const bool hasT = e.target != nullptr;
    const rsrc_t rT = make_rsrc(uniptr(hasT ? e.target + (long long)slot * e.PT + e.w_off[gi] + (long long)y * e.ens
                                            : e.m + pb), nleaf);
    const float t = (float)(e.count[slot] + 1);
    const float bc1 = 1.0f - powf(0.9f, t), bc2 = 1.0f - powf(0.999f, t);
    const float rbc1 = 1.0f / bc1, rbc2 = 1.0f / bc2;
    const float lr = e.lr, tau = e.tau;
    float mx = -INFINITY, mn = INFINITY, ss = 0.f;
    const int rows = min(BM, gM - i0);
    const bool run = e.mode != 1;  // mode 1: timing probe only (no optimiser traffic)
    // pass 1: thread -> 4 consecutive columns of a row, U rows per batch, two batches in
    // flight (p, m, v, target do not depend on the gradient: batch 0 is issued before the
    // gradient tile is staged); m, v and the target stream non-temporally
    constexpr int TPR = BN / 4, RPI = 256 / TPR, U = ADAM_U, NB = BM / (RPI * U);
    static_assert(NB * RPI * U == BM && NB >= 2, "");
    const int cj = (tid % TPR) * 4, ri = tid / TPR;
    float4 p4[2][U], m4[2][U], v4[2][U], t4[2][U];
    auto issue = [&](int bi, int q) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int i = bi * RPI * U + u * RPI + ri;
            const int off = ((i0 + i) * ldc + j0 + cj) * 4;
            p4[q][u] = bload4_aux(rP, off, 0);
            m4[q][u] = bload4_aux(rM, off, 1);
            v4[q][u] = bload4_aux(rV, off, 1);
            t4[q][u] = hasT ? bload4_aux(rT, off, 1) : float4{0.f, 0.f, 0.f, 0.f};
        }
    };
    if (PRE) {  // batch 0 issued by the k-loop's last slice (adam_issue0)
#pragma unroll
        for (int u = 0; u < U; ++u) {
            p4[0][u] = pre.p[u];
            m4[0][u] = pre.m[u];
            v4[0][u] = pre.v[u];
            t4[0][u] = pre.t[u];
        }
    } else if (run) {
        issue(0, 0);
    }
    __syncthreads();  // every wave is done with the operand buffers
#pragma unroll
    for (int a = 0; a < TM; ++a)
#pragma unroll
        for (int b = 0; b < TN; ++b) {
            if constexpr (DUAL) acc[a][b] += acc2[a][b];
#pragma unroll
            for (int r = 0; r < 16; ++r)
                smem[(wi + a * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh) * PT + wj + b * 32 + l32] = acc[a][b][r];
        }
    __syncthreads();
    if (run) {
#pragma unroll
        for (int bi = 0; bi < NB; ++bi) {
            const int q = bi & 1;
            if (bi + 1 < NB) issue(bi + 1, q ^ 1);
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int i = bi * RPI * U + u * RPI + ri;
                const int off = ((i0 + i) * ldc + j0 + cj) * 4;
                const bool live = i < rows;
                float* gs = smem + i * PT + cj;
                float pp[4] = {p4[q][u].x, p4[q][u].y, p4[q][u].z, p4[q][u].w};
                float mm[4] = {m4[q][u].x, m4[q][u].y, m4[q][u].z, m4[q][u].w};
                float vv[4] = {v4[q][u].x, v4[q][u].y, v4[q][u].z, v4[q][u].w};
                float tt[4] = {t4[q][u].x, t4[q][u].y, t4[q][u].z, t4[q][u].w};
#pragma unroll
                for (int c = 0; c < 4; ++c) {
                    const float gr = gs[c];
                    // bias corrections by reciprocal and the step by v_sqrt + v_rcp: <= 2 ulp from
                    // optax's IEEE divisions, and 3 IEEE division sequences fewer per element
                    adam_moments(gr, mm[c], vv[c]);
                    tt[c] = ema_target(pp[c], tt[c], tau);
                    pp[c] = adam_step_fast(pp[c], mm[c], vv[c], rbc1, rbc2, lr);
                    gs[c] = pp[c];
                    mx = live ? fmaxf(mx, gr) : mx;
                    mn = live ? fminf(mn, gr) : mn;
                    ss = live ? fmaf(gr, gr, ss) : ss;
                }
                bstore4_aux(rPo, float4{pp[0], pp[1], pp[2], pp[3]}, off, 0);
                bstore4_aux(rM, float4{mm[0], mm[1], mm[2], mm[3]}, off, 1);
                bstore4_aux(rV, float4{vv[0], vv[1], vv[2], vv[3]}, off, 1);
                if (hasT) bstore4_aux(rT, float4{tt[0], tt[1], tt[2], tt[3]}, off, 1);
            }
        }
    }
    __shared__ float red[3 * 8];
    float st3[3] = {mx, mn, ss};
    block_reduce_n<3>(st3, {1, 2, 0}, red);  // (its barriers also publish the new p in LDS)
    mx = st3[0];
    mn = st3[1];
    ss = st3[2];
    if (tid == 0) {
        float* st = e.stats + ((long long)slot * e.n_total_chunks + e.stat_base[gi] + y * per + tile) * 3;
        st[0] = mx;
        st[1] = mn;
        st[2] = ss;
    }
    // pass 2 (hidden layers: M = H, full tiles): W^T[j][i0 .. i0+BM) as float4 runs along i
    const int nt = e.nt;
    if (e.wt_off[gi] >= 0 && e.mode != 1 && e.mode != 3) {  // mode 3: timing probe without the W^T pass
        float* __restrict__ WT = e.wt_out + (long long)slot * e.PTT + e.wt_off[gi] + (long long)y * e.wt_sy;
        constexpr int TPC = BM / 4;  // threads per W^T row segment
#pragma unroll 4
        for (int q = tid; q < BM * BN / 4; q += 256) {
            const int jj = q / TPC, ii = (q % TPC) * 4;
            const float* src = smem + ii * PT + jj;
            st4(WT + (long long)(j0 + jj) * gM + i0 + ii, float4{src[0], src[PT], src[2 * PT], src[3 * PT]}, nt & 8);
        }
    }
}

// One output tile (logical block id w of the problem g) of the register-staged GEMM.
template <int BM, int BN, int BK, bool DUAL, bool ARC, bool BRC, int EPI>
DEV void gemm_body(const GemmArgs& g, int w, float* smem, const AdamEpi* ae = nullptr, int gi = 0) {
    constexpr int WM = BM / 2, WN = BN / 2, TM = WM / 32, TN = WN / 32;
    constexpr bool KB = gemm_kb<BM, BN, BK, ARC, BRC, EPI>();
    constexpr int RP = rc_pitch<BK, KB>();
    constexpr int A_SZ = ARC ? BM * RP : BK * BM;
    constexpr int B_SZ = BRC ? BN * RP : BK * BN;
    constexpr int A_LD = BM * BK / 1024;  // float4 loads per thread
    constexpr int B_LD = BN * BK / 1024;

    // (every block-level value through readfirstlane: in the grouped launch g is ga.g[gi]
    // with a run-time gi, its fields come back in VGPRs, and buffer resources built from
    // them were re-read through waterfall loops around every operand load of the k-loop)
    const int gM = uni(g.M), gN = uni(g.N), gK = uni(g.K), lda = uni(g.lda), ldb = uni(g.ldb);
    const int tiles_m = gM / BM + (gM % BM != 0), tiles_n = gN / BN;  // host guarantees N % BN == 0
    const int per = tiles_m * tiles_n;
    const int tile = w % per, yz = w / per;
    const int gny = uni(g.ny);
    const int y = yz % gny, z = yz / gny;
    const int slot = uni(g.slots[z]);
    const int i0 = (tile / tiles_n) * BM, j0 = (tile % tiles_n) * BN;

    // valid extents (elements) of the two operands from their base
    const rsrc_t rA = make_rsrc(uniptr(at(g.A, slot, y)), ARC ? (long long)(gM - 1) * lda + gK : (long long)(gK - 1) * lda + gM);
    const rsrc_t rB = make_rsrc(uniptr(at(g.B, slot, y)), BRC ? (long long)(gN - 1) * ldb + gK : (long long)(gK - 1) * ldb + gN);

    float* As0 = smem;
    float* Bs0 = smem + A_SZ;
    float* As1 = smem + A_SZ + B_SZ;
    float* Bs1 = As1 + A_SZ;
    float* bias_s = smem + 2 * (A_SZ + B_SZ);
    if constexpr (EPI != EPI_STORE && EPI != EPI_ADAM) {
        if (threadIdx.x < BM) {
            const int i = i0 + threadIdx.x;
            bias_s[threadIdx.x] = i < gM ? at(g.bias, slot, y)[i] : 0.f;
        }
    }

    const int tid = threadIdx.x;
    const int lane = tid & 63, wave = tid >> 6;
    const int wi = (wave >> 1) * WM, wj = (wave & 1) * WN;
    const int l32 = lane & 31, lh = lane >> 5;

    // DUAL: even / odd k-pairs accumulate into separate registers (two
    // independent MFMA chains), summed once in the epilogue
    f32x16 acc[TM][TN], acc2[TM][TN];
#pragma unroll
    for (int a = 0; a < TM; ++a)
#pragma unroll
        for (int b = 0; b < TN; ++b)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                acc[a][b][r] = 0.f;
                acc2[a][b][r] = 0.f;
            }

    float4 ra[A_LD], rb[B_LD];
    const int nk = (EPI == EPI_ADAM && ae->mode == 2) ? 1 : (gK + BK - 1) / BK;  // mode 2: timing probe only
#pragma unroll
    for (int p = 0; p < A_LD; ++p) ra[p] = stage_load<BM, BK, ARC>(rA, lda, p, i0, 0);
#pragma unroll
    for (int p = 0; p < B_LD; ++p) rb[p] = stage_load<BN, BK, BRC>(rB, ldb, p, j0, 0);
#pragma unroll
    for (int p = 0; p < A_LD; ++p) stage_store<BM, BK, ARC, RP>(As0, p, ra[p]);
#pragma unroll
    for (int p = 0; p < B_LD; ++p) stage_store<BN, BK, BRC, RP>(Bs0, p, rb[p]);
    __syncthreads();
    // EPI_ADAM: the last slice is peeled; instead of the (unused) prefetch it issues the
    // optimiser epilogue's first batch (adam_issue0).  (Issued one slice earlier, behind that
    // slice's prefetch, it measured slower: 156.6 against 154.6 us serial.)
    constexpr bool PEEL = EPI == EPI_ADAM;
    AdamPre pre;
    auto slice = [&](int kt, auto last_c, auto issue_c) {
        constexpr bool LAST = decltype(last_c)::value, ISSUE = decltype(issue_c)::value;
        const float* Ac = (kt & 1) ? As1 : As0;
        const float* Bc = (kt & 1) ? Bs1 : Bs0;
        if constexpr (ISSUE) {
            if (ae->mode != 1) adam_issue0<BM, BN>(*ae, gi, g, slot, y, i0, j0, pre);
        }
        if constexpr (!LAST) {
            // prefetch the next slice (the last iteration re-reads a valid slice:
            // no branch, so the loads stay in flight across the MFMAs)
            const int kn = (kt + 1 < nk ? kt + 1 : kt) * BK;
#pragma unroll
            for (int p = 0; p < A_LD; ++p) ra[p] = stage_load<BM, BK, ARC>(rA, lda, p, i0, kn);
#pragma unroll
            for (int p = 0; p < B_LD; ++p) rb[p] = stage_load<BN, BK, BRC>(rB, ldb, p, j0, kn);
        }
        // keep the prefetch at the top of the iteration (hipcc otherwise sinks
        // it next to its ds_write and exposes the whole global latency)
        __builtin_amdgcn_sched_barrier(0);
        // all fragments of the slice first, then the MFMA chain
        float av[BK / 2][TM], bv[BK / 2][TN];
        if constexpr (KB) {
            // k-blocked: MFMA kk of lane half lh takes k = 8 lh + kk (BK = 16)
#pragma unroll
            for (int a = 0; a < TM; ++a) {
                const float* r = Ac + (wi + a * 32 + l32) * RP + 8 * lh;
                const float4 x0 = *reinterpret_cast<const float4*>(r), x1 = *reinterpret_cast<const float4*>(r + 4);
                av[0][a] = x0.x; av[1][a] = x0.y; av[2][a] = x0.z; av[3][a] = x0.w;
                av[4][a] = x1.x; av[5][a] = x1.y; av[6][a] = x1.z; av[7][a] = x1.w;
            }
#pragma unroll
            for (int b = 0; b < TN; ++b) {
                const float* r = Bc + (wj + b * 32 + l32) * RP + 8 * lh;
                const float4 x0 = *reinterpret_cast<const float4*>(r), x1 = *reinterpret_cast<const float4*>(r + 4);
                bv[0][b] = x0.x; bv[1][b] = x0.y; bv[2][b] = x0.z; bv[3][b] = x0.w;
                bv[4][b] = x1.x; bv[5][b] = x1.y; bv[6][b] = x1.z; bv[7][b] = x1.w;
            }
        } else {
#pragma unroll
            for (int kk = 0; kk < BK / 2; ++kk) {
                const int rr = 2 * kk + lh;
#pragma unroll
                for (int a = 0; a < TM; ++a)
                    av[kk][a] = ARC ? Ac[(wi + a * 32 + l32) * RP + rr] : Ac[rr * BM + wi + a * 32 + l32];
#pragma unroll
                for (int b = 0; b < TN; ++b)
                    bv[kk][b] = BRC ? Bc[(wj + b * 32 + l32) * RP + rr] : Bc[rr * BN + wj + b * 32 + l32];
            }
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int kk = 0; kk < BK / 2; ++kk)
#pragma unroll
            for (int a = 0; a < TM; ++a)
#pragma unroll
                for (int b = 0; b < TN; ++b)
                    if (DUAL && (kk & 1))
                        acc2[a][b] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[kk][a], bv[kk][b], acc2[a][b], 0, 0, 0);
                    else
                        acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[kk][a], bv[kk][b], acc[a][b], 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
        if constexpr (!LAST) {
            float* An = (kt & 1) ? As0 : As1;
            float* Bn = (kt & 1) ? Bs0 : Bs1;
#pragma unroll
            for (int p = 0; p < A_LD; ++p) stage_store<BM, BK, ARC, RP>(An, p, ra[p]);
#pragma unroll
            for (int p = 0; p < B_LD; ++p) stage_store<BN, BK, BRC, RP>(Bn, p, rb[p]);
            __syncthreads();
        }
    };
    if constexpr (PEEL) {
        for (int kt = 0; kt < nk - 1; ++kt) slice(kt, std::false_type{}, std::false_type{});
        slice(nk - 1, std::true_type{}, std::true_type{});
    } else {
        for (int kt = 0; kt < nk; ++kt) slice(kt, std::false_type{}, std::false_type{});
    }

    // epilogue: accumulator register r of a 32x32 tile holds
    // row i = (r&3) + 8*(r>>2) + 4*(lane>>5), column j = lane&31.
    if constexpr (EPI == EPI_ADAM) {
        adam_epilogue<BM, BN, DUAL, true>(*ae, gi, g, acc, acc2, slot, y, tile, per, i0, j0, wi, wj, l32, lh, smem, pre);
        return;
    }
    float* __restrict__ C = at(g.C, slot, y);
    float* __restrict__ C2 = (EPI == EPI_BIAS_GELU2) ? at(g.C2, slot, y) : nullptr;
    const int ldc = g.ldc;
    const bool full = i0 + BM <= gM;  // uniform: no row guard needed
    if constexpr (DUAL) {
#pragma unroll
        for (int a = 0; a < TM; ++a)
#pragma unroll
            for (int b = 0; b < TN; ++b) acc[a][b] += acc2[a][b];
    }
#pragma unroll
    for (int a = 0; a < TM; ++a) {
        float bsv[16];
#pragma unroll
        for (int r = 0; r < 16; ++r)
            bsv[r] = (EPI != EPI_STORE) ? bias_s[wi + a * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh] : 0.f;
#pragma unroll
        for (int b = 0; b < TN; ++b)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int i = i0 + wi + a * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
                const int j = j0 + wj + b * 32 + l32;
                if (full || i < gM) {
                    float v = acc[a][b][r];
                    const long long o = (long long)i * ldc + j;
                    if constexpr (EPI == EPI_STORE) {
                        C[o] = v;
                    } else if constexpr (EPI == EPI_BIAS) {
                        C[o] = v + bsv[r];
                    } else if constexpr (EPI == EPI_BIAS_GELU2) {
                        v += bsv[r];
                        C[o] = v;
                        C2[o] = gelu_f(v);
                    } else {
                        C[o] = gelu_f(v + bsv[r]);
                    }
                }
            }
    }
}

template <int BM, int BN, int BK, bool DUAL, bool ARC, bool BRC, int EPI>
__global__ __launch_bounds__(256, 2) void gemm_kernel(const GemmArgs g) {
    __shared__ __attribute__((aligned(16))) float smem[gemm_smem_floats<BM, BN, BK, ARC, BRC>()];
    const int tiles_m = g.M / BM + (g.M % BM != 0), tiles_n = g.N / BN;
    const int total = tiles_m * tiles_n * g.ny * g.nz;
    gemm_body<BM, BN, BK, DUAL, ARC, BRC, EPI>(g, xcd_remap(blockIdx.x, total), smem);
}

// Grouped launch of independent problems of one layout (the dW GEMMs of every
// layer of a network): block -> problem by the prefix of tile counts.
// LDS of a grouped dW launch: the operand double buffer, or the fused optimiser's
// gradient tile (BM rows of BN + 1) when that is larger (BK = 16 slices)
template <int BM, int BN, int BK, bool ARC, bool BRC, int EPI>
constexpr int group_smem_floats() {
    constexpr int G = gemm_smem_floats<BM, BN, BK, ARC, BRC, gemm_kb<BM, BN, BK, ARC, BRC, EPI>()>();
    return (EPI == EPI_ADAM && BM * (BN + 1) > G) ? BM * (BN + 1) : G;
}

template <int BM, int BN, bool ARC, bool BRC, int EPI, int BK>
DEV void gemm_group_body(const GemmGroupArgs& ga, float* smem) {
    if (EPI == EPI_ADAM && (int)blockIdx.x >= ga.first[ga.ng]) {
        // the net's small leaves: raw block ids past the tiles (the dispatcher spreads
        // consecutive ids over the XCDs, so they add no per-XCD imbalance)
        const int sb = blockIdx.x - ga.first[ga.ng], nch = ga.adam.small.n_chunks;
        adam_chunk(ga.adam.small, sb % nch, sb / nch);
        return;
    }
    const int bid = xcd_remap(blockIdx.x, ga.first[ga.ng]);
    int gi = 0;
#pragma unroll
    for (int i = 1; i < GEMM_GROUP_MAX; ++i)
        if (i < ga.ng && bid >= ga.first[i]) gi = i;
    gemm_body<BM, BN, BK, false, ARC, BRC, EPI>(ga.g[gi], bid - ga.first[gi], smem, &ga.adam, gi);
}

template <int BM, int BN, bool ARC, bool BRC, int EPI = EPI_STORE, int BK = 32>
__global__ __launch_bounds__(256, 2) void gemm_group_kernel(const GemmGroupArgs ga) {
    __shared__ __attribute__((aligned(16))) float smem[group_smem_floats<BM, BN, BK, ARC, BRC, EPI>()];
    gemm_group_body<BM, BN, ARC, BRC, EPI, BK>(ga, smem);
}

// the same at <= 128 VGPRs: 4 blocks per CU (33 KB of LDS each at 64 x 128, BK 16)
template <int BM, int BN, bool ARC, bool BRC, int EPI, int BK>
__global__ __launch_bounds__(256, 4) void gemm_group_kernel_o4(const GemmGroupArgs ga) {
    __shared__ __attribute__((aligned(16))) float smem[group_smem_floats<BM, BN, BK, ARC, BRC, EPI>()];
    gemm_group_body<BM, BN, ARC, BRC, EPI, BK>(ga, smem);
}

int gemm_group_tiles(int tile, int M, int N) {
    const int bm = (tile & 1) ? 128 : 64, bn = (tile & 2) ? 128 : 64;
    return ((M + bm - 1) / bm) * (N / bn);
}

void launch_gemm_group_dw(int tile, const GemmArgs* gs, int ng, hipStream_t s, const AdamEpi* adam) {
    GemmGroupArgs ga{};
    int tot = 0;
    for (int i = 0; i < ng; ++i) {
        ga.g[i] = gs[i];
        ga.first[i] = tot;
        tot += gemm_group_tiles(tile, gs[i].M, gs[i].N) * gs[i].ny * gs[i].nz;
    }
    ga.first[ng] = tot;
    ga.ng = ng;
    if (adam) {
        ga.adam = *adam;
        tot += adam->small_blocks;
        switch (tile == 6 || tile == 10 ? tile : tile & 3) {
            case 0: hipLaunchKernelGGL((gemm_group_kernel<64, 64, true, true, EPI_ADAM>), dim3(tot), dim3(256), 0, s, ga); break;
            case 1: hipLaunchKernelGGL((gemm_group_kernel<128, 64, true, true, EPI_ADAM>), dim3(tot), dim3(256), 0, s, ga); break;
            case 2: hipLaunchKernelGGL((gemm_group_kernel<64, 128, true, true, EPI_ADAM>), dim3(tot), dim3(256), 0, s, ga); break;
            case 6: hipLaunchKernelGGL((gemm_group_kernel<64, 128, true, true, EPI_ADAM, 16>), dim3(tot), dim3(256), 0, s, ga); break;
            case 10: hipLaunchKernelGGL((gemm_group_kernel_o4<64, 128, true, true, EPI_ADAM, 16>), dim3(tot), dim3(256), 0, s, ga); break;
            default: hipLaunchKernelGGL((gemm_group_kernel<128, 128, true, true, EPI_ADAM>), dim3(tot), dim3(256), 0, s, ga); break;
        }
        return;
    }
    switch (tile & 3) {  // (BK 16 only in the fused-optimiser launch)
        case 0: hipLaunchKernelGGL((gemm_group_kernel<64, 64, true, true>), dim3(tot), dim3(256), 0, s, ga); break;
        case 1: hipLaunchKernelGGL((gemm_group_kernel<128, 64, true, true>), dim3(tot), dim3(256), 0, s, ga); break;
        case 2: hipLaunchKernelGGL((gemm_group_kernel<64, 128, true, true>), dim3(tot), dim3(256), 0, s, ga); break;
        default: hipLaunchKernelGGL((gemm_group_kernel<128, 128, true, true>), dim3(tot), dim3(256), 0, s, ga); break;
    }
}

// ---------------------------------------------------------------------------
// Forward GEMM (both operands i-contiguous: W[k][n] and x'[k][m]) on an
// LDS-DMA ring.  `buffer_load_dwordx4 ... lds` writes a wave's 64 x 16 B
// straight into a lane-linear LDS image, so each K slice [BK][TILE] is moved
// with no VGPR staging and no ds_write; STAGES-1 slices are in flight while
// one is consumed.  Per iteration: counted vmcnt (own DMAs of slice kt
// landed) -> raw s_barrier (everyone's landed, everyone done with kt-1) ->
// DMA slice kt+STAGES-1 into the freed buffer -> fragments -> MFMAs.
// K tail (first layer, K = 33/34): the buffer range check returns zeros.
DEV constexpr int vmcnt_imm(int n) { return (n & 15) | (7 << 4) | (15 << 8) | (((n >> 4) & 3) << 14); }

template <int TILE, int BK>
DEV void dma_slice(rsrc_t r, int ld, int i0, int k0, float* lds_slice, int wave, int lane) {
    constexpr int NQ = TILE * BK / 256 / 4;  // 1 KB DMA instructions per wave per slice
#pragma unroll
    for (int t = 0; t < NQ; ++t) {
        const int q = wave * NQ + t;  // instruction index within the slice
        const int f = q * 256 + lane * 4;  // float offset of this lane's 16 B
        const int row = f / TILE, col = f % TILE;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(
            r, (__attribute__((address_space(3))) void*)(lds_slice + q * 256), 16,
            ((k0 + row) * ld + i0 + col) * 4, 0, 0, 0);
    }
}

// TAG only separates instantiations (the Euler-flow hidden layers get their own
// kernel symbol so profilers report exactly those launches).
template <int BM, int BN, int STAGES, int EPI, int TAG = 0>
__global__ __launch_bounds__(256, 2) void gemm_fwd_dma_kernel(const GemmArgs g) {
    constexpr int BK = 32;
    constexpr int WM = BM / 2, WN = BN / 2, TM = WM / 32, TN = WN / 32;
    constexpr int SA = BK * BM, SB = BK * BN, SS = SA + SB;  // floats per stage
    constexpr int NQ = (SA + SB) / 1024;                       // DMA instructions per wave per stage
    __shared__ __attribute__((aligned(16))) float smem[STAGES * SS + BM];

    const int tiles_m = g.M / BM, tiles_n = g.N / BN;  // host guarantees divisibility
    const int per = tiles_m * tiles_n;
    const int total = per * g.ny * g.nz;
    const int w = xcd_remap(blockIdx.x, total);
    const int tile = w % per, yz = w / per;
    const int y = yz % g.ny, z = yz / g.ny;
    const int slot = g.slots[z];
    const int i0 = (tile / tiles_n) * BM, j0 = (tile % tiles_n) * BN;
    const int gM = g.M, gN = g.N, gK = g.K, lda = g.lda, ldb = g.ldb;
    const rsrc_t rA = make_rsrc(at(g.A, slot, y), (long long)(gK - 1) * lda + gM);
    const rsrc_t rB = make_rsrc(at(g.B, slot, y), (long long)(gK - 1) * ldb + gN);

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wi = (wave >> 1) * WM, wj = (wave & 1) * WN;
    const int l32 = lane & 31, lh = lane >> 5;
    if constexpr (TAG == 1) {  // per-block start stamp (plain store: no contention)
        if (g.probe != nullptr && tid == 0) g.probe[2 * blockIdx.x] = __builtin_amdgcn_s_memrealtime();
    }
    float* bias_s = smem + STAGES * SS;
    if constexpr (EPI != EPI_STORE) {
        if (tid < BM) bias_s[tid] = at(g.bias, slot, y)[i0 + tid];
    }

    const int nk = (gK + BK - 1) / BK;
#pragma unroll
    for (int st = 0; st < STAGES - 1; ++st) {
        const int k0 = (st < nk ? st : nk - 1) * BK;
        dma_slice<BM, BK>(rA, lda, i0, k0, smem + st * SS, wave, lane);
        dma_slice<BN, BK>(rB, ldb, j0, k0, smem + st * SS + SA, wave, lane);
    }

    f32x16 acc[TM][TN];
#pragma unroll
    for (int a = 0; a < TM; ++a)
#pragma unroll
        for (int b = 0; b < TN; ++b)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[a][b][r] = 0.f;

    for (int kt = 0; kt < nk; ++kt) {
        __builtin_amdgcn_s_waitcnt(vmcnt_imm((STAGES - 2) * NQ));
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_sched_barrier(0);
        {
            const int kn = kt + STAGES - 1;
            const int k0 = (kn < nk ? kn : nk - 1) * BK;  // past the end: harmless re-load, keeps counts uniform
            float* dst = smem + (kn % STAGES) * SS;
            dma_slice<BM, BK>(rA, lda, i0, k0, dst, wave, lane);
            dma_slice<BN, BK>(rB, ldb, j0, k0, dst + SA, wave, lane);
        }
        __builtin_amdgcn_sched_barrier(0);
        const float* Ac = smem + (kt % STAGES) * SS;
        const float* Bc = Ac + SA;
        float av[BK / 2][TM], bv[BK / 2][TN];
#pragma unroll
        for (int kk = 0; kk < BK / 2; ++kk) {
            const int rr = 2 * kk + lh;
#pragma unroll
            for (int a = 0; a < TM; ++a) av[kk][a] = Ac[rr * BM + wi + a * 32 + l32];
#pragma unroll
            for (int b = 0; b < TN; ++b) bv[kk][b] = Bc[rr * BN + wj + b * 32 + l32];
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int kk = 0; kk < BK / 2; ++kk)
#pragma unroll
            for (int a = 0; a < TM; ++a)
#pragma unroll
                for (int b = 0; b < TN; ++b)
                    acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[kk][a], bv[kk][b], acc[a][b], 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
    }
    __builtin_amdgcn_s_waitcnt(vmcnt_imm(0));

    float* __restrict__ C = at(g.C, slot, y);
    float* __restrict__ C2 = (EPI == EPI_BIAS_GELU2) ? at(g.C2, slot, y) : nullptr;
    const int ldc = g.ldc;
#pragma unroll
    for (int a = 0; a < TM; ++a) {
        float bsv[16];
#pragma unroll
        for (int r = 0; r < 16; ++r)
            bsv[r] = (EPI != EPI_STORE) ? bias_s[wi + a * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh] : 0.f;
#pragma unroll
        for (int b = 0; b < TN; ++b)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int i = i0 + wi + a * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
                const int j = j0 + wj + b * 32 + l32;
                float v = acc[a][b][r];
                const long long o = (long long)i * ldc + j;
                if constexpr (EPI == EPI_STORE) {
                    C[o] = v;
                } else if constexpr (EPI == EPI_BIAS) {
                    C[o] = v + bsv[r];
                } else if constexpr (EPI == EPI_BIAS_GELU2) {
                    v += bsv[r];
                    C[o] = v;
                    C2[o] = gelu_f(v);
                } else {
                    C[o] = gelu_f(v + bsv[r]);
                }
            }
    }
    if constexpr (TAG == 1) {  // per-block end stamp once every wave has issued its stores
        if (g.probe != nullptr) {
            __syncthreads();
            if (tid == 0) g.probe[2 * blockIdx.x + 1] = __builtin_amdgcn_s_memrealtime();
        }
    }
}

// Register-staged kernel: K slice 32, one accumulator chain.  (BK 64 and dual
// accumulator chains were measured slower on every shape of the step:
// profiles/round1_gemm_variants.txt; the template keeps both knobs.)
template <int BM, int BN, bool ARC, bool BRC, int EPI>
static void gemm_dispatch_variant(int /*variant*/, dim3 grid, const GemmArgs& a, hipStream_t s) {
    hipLaunchKernelGGL((gemm_kernel<BM, BN, 32, false, ARC, BRC, EPI>), grid, dim3(256), 0, s, a);
}

template <int EPI>
static void gemm_fwd_dma_dispatch(int tile, int stages, const GemmArgs& a, hipStream_t s) {
    auto grid = [&](int bm, int bn) { return dim3((a.M / bm) * (a.N / bn) * a.ny * a.nz); };
#define FQ_DMA(BM, BN, ST) hipLaunchKernelGGL((gemm_fwd_dma_kernel<BM, BN, ST, EPI>), grid(BM, BN), dim3(256), 0, s, a)
    if (tile == 0) {
        if (stages == 3) FQ_DMA(64, 64, 3);
        else FQ_DMA(64, 64, 4);
    } else if (tile == 1) {
        FQ_DMA(128, 64, 3);
    } else {
        FQ_DMA(64, 128, 3);
    }
#undef FQ_DMA
}

template <bool ARC, bool BRC, int EPI>
static void gemm_dispatch_tile(int tile, int variant, const GemmArgs& a, hipStream_t s) {
    if constexpr (!ARC && !BRC) {
        // variants 4 / 5: LDS-DMA ring with 3 / 4 stages (needs M % BM == 0)
        if (variant >= 4 && a.M % ((tile & 1) ? 128 : 64) == 0) {
            gemm_fwd_dma_dispatch<EPI>(tile, variant == 4 ? 3 : 4, a, s);
            return;
        }
    }
    variant &= 3;
    auto grid = [&](int bm, int bn) { return dim3(((a.M + bm - 1) / bm) * (a.N / bn) * a.ny * a.nz); };
    switch (tile) {
        case 0: gemm_dispatch_variant<64, 64, ARC, BRC, EPI>(variant, grid(64, 64), a, s); break;
        case 1: gemm_dispatch_variant<128, 64, ARC, BRC, EPI>(variant, grid(128, 64), a, s); break;
        case 2: gemm_dispatch_variant<64, 128, ARC, BRC, EPI>(variant, grid(64, 128), a, s); break;
        default: gemm_dispatch_variant<128, 128, ARC, BRC, EPI>(variant & 2, grid(128, 128), a, s); break;
    }
}

void launch_gemm_variant(int layout, int epi, int tile, int variant, const GemmArgs& a, hipStream_t s) {
    // column tiles must divide N exactly (no column guard in the kernel)
    if ((tile & 2) && a.N % 128 != 0) tile &= ~2;
    if (layout != LAYOUT_FWD) variant &= 3;
    const int bk = (variant & 1) ? 64 : 32;
    if (layout != LAYOUT_FWD && a.K % bk != 0) variant &= ~1;  // r-contiguous slices must be whole
    if (layout == LAYOUT_FWD) {
        switch (epi) {
            case EPI_BIAS: gemm_dispatch_tile<false, false, EPI_BIAS>(tile, variant, a, s); break;
            case EPI_BIAS_GELU2: gemm_dispatch_tile<false, false, EPI_BIAS_GELU2>(tile, variant, a, s); break;
            default: gemm_dispatch_tile<false, false, EPI_BIAS_GELU>(tile, variant, a, s); break;
        }
    } else if (layout == LAYOUT_DX) {
        gemm_dispatch_tile<true, false, EPI_STORE>(tile, variant, a, s);
    } else {
        gemm_dispatch_tile<true, true, EPI_STORE>(tile, variant, a, s);
    }
}

void launch_gemm(int layout, int epi, int tile, const GemmArgs& a, hipStream_t s) {
    launch_gemm_variant(layout, epi, tile, 0, a, s);
}

void launch_gemm_euler_hidden(const GemmArgs& a, hipStream_t s) {
    const dim3 grid((a.M / 64) * (a.N / 64) * a.ny * a.nz);
    hipLaunchKernelGGL((gemm_fwd_dma_kernel<64, 64, 4, EPI_BIAS_GELU, 1>), grid, dim3(256), 0, s, a);
}

// ==================================================== persistent Euler flow ==
// compute_flow_actions ([EXT] fql/agents/fql.py; SURVEY.md App. A "Flow
// target"): x <- x + v_theta(s, x, i/S) / S for i = first..S-1, then clip.
// One block = 16 minibatch columns of one member for the WHOLE chain, so the
// activation slab x'[512][16] never leaves LDS and there is one launch per
// population step instead of 5 per Euler step.  8 waves split the 512 output
// features (64 each).  The weights stream from L2 straight into MFMA A
// fragments (v_mfma_f32_16x16x4_f32): lane (li = l&15, lk = l>>4) loads the
// float4 W[4s+lk][64w+4li .. +3], whose component c feeds accumulator tile c,
// so tile c row li is feature 64w + 4li + c (a fixed permutation the epilogue
// undoes).  An 8-deep register ring of W loads runs across layer boundaries
// (the refill of a layer's last 8 k-steps fetches the next layer's first 8);
// the B fragment (x'[4s+lk][li], LDS) is read one k-step ahead.
// Layer 0 input [s; x; t] is K0 = D+A+1 rows, zero-padded to a multiple of 32
// (the padded rows multiply finite parameter words by exact zeros).
constexpr int EF_H = 512, EF_NC = 16, EF_NW = 8, EF_PF = 8, EF_K0MAX = 64;

// GELU-tanh in sigmoid form: 0.5 x (1 + tanh(y)) = x sigmoid(2y), y = k (x +
// 0.044715 x^3), sigmoid on v_exp_f32 + v_rcp_f32 (no libm branches).  For x
// very negative exp2 overflows to +inf and rcp gives 0 (gelu -> -0); for x
// very positive exp2 underflows to 0 (gelu -> x).  5 VALU + 2 transcendental.
constexpr float kG0 = -2.0f * 0.7978845608028654f * 1.4426950408889634f;  // -2k log2(e)
constexpr float kG1 = kG0 * 0.044715f;
DEV float gelu_sig(float x, float x2) {  // sigmoid(2y)
    return __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(x * fmaf(x2, kG1, kG0)));
}
DEV float gelu_fast(float x) { return x * gelu_sig(x, x * x); }
// d/dx [x s] = s + x s (1 - s) d(2y)/dx,  d(2y)/dx = 2k (1 + 3 * 0.044715 x^2)
constexpr float kD0 = 2.0f * 0.7978845608028654f, kD1 = kD0 * 3.0f * 0.044715f;
DEV void gelu_and_grad_fast(float x, float& g, float& gp) {
    const float x2 = x * x, sg = gelu_sig(x, x2);
    g = x * sg;
    gp = fmaf(sg, x * (1.0f - sg) * fmaf(x2, kD1, kD0), sg);
}
DEV float gelu_grad_fast(float x) {
    const float x2 = x * x, sg = gelu_sig(x, x2);
    return fmaf(sg, x * (1.0f - sg) * fmaf(x2, kD1, kD0), sg);
}

// LayerNorm arithmetic with every rounding explicit (fp contraction off, fmaf where a
// fused multiply-add is meant), so that the unsplit and the split kernels, whose code around
// these sums differs, give bit-identical results.
DEV void ln_acc(float v, float& s1, float& s2) {  // column sums of x and x^2
#pragma clang fp contract(off)
    s1 = s1 + v;
    s2 = fmaf(v, v, s2);
}
DEV void ln_stats(float S1, float S2, float h, float& mean, float& rs) {  // from the feature sums
#pragma clang fp contract(off)
    mean = S1 / h;
    const float var = fmaxf(fmaf(-mean, mean, S2 / h), 0.f);
    rs = 1.0f / sqrtf(var + 1e-6f);
}
DEV float ln_apply(float v, float mean, float rs, float ga, float be) {
#pragma clang fp contract(off)
    return fmaf((v - mean) * rs, ga, be);
}
// backward: d = dh gamma (rounded), its column sums s1 += d, s2 += d xhat
DEV float ln_bwd_acc(float dh, float gm, float xh, float& s1, float& s2) {
#pragma clang fp contract(off)
    const float d = dh * gm;
    s1 = s1 + d;
    s2 = fmaf(d, xh, s2);
    return d;
}
// du = rstd (d - c1 - xhat c2) gelu'(u)
DEV float ln_bwd_du(float d, float xh, float c1, float c2, float rs, float gp) {
#pragma clang fp contract(off)
    return (rs * fmaf(-xh, c2, d - c1)) * gp;
}
// one product rounded on its own, then summed (LN scale grads: sum over columns of dh xhat)
DEV float mul_rn(float a, float b) {
#pragma clang fp contract(off)
    return a * b;
}

// One streamed layer's k-loop: acc[c] += W[k][64w + 4li + c] * xs[k][li] over
// k < 4 NS (NS a multiple of EF_PF).  ring[] holds the next EF_PF k-steps' A
// fragments on entry; on exit it holds the first EF_PF of the layer at
// w_next (element offset of the next layer's Dense kernel).
// tail >= 0 (layer 0 of the Euler flow): the last pass refills ring[0] from element
// offset tail (+ lo) instead of the next layer's first k-step; the caller consumes it
// (ef_tail) and loads the next layer's k-step 0 itself.
template <int PF = EF_PF>
DEV void ef_kloop(f32x4 (&acc)[4], float4 (&ring)[PF], rsrc_t rW, const float* xs, int NS, int w_cur,
                  int w_next, int lo, int lk, int li, int tail = -1) {
    constexpr int H = EF_H, NC = EF_NC;
    float bnext = xs[lk * NC + li];
    // do-while (NS >= PF always): with no zero-trip path the waitcnt pass can prove that
    // the loads issued before the loop (the caller's epilogue operands) are complete at
    // the exit, instead of waiting there for the next layer's ring refills too
    int s0 = 0;
    do {
        // refill targets: k-steps s0+PF.. of this layer, or the next layer's first PF
        const int rbase = (s0 + PF < NS ? w_cur + 4 * (s0 + PF) * H : w_next) + lo;
        const int r0 = (s0 + PF >= NS && tail >= 0 ? tail : rbase - lo) + lo;  // ring[0]'s refill
#pragma unroll
        for (int p = 0; p < PF; ++p) {
            const int s = s0 + p;
            const float b = bnext;
            bnext = xs[(4 * (s + 1) + lk) * NC + li];  // one k-step ahead (past the end: unused)
            __builtin_amdgcn_sched_barrier(0);
            const float4 a = ring[p];
            acc[0] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.x, b, acc[0], 0, 0, 0);
            acc[1] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.y, b, acc[1], 0, 0, 0);
            acc[2] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.z, b, acc[2], 0, 0, 0);
            acc[3] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.w, b, acc[3], 0, 0, 0);
            __builtin_amdgcn_sched_barrier(0);
            ring[p] = bload4(rW, p == 0 ? r0 : rbase + 4 * p * H);
            __builtin_amdgcn_sched_barrier(0);
        }
        s0 += PF;
    } while (s0 < NS);
}

// Layer 0's k-step PF (rows 4 PF .. 4 PF + 3) when the ring pass covered k-steps 0 .. PF-1:
// a = W[4 PF + lk][64w + 4li .. +3], loaded before the k-loop.
DEV void ef_tail(f32x4 (&acc)[4], float4 a, const float* xs, int lk, int li) {
    constexpr int NC = EF_NC;
    const float b = xs[(4 * EF_PF + lk) * NC + li];
    acc[0] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.x, b, acc[0], 0, 0, 0);
    acc[1] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.y, b, acc[1], 0, 0, 0);
    acc[2] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.z, b, acc[2], 0, 0, 0);
    acc[3] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.w, b, acc[3], 0, 0, 0);
}

bool euler_flow_supported(int H, int L, int D, int A, int B) {
    return H == EF_H && L >= 1 && L <= EF_MAX_LAYERS && D + A + 1 <= EF_K0MAX && A <= 8 && B % EF_NC == 0;
}

__global__ __launch_bounds__(EF_NW * 64, 1) void euler_flow_kernel(const EulerArgs g) {
    constexpr int H = EF_H, NC = EF_NC, NT = EF_NW * 64, PF = EF_PF;
    // LDS kept to ~69 KB so that blocks of the kernels running concurrently on
    // the other streams still fit beside this one on a CU (biases and the head
    // weights live in registers; the head reduction reuses the idle slab)
    __shared__ __attribute__((aligned(16))) float slab[2][H * NC];
    __shared__ __attribute__((aligned(16))) float in0[EF_K0MAX * NC + 64];  // + slack for the look-ahead read
    __shared__ float b5s[8];

    const int tiles = g.B / NC;
    const int total = tiles * g.nz;
    const int bid = xcd_remap(blockIdx.x, total);
    const int z = bid / tiles, c0 = (bid % tiles) * NC;
    const int slot = g.slots[z];
    const int tid = threadIdx.x, lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int li = lane & 15, lk = lane >> 4;
    if (g.probe != nullptr && tid == 0) g.probe[2 * blockIdx.x] = __builtin_amdgcn_s_memrealtime();
#ifdef FQ_PHASE_PROBE  // diagnostic build only (make PHASE=1): the disabled branch cost 0.3 % in the step
    unsigned long long* const ph = g.phase != nullptr ? g.phase + (long long)blockIdx.x * EF_PHASE_STRIDE : nullptr;
    auto stamp = [&](int i) {
        if (ph != nullptr && tid == 0) ph[i] = __builtin_amdgcn_s_memrealtime();
    };
#else
    auto stamp = [](int) {};
#endif
    stamp(0);

    const int D = g.D, A = g.A, L = g.L, B = g.B, S = g.S;
    // layer 0's k-steps: K0 <= 4 (PF + 1) runs one ring pass of PF k-steps plus one tail k-step
    // (ef_tail) instead of 2 PF, of which the padded ones multiply exact zeros
    const int K0 = D + A + 1;
#ifdef FQ_NO_EULER_TAIL  // A/B switch
    const bool tail0 = false;
#else
    const bool tail0 = K0 > 4 * PF && K0 <= 4 * (PF + 1);
#endif
    const int NS0 = tail0 ? PF : (K0 + 4 * PF - 1) / (4 * PF) * PF;
    const float* __restrict__ P = g.params + (long long)slot * g.P;
    const float* __restrict__ eu = at(g.eu, slot);
    load_in0<NT>(in0, eu, D + A, B, c0);
    if (tid < A) b5s[tid] = P[g.b_off[L] + tid];
    const rsrc_t rW = make_rsrc(P, g.P);
    // head A fragments (constant over the flow): W_L[64w + 4s + lk][li], li < A (unguarded
    // loads inside the arena, then a select)
    float w5r[16];
#pragma unroll
    for (int s = 0; s < 16; ++s) w5r[s] = bload1(rW, ((int)g.w_off[L] + (64 * w + 4 * s + lk) * A + li) * 4, 0);
#pragma unroll
    for (int s = 0; s < 16; ++s) w5r[s] = li < A ? w5r[s] : 0.f;

    const int lo = lk * H + 64 * w + 4 * li;
    float4 ring[PF];
#pragma unroll
    for (int p = 0; p < PF; ++p) ring[p] = bload4(rW, (int)g.w_off[0] + 4 * p * H + lo);
    __syncthreads();

    for (int step = g.first; step < S; ++step) {
        if (step == g.first) {  // later steps' time rows are written with the x update
            if (tid < NC) in0[(D + A) * NC + tid] = (float)((double)step / (double)S);
            __syncthreads();
        }
        for (int l = 0; l < L; ++l) {
            const int NS = l == 0 ? NS0 : H / 4;
            const float* xs = l == 0 ? in0 : slab[(l - 1) & 1];
            float* xo = slab[l & 1];
            const int nl = l + 1 < L ? l + 1 : 0;
            f32x4 acc[4];
#pragma unroll
            for (int c = 0; c < 4; ++c) acc[c] = f32x4{0.f, 0.f, 0.f, 0.f};
            // this lane's 16 bias values (features 64w + 16lk + 4r + c), in flight during the k-loop
            float4 bias4[4];
#pragma unroll
            for (int r = 0; r < 4; ++r) bias4[r] = bload4(rW, (int)g.b_off[l] + 64 * w + 16 * lk + 4 * r);
            // vmcnt(4): everything but the 4 bias loads is complete (the ring was filled a layer
            // ago); otherwise the loop head merges layer 0's late ring[0] refill (tail) into
            // its wait and every 8-k-step pass starts at vmcnt(4) instead of vmcnt(7)
            __builtin_amdgcn_s_waitcnt(0x0F74);
            // both layer offsets waited for here, with the bias loads' scalar loads: an SMEM
            // load left in flight into the k-loop made its first LDS wait lgkmcnt(0) (SMEM
            // returns out of order), exposing a B-fragment read every 8 k-steps
            const int wcur = (int)g.w_off[l], wnext = (int)g.w_off[nl];
            asm volatile("" ::"s"(wcur), "s"(wnext));
            const int pi = 1 + 4 * ((step - g.first) * (L + 1) + l);
            stamp(pi);
            const bool tl = l == 0 && tail0;
            // layer 0's tail k-step rides in ring[0] (no extra registers: this kernel's
            // throughput in the step drops by ~5 % at 107 VGPRs against 101)
            ef_kloop(acc, ring, rW, xs, NS, wcur, wnext, lo, lk, li, tl ? wcur + 4 * PF * H : -1);
            if (tl) {
                ef_tail(acc, ring[0], xs, lk, li);
                __builtin_amdgcn_sched_barrier(0);
                ring[0] = bload4(rW, wnext + lo);
            }
            stamp(pi + 1);
            // tile c, reg r, lane (lk, li): feature 64w + 4(4lk + r) + c, column li
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const float bb[4] = {bias4[r].x, bias4[r].y, bias4[r].z, bias4[r].w};
#pragma unroll
                for (int c = 0; c < 4; ++c) {
                    const int f = 64 * w + 4 * (4 * lk + r) + c;
                    xo[f * NC + li] = gelu_fast(acc[c][r] + bb[c]);
                }
            }
            stamp(pi + 2);
            __syncthreads();
            stamp(pi + 3);
        }
        // head: v[a][j] = sum_k W_L[k][a] h[k][j] + b_L[a]; wave w sums k in [64w, 64w+64)
        const int ph0 = 1 + 4 * ((step - g.first) * (L + 1) + L);
        stamp(ph0);
        float* red = slab[L & 1];  // [EF_NW][16 x NC] partial head tiles (this slab is idle now)
        {
            const float* hs = slab[(L - 1) & 1];
            f32x4 hacc = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int s = 0; s < 16; ++s) {
                const int k = 64 * w + 4 * s + lk;
                hacc = __builtin_amdgcn_mfma_f32_16x16x4f32(w5r[s], hs[k * NC + li], hacc, 0, 0, 0);
            }
#pragma unroll
            for (int r = 0; r < 4; ++r) red[w * 16 * NC + (4 * lk + r) * NC + li] = hacc[r];
        }
        __syncthreads();
        if (tid < A * NC) {
            const int a = tid / NC, j = tid % NC;
            float v = red[tid];
#pragma unroll
            for (int q = 1; q < EF_NW; ++q) v += red[q * 16 * NC + tid];
            v += b5s[a];
            float* xp = &in0[(D + a) * NC + j];
            *xp = *xp + v / g.steps_f;
        } else if (tid < (A + 1) * NC && step + 1 < S) {  // the next step's time row
            in0[(D + A) * NC + tid - A * NC] = (float)((double)(step + 1) / (double)S);
        }
        __syncthreads();
        stamp(ph0 + 3);
    }
    if (tid < A * NC) {
        const int a = tid / NC, j = tid % NC;
        at(g.aflow, slot)[(long long)a * B + c0 + j] = clip1(in0[(D + a) * NC + j]);
    }
    if (g.probe != nullptr) {
        __syncthreads();
        if (tid == 0) g.probe[2 * blockIdx.x + 1] = __builtin_amdgcn_s_memrealtime();
    }
}

void launch_euler_flow(const EulerArgs& a, hipStream_t s) {
    const dim3 grid((a.B / EF_NC) * a.nz);
    hipLaunchKernelGGL(euler_flow_kernel, grid, dim3(EF_NW * 64), 0, s, a);
}

// ================================================= column-reduction kernels ==
// Kernels that reduce over the FEATURE axis for every column (minibatch row)
// m: LayerNorm statistics, the narrow last Dense layer, the LN backward row
// statistics and the critic input gradient.  A block owns 64 columns (one per
// lane, coalesced 256 B rows) and 16 waves split the H features, KPT = H/16
// each; every thread issues its KPT loads before consuming any of them (the
// latency of one HBM round trip per block instead of KPT of them) and the 16
// partial results meet in LDS.
constexpr int CW = 16;  // waves per column block

#define FQ_KPT_DISPATCH(H, KERNEL, ...)                                      \
    switch ((H) / CW) {                                                      \
        case 4: KERNEL(4, __VA_ARGS__); break;                               \
        case 8: KERNEL(8, __VA_ARGS__); break;                               \
        case 16: KERNEL(16, __VA_ARGS__); break;                             \
        case 32: KERNEL(32, __VA_ARGS__); break;                             \
        default: KERNEL(64, __VA_ARGS__); break;                             \
    }

// ======================================================= LayerNorm fwd =====
// h'[k][m] = (gelu(u'[k][m]) - mu[m]) * rstd[m] * gamma[k] + beta[k]
// (flax LayerNorm eps 1e-6, fast variance E[g^2]-E[g]^2 clipped at 0, applied
// after GELU).  gelu(u) stays in registers between the statistics and the
// normalisation.
template <int KPT>
__global__ __launch_bounds__(1024) void ln_gelu_fwd_kernel(const LnArgs a) {
    const int ncb = a.M / 64;
    const int cb = blockIdx.x % ncb, yz = blockIdx.x / ncb;
    const int y = yz % a.ny, z = yz / a.ny;
    const int slot = a.slots[z];
    const int lane = threadIdx.x & 63;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int m = cb * 64 + lane;
    const long long ld = a.ld;
    const float* __restrict__ u = at(a.u, slot, y) + m;
    const int k0 = w * KPT;
    float g[KPT];
#pragma unroll
    for (int i = 0; i < KPT; ++i) g[i] = u[(k0 + i) * ld];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int i = 0; i < KPT; ++i) {
        g[i] = gelu_f(g[i]);
        s1 += g[i];
        s2 += g[i] * g[i];
    }
    __shared__ float red[2][CW][64];
    red[0][w][lane] = s1;
    red[1][w][lane] = s2;
    __syncthreads();
    float S1 = 0.f, S2 = 0.f;
#pragma unroll
    for (int q = 0; q < CW; ++q) {
        S1 += red[0][q][lane];
        S2 += red[1][q][lane];
    }
    const float mean = S1 / (float)a.H;
    const float var = fmaxf(S2 / (float)a.H - mean * mean, 0.f);
    const float rs = 1.0f / sqrtf(var + 1e-6f);
    float* __restrict__ h = at(a.h, slot, y) + m;
    const float* __restrict__ gam = at(a.gamma, slot, y) + k0;
    const float* __restrict__ bet = at(a.beta, slot, y) + k0;
#pragma unroll
    for (int i = 0; i < KPT; ++i) h[(k0 + i) * ld] = (g[i] - mean) * rs * gam[i] + bet[i];
    if (w == 0) {
        at(a.mu, slot, y)[m] = mean;
        at(a.rstd, slot, y)[m] = rs;
    }
}

#define FQ_LN_LAUNCH(KPT, grid, s, a) hipLaunchKernelGGL(ln_gelu_fwd_kernel<KPT>, grid, dim3(1024), 0, s, a)
void launch_ln_gelu_fwd(const LnArgs& a, hipStream_t s) {
    const dim3 grid((a.M / 64) * a.ny * a.nz);
    FQ_KPT_DISPATCH(a.H, FQ_LN_LAUNCH, grid, s, a)
}

// ============================================================ head fwd =====
// Last Dense layer (out width 1 or action_dim <= 8): weights are wave-uniform
// (scalar loads).  Modes fuse what consumes the head output:
//   HEAD_STORE    o0[j][m] = v                              (critic Q)
//   HEAD_BC_FUSED M = 2B: m <  B -> o0 = v_theta prediction (BC loss)
//                         m >= B -> Euler step 0: x1 = z_d + v/steps into o2
//                         (= Euler input rows D..D+A-1), time row D+A = t_next
//   HEAD_EULER    x += v/steps in o2 rows; last step: o0 = clip(x) (a_flow)
//   HEAD_OS       M = 3B: [0,B) a' = clip(v) -> o1 (target-critic input rows)
//                 [B,2B) a_pi = v -> o0, clip(a_pi) -> o2 cols B.. (critic input)
//                 [2B,3B) clip(v) -> o3 (mse metric actions)
//   HEAD_ACT      o0 = clip(v)                              (sample_actions)
template <int MODE>
DEV void head_write(const HeadArgs& a, int slot, int y, int j, int m, float v) {
    const int B = a.B, D = a.D;
    if constexpr (MODE == HEAD_STORE) {
        at(a.o0, slot, y)[(long long)j * a.ld0 + m] = v;
    } else if constexpr (MODE == HEAD_ACT) {
        at(a.o0, slot, y)[(long long)j * a.ld0 + m] = clip1(v);
    } else if constexpr (MODE == HEAD_BC_FUSED) {
        if (m < B) {
            at(a.o0, slot)[(long long)j * a.ld0 + m] = v;
        } else {
            const int mm = m - B;
            const float x = at(a.o1, slot)[(long long)(D + j) * a.ld1 + m];
            float* eu = at(a.o2, slot);
            eu[(long long)(D + j) * a.ld2 + mm] = x + v / a.steps_f;
            if (j == 0) eu[(long long)(D + a.nout) * a.ld2 + mm] = a.t_next;
        }
    } else if constexpr (MODE == HEAD_EULER) {
        float* eu = at(a.o2, slot);
        const long long o = (long long)(D + j) * a.ld2 + m;
        const float xn = eu[o] + v / a.steps_f;
        if (a.last) {
            at(a.o0, slot)[(long long)j * a.ld0 + m] = clip1(xn);
        } else {
            eu[o] = xn;
            if (j == 0) eu[(long long)(D + a.nout) * a.ld2 + m] = a.t_next;
        }
    } else if constexpr (MODE == HEAD_OS) {
        if (m < B) {
            at(a.o1, slot)[(long long)(D + j) * a.ld1 + m] = clip1(v);
        } else if (m < 2 * B) {
            const int mm = m - B;
            at(a.o0, slot)[(long long)j * a.ld0 + mm] = v;
            at(a.o2, slot)[(long long)(D + j) * a.ld2 + B + mm] = clip1(v);
        } else {
            at(a.o3, slot)[(long long)j * a.ld3 + (m - 2 * B)] = clip1(v);
        }
    }
}

template <int MODE, int KPT>
__global__ __launch_bounds__(1024) void head_fwd_kernel(const HeadArgs a) {
    const int ncb = a.M / 64;
    const int cb = blockIdx.x % ncb, yz = blockIdx.x / ncb;
    const int y = yz % a.ny, z = yz / a.ny;
    const int slot = a.slots[z];
    const int lane = threadIdx.x & 63;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int m = cb * 64 + lane;
    const long long ld = a.ld;
    const int nout = a.nout;
    const int k0 = w * KPT;
    const float* __restrict__ h = at(a.h, slot, y) + m;
    const float* __restrict__ W = at(a.W, slot, y) + (long long)k0 * nout;
    float hv[KPT];
#pragma unroll
    for (int i = 0; i < KPT; ++i) hv[i] = h[(k0 + i) * ld];
    float acc[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] = 0.f;
#pragma unroll
    for (int i = 0; i < KPT; ++i)
#pragma unroll
        for (int j = 0; j < 8; ++j)
            if (j < nout) acc[j] += W[i * nout + j] * hv[i];
    __shared__ float red[CW][8][64];
#pragma unroll
    for (int j = 0; j < 8; ++j) red[w][j][lane] = acc[j];
    __syncthreads();
    const int t = threadIdx.x;
    if (t < nout * 64) {
        const int j = t >> 6, l2 = t & 63;
        float v = 0.f;
#pragma unroll
        for (int q = 0; q < CW; ++q) v += red[q][j][l2];
        v += at(a.b, slot, y)[j];
        head_write<MODE>(a, slot, y, j, cb * 64 + l2, v);
    }
}

#define FQ_HEAD_LAUNCH(KPT, MODE, grid, s, a) \
    hipLaunchKernelGGL((head_fwd_kernel<MODE, KPT>), grid, dim3(1024), 0, s, a)
void launch_head_fwd(int mode, const HeadArgs& a, hipStream_t s) {
    const dim3 grid((a.M / 64) * a.ny * a.nz);
    switch (mode) {
        case HEAD_STORE: FQ_KPT_DISPATCH(a.H, FQ_HEAD_LAUNCH, HEAD_STORE, grid, s, a) break;
        case HEAD_BC_FUSED: FQ_KPT_DISPATCH(a.H, FQ_HEAD_LAUNCH, HEAD_BC_FUSED, grid, s, a) break;
        case HEAD_EULER: FQ_KPT_DISPATCH(a.H, FQ_HEAD_LAUNCH, HEAD_EULER, grid, s, a) break;
        case HEAD_OS: FQ_KPT_DISPATCH(a.H, FQ_HEAD_LAUNCH, HEAD_OS, grid, s, a) break;
        default: FQ_KPT_DISPATCH(a.H, FQ_HEAD_LAUNCH, HEAD_ACT, grid, s, a) break;
    }
}

// ===================================================== streamed MLP forward ==
// The whole forward pass of one network in one launch (StreamArgs, kernels.h):
// block = 16 columns x all 512 features of one (member, ensemble member); the
// same weight-streaming k-loop as the Euler flow.  One LDS slab holds the
// layer input; after a barrier (every wave done reading it) the epilogue
// overwrites it with the layer output, so LDS stays ~38 KB and blocks of other
// kernels fit beside this one.  Epilogue per hidden layer: u = acc + b
// (stored if requested), g = gelu(u), LayerNorm over the 512 features of each
// column when LN (statistics: lane partials -> shuffles over lk -> LDS over
// the 8 waves), layer output stored if requested and written to the slab.
// The head (nout <= 8) is a 16x16x4 MFMA per wave over its 64 features,
// reduced over waves in LDS, and handed to head_write<MODE>.
bool stream_fwd_supported(int H, int L, int K0, int nout, int M) {
    return H == EF_H && L >= 1 && L <= EF_MAX_LAYERS && K0 <= EF_K0MAX && nout <= 8 && M % EF_NC == 0;
}

template <int MODE, bool LN>
__global__ __launch_bounds__(EF_NW * 64, 1) void stream_fwd_kernel(const StreamArgs g) {
    constexpr int H = EF_H, NC = EF_NC, NT = EF_NW * 64, PF = EF_PF;
    __shared__ __attribute__((aligned(16))) float slab[H * NC + 64];          // + slack for the look-ahead read
    __shared__ __attribute__((aligned(16))) float in0[EF_K0MAX * NC + 64];   // layer-0 input, then head partials
    __shared__ float lnred[2][EF_NW][NC];
    __shared__ float lnp[3][H];  // this layer's bias, LN scale, LN bias

    const int tiles = g.M / NC;
    const int total = tiles * g.ny * g.nz;
    const int bid = xcd_remap(blockIdx.x, total);
    const int tile = bid % tiles, yz = bid / tiles;
    const int y = yz % g.ny, z = yz / g.ny;
    const int slot = g.slots[z];
    const int c0 = tile * NC;
    const int tid = threadIdx.x, lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int li = lane & 15, lk = lane >> 4;
    const int L = g.L, K0 = g.K0, nout = g.head.nout;
    const bool tail0 = K0 > 4 * PF && K0 <= 4 * (PF + 1);  // layer 0 as in euler_flow_kernel
    const int NS0 = tail0 ? PF : (K0 + 4 * PF - 1) / (4 * PF) * PF;
    const float* __restrict__ P = g.params + (long long)slot * g.P + (long long)y * g.ens;
    const float* __restrict__ x0 = g.x0 + (long long)slot * g.x0_ss;
    load_in0<NT>(in0, x0, K0, g.ld_x, c0);
    const rsrc_t rW = make_rsrc(P, g.P);
    const int lo = lk * H + 64 * w + 4 * li;
    float4 ring[PF];
#pragma unroll
    for (int p = 0; p < PF; ++p) ring[p] = bload4(rW, (int)g.w_off[0] + 4 * p * H + lo);
    const bool st = c0 >= g.st_lo && c0 + NC <= g.st_hi;  // block stores activations
    const int m = c0 + li;
    if constexpr (LN) {
        // LN variant: layer l's bias / LN scale / LN bias are staged one layer ahead (see below)
        lnp[0][tid] = P[g.b_off[0] + tid];
        lnp[1][tid] = P[g.g_off[0] + tid];
        lnp[2][tid] = P[g.be_off[0] + tid];
    }
    __syncthreads();

    for (int l = 0; l < L; ++l) {
        const int NS = l == 0 ? NS0 : H / 4;
        const float* xs = l == 0 ? in0 : slab;
        const int nl = l + 1 < L ? l + 1 : 0;
        f32x4 acc[4];
#pragma unroll
        for (int c = 0; c < 4; ++c) acc[c] = f32x4{0.f, 0.f, 0.f, 0.f};
        // feature tid's bias (LN: and LN scale / bias) in flight during the k-loop, then to LDS.
        // LN: those of the NEXT layer, written after this layer's barriers that retire the
        // current ones (bias after the stats barrier, scale / bias after the slab barrier), so
        // that no barrier is needed between the k-loop and the epilogue: the stats barrier
        // already orders every wave's slab reads before the slab writes
        const int lp = LN ? nl : l;
        const float pb = P[g.b_off[lp] + tid];
        const float pg = LN ? P[g.g_off[lp] + tid] : 0.f;
        const float pe = LN ? P[g.be_off[lp] + tid] : 0.f;
        const int wcur = (int)g.w_off[l], wnext = (int)g.w_off[nl];
        asm volatile("" ::"s"(wcur), "s"(wnext));  // no SMEM load in flight into the k-loop (see euler_flow_kernel)
        const float4 at0 = bload4(rW, wcur + 4 * PF * H + lo);  // layer 0's tail k-step (l > 0: unused)
        ef_kloop(acc, ring, rW, xs, NS, wcur, wnext, lo, lk, li);
        if (l == 0 && tail0) ef_tail(acc, at0, xs, lk, li);
        if constexpr (!LN) {
            lnp[0][tid] = pb;
            __syncthreads();  // every wave is done reading the slab; lnp visible
        }

        // activation stores: buffer ops, per-lane offset + wave-uniform row offset (no 64-bit address VGPRs)
        const bool stU = st && g.U[l], stG = st && g.G[l] && c0 + NC <= g.g_hi;
        const long long sbase = (long long)slot * g.s_ss + (long long)y * g.s_sy + c0;
        const rsrc_t rU = make_rsrc(stU ? g.U[l] + sbase : g.params, stU ? (long long)H * g.ld_s : 0);
        const rsrc_t rG = make_rsrc(stG ? g.G[l] + sbase : g.params, stG ? (long long)H * g.ld_s : 0);
        const int svo = ((64 * w + 16 * lk) * g.ld_s + li) * 4;
        float v[4][4];  // [r][c]: feature 64w + 16lk + 4r + c, column li
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const float4 bb = *reinterpret_cast<const float4*>(&lnp[0][64 * w + 16 * lk + 4 * r]);
            const float bv[4] = {bb.x, bb.y, bb.z, bb.w};
#pragma unroll
            for (int c = 0; c < 4; ++c) {
                const float u = acc[c][r] + bv[c];
                if (stU) bstore1(rU, u, svo, (4 * r + c) * g.ld_s * 4);
                v[r][c] = gelu_fast(u);
            }
        }
        if constexpr (LN) {
            float s1 = 0.f, s2 = 0.f;
#pragma unroll
            for (int r = 0; r < 4; ++r)
#pragma unroll
                for (int c = 0; c < 4; ++c) ln_acc(v[r][c], s1, s2);
            s1 = lk_sum(s1);
            s2 = lk_sum(s2);
            if (lk == 0) {
                lnred[0][w][li] = s1;
                lnred[1][w][li] = s2;
            }
            __syncthreads();  // lnred visible; every wave is done reading the slab and lnp[0]
            lnp[0][tid] = pb;  // next layer's bias (visible after the slab barrier)
            float S1 = 0.f, S2 = 0.f;
#pragma unroll
            for (int q = 0; q < EF_NW; ++q) {
                S1 += lnred[0][q][li];
                S2 += lnred[1][q][li];
            }
            float mean, rs;
            ln_stats(S1, S2, (float)H, mean, rs);
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const float4 g4 = *reinterpret_cast<const float4*>(&lnp[1][64 * w + 16 * lk + 4 * r]);
                const float4 b4 = *reinterpret_cast<const float4*>(&lnp[2][64 * w + 16 * lk + 4 * r]);
                const float ga[4] = {g4.x, g4.y, g4.z, g4.w};
                const float be[4] = {b4.x, b4.y, b4.z, b4.w};
#pragma unroll
                for (int c = 0; c < 4; ++c) v[r][c] = ln_apply(v[r][c], mean, rs, ga[c], be[c]);
            }
            if (st && w == 0 && lk == 0 && g.MU[l]) {
                const long long so = (long long)slot * g.st_ss + (long long)y * g.st_sy + m;
                g.MU[l][so] = mean;
                g.RS[l][so] = rs;
            }
        }
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
            for (int c = 0; c < 4; ++c) {
                const int f = 64 * w + 16 * lk + 4 * r + c;
                if (stG) bstore1(rG, v[r][c], svo, (4 * r + c) * g.ld_s * 4);
                slab[f * NC + li] = v[r][c];
            }
        __syncthreads();
        if constexpr (LN) {
            lnp[1][tid] = pg;  // next layer's LN scale / bias (visible after its stats barrier)
            lnp[2][tid] = pe;
        }
    }
    // head: out[j][col] = sum_k W_L[k][j] h[k][col] + b_L[j]
    {
        float w5r[16];  // A fragments: W_L[64w + 4s + lk][li], li < nout
#pragma unroll
        for (int s = 0; s < 16; ++s) w5r[s] = bload1(rW, ((int)g.w_off[L] + (64 * w + 4 * s + lk) * nout + li) * 4, 0);
#pragma unroll
        for (int s = 0; s < 16; ++s) w5r[s] = li < nout ? w5r[s] : 0.f;  // unguarded loads, then a select
        f32x4 hacc = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int s = 0; s < 16; ++s)
            hacc = __builtin_amdgcn_mfma_f32_16x16x4f32(w5r[s], slab[(64 * w + 4 * s + lk) * NC + li], hacc, 0, 0, 0);
        float* hred = in0;  // [EF_NW][8 x NC]
        if (lk < 2) {
#pragma unroll
            for (int r = 0; r < 4; ++r) hred[w * 8 * NC + (4 * lk + r) * NC + li] = hacc[r];
        }
        __syncthreads();
        if (tid < nout * NC) {
            const int j = tid / NC, col = tid % NC;
            float v = hred[tid];
#pragma unroll
            for (int q = 1; q < EF_NW; ++q) v += hred[q * 8 * NC + tid];
            v += P[g.b_off[L] + j];
            head_write<MODE>(g.head, slot, y, j, c0 + col, v);
        }
    }
}

void launch_stream_fwd(int head_mode, bool ln, const StreamArgs& a, hipStream_t s) {
    const dim3 grid((a.M / EF_NC) * a.ny * a.nz), block(EF_NW * 64);
#define FQ_SF(MODE, LNV) hipLaunchKernelGGL((stream_fwd_kernel<MODE, LNV>), grid, block, 0, s, a)
    switch (head_mode) {
        case HEAD_BC_FUSED: if (ln) FQ_SF(HEAD_BC_FUSED, true); else FQ_SF(HEAD_BC_FUSED, false); break;
        case HEAD_OS: if (ln) FQ_SF(HEAD_OS, true); else FQ_SF(HEAD_OS, false); break;
        default: if (ln) FQ_SF(HEAD_STORE, true); else FQ_SF(HEAD_STORE, false); break;
    }
#undef FQ_SF
}

// ============================================ split streamed forward (small populations) ==
// The streamed forward and the Euler flow with every 16-column tile computed by a CLUSTER of
// F blocks (F = 2, 4 or 8), so that a population of one to four members still fills the chip
// (the unsplit kernels give a 2-member population 32 to 128 blocks).  Block f of a cluster
// owns the 512/F features [fb, fb + 512/F) of every hidden layer after the first; each of its
// 4 waves runs TPW = 8/F 16x16 output tiles over the FULL K in the unsplit k order, so every
// output element is the same fp32 chain as in stream_fwd_kernel / euler_flow_kernel: the
// split results are bit-identical to the unsplit ones (and so independent of the split
// chosen, the members per GPU and the world size).
//   * layer 0 (K0 <= 64 inputs) is computed redundantly by every block of the cluster, with
//     the unsplit lane layout (two "unsplit waves" per wave), into the LDS slab: no hand-off;
//   * hidden layer l >= 1: A fragments W_l[4s + lk][feature] (TPW consecutive features per
//     lane: dword / dwordx2 / dwordx4 loads, an 8-deep ring that runs across layers), B from
//     the LDS slab in FRAGMENT ORDER (sp_fidx: one ds_read_b128 gives a lane the B values of
//     4 k-steps); the epilogue publishes GELU(u) of the block's features, and LayerNorm's
//     column partials of the block's "unsplit waves" (summed in the unsplit order from an LDS
//     image of the block's tile);
//   * hand-off by tagged granules (MI355X_MICROARCH.md price list, handoff-1to1 / allgather;
//     cdna_hip_programming.md Guideline 16, R2): every published value is one 8-byte
//     {value, tag} word written by one agent-scope atomic store; a consumer re-reads the
//     words of a layer (16-byte sc1 loads) until every tag is the hand-off's, and writes the
//     values into its LDS slab.  The data is its own flag: no drain, no counter, no poll of a
//     separate word.  tag = launch generation << 8 | hand-off index + 1; the generation is a
//     per-site word the last exiting block of every launch increments, so words left by an
//     earlier launch never match;
//   * head: the Euler flow publishes every block's unsplit-wave head partials and every block
//     sums the 8 in the unsplit order (x += v / S for the next step); the forward's head is
//     computed by the cluster's LAST arriver (told by its add to the cluster's counter), which
//     stages the last hidden layer, stores its G (and LN statistics) and calls head_write.
// The counters (cluster, ticket, exit) are zeroed by the last block to exit each launch (and
// at allocation, and by the runtime after an error); spins give up after ~2 s and set
// sync.err (the runtime then reports an error instead of hanging).
// Residency: a block takes its (cluster, slice) from a launch-wide ticket counter when it
// starts (sp_begin), so clusters are formed in the order blocks become resident: at any time
// a launch has at most one cluster whose blocks are not all resident, and every other cluster
// can finish and free its CUs.  No split launch can therefore wait for blocks that cannot be
// scheduled, whatever else runs on the device (other streams, other processes), as long as
// one cluster's F blocks fit on the chip.
constexpr int SP_NW = 4, SP_NT = SP_NW * 64;
constexpr int SP_XG = EF_H * EF_NC;                              // granules of one hidden layer of a tile
constexpr int SP_G_HP = 2 * SP_XG;                               // head partials [8 waves][8 outputs][16]
constexpr int SP_G_LP = SP_G_HP + 8 * 8 * EF_NC;                 // LN partials [2 parities][8 waves][2][16]
constexpr int SP_G_N = SP_G_LP + 2 * 8 * 2 * EF_NC;
constexpr long long SP_CLUSTER_GRANULES = (SP_G_N + 31) / 32 * 32;
constexpr int SP_CNT_STRIDE = 16;                                // counters 64 B apart
constexpr unsigned SP_SPIN_LIMIT = 1u << 21;

long long split_cluster_bytes() { return SP_CLUSTER_GRANULES * 8; }
int split_counter_stride() { return SP_CNT_STRIDE; }

typedef __attribute__((address_space(1))) unsigned int gu32_t;
typedef __attribute__((address_space(1))) unsigned long long gu64_t;

// element index of (feature k, column col) in the fragment-order slab / exchange: k-step
// s = k >> 2 of lane (lk = k & 3, col) is component s & 3 of float4 (s >> 2) * 64 + lane
DEV int sp_fidx(int k, int col) { return ((((k >> 4) << 6) + ((k & 3) << 4) + col) << 2) + ((k >> 2) & 3); }

DEV void sp_fail(const SplitSync& sy) {
    __hip_atomic_store((gu32_t*)sy.err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);  // host-mapped word
}
// block start: the ticket (cluster * F + slice) and the launch generation, block-uniform.
// readfirstlane: values read from LDS are not known to be uniform, and everything derived
// from the ticket (slot, parameter base, buffer resources) would sit in VGPRs, every buffer
// load then in a waterfall loop (round 4: the split k-loops ran 4x their MFMA time)
DEV int sp_begin(const SplitSync& sy, int clusters, unsigned* bc) {
    if (threadIdx.x == 0) {
        bc[0] = __hip_atomic_fetch_add((gu32_t*)(sy.cnt + (long long)clusters * SP_CNT_STRIDE), 1u, __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);
        bc[1] = __hip_atomic_load((const gu32_t*)sy.gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
    return __builtin_amdgcn_readfirstlane((int)bc[0]);
}
// block end (every block, every path): the last one to exit advances the site's generation and
// zeroes the launch's counters (every other block has taken its ticket, made its last-arriver
// add and exited), so the next launch of the site needs no memset node
DEV void sp_end(const SplitSync& sy, int clusters, int blocks, unsigned* bc) {
    __syncthreads();
    if (threadIdx.x == 0)
        bc[0] = __hip_atomic_fetch_add((gu32_t*)(sy.cnt + (long long)(clusters + 1) * SP_CNT_STRIDE), 1u, __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    if (__builtin_amdgcn_readfirstlane(bc[0]) == (unsigned)blocks - 1) {
        for (int c = threadIdx.x; c < clusters + 2; c += blockDim.x)
            __hip_atomic_store((gu32_t*)(sy.cnt + (long long)c * SP_CNT_STRIDE), 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (threadIdx.x == 0) __hip_atomic_fetch_add((gu32_t*)sy.gen, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}
DEV unsigned sp_tag(unsigned gen, unsigned phase) { return (gen << 8) | ((phase + 1) & 255u); }
// publish one value (an 8-byte {value, tag} word, one atomic store)
DEV void gx_put(unsigned long long* X, int gi, float v, unsigned tag) {
    __hip_atomic_store((gu64_t*)(X + gi), ((unsigned long long)tag << 32) | __builtin_bit_cast(unsigned, v), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
}
// read one published value, waiting for its tag
DEV float gx_get(const unsigned long long* X, int gi, unsigned tag, const SplitSync& sy) {
    unsigned spins = 0;
    while (true) {
        const unsigned long long x = __hip_atomic_load((const gu64_t*)(X + gi), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if ((unsigned)(x >> 32) == tag) return __builtin_bit_cast(float, (unsigned)x);
        if (++spins > SP_SPIN_LIMIT) {
            sp_fail(sy);
            return 0.f;
        }
        __builtin_amdgcn_s_sleep(1);
    }
}
// stage one published layer (SP_XG words from granule g0) into the fragment-order slab: each
// thread re-reads its 16-byte chunks (two words, sc1 loads) until both tags match
DEV void gx_stage(rsrc_t rX, int g0, unsigned tag, float* slab, const SplitSync& sy) {
    constexpr int CH = 8, PASSES = SP_XG / 2 / SP_NT / CH;  // 2 passes of 8 chunks per thread (32 VGPRs)
#pragma unroll
    for (int ps = 0; ps < PASSES; ++ps) {
        unsigned pending = (1u << CH) - 1u, spins = 0;
        uint4 v[CH];
        while (true) {
#pragma unroll
            for (int i = 0; i < CH; ++i)
                if (pending & (1u << i))
                    v[i] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(
                                                         rX, (g0 + 2 * ((int)threadIdx.x + (ps * CH + i) * SP_NT)) * 8, 0, 16));
#pragma unroll
            for (int i = 0; i < CH; ++i)
                if ((pending & (1u << i)) && v[i].y == tag && v[i].w == tag) {
                    *reinterpret_cast<float2*>(&slab[2 * ((int)threadIdx.x + (ps * CH + i) * SP_NT)]) =
                        float2{__builtin_bit_cast(float, v[i].x), __builtin_bit_cast(float, v[i].z)};
                    pending &= ~(1u << i);
                }
            if (pending == 0) break;
            if (++spins > SP_SPIN_LIMIT) {
                sp_fail(sy);
                break;
            }
            __builtin_amdgcn_s_sleep(1);
        }
    }
}
// the cluster's last arriver (after its words are written): one add to the cluster's counter
DEV bool sp_last(const SplitSync& sy, int cl, int F, unsigned* bc) {
    if (threadIdx.x == 0)
        bc[0] = __hip_atomic_fetch_add((gu32_t*)(sy.cnt + (long long)cl * SP_CNT_STRIDE), 1u, __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    return __builtin_amdgcn_readfirstlane(bc[0]) == (unsigned)F - 1;
}

// A fragments of TPW consecutive features: W[k][col .. col + TPW - 1] (components 0..TPW-1)
template <int TPW>
DEV float4 sp_aload(rsrc_t r, int elem_off) {
    if constexpr (TPW == 4) {
        return bload4(r, elem_off);
    } else if constexpr (TPW == 2) {
        const auto v = __builtin_amdgcn_raw_buffer_load_b64(r, elem_off * 4, 0, 0);
        const float2 f = __builtin_bit_cast(float2, v);
        return float4{f.x, f.y, 0.f, 0.f};
    } else {
        return float4{bload1(r, elem_off * 4, 0), 0.f, 0.f, 0.f};
    }
}

// One split hidden layer's k-loop (see ef_kloop): acc[t] += W[k][col + t] x[k][li] over the
// NS k-steps, B from the fragment-order slab (one float4 = 4 k-steps, read a group ahead);
// ring[] holds this layer's first sp_pf<TPW> k-steps on entry and the next layer's (w_next)
// on exit.  lo = lk * H + col.
// Prefetch depth: a k-step issues TPW dependent-latency MFMAs (40 cycles each), so an 8-deep
// ring covers only 320 cycles at TPW = 1, less than one Infinity-Cache hit (545 cycles idle,
// more under load): the ring holds SP_PFW / TPW k-steps (the same SP_PFW VGPRs at every TPW).
#ifndef FQ_SP_PFW
#define FQ_SP_PFW 32
#endif
constexpr int SP_PFW = FQ_SP_PFW;
template <int TPW>
constexpr int sp_pf() { return SP_PFW / TPW < 8 ? 8 : SP_PFW / TPW; }
template <int TPW, int PF = sp_pf<TPW>(), int INFLIGHT = 0>
DEV void sp_kloop(f32x4 (&acc)[TPW], float4 (&ring)[PF], rsrc_t rW, const float* xs, int NS, int w_cur,
                  int w_next, int lo, int lane) {
    constexpr int H = EF_H;
    const float4* x4 = reinterpret_cast<const float4*>(xs);
    float4 bn = x4[lane], b4 = bn;
    int s0 = 0;
    // Every vector-memory op older than the caller's last INFLIGHT loads is complete here
    // (vmcnt(INFLIGHT); the ring was filled a layer ago, the stage already drained).
    // Without it the waitcnt pass merges, at the loop head, the ring's in-order state of
    // the loop's back edge with the entry paths' (ring[0] refilled last on some of them)
    // and waits vmcnt(1) at the top of EVERY pass: the whole ring drained every PF k-steps
    // (TPW = 1: vmcnt(1) instead of vmcnt(31), 3.7 us per layer against a 1.9 us chain).
    static_assert(INFLIGHT >= 0 && INFLIGHT < 16, "");
    __builtin_amdgcn_s_waitcnt(0x0F70 | INFLIGHT);
    do {
        const int rbase = (s0 + PF < NS ? w_cur + 4 * (s0 + PF) * H : w_next) + lo;
#pragma unroll
        for (int p = 0; p < PF; ++p) {
            const int s = s0 + p;
            if ((p & 3) == 0) {
                b4 = bn;
                bn = x4[((s >> 2) + 1) * 64 + lane];  // the next group (past the end: slack)
            }
            const float b = (p & 3) == 0 ? b4.x : (p & 3) == 1 ? b4.y : (p & 3) == 2 ? b4.z : b4.w;
            __builtin_amdgcn_sched_barrier(0);
            const float4 a = ring[p];
            acc[0] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.x, b, acc[0], 0, 0, 0);
            if constexpr (TPW > 1) acc[1] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.y, b, acc[1], 0, 0, 0);
            if constexpr (TPW > 2) {
                acc[2] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.z, b, acc[2], 0, 0, 0);
                acc[3] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.w, b, acc[3], 0, 0, 0);
            }
            __builtin_amdgcn_sched_barrier(0);
            ring[p] = sp_aload<TPW>(rW, rbase + 4 * p * H);
            __builtin_amdgcn_sched_barrier(0);
        }
        s0 += PF;
    } while (s0 < NS);
}

bool split_fwd_supported(int H, int L, int K0, int nout, int M) {
    // L >= 3: a hand-off lies between two steps' head-partial writes (Euler)
    return H == EF_H && L >= 3 && L <= EF_MAX_LAYERS && K0 <= EF_K0MAX && nout <= 8 && M % EF_NC == 0;
}

// The Euler flow's layer-0 form (split_fwd_kernel's PRE0): the observation rows' k-steps
// once per launch, at most 2 k-steps of its own per flow step (see pre0g in the kernel)
constexpr int sp_ns0(int K0, bool tail0) { return tail0 ? EF_PF : (K0 + 4 * EF_PF - 1) / (4 * EF_PF) * EF_PF; }
bool split_euler_pre0(int K0, int D) {
    const bool tail0 = K0 > 4 * EF_PF && K0 <= 4 * (EF_PF + 1);
    const int npre = D / 4, nps = sp_ns0(K0, tail0) + (tail0 ? 1 : 0) - npre;
    return npre > 0 && nps >= 1 && nps <= 2;
}

template <int MODE, bool LN, bool EULER, int TPW, bool PRE0 = false>
__global__ __launch_bounds__(SP_NT, 2) void split_fwd_kernel(const SplitFwdArgs a) {
    constexpr int H = EF_H, NC = EF_NC, NT = SP_NT, PF = EF_PF, F = 8 / TPW, FB = H / F;
    const StreamArgs& g = a.s;
    __shared__ __attribute__((aligned(16))) float slab[H * NC + 256];        // layer input, fragment order (+ slack)
    __shared__ __attribute__((aligned(16))) float in0[EF_K0MAX * NC + 64];   // layer-0 input [K0][NC]
    __shared__ __attribute__((aligned(16))) float tile[FB * NC];             // the block's layer output [FB][NC]
    __shared__ float lnred[2][8][NC];                                        // unsplit-wave LN partials
    __shared__ float stat[2][NC];                                            // column mean / rstd
    __shared__ float lng[2][H];                                              // LN scale / bias of a staged layer
    __shared__ float hred[8][8][NC];                                         // unsplit-wave head partials
    __shared__ unsigned bc[2];

    const int tiles = g.M / NC, clusters = tiles * g.ny * g.nz;
    const int ticket = sp_begin(a.sync, clusters, bc);
    const unsigned gen = __builtin_amdgcn_readfirstlane(bc[1]);
    const int cl = ticket / F, f = ticket % F, fb = f * FB;
    const int tl = __builtin_amdgcn_readfirstlane(cl % tiles), yz = cl / tiles;
    const int y = __builtin_amdgcn_readfirstlane(yz % g.ny), z = __builtin_amdgcn_readfirstlane(yz / g.ny);
    const int slot = __builtin_amdgcn_readfirstlane(g.slots[z]);
    const int c0 = tl * NC;
    const int tid = threadIdx.x, lane = tid & 63;
    const int q = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int li = lane & 15, lk = lane >> 4;
    const int L = g.L, K0 = g.K0, nout = g.head.nout;
    if (a.probe != nullptr && tid == 0) a.probe[2 * blockIdx.x] = __builtin_amdgcn_s_memrealtime();
#ifdef FQ_PHASE_PROBE  // diagnostic build only (make PHASE=1): the Euler flow's per-layer phases
    // [0] start, [1] inputs loaded; step st, layer l: 1 + 4 (st (L + 1) + l) + {0 layer start,
    // 1 input staged, 2 k-loop end, 3 published}; head (l = L): {0 start, 3 state updated};
    // [STRIDE - 1] XCC_ID, [STRIDE - 2] HW_ID, [STRIDE - 3] ticket
    unsigned long long* const ph = EULER && a.phase != nullptr ? a.phase + (long long)blockIdx.x * EF_PHASE_STRIDE : nullptr;
    auto stamp = [&](int st, int l, int i) {
        if (ph != nullptr && tid == 0) ph[st < 0 ? i : 1 + 4 * (st * (L + 1) + l) + i] = __builtin_amdgcn_s_memrealtime();
    };
    if (ph != nullptr && tid == 0) {
        ph[EF_PHASE_STRIDE - 1] = (unsigned)__builtin_amdgcn_s_getreg(20 | (31 << 11));
        ph[EF_PHASE_STRIDE - 2] = (unsigned)__builtin_amdgcn_s_getreg(4 | (31 << 11));
        ph[EF_PHASE_STRIDE - 3] = (unsigned)ticket;
    }
    stamp(-1, 0, 0);
#else
    auto stamp = [](int, int, int) {};
#endif
    const bool tail0 = K0 > 4 * PF && K0 <= 4 * (PF + 1);
    const int NS0 = sp_ns0(K0, tail0);
    const float* __restrict__ P = g.params + (long long)slot * g.P + (long long)y * g.ens;
    const rsrc_t rW = make_rsrc(P, g.P);
    unsigned long long* const X = a.sync.xch + (long long)cl * SP_CLUSTER_GRANULES;
    const rsrc_t rX = __builtin_amdgcn_make_buffer_rsrc((void*)X, (short)0, (int)(SP_CLUSTER_GRANULES * 8), 0x00020000);
    unsigned phase = 0;  // hand-offs of this launch so far
    const bool st = c0 >= g.st_lo && c0 + NC <= g.st_hi;
    const long long sbase = (long long)slot * g.s_ss + (long long)y * g.s_sy + c0;
    load_in0<NT>(in0, g.x0 + (long long)slot * g.x0_ss, K0, g.ld_x, c0);
    __syncthreads();
    stamp(-1, 0, 1);

    // Euler flow, layer 0 (computed in every block, all 512 features): its observation rows
    // are the same at every flow step, so the first NPRE k-steps of each feature's chain
    // (rows < 4 NPRE <= D) run once per launch, and every step resumes the chain from their
    // accumulators with its own k-steps (action and time rows, then the zero rows up to the
    // unsplit kernel's k-step count, tail included): the same MFMAs in the same order as
    // the full chain, bit-identical.  The accumulators (32 per thread) live in a global
    // scratch slab of the block's ticket (a.pre0; each thread reads back only its own
    // words): 32 KB of LDS per block would cost the kernels beside the flow their
    // co-residency.  A step's own A fragments are loaded before the
    // previous step's head wait, the accumulators at the start of its layer 0.  Taken when a step has at most 2
    // k-steps of its own (cube: 7 of 9 k-steps once per launch).
    const int NPRE = EULER ? a.D / 4 : 0, NPS = NS0 + (tail0 ? 1 : 0) - NPRE;
    constexpr bool fast0 = EULER && PRE0;  // the host checked split_euler_pre0(K0, D)
    float4 a0[2][2], pv[2][4];
    float* const pre0g = fast0 ? a.pre0 + ((long long)ticket * 2 * NT + tid) * 16 : nullptr;  // [h] at + h NT 16
    auto load_step0 = [&]() {
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int lo0 = lk * H + 64 * (2 * q + h) + 4 * li;
#pragma unroll
            for (int j = 0; j < 2; ++j)
                a0[h][j] = j < NPS ? bload4(rW, (int)g.w_off[0] + 4 * (NPRE + j) * H + lo0) : float4{0.f, 0.f, 0.f, 0.f};
        }
    };
    auto load_pv = [&]() {  // the accumulators: at layer 0 (across the head wait they would spill)
#pragma unroll
        for (int h = 0; h < 2; ++h)
#pragma unroll
            for (int c = 0; c < 4; ++c) pv[h][c] = *reinterpret_cast<const float4*>(pre0g + (long long)h * NT * 16 + 4 * c);
    };
    if constexpr (fast0) {
        // both unsplit waves' loads of a batch of 8 k-steps in flight together
        f32x4 acc[2][4];
#pragma unroll
        for (int h = 0; h < 2; ++h)
#pragma unroll
            for (int c = 0; c < 4; ++c) acc[h][c] = f32x4{0.f, 0.f, 0.f, 0.f};
        for (int s0 = 0; s0 < NPRE; s0 += 8) {
            float4 t[2][8];
#pragma unroll
            for (int h = 0; h < 2; ++h)
#pragma unroll
                for (int j = 0; j < 8; ++j)
                    t[h][j] = s0 + j < NPRE ? bload4(rW, (int)g.w_off[0] + 4 * (s0 + j) * H + lk * H + 64 * (2 * q + h) + 4 * li)
                                            : float4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int h = 0; h < 2; ++h)
#pragma unroll
                for (int j = 0; j < 8; ++j)
                    if (s0 + j < NPRE) {
                        const float b = in0[(4 * (s0 + j) + lk) * NC + li];
                        acc[h][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(t[h][j].x, b, acc[h][0], 0, 0, 0);
                        acc[h][1] = __builtin_amdgcn_mfma_f32_16x16x4f32(t[h][j].y, b, acc[h][1], 0, 0, 0);
                        acc[h][2] = __builtin_amdgcn_mfma_f32_16x16x4f32(t[h][j].z, b, acc[h][2], 0, 0, 0);
                        acc[h][3] = __builtin_amdgcn_mfma_f32_16x16x4f32(t[h][j].w, b, acc[h][3], 0, 0, 0);
                    }
        }
#pragma unroll
        for (int h = 0; h < 2; ++h)
#pragma unroll
            for (int c = 0; c < 4; ++c)
                *reinterpret_cast<float4*>(pre0g + (long long)h * NT * 16 + 4 * c) =
                    float4{acc[h][c][0], acc[h][c][1], acc[h][c][2], acc[h][c][3]};
        load_step0();
    }

    // LayerNorm statistics of one column from the 8 unsplit-wave partials (stream_fwd_kernel's sums)
    auto col_stats = [&](int col, float& mean, float& rs) {
        float S1 = 0.f, S2 = 0.f;
#pragma unroll
        for (int w8 = 0; w8 < EF_NW; ++w8) {
            S1 += lnred[0][w8][col];
            S2 += lnred[1][w8][col];
        }
        ln_stats(S1, S2, (float)H, mean, rs);
    };
    // normalise the fragment-order slab in place with stat[] and lng[] (thread: 8 float4)
    auto ln_slab = [&]() {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const int f4 = tid * 8 + i, gq = f4 >> 6, ln = f4 & 63, col = ln & 15, kk = ln >> 4;
            float4 v = reinterpret_cast<float4*>(slab)[f4];
            const float m = stat[0][col], r = stat[1][col];
            v.x = ln_apply(v.x, m, r, lng[0][16 * gq + kk], lng[1][16 * gq + kk]);
            v.y = ln_apply(v.y, m, r, lng[0][16 * gq + 4 + kk], lng[1][16 * gq + 4 + kk]);
            v.z = ln_apply(v.z, m, r, lng[0][16 * gq + 8 + kk], lng[1][16 * gq + 8 + kk]);
            v.w = ln_apply(v.w, m, r, lng[0][16 * gq + 12 + kk], lng[1][16 * gq + 12 + kk]);
            reinterpret_cast<float4*>(slab)[f4] = v;
        }
    };
    // layer outputs in the slab (features [k0, k0 + nk)) -> G [feature][ld_s]
    auto store_slab_rows = [&](int l, int k0, int nk) {
        if (!st || g.G[l] == nullptr || c0 + NC > g.g_hi) return;
        float* Gp = g.G[l] + sbase;
        for (int e = tid; e < nk * NC; e += NT) {
            const int k = k0 + e / NC, col = e % NC;
            Gp[(long long)k * g.ld_s + col] = slab[sp_fidx(k, col)];
        }
    };
    auto store_stats = [&](int l) {
        if (LN && st && tid < NC && g.MU[l]) {
            const long long so = (long long)slot * g.st_ss + (long long)y * g.st_sy + c0 + tid;
            g.MU[l][so] = stat[0][tid];
            g.RS[l][so] = stat[1][tid];
        }
    };
    // stage a published layer output (+ LN partials, scale and bias of layer l) into the slab
    auto stage = [&](int par, unsigned tag, int l) {
        if (LN) {
            lng[0][tid] = P[g.g_off[l] + tid];
            lng[0][tid + NT] = P[g.g_off[l] + tid + NT];
            lng[1][tid] = P[g.be_off[l] + tid];
            lng[1][tid + NT] = P[g.be_off[l] + tid + NT];
            // the words hold [w][s][c] (tid < 256 = 8 x 2 x 16); lnred is [s][w][c]
            lnred[(tid / NC) & 1][tid / (2 * NC)][tid % NC] = gx_get(X, SP_G_LP + par * 8 * 2 * NC + tid, tag, a.sync);
        }
        gx_stage(rX, par * SP_XG, tag, slab, a.sync);
        __syncthreads();
        if (LN) {
            if (tid < NC) col_stats(tid, stat[0][tid], stat[1][tid]);
            __syncthreads();
        }
    };

    const int EUS = EULER ? a.S : 1;
    for (int step = EULER ? a.first : 0; step < EUS; ++step) {
        if (EULER && step == a.first) {
            if (tid < NC) in0[(a.D + a.A) * NC + tid] = (float)((double)step / (double)a.S);
            __syncthreads();
        }
        const int pst = step - a.first;  // (phase stamps)
        (void)pst;
        // ---- layer 0, redundantly in every block: unsplit waves 2q, 2q + 1 ----
        stamp(pst, 0, 0);
        if constexpr (fast0) load_pv();
        stamp(pst, 0, 1);
        {
            float v[2][4][4];
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const int w = 2 * q + h;
                float4 bias4[4];
                f32x4 acc[4];
                bool done0 = false;
                if constexpr (EULER) {
                    if constexpr (fast0) {  // resume the chain after the observation rows (see pre0g)
#pragma unroll
                        for (int r = 0; r < 4; ++r) bias4[r] = bload4(rW, (int)g.b_off[0] + 64 * w + 16 * lk + 4 * r);
#pragma unroll
                        for (int c = 0; c < 4; ++c) acc[c] = f32x4{pv[h][c].x, pv[h][c].y, pv[h][c].z, pv[h][c].w};
#pragma unroll
                        for (int j = 0; j < 2; ++j)
                            if (j < NPS) {
                                const float b = in0[(4 * (NPRE + j) + lk) * NC + li];
                                acc[0] = __builtin_amdgcn_mfma_f32_16x16x4f32(a0[h][j].x, b, acc[0], 0, 0, 0);
                                acc[1] = __builtin_amdgcn_mfma_f32_16x16x4f32(a0[h][j].y, b, acc[1], 0, 0, 0);
                                acc[2] = __builtin_amdgcn_mfma_f32_16x16x4f32(a0[h][j].z, b, acc[2], 0, 0, 0);
                                acc[3] = __builtin_amdgcn_mfma_f32_16x16x4f32(a0[h][j].w, b, acc[3], 0, 0, 0);
                            }
                        done0 = true;
                    }
                }
                if (!done0) {
                    const int lo = lk * H + 64 * w + 4 * li;
                    float4 ring[PF];
#pragma unroll
                    for (int p = 0; p < PF; ++p) ring[p] = bload4(rW, (int)g.w_off[0] + 4 * p * H + lo);
                    const float4 at0 = bload4(rW, (int)g.w_off[0] + 4 * PF * H + lo);
#pragma unroll
                    for (int r = 0; r < 4; ++r) bias4[r] = bload4(rW, (int)g.b_off[0] + 64 * w + 16 * lk + 4 * r);
#pragma unroll
                    for (int c = 0; c < 4; ++c) acc[c] = f32x4{0.f, 0.f, 0.f, 0.f};
                    ef_kloop(acc, ring, rW, in0, NS0, (int)g.w_off[0], (int)g.w_off[0], lo, lk, li);
                    if (tail0) ef_tail(acc, at0, in0, lk, li);
                }
                const bool stU = st && g.U[0] && 64 * w >= fb && 64 * w < fb + FB;
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const float bv[4] = {bias4[r].x, bias4[r].y, bias4[r].z, bias4[r].w};
#pragma unroll
                    for (int c = 0; c < 4; ++c) {
                        const float u = acc[c][r] + bv[c];
                        if (stU) g.U[0][sbase + (long long)(64 * w + 16 * lk + 4 * r + c) * g.ld_s + li] = u;
                        v[h][r][c] = gelu_fast(u);
                    }
                }
                if constexpr (LN) {
                    float s1 = 0.f, s2 = 0.f;
#pragma unroll
                    for (int r = 0; r < 4; ++r)
#pragma unroll
                        for (int c = 0; c < 4; ++c) ln_acc(v[h][r][c], s1, s2);
                    s1 = lk_sum(s1);
                    s2 = lk_sum(s2);
                    if (lk == 0) {
                        lnred[0][w][li] = s1;
                        lnred[1][w][li] = s2;
                    }
                }
            }
            __syncthreads();  // lnred visible; every wave is done reading the slab (previous layer)
            stamp(pst, 0, 2);
            float mean = 0.f, rs = 0.f;
            if constexpr (LN) col_stats(li, mean, rs);
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const int w = 2 * q + h;
                float ga[16], be[16];
                if constexpr (LN) {
#pragma unroll
                    for (int e = 0; e < 16; ++e) {
                        ga[e] = P[g.g_off[0] + 64 * w + 16 * lk + e];
                        be[e] = P[g.be_off[0] + 64 * w + 16 * lk + e];
                    }
                }
                // feature 64 w + 16 lk + 4 r + c, column li: fragment-order float4 over r
#pragma unroll
                for (int c = 0; c < 4; ++c) {
                    float x[4];
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        x[r] = v[h][r][c];
                        if constexpr (LN) x[r] = ln_apply(x[r], mean, rs, ga[4 * r + c], be[4 * r + c]);
                    }
                    reinterpret_cast<float4*>(slab)[(4 * w + lk) * 64 + c * 16 + li] = float4{x[0], x[1], x[2], x[3]};
                }
            }
            if constexpr (LN) {
                if (tid < NC) col_stats(tid, stat[0][tid], stat[1][tid]);
            }
            __syncthreads();
            if (!EULER) {
                store_slab_rows(0, fb, FB);
                if (f == 0) store_stats(0);
            }
            stamp(pst, 0, 3);
        }
        // ---- hidden layers 1 .. L-1, split ----
        // ring depth per form, the deepest that does not spill (256 VGPRs at 2 waves per SIMD):
        // a k-step's loads wait ~1 us under load, its MFMAs take TPW x 32-40 cycles
        constexpr int RPF = EULER ? (TPW == 1 ? 32 : 8)
                                  : (TPW == 4 ? (LN ? 8 : 16) : TPW == 2 ? 32 : 64);
        float4 ring[RPF];
        const int col = fb + 16 * TPW * q + TPW * li;
        const int lo = lk * H + col;
#pragma unroll
        for (int p = 0; p < RPF; ++p) ring[p] = sp_aload<TPW>(rW, (int)g.w_off[1] + 4 * p * H + lo);
        for (int l = 1; l < L; ++l) {
            stamp(pst, l, 0);
            if (l >= 2) {
                stage((l - 1) & 1, sp_tag(gen, phase - 1), l - 1);
                if constexpr (LN) {
                    ln_slab();
                    __syncthreads();
                    // (without LN the producers stored G_{l-1} themselves)
                    store_slab_rows(l - 1, fb, FB);
                    if (f == 0) store_stats(l - 1);
                }
            }
            f32x4 acc[TPW];
#pragma unroll
            for (int t = 0; t < TPW; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
            // bias of the lane's 4 TPW features fb + 16 TPW q + 4 TPW lk + (TPW r + t)
            float bias[4 * TPW];
#pragma unroll
            for (int i = 0; i < TPW; ++i) {
                const float4 b4 = bload4(rW, (int)g.b_off[l] + fb + 16 * TPW * q + 4 * TPW * lk + 4 * i);
                bias[4 * i] = b4.x; bias[4 * i + 1] = b4.y; bias[4 * i + 2] = b4.z; bias[4 * i + 3] = b4.w;
            }
            const int wcur = (int)g.w_off[l], wnext = (int)g.w_off[l + 1 < L ? l + 1 : 1];
            asm volatile("" ::"s"(wcur), "s"(wnext));
            stamp(pst, l, 1);
            sp_kloop<TPW, RPF, TPW>(acc, ring, rW, slab, H / 4, wcur, wnext, lo, lane);  // the bias loads stay in flight
            stamp(pst, l, 2);
            // epilogue: tile t, reg r: feature fb + 16 TPW q + TPW (4 lk + r) + t, column li
            const bool last = l == L - 1;
            const bool stU = st && g.U[l];
            const bool stG = !LN && st && g.G[l] && c0 + NC <= g.g_hi;
            const unsigned tag = sp_tag(gen, phase);
#pragma unroll
            for (int r = 0; r < 4; ++r)
#pragma unroll
                for (int t = 0; t < TPW; ++t) {
                    const int fl = 16 * TPW * q + TPW * (4 * lk + r) + t;  // feature - fb
                    const float u = acc[t][r] + bias[TPW * r + t];
                    if (stU) g.U[l][sbase + (long long)(fb + fl) * g.ld_s + li] = u;
                    const float gv = gelu_fast(u);
                    if (stG) g.G[l][sbase + (long long)(fb + fl) * g.ld_s + li] = gv;
                    tile[fl * NC + li] = gv;
                    if (!EULER || !last) gx_put(X, (l & 1) * SP_XG + sp_fidx(fb + fl, li), gv, tag);
                }
            __syncthreads();  // tile complete
            if (LN && q < TPW) {
                // LN partials of unsplit wave f TPW + q, in its order (features 64 q + 16 lk + e)
                float s1 = 0.f, s2 = 0.f;
#pragma unroll
                for (int e = 0; e < 16; ++e) ln_acc(tile[(64 * q + 16 * lk + e) * NC + li], s1, s2);
                s1 = lk_sum(s1);
                s2 = lk_sum(s2);
                if (lk == 0) {
                    const int w8 = f * TPW + q;
                    gx_put(X, SP_G_LP + ((l & 1) * 8 + w8) * 2 * NC + li, s1, tag);
                    gx_put(X, SP_G_LP + ((l & 1) * 8 + w8) * 2 * NC + NC + li, s2, tag);
                }
            }
            if (EULER && last && q < TPW) {
                // head partials of unsplit wave f TPW + q (euler_flow_kernel's head)
                const int w8 = f * TPW + q;
                float w5r[16];
#pragma unroll
                for (int s = 0; s < 16; ++s) w5r[s] = bload1(rW, ((int)g.w_off[L] + (64 * w8 + 4 * s + lk) * a.A + li) * 4, 0);
#pragma unroll
                for (int s = 0; s < 16; ++s) w5r[s] = li < a.A ? w5r[s] : 0.f;
                f32x4 hacc = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
                for (int s = 0; s < 16; ++s)
                    hacc = __builtin_amdgcn_mfma_f32_16x16x4f32(w5r[s], tile[(64 * q + 4 * s + lk) * NC + li], hacc, 0, 0, 0);
                if (lk < 2) {
#pragma unroll
                    for (int r = 0; r < 4; ++r) gx_put(X, SP_G_HP + (w8 * 8 + 4 * lk + r) * NC + li, hacc[r], tag);
                }
            }
            ++phase;
            stamp(pst, l, 3);
            if (!EULER && last) {
                // the cluster's last arriver: stage the last hidden layer, store it, run the head
                if (!sp_last(a.sync, cl, F, bc)) break;
                stage(l & 1, tag, l);
                if constexpr (LN) {
                    ln_slab();
                    __syncthreads();
                    store_slab_rows(l, 0, H);
                    store_stats(l);
                }
                // head partials of all 8 unsplit waves (wave q: 2q, 2q + 1), stream_fwd_kernel's order
#pragma unroll
                for (int h = 0; h < 2; ++h) {
                    const int w8 = 2 * q + h;
                    float w5r[16];
#pragma unroll
                    for (int s = 0; s < 16; ++s) w5r[s] = bload1(rW, ((int)g.w_off[L] + (64 * w8 + 4 * s + lk) * nout + li) * 4, 0);
#pragma unroll
                    for (int s = 0; s < 16; ++s) w5r[s] = li < nout ? w5r[s] : 0.f;
                    f32x4 hacc = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
                    for (int s = 0; s < 16; ++s)
                        hacc = __builtin_amdgcn_mfma_f32_16x16x4f32(w5r[s], slab[sp_fidx(64 * w8 + 4 * s + lk, li)], hacc, 0, 0, 0);
                    if (lk < 2) {
#pragma unroll
                        for (int r = 0; r < 4; ++r) hred[w8][4 * lk + r][li] = hacc[r];
                    }
                }
                __syncthreads();
                if (tid < nout * NC) {
                    const int j = tid / NC, cc = tid % NC;
                    float v = hred[0][j][cc];
#pragma unroll
                    for (int w8 = 1; w8 < EF_NW; ++w8) v += hred[w8][j][cc];
                    v += P[g.b_off[L] + j];
                    head_write<MODE>(g.head, slot, y, j, c0 + cc, v);
                }
            }
        }
        if constexpr (EULER) {
            // every block: the 8 unsplit-wave head partials, summed in euler_flow_kernel's order
            const unsigned tag = sp_tag(gen, phase - 1);
            stamp(pst, L, 0);
            if (fast0 && step + 1 < a.S) load_step0();  // the next step's layer-0 operands, during the wait
            if (tid < a.A * NC) {
                const int aa = tid / NC, j = tid % NC;
                float v = gx_get(X, SP_G_HP + aa * NC + j, tag, a.sync);
#pragma unroll
                for (int w8 = 1; w8 < EF_NW; ++w8) v += gx_get(X, SP_G_HP + (w8 * 8 + aa) * NC + j, tag, a.sync);
                v += P[g.b_off[L] + aa];
                float* xp = &in0[(a.D + aa) * NC + j];
                *xp = *xp + v / a.steps_f;
            } else if (tid < (a.A + 1) * NC && step + 1 < a.S) {
                in0[(a.D + a.A) * NC + tid - a.A * NC] = (float)((double)(step + 1) / (double)a.S);
            }
            __syncthreads();
            stamp(pst, L, 3);
        }
    }
    if (EULER && f == 0 && tid < a.A * NC) {
        const int aa = tid / NC, j = tid % NC;
        at(a.aflow, slot)[(long long)aa * a.s.M + c0 + j] = clip1(in0[(a.D + aa) * NC + j]);
    }
    if (a.probe != nullptr) {
        __syncthreads();
        if (tid == 0) a.probe[2 * blockIdx.x + 1] = __builtin_amdgcn_s_memrealtime();
    }
    sp_end(a.sync, clusters, clusters * F, bc);
}

void launch_split_fwd(int head_mode, bool ln, bool euler, int F, const SplitFwdArgs& a, hipStream_t s) {
    const dim3 grid((a.s.M / EF_NC) * a.s.ny * a.s.nz * F), block(SP_NT);
#define FQ_SPF(MODE, LNV, EU, T) hipLaunchKernelGGL((split_fwd_kernel<MODE, LNV, EU, T>), grid, block, 0, s, a)
#define FQ_SPF0(T) hipLaunchKernelGGL((split_fwd_kernel<HEAD_EULER, false, true, T, true>), grid, block, 0, s, a)
#define FQ_SPF_T(MODE, LNV, EU)                          \
    switch (F) {                                         \
        case 8: FQ_SPF(MODE, LNV, EU, 1); break;         \
        case 4: FQ_SPF(MODE, LNV, EU, 2); break;         \
        default: FQ_SPF(MODE, LNV, EU, 4); break;        \
    }
    if (euler) {
        const bool pre0 = a.pre0 != nullptr && split_euler_pre0(a.s.K0, a.D);
        if (F == 8) {
            if (pre0) FQ_SPF0(1); else FQ_SPF(HEAD_EULER, false, true, 1);
        } else {
            if (pre0) FQ_SPF0(2); else FQ_SPF(HEAD_EULER, false, true, 2);
        }
    } else {
        switch (head_mode) {
            // (the actors have no LayerNorm: actor_layer_norm is refused at create)
            case HEAD_BC_FUSED: FQ_SPF_T(HEAD_BC_FUSED, false, false) break;
            case HEAD_OS: FQ_SPF_T(HEAD_OS, false, false) break;
            default: if (ln) { FQ_SPF_T(HEAD_STORE, true, false) } else { FQ_SPF_T(HEAD_STORE, false, false) } break;
        }
    }
#undef FQ_SPF_T
#undef FQ_SPF0
#undef FQ_SPF
}

// ============================================================ backward =====
// Gradient w.r.t. a hidden layer's output, either from memory (dh') or, for
// the last hidden layer, recomputed from the head: dh[k][m] = sum_j W5[k][j] dout[j][m].
template <bool HEAD>
DEV float load_dh(const float* __restrict__ dh, const float* __restrict__ W5, const float* dov,
                  int nout, int k, int m, int ld_d) {
    if constexpr (HEAD) {
        float s = 0.f;
        const float* wr = W5 + (long long)k * nout;
#pragma unroll
        for (int j = 0; j < 8; ++j)
            if (j < nout) s += wr[j] * dov[j];
        return s;
    } else {
        return dh[(long long)k * ld_d + m];
    }
}

// LN backward row statistics: c1[m] = mean_k(dxhat), c2[m] = mean_k(dxhat*xhat)
// with dxhat = dh*gamma, xhat = (gelu(u)-mu)*rstd.
template <bool HEAD, int KPT>
__global__ __launch_bounds__(1024) void bwd_rowstats_kernel(const BwdArgs a) {
    const int ncb = a.M / 64;
    const int cb = blockIdx.x % ncb, yz = blockIdx.x / ncb;
    const int y = yz % a.ny, z = yz / a.ny;
    const int slot = a.slots[z];
    const int lane = threadIdx.x & 63;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int m = cb * 64 + lane;
    const int k0 = w * KPT;
    const float* __restrict__ u = at(a.u, slot, y) + m;
    const float* __restrict__ gam = at(a.gamma, slot, y) + k0;
    const float mu = at(a.mu, slot, y)[m], rs = at(a.rstd, slot, y)[m];
    float dov[8];
    const float* W5 = nullptr;
    const float* dh = nullptr;
    if constexpr (HEAD) {
        const float* dout = at(a.dout, slot, y) + m;
        W5 = at(a.W5, slot, y) + (long long)k0 * a.nout;
#pragma unroll
        for (int j = 0; j < 8; ++j) dov[j] = (j < a.nout) ? dout[(long long)j * a.ld_o] : 0.f;
    } else {
        dh = at(a.dh, slot, y) + m;
    }
    float s1 = 0.f, s2 = 0.f;
    constexpr int CH = KPT < 16 ? KPT : 16;  // loads in flight per array
#pragma unroll 1
    for (int c = 0; c < KPT; c += CH) {
        float uv[CH], dhv[CH];
#pragma unroll
        for (int i = 0; i < CH; ++i) uv[i] = u[(long long)(k0 + c + i) * a.ld];
        if constexpr (HEAD) {
#pragma unroll
            for (int i = 0; i < CH; ++i) {
                float sv = 0.f;
#pragma unroll
                for (int j = 0; j < 8; ++j)
                    if (j < a.nout) sv += W5[(c + i) * a.nout + j] * dov[j];
                dhv[i] = sv;
            }
        } else {
#pragma unroll
            for (int i = 0; i < CH; ++i) dhv[i] = dh[(long long)(k0 + c + i) * a.ld_d];
        }
#pragma unroll
        for (int i = 0; i < CH; ++i) {
            const float xh = (gelu_f(uv[i]) - mu) * rs;
            const float dxh = dhv[i] * gam[c + i];
            s1 += dxh;
            s2 += dxh * xh;
        }
    }
    __shared__ float red[2][CW][64];
    red[0][w][lane] = s1;
    red[1][w][lane] = s2;
    __syncthreads();
    if (w == 0) {
        float S1 = 0.f, S2 = 0.f;
#pragma unroll
        for (int q = 0; q < CW; ++q) {
            S1 += red[0][q][lane];
            S2 += red[1][q][lane];
        }
        at(a.c1, slot, y)[m] = S1 / (float)a.H;
        at(a.c2, slot, y)[m] = S2 / (float)a.H;
    }
}

// One wave per feature k: du'[k][m] for every column m, plus the parameter
// gradients that are sums over the batch (only columns m < Mg contribute):
//   bias  db[k] = sum du ;  LN: dgamma[k] = sum dh*xhat, dbeta[k] = sum dh ;
//   head: dW5[k][j] = sum x_head[k][m] dout[j][m].
template <bool HEAD, bool LN>
__global__ __launch_bounds__(256) void bwd_cols_kernel(const BwdArgs a) {
    const int nkb = a.H / 4;
    const int kb = blockIdx.x % nkb, yz = blockIdx.x / nkb;
    const int y = yz % a.ny, z = yz / a.ny;
    const int slot = a.slots[z];
    const int lane = threadIdx.x & 63;
    const int k = kb * 4 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const float* __restrict__ u = at(a.u, slot, y);
    const float* __restrict__ dh = HEAD ? nullptr : at(a.dh, slot, y);
    const float* __restrict__ W5 = HEAD ? at(a.W5, slot, y) : nullptr;
    const float* __restrict__ dout = HEAD ? at(a.dout, slot, y) : nullptr;
    const float* __restrict__ xhd = HEAD ? at(a.x_head, slot, y) : nullptr;
    const float* __restrict__ mu = LN ? at(a.mu, slot, y) : nullptr;
    const float* __restrict__ rs = LN ? at(a.rstd, slot, y) : nullptr;
    const float* __restrict__ c1 = LN ? at(a.c1, slot, y) : nullptr;
    const float* __restrict__ c2 = LN ? at(a.c2, slot, y) : nullptr;
    const float gam = LN ? at(a.gamma, slot, y)[k] : 1.f;
    float* __restrict__ du = at(a.du, slot, y);
    float sb = 0.f, sg = 0.f, sbeta = 0.f;
    float sw[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) sw[j] = 0.f;
    for (int m = lane; m < a.M; m += 64) {
        float dov[8];
        if constexpr (HEAD) {
#pragma unroll
            for (int j = 0; j < 8; ++j) dov[j] = (j < a.nout) ? dout[(long long)j * a.ld_o + m] : 0.f;
        }
        const float dhv = load_dh<HEAD>(dh, W5, dov, a.nout, k, m, a.ld_d);
        const float uv = u[(long long)k * a.ld + m];
        float dg;
        if constexpr (LN) {
            const float xh = (gelu_f(uv) - mu[m]) * rs[m];
            dg = rs[m] * (dhv * gam - c1[m] - xh * c2[m]);
            if (m < a.Mg) {
                sg += dhv * xh;
                sbeta += dhv;
            }
        } else {
            dg = dhv;
        }
        const float duv = dg * gelu_grad_f(uv);
        du[(long long)k * a.ld_d + m] = duv;
        if (m < a.Mg) {
            sb += duv;
            if constexpr (HEAD) {
                const float xv = xhd[(long long)k * a.ld + m];
#pragma unroll
                for (int j = 0; j < 8; ++j) sw[j] += xv * dov[j];
            }
        }
    }
    sb = wave_sum(sb);
    if constexpr (LN) {
        sg = wave_sum(sg);
        sbeta = wave_sum(sbeta);
    }
    if constexpr (HEAD) {
#pragma unroll
        for (int j = 0; j < 8; ++j) sw[j] = wave_sum(sw[j]);
    }
    if (lane == 0) {
        at(a.g_b, slot, y)[k] = sb;
        if constexpr (LN) {
            at(a.g_gamma, slot, y)[k] = sg;
            at(a.g_beta, slot, y)[k] = sbeta;
        }
        if constexpr (HEAD) {
            float* gw = at(a.g_W5, slot, y) + (long long)k * a.nout;
            for (int j = 0; j < a.nout; ++j) gw[j] = sw[j];
        }
    }
}

#define FQ_RS_LAUNCH(KPT, HEAD, grid, s, a) \
    hipLaunchKernelGGL((bwd_rowstats_kernel<HEAD, KPT>), grid, dim3(1024), 0, s, a)
void launch_bwd_rowstats(bool head, const BwdArgs& a, hipStream_t s) {
    const dim3 grid((a.M / 64) * a.ny * a.nz);
    if (head) {
        FQ_KPT_DISPATCH(a.H, FQ_RS_LAUNCH, true, grid, s, a)
    } else {
        FQ_KPT_DISPATCH(a.H, FQ_RS_LAUNCH, false, grid, s, a)
    }
}

void launch_bwd_cols(bool head, bool ln, const BwdArgs& a, hipStream_t s) {
    const dim3 grid((a.H / 4) * a.ny * a.nz), blk(256);
    if (head && ln) hipLaunchKernelGGL((bwd_cols_kernel<true, true>), grid, blk, 0, s, a);
    else if (head) hipLaunchKernelGGL((bwd_cols_kernel<true, false>), grid, blk, 0, s, a);
    else if (ln) hipLaunchKernelGGL((bwd_cols_kernel<false, true>), grid, blk, 0, s, a);
    else hipLaunchKernelGGL((bwd_cols_kernel<false, false>), grid, blk, 0, s, a);
}

// dq/da for the actor's Q term: the critic's first-layer input gradient,
// restricted to the action rows and summed over the ensemble.
template <int KPT>
__global__ __launch_bounds__(1024) void input_grad_kernel(const InGradArgs a) {
    const int ncb = a.M / 64;
    const int cb = blockIdx.x % ncb, z = blockIdx.x / ncb;
    const int slot = a.slots[z];
    const int lane = threadIdx.x & 63;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int m = cb * 64 + lane;
    const int n0 = w * KPT;
    float acc[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] = 0.f;
    for (int e = 0; e < a.E; ++e) {
        const float* __restrict__ W0 = at(a.W0, slot, e) + (long long)a.D * a.H + n0;
        const float* __restrict__ du = at(a.du0, slot, e) + a.off + m;
        float dv[KPT];
#pragma unroll
        for (int i = 0; i < KPT; ++i) dv[i] = du[(long long)(n0 + i) * a.ld];
#pragma unroll
        for (int j = 0; j < 8; ++j)
            if (j < a.A) {
#pragma unroll
                for (int i = 0; i < KPT; ++i) acc[j] += W0[(long long)j * a.H + i] * dv[i];
            }
    }
    __shared__ float red[CW][8][64];
#pragma unroll
    for (int j = 0; j < 8; ++j) red[w][j][lane] = acc[j];
    __syncthreads();
    const int t = threadIdx.x;
    if (t < a.A * 64) {
        const int j = t >> 6, l2 = t & 63;
        float v = 0.f;
#pragma unroll
        for (int q = 0; q < CW; ++q) v += red[q][j][l2];
        at(a.da, slot)[(long long)j * a.M + cb * 64 + l2] = v;
    }
}

#define FQ_IG_LAUNCH(KPT, grid, s, a) hipLaunchKernelGGL(input_grad_kernel<KPT>, grid, dim3(1024), 0, s, a)
void launch_input_grad(const InGradArgs& a, hipStream_t s) {
    const dim3 grid((a.M / 64) * a.nz);
    FQ_KPT_DISPATCH(a.H, FQ_IG_LAUNCH, grid, s, a)
}

// ==================================================== streamed MLP backward ==
// jax.grad through the MLP ([EXT] fql/utils/networks.py MLP)
// of one network in one launch (StreamBwdArgs, kernels.h).  Block = 16 columns
// x all 512 features of one (member, ensemble member), 8 waves.  Lane (li =
// lane & 15, lk = lane >> 4) of wave w owns features kq = 64w + 16q + li
// (q = 0..3) and columns 4lk + r (r = accumulator register), because the dX
// product is computed TRANSPOSED:
//   dh^T[m][k] = sum_j du^T[m][j] W_l[k][j]     (v_mfma_f32_16x16x4_f32)
// with A = du^T from LDS (one ds_read_b128 per k-step of 16 j) and B = rows of
// W_l streamed from L2 (lane float4 W[kq][16s + 4lk .. +3]: component c feeds
// MFMA c of k-step s, whose reduction slot lk is j = 16s + 4lk + c).  In this
// layout the LayerNorm column statistics take one 16-lane DPP row sum and the
// per-feature sums over the block's columns (parameter grads) two shuffles.
// float4 W^T loads in flight per lane: the LN (critic) kernel runs 2 blocks per CU
// (1024 blocks; <= 128 VGPRs), whose other block hides what a 4-deep ring does not;
// the one-step / BC kernels (256 blocks, 1 per CU) keep the 8-deep ring
template <bool LN> constexpr int sb_pf() { return LN ? 4 : 8; }

template <int CTRL>
DEV float dpp_mov(float v) {
    return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL, 0xF, 0xF, true));
}
// Sum over the 16 lanes of a DPP row (every lane gets the row's sum):
// quad_perm [1,0,3,2], quad_perm [2,3,0,1], row_half_mirror, row_mirror.
DEV float row16_sum(float v) {
    v += dpp_mov<0xB1>(v);
    v += dpp_mov<0x4E>(v);
    v += dpp_mov<0x141>(v);
    v += dpp_mov<0x140>(v);
    return v;
}
// Reduce-scatter over the 16 lanes of a DPP row: lane li of the row returns the sum of
// v[li] over the row's lanes (butterfly on li's bits 3..0: row_ror:8, row_half_mirror,
// quad_perm [2,3,0,1], quad_perm [1,0,3,2]; each level keeps the half named by the bit
// and adds the partner's other half). 45 VALU, no LDS.
DEV float row16_reduce_scatter(const float (&v)[16], int li) {
    const bool b3 = li & 8, b2 = li & 4, b1 = li & 2, b0 = li & 1;
    float a[8], b[4], c[2];
#pragma unroll
    for (int j = 0; j < 8; ++j) a[j] = (b3 ? v[j + 8] : v[j]) + dpp_mov<0x128>(b3 ? v[j] : v[j + 8]);
#pragma unroll
    for (int j = 0; j < 4; ++j) b[j] = (b2 ? a[j + 4] : a[j]) + dpp_mov<0x141>(b2 ? a[j] : a[j + 4]);
#pragma unroll
    for (int j = 0; j < 2; ++j) c[j] = (b1 ? b[j + 2] : b[j]) + dpp_mov<0x4E>(b1 ? b[j] : b[j + 2]);
    return (b0 ? c[1] : c[0]) + dpp_mov<0xB1>(b0 ? c[0] : c[1]);
}

bool stream_bwd_supported(int H, int L, int nout, int M, int Mg) {
    return H == EF_H && L >= 1 && L <= EF_MAX_LAYERS && nout >= 1 && nout <= 8 && M % EF_NC == 0 &&
           Mg % EF_NC == 0 && Mg <= M;
}

template <bool LN>
__global__ __launch_bounds__(EF_NW * 64, LN ? 4 : 1) void stream_bwd_kernel(const StreamBwdArgs g) {
    constexpr int H = EF_H, NC = EF_NC, NT = EF_NW * 64, PF = sb_pf<LN>();
    __shared__ __attribute__((aligned(16))) float slab[H * NC + 64];  // du_l [H][NC] (+ look-ahead slack)
    __shared__ __attribute__((aligned(16))) float scr[H * NC];         // head kernel W_L [H][nout]; then LN-grad products
    __shared__ float colred[2][EF_NW][NC];                            // LN column-stat partials per wave
    __shared__ float dos[8][NC];                                      // dout of the block's columns

    const int tiles = g.M / NC;
    const int total = tiles * g.ny * g.nz;
    const int bid = xcd_remap(blockIdx.x, total);
    const int tile = bid % tiles, yz = bid / tiles;
    const int y = yz % g.ny, z = yz / g.ny;
    const int slot = g.slots[z];
    const int c0 = tile * NC;
    const int tid = threadIdx.x, lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int li = lane & 15, lk = lane >> 4;
    const int L = g.L, nout = g.nout;
    const bool gp = c0 < g.Mg;  // the block's columns feed the parameter grads
    const float* __restrict__ P = g.params + (long long)slot * g.P + (long long)y * g.ens;
    const float* __restrict__ PTb = g.paramsT + (long long)slot * g.PT + (long long)y * g.ensT;
    const rsrc_t rT = make_rsrc(PTb, g.ensT);
    // element offsets of column c0 in the activation / stats / du buffers
    const long long so = (long long)slot * g.s_ss + (long long)y * g.s_sy + g.coff + c0;
    const long long sto = (long long)slot * g.st_ss + (long long)y * g.st_sy + g.coff + c0;
    const long long dso = (long long)slot * g.d_ss + (long long)y * g.d_sy + c0;
    float* __restrict__ part = gp ? g.part + ((long long)(slot * g.ny + y) * (g.Mg / NC) + tile) * g.NP : nullptr;
    // block-uniform buffer resources + 32-bit lane offsets for the per-layer accesses (no
    // 64-bit per-lane addresses to keep live across the layer loop)
    const rsrc_t rPart = make_rsrc(gp ? part : g.params, gp ? g.NP : 0);
    const rsrc_t rPe = make_rsrc(P, g.ens);
    // diagnostics only (null unless FQLPOP_PHASE_PROBE): wave 0's view of the phases
#ifdef FQ_PHASE_PROBE  // diagnostic build only (make PHASE=1)
    unsigned long long* const ph = g.phase != nullptr ? g.phase + (long long)blockIdx.x * SB_PHASE_STRIDE : nullptr;
    auto stamp = [&](int i) {
        if (ph != nullptr && tid == 0) ph[i] = __builtin_amdgcn_s_memrealtime();
    };
    if (ph != nullptr && tid == 0) {  // where the block ran: HW_ID (CU, SH, SE) and XCC_ID
        ph[SB_PHASE_STRIDE - 1] = (unsigned)__builtin_amdgcn_s_getreg(4 | (31 << 11));
        ph[SB_PHASE_STRIDE - 2] = (unsigned)__builtin_amdgcn_s_getreg(20 | (31 << 11));
    }
#else
    auto stamp = [](int) {};
#endif
    stamp(0);


    // epilogue inputs of layer l (u, LN stats, LN scale), loaded one layer ahead
    // so that their latency hides under the previous dX product
    float u[4][4], mu = 0.f, rs = 0.f;
    // (lane indices as arguments: inside the layer loop they come from an opaque copy of
    // tid, so that per-lane addresses are recomputed where they are used instead of
    // being hoisted out of the loop and spilled: every spill reload was a vmcnt(0) that
    // also waited for the ring refills and the du stores in flight)
    auto load_epi = [&](int l, int tid_, int li_, int lk_) {
        const rsrc_t rU = make_rsrc(g.U[l] + so, (long long)H * g.ld_s);
        const int vo = ((64 * w + 16 * lk_) * g.ld_s + li_) * 4;
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
            for (int c = 0; c < 4; ++c) u[r][c] = bload1(rU, vo, (4 * r + c) * g.ld_s * 4);
        if constexpr (LN) {
            mu = bload1(make_rsrc(g.MU[l] + sto, NC), li_ * 4, 0);
            rs = bload1(make_rsrc(g.RS[l] + sto, NC), li_ * 4, 0);
        }
    };
    // W^T ring: the first PF k-steps of the first dX product (W_{L-1}^T), issued after the
    // epilogue loads as in the layer loop, so that the loop head waits for the epilogue
    // loads only (vmcnt(PF)) instead of for everything in flight (a vmcnt(0) that also
    // waited for the ring refills of the next product, every layer)
    const int lo = lk * H + 64 * w + 4 * li;
    float4 ring[PF];
    auto load_first = [&]() {
        load_epi(L - 1, tid, li, lk);
        const int wf = L > 1 ? (int)g.wt_off[L - 1] : 0;
#pragma unroll
        for (int p = 0; p < PF; ++p) ring[p] = bload4(rT, wf + 4 * p * H + lo);
    };
    // lane layout (as ef_kloop's accumulators): column li, features f = 64w + 16lk + 4r + c
    // last hidden layer: dh = W_L dout (nout <= 8, VALU)
    float dh[4][4];  // [r][c]
    const int w5 = (LN ? 3 : 1) * L * H;  // head kernel grads in the partials
    // The head's operands are loaded before the first layer's epilogue inputs and ring: loads
    // complete in order, so a wait for one issued after those would wait for them too (the
    // head is on the block's critical path, the ring and epilogue inputs are needed later)
    if (nout == 1) {
        // (the critic: a scalar head) no LDS staging: W_L[f] as float4 runs, this lane's dout,
        // and G_{L-1} in the accumulator layout, all issued in one batch (one memory round
        // trip, no barrier); the head kernel grads sum_col G_{L-1}[f][col] dout[col] by the
        // DPP reduce-scatter over the column lanes (lane li ends with feature 64w + 16lk + li =
        // tid)
        const rsrc_t rH = make_rsrc(P + g.w_off[L], (long long)H);
        float4 wl[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) wl[r] = bload4(rH, 64 * w + 16 * lk + 4 * r);
        const float dv = g.dout[(long long)slot * g.dout_ss + (long long)y * g.dout_sy + c0 + li];
        float gh[16];
        if (gp) {
            const rsrc_t rG = make_rsrc(g.Ghead + so, (long long)H * g.ld_s);
            const int vo = ((64 * w + 16 * lk) * g.ld_s + li) * 4;
#pragma unroll
            for (int e = 0; e < 16; ++e) gh[e] = bload1(rG, vo, e * g.ld_s * 4);
        }
        load_first();
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const float wv[4] = {wl[r].x, wl[r].y, wl[r].z, wl[r].w};
#pragma unroll
            for (int c = 0; c < 4; ++c) dh[r][c] = mul_rn(wv[c], dv);
        }
        if (gp) {
#pragma unroll
            for (int e = 0; e < 16; ++e) gh[e] = mul_rn(gh[e], dv);
            bstore1(rPart, row16_reduce_scatter(gh, li), tid * 4, w5 * 4);
        }
    } else {
        // dout of the block's columns, row tid (= feature, NT = H) of the head kernel W_L
        // [H][nout] (nout <= 8), zero-padded to 8 outputs, and this thread's G_{L-1} row (head
        // kernel grad partials, thread = feature), one batch
        static_assert(NT == H, "one thread per feature");
        const bool dl = tid < 8 * NC;
        float dov = 0.f;
        if (dl && tid / NC < nout) {
            const int j = tid / NC, col = tid % NC;
            dov = g.dout[(long long)slot * g.dout_ss + (long long)y * g.dout_sy + (long long)j * g.ld_o + c0 + col];
        }
        const rsrc_t rH = make_rsrc(P + g.w_off[L], (long long)H * nout);
        float hv[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) hv[j] = bload1(rH, (tid * nout + j) * 4, 0);
        float gv[NC];
        if (gp) {
            const rsrc_t rG = make_rsrc(g.Ghead + so, (long long)H * g.ld_s);
#pragma unroll
            for (int q = 0; q < NC / 4; ++q) {
                const float4 t4 = bload4(rG, tid * g.ld_s + 4 * q);
                gv[4 * q] = t4.x; gv[4 * q + 1] = t4.y; gv[4 * q + 2] = t4.z; gv[4 * q + 3] = t4.w;
            }
        }
        load_first();
        if (dl) dos[tid / NC][tid % NC] = dov;  // 0 for outputs j >= nout
#pragma unroll
        for (int j = 0; j < 8; ++j) hv[j] = j < nout ? hv[j] : 0.f;
        reinterpret_cast<float4*>(scr)[2 * tid] = float4{hv[0], hv[1], hv[2], hv[3]};
        reinterpret_cast<float4*>(scr)[2 * tid + 1] = float4{hv[4], hv[5], hv[6], hv[7]};
        stamp(40);
        __syncthreads();
        stamp(41);
        if (gp) {
            for (int j = 0; j < nout; ++j) {
                float v = 0.f;
#pragma unroll
                for (int col = 0; col < NC; ++col) v = fmaf(gv[col], dos[j][col], v);
                part[w5 + tid * nout + j] = v;
            }
        }
        stamp(42);
        // dh = W_L dout: branch-free over the 8 padded outputs (the padding adds exact zeros),
        // every LDS read of the 16 features issued before the first FMA
        float dj[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) dj[j] = dos[j][li];
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
            for (int c = 0; c < 4; ++c) {
                const int f = 64 * w + 16 * lk + 4 * r + c;
                const float4 wa = reinterpret_cast<const float4*>(scr)[2 * f];
                const float4 wb = reinterpret_cast<const float4*>(scr)[2 * f + 1];
                const float wv[8] = {wa.x, wa.y, wa.z, wa.w, wb.x, wb.y, wb.z, wb.w};
                float s = 0.f;
#pragma unroll
                for (int j = 0; j < 8; ++j) s = fmaf(wv[j], dj[j], s);
                dh[r][c] = s;
            }
        __syncthreads();  // scr (head kernel image) is reused by the first epilogue
        stamp(43);
    }
    // parameter-grad partials, thread = feature: sums over the block's 16 columns of an LDS image
    auto row_sum = [&](const float* a, int tid_) {
        const float4* row = reinterpret_cast<const float4*>(&a[tid_ * NC]);
        float sv = 0.f;
#pragma unroll
        for (int q = 0; q < NC / 4; ++q) {
            const float4 t4 = row[q];
            sv += t4.x + t4.y + t4.z + t4.w;
        }
        return sv;
    };
    for (int l = L - 1; l >= 0; --l) {
        // (the critic's LN variant only: the actor backward has no spills, and the opaque
        // lane indices slowed its in-step launch 2x beside the flow)
        // (the lane id from mbcnt, not from tid: a kept tid was itself spilled, and its reload
        // at the loop head was a vmcnt(0))
        const int lane_l = LN ? lane_id_asm() : lane;
        const int tid_l = 64 * w + lane_l, li_l = lane_l & 15, lk_l = lane_l >> 4;
        // this lane's element (feature 64w + 16lk, column li_l) of an [H][NC] LDS image; element
        // (r, c) is at + (4r + c) * NC (ds_write immediate offsets, one address VGPR)
        float* const slab_l = slab + (64 * w + 16 * lk_l) * NC + li_l;
        float* const scr_l = scr + (64 * w + 16 * lk_l) * NC + li_l;
        const int pi = 2 + 5 * (L - 1 - l);
        stamp(pi);
        // ---- du_l from dh = dL/dG_l (GELU', LayerNorm backward), in place in dh ----
        if constexpr (LN) {
            // this lane's 16 LN scales (features 64w + 16lk + 4r + c), in flight during the
            // DPP reduction and the GELU math below
            float4 gq[4];
#pragma unroll
            for (int r = 0; r < 4; ++r) gq[r] = bload4(rPe, (int)g.g_off[l] + 64 * w + 16 * lk_l + 4 * r);
            // LN bias grads: feature 64w + 16lk + li = tid_l, sum over the block's columns of
            // dh (DPP reduce-scatter over the column lanes; done before xhat is live)
            if (gp) bstore1(rPart, row16_reduce_scatter(reinterpret_cast<const float(&)[16]>(dh), li_l), tid_l * 4,
                            (2 * L + l) * H * 4);
            // pass 1: xhat, GELU' (kept in u); dh * xhat to LDS (LN scale grads, thread =
            // feature); the column partials of dh*gamma and dh*gamma*xhat. No slab write and
            // no barrier before the column stats: the previous product needs no barrier after it
            float xh[4][4], s1 = 0.f, s2 = 0.f;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const float gr[4] = {gq[r].x, gq[r].y, gq[r].z, gq[r].w};
#pragma unroll
                for (int c = 0; c < 4; ++c) {
                    float gv, gpr;
                    gelu_and_grad_fast(u[r][c], gv, gpr);
                    u[r][c] = gpr;
                    xh[r][c] = (gv - mu) * rs;
                    scr_l[(4 * r + c) * NC] = mul_rn(dh[r][c], xh[r][c]);
                    dh[r][c] = ln_bwd_acc(dh[r][c], gr[c], xh[r][c], s1, s2);  // dh * gamma from here on
                }
            }
            s1 = lk_sum(s1);
            s2 = lk_sum(s2);
            if (lk_l == 0) {
                colred[0][w][li_l] = s1;
                colred[1][w][li_l] = s2;
            }
            stamp(pi + 1);
            __syncthreads();  // colred, scr visible
            stamp(pi + 2);
            if (gp) bstore1(rPart, row_sum(scr, tid_l), tid_l * 4, (L + l) * H * 4);  // LN scale: sum dh * xhat
            float c1 = 0.f, c2 = 0.f;
#pragma unroll
            for (int q8 = 0; q8 < EF_NW; ++q8) {
                c1 += colred[0][q8][li_l];
                c2 += colred[1][q8][li_l];
            }
            c1 = c1 / (float)H;
            c2 = c2 / (float)H;
            // pass 2: du = rstd (dh gamma - c1 - xhat c2) gelu'(u)
#pragma unroll
            for (int r = 0; r < 4; ++r)
#pragma unroll
                for (int c = 0; c < 4; ++c) dh[r][c] = ln_bwd_du(dh[r][c], xh[r][c], c1, c2, rs, u[r][c]);
        } else {
#pragma unroll
            for (int r = 0; r < 4; ++r)
#pragma unroll
                for (int c = 0; c < 4; ++c) dh[r][c] *= gelu_grad_fast(u[r][c]);
        }
        if (gp || g.da == nullptr) {
            // du_l is the dW GEMMs' operand (grad columns) or input_grad_kernel's; the dQ/da
            // columns of a fused backward need it only in LDS
            const rsrc_t rD = make_rsrc(g.DU[l] + dso, (long long)H * g.ld_d);
            const int vo = ((64 * w + 16 * lk_l) * g.ld_d + li_l) * 4;
#pragma unroll
            for (int r = 0; r < 4; ++r)
#pragma unroll
                for (int c = 0; c < 4; ++c) {
                    bstore1(rD, dh[r][c], vo, (4 * r + c) * g.ld_d * 4);
                    slab_l[(4 * r + c) * NC] = dh[r][c];
                }
        } else {
#pragma unroll
            for (int r = 0; r < 4; ++r)
#pragma unroll
                for (int c = 0; c < 4; ++c) slab_l[(4 * r + c) * NC] = dh[r][c];
        }
        __syncthreads();
        stamp(pi + 3);
        if (gp) bstore1(rPart, row_sum(slab, tid_l), tid_l * 4, l * H * 4);  // bias: sum du
        if (l == 0 && g.da != nullptr && !gp) {
            // dQ/da for the actor's Q-loss columns (replaces input_grad_kernel): output (j, col)
            // = thread & 127, feature quarter = thread >> 7, then a fixed-order fold in scr
            // W_0's action rows D0 .. D0 + na - 1 (na H <= 8 NT floats) staged into scr (free
            // after the slab barrier) with one batch of loads, instead of one dependent L2
            // round trip per 8 features in the loop below
            const int o = tid_l & 127, q = tid_l >> 7, j = o >> 4, col = o & 15;
            float* const wa = scr + 512;
            {
                const rsrc_t rA = make_rsrc(P + g.w_off[0] + (long long)g.D0 * H, (long long)g.na * H);
                float t[8];
#pragma unroll
                for (int i = 0; i < 8; ++i) t[i] = bload1(rA, (tid_l + i * NT) * 4, 0);  // past na H: 0
#pragma unroll
                for (int i = 0; i < 8; ++i)
                    if (tid_l + i * NT < g.na * H) wa[tid_l + i * NT] = t[i];
            }
            __syncthreads();
            float s = 0.f;
            if (j < g.na) {
                const float* const wr = wa + j * H;
#pragma unroll 8
                for (int f = q * (H / 4); f < (q + 1) * (H / 4); ++f) s = fmaf(wr[f], slab[f * NC + col], s);
            }
            scr[q * 128 + o] = s;
            __syncthreads();
            if (tid_l < g.na * NC)
                g.da[(long long)slot * g.da_ss + (long long)y * g.da_sy + (long long)(tid_l >> 4) * g.ld_da +
                     (c0 - g.Mg) + (tid_l & 15)] = scr[tid_l] + scr[128 + tid_l] + scr[256 + tid_l] + scr[384 + tid_l];
        }
        if (l == 0) break;

        // ---- dh_{l-1} = W_l du_l = (W_l^T)^T du_l: the forward k-loop on W_l^T ----
        load_epi(l - 1, tid_l, li_l, lk_l);
        f32x4 acc[4];
#pragma unroll
        for (int c = 0; c < 4; ++c) acc[c] = f32x4{0.f, 0.f, 0.f, 0.f};
        const int wn = (int)g.wt_off[l >= 2 ? l - 1 : l];  // next product's W^T (l-1 >= 1), else a harmless re-load
        ef_kloop<PF>(acc, ring, rT, slab, H / 4, (int)g.wt_off[l], wn, lk_l * H + 64 * w + 4 * li_l, lk_l, li_l);
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
            for (int c = 0; c < 4; ++c) dh[r][c] = acc[c][r];
        stamp(pi + 4);
        // the actor variant writes the slab right away (du of the next layer): wait for every
        // wave's product; the LN variant's next LDS writes (scr, colred) are not read by the
        // product, and its slab write follows the next barrier
        if constexpr (!LN) __syncthreads();
    }
    stamp(1);
}

void launch_stream_bwd(bool ln, const StreamBwdArgs& a, hipStream_t s) {
    const dim3 grid((a.M / EF_NC) * a.ny * a.nz), block(EF_NW * 64);
    if (ln) hipLaunchKernelGGL((stream_bwd_kernel<true>), grid, block, 0, s, a);
    else hipLaunchKernelGGL((stream_bwd_kernel<false>), grid, block, 0, s, a);
}

// ============================================ split streamed backward (small populations) ==
// stream_bwd_kernel with each 16-column tile computed by a cluster of F = 2, 4 or 8 blocks
// (the split streamed forward's scheme and hand-off): block f owns the 512/F features
// [fb, fb + 512/F) of every dh_l / du_l; its 4 waves run TPW = 8/F 16x16 tiles of the dX
// products over the full K (the unsplit k order, W_l^T rows as the A fragments, du_l from the
// fragment-order slab), so every value is the unsplit fp32 chain.  The sums over features
// (LayerNorm backward column statistics) and over columns (bias / LN / head-kernel grad
// partials) are re-done from LDS images of the block's features in the unsplit order and
// lane layout ("unsplit wave" w = f TPW + q), so the results are bit-identical to
// stream_bwd_kernel's.  Hand-offs per layer: the LN column partials (LN only), then du_l
// (the next product's B operand).  The critic's dQ/da (columns >= Mg, layer 0) is computed
// by the cluster's last arriver from the staged du_0, in the unsplit order.
bool split_bwd_supported(int H, int L, int nout, int M, int Mg) {
    return H == EF_H && L >= 2 && L <= EF_MAX_LAYERS && nout >= 1 && nout <= 8 && M % EF_NC == 0 &&
           Mg % EF_NC == 0 && Mg <= M;
}

template <bool LN, int TPW>
__global__ __launch_bounds__(SP_NT, 2) void split_bwd_kernel(const StreamBwdArgs g, const SplitSync sync) {
    constexpr int H = EF_H, NC = EF_NC, F = 8 / TPW, FB = H / F;
    __shared__ __attribute__((aligned(16))) float slab[H * NC + 256];  // du_l, fragment order (+ slack)
    __shared__ __attribute__((aligned(16))) float ta[FB * NC];          // the block's dh (raw), then du
    __shared__ __attribute__((aligned(16))) float tb[FB * NC];          // the block's xhat (LN)
    __shared__ float cst[2][NC];                                        // c1, c2 per column
    __shared__ float dos[8][NC];
    __shared__ unsigned bc[2];

    const int tiles = g.M / NC, clusters = tiles * g.ny * g.nz;
    const int ticket = sp_begin(sync, clusters, bc);
    const unsigned gen = __builtin_amdgcn_readfirstlane(bc[1]);
    const int cl = ticket / F, f = ticket % F, fb = f * FB;
    const int tl = __builtin_amdgcn_readfirstlane(cl % tiles), yz = cl / tiles;
    const int y = __builtin_amdgcn_readfirstlane(yz % g.ny), z = __builtin_amdgcn_readfirstlane(yz / g.ny);
    const int slot = __builtin_amdgcn_readfirstlane(g.slots[z]);
    const int c0 = tl * NC;
    const int tid = threadIdx.x, lane = tid & 63;
    const int q = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int li = lane & 15, lk = lane >> 4;
    const int L = g.L, nout = g.nout;
    const bool gp = c0 < g.Mg;
    const float* __restrict__ P = g.params + (long long)slot * g.P + (long long)y * g.ens;
    const float* __restrict__ PTb = g.paramsT + (long long)slot * g.PT + (long long)y * g.ensT;
    const rsrc_t rT = make_rsrc(PTb, g.ensT);
    const long long so = (long long)slot * g.s_ss + (long long)y * g.s_sy + g.coff + c0;
    const long long sto = (long long)slot * g.st_ss + (long long)y * g.st_sy + g.coff + c0;
    const long long dso = (long long)slot * g.d_ss + (long long)y * g.d_sy + c0;
    float* __restrict__ part = gp ? g.part + ((long long)(slot * g.ny + y) * (g.Mg / NC) + tl) * g.NP : nullptr;
    unsigned long long* const X = sync.xch + (long long)cl * SP_CLUSTER_GRANULES;
    const rsrc_t rX = __builtin_amdgcn_make_buffer_rsrc((void*)X, (short)0, (int)(SP_CLUSTER_GRANULES * 8), 0x00020000);
    unsigned phase = 0;
    const int w5 = (LN ? 3 : 1) * L * H;
    // lane layout: tile t, reg r -> feature fb + fl, fl = 16 TPW q + TPW (4 lk + r) + t, column li
    auto flo = [&](int r, int t) { return 16 * TPW * q + TPW * (4 * lk + r) + t; };

    // ---- head: dh_{L-1} = W_L dout (own features), head-kernel grad partials ----
    float dh[4][TPW];
    if (nout == 1) {
        const float dv = g.dout[(long long)slot * g.dout_ss + (long long)y * g.dout_sy + c0 + li];
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
            for (int t = 0; t < TPW; ++t) dh[r][t] = mul_rn(P[g.w_off[L] + fb + flo(r, t)], dv);
        if (gp && q < TPW) {
            // unsplit wave f TPW + q: G_{L-1}[64 w + 16 lk + e][li] dout, DPP reduce-scatter over the columns
            const int w8 = f * TPW + q;
            float gh[16];
            const float* Gp = g.Ghead + so;
#pragma unroll
            for (int e = 0; e < 16; ++e) gh[e] = Gp[(long long)(64 * w8 + 16 * lk + e) * g.ld_s + li];
#pragma unroll
            for (int e = 0; e < 16; ++e) gh[e] = mul_rn(gh[e], dv);
            part[w5 + 64 * w8 + 16 * lk + li] = row16_reduce_scatter(gh, li);
        }
    } else {
        if (tid < 8 * NC) {
            const int j = tid / NC, col = tid % NC;
            dos[j][col] = j < nout ? g.dout[(long long)slot * g.dout_ss + (long long)y * g.dout_sy +
                                            (long long)j * g.ld_o + c0 + col] : 0.f;
        }
        __syncthreads();
        float dj[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) dj[j] = dos[j][li];
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
            for (int t = 0; t < TPW; ++t) {
                const int fe = fb + flo(r, t);
                float wv[8];
#pragma unroll
                for (int j = 0; j < 8; ++j) wv[j] = j < nout ? P[g.w_off[L] + fe * nout + j] : 0.f;
                float s = 0.f;
#pragma unroll
                for (int j = 0; j < 8; ++j) s = fmaf(wv[j], dj[j], s);
                dh[r][t] = s;
            }
        if (gp && tid < FB) {
            const int fe = fb + tid;
            float gv[NC];
            const float* Gr = g.Ghead + so + (long long)fe * g.ld_s;
#pragma unroll
            for (int c = 0; c < NC; ++c) gv[c] = Gr[c];
            for (int j = 0; j < nout; ++j) {
                float v = 0.f;
#pragma unroll
                for (int col = 0; col < NC; ++col) v = fmaf(gv[col], dos[j][col], v);
                part[w5 + fe * nout + j] = v;
            }
        }
    }
    // row sum over the 16 columns of an [FB][NC] LDS image, stream_bwd_kernel's order
    auto row_sum = [&](const float* a, int fl) {
        const float4* row = reinterpret_cast<const float4*>(&a[fl * NC]);
        float sv = 0.f;
#pragma unroll
        for (int qq = 0; qq < NC / 4; ++qq) {
            const float4 t4 = row[qq];
            sv += t4.x + t4.y + t4.z + t4.w;
        }
        return sv;
    };

    float4 ring[sp_pf<TPW>()];
    const int lo = lk * H + fb + 16 * TPW * q + TPW * li;
#pragma unroll
    for (int p = 0; p < sp_pf<TPW>(); ++p) ring[p] = sp_aload<TPW>(rT, (int)g.wt_off[L - 1] + 4 * p * H + lo);
    for (int l = L - 1; l >= 0; --l) {
        // epilogue inputs of layer l (own features)
        float u[4][TPW];
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
            for (int t = 0; t < TPW; ++t) u[r][t] = g.U[l][so + (long long)(fb + flo(r, t)) * g.ld_s + li];
        if constexpr (LN) {
            const float mu = g.MU[l][sto + li], rs = g.RS[l][sto + li];
            float xh[4][TPW], gpr[4][TPW];
#pragma unroll
            for (int r = 0; r < 4; ++r)
#pragma unroll
                for (int t = 0; t < TPW; ++t) {
                    float gv;
                    gelu_and_grad_fast(u[r][t], gv, gpr[r][t]);
                    xh[r][t] = (gv - mu) * rs;
                    ta[flo(r, t) * NC + li] = dh[r][t];
                    tb[flo(r, t) * NC + li] = xh[r][t];
                }
            __syncthreads();
            const unsigned tag = sp_tag(gen, phase);
            if (q < TPW) {
                // unsplit wave w8 = f TPW + q: LN bias grads (reduce-scatter of dh), column partials of
                // dh gamma and dh gamma xhat (16 consecutive features per lane, then the lk sum)
                const int w8 = f * TPW + q;
                float v[16];
#pragma unroll
                for (int e = 0; e < 16; ++e) v[e] = ta[(64 * q + 16 * lk + e) * NC + li];
                if (gp) part[(2 * L + l) * H + 64 * w8 + 16 * lk + li] = row16_reduce_scatter(v, li);
                float s1 = 0.f, s2 = 0.f;
#pragma unroll
                for (int e = 0; e < 16; ++e)
                    (void)ln_bwd_acc(v[e], P[g.g_off[l] + 64 * w8 + 16 * lk + e], tb[(64 * q + 16 * lk + e) * NC + li], s1,
                                     s2);
                s1 = lk_sum(s1);
                s2 = lk_sum(s2);
                if (lk == 0) {
                    gx_put(X, SP_G_LP + ((l & 1) * 8 + w8) * 2 * NC + li, s1, tag);
                    gx_put(X, SP_G_LP + ((l & 1) * 8 + w8) * 2 * NC + NC + li, s2, tag);
                }
            }
            if (gp && tid < FB) {
                // LN scale grads: sum over the columns of dh * xhat (thread = feature)
                float sv = 0.f;
                const float4* ra = reinterpret_cast<const float4*>(&ta[tid * NC]);
                const float4* rb = reinterpret_cast<const float4*>(&tb[tid * NC]);
#pragma unroll
                for (int qq = 0; qq < NC / 4; ++qq) {
                    const float4 a4 = ra[qq], b4 = rb[qq];
                    sv += mul_rn(a4.x, b4.x) + mul_rn(a4.y, b4.y) + mul_rn(a4.z, b4.z) + mul_rn(a4.w, b4.w);
                }
                part[(L + l) * H + fb + tid] = sv;
            }
            ++phase;
            if (tid < NC) {
                float c1 = 0.f, c2 = 0.f;
#pragma unroll
                for (int w8 = 0; w8 < EF_NW; ++w8) {
                    c1 += gx_get(X, SP_G_LP + ((l & 1) * 8 + w8) * 2 * NC + tid, tag, sync);
                    c2 += gx_get(X, SP_G_LP + ((l & 1) * 8 + w8) * 2 * NC + NC + tid, tag, sync);
                }
                cst[0][tid] = c1 / (float)H;
                cst[1][tid] = c2 / (float)H;
            }
            __syncthreads();
            const float c1 = cst[0][li], c2 = cst[1][li];
#pragma unroll
            for (int r = 0; r < 4; ++r)
#pragma unroll
                for (int t = 0; t < TPW; ++t) {
                    const float d = mul_rn(dh[r][t], P[g.g_off[l] + fb + flo(r, t)]);  // dh gamma
                    dh[r][t] = ln_bwd_du(d, xh[r][t], c1, c2, rs, gpr[r][t]);
                }
        } else {
#pragma unroll
            for (int r = 0; r < 4; ++r)
#pragma unroll
                for (int t = 0; t < TPW; ++t) dh[r][t] *= gelu_grad_fast(u[r][t]);
        }
        // du_l: DU (dW operand), the LDS image (bias grads), the exchange (next product / dQ/da)
        const bool need_x = l > 0 || (g.da != nullptr && !gp);
        const unsigned tag = sp_tag(gen, phase);
        __syncthreads();  // ta is free (LN: read above)
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
            for (int t = 0; t < TPW; ++t) {
                const int fl = flo(r, t);
                if (gp || g.da == nullptr) g.DU[l][dso + (long long)(fb + fl) * g.ld_d + li] = dh[r][t];
                ta[fl * NC + li] = dh[r][t];
                if (need_x) gx_put(X, (l & 1) * SP_XG + sp_fidx(fb + fl, li), dh[r][t], tag);
            }
        __syncthreads();
        if (gp && tid < FB) part[l * H + fb + tid] = row_sum(ta, tid);  // bias: sum du
        if (!need_x) break;
        ++phase;
        if (l == 0) {
            // dQ/da of the Q-loss columns by the cluster's last arriver (stream_bwd_kernel's order:
            // 4 feature quarters of W_0[D0 + j][f] du_0[f][col], then their sum in quarter order)
            if (!sp_last(sync, cl, F, bc)) break;
            gx_stage(rX, 0, tag, slab, sync);  // du_0 (exchange parity 0)
            __syncthreads();
            float* const scr = tb;  // [4 quarters][128] (FB NC >= 1024 floats)
#pragma unroll
            for (int qq = 0; qq < 2; ++qq) {
                const int o = tid & 127, qd = (tid >> 7) + 2 * qq, j = o >> 4, col = o & 15;
                float sacc = 0.f;
                if (j < g.na) {
                    const float* wr = P + g.w_off[0] + (long long)(g.D0 + j) * H;
#pragma unroll 8
                    for (int fe = qd * (H / 4); fe < (qd + 1) * (H / 4); ++fe)
                        sacc = fmaf(wr[fe], slab[sp_fidx(fe, col)], sacc);
                }
                scr[qd * 128 + o] = sacc;
            }
            __syncthreads();
            if (tid < g.na * NC)
                g.da[(long long)slot * g.da_ss + (long long)y * g.da_sy + (long long)(tid >> 4) * g.ld_da + (c0 - g.Mg) +
                     (tid & 15)] = scr[tid] + scr[128 + tid] + scr[256 + tid] + scr[384 + tid];
            break;
        }
        // ---- dh_{l-1} = W_l du_l over the staged du_l (all 512 features) ----
        gx_stage(rX, (l & 1) * SP_XG, tag, slab, sync);
        __syncthreads();
        f32x4 acc[TPW];
#pragma unroll
        for (int t = 0; t < TPW; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
        const int wn = (int)g.wt_off[l >= 2 ? l - 1 : l];
        sp_kloop<TPW>(acc, ring, rT, slab, H / 4, (int)g.wt_off[l], wn, lo, lane);
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
            for (int t = 0; t < TPW; ++t) dh[r][t] = acc[t][r];
    }
    sp_end(sync, clusters, clusters * F, bc);
}

void launch_split_bwd(bool ln, int F, const StreamBwdArgs& a, const SplitSync& sy, hipStream_t s) {
    const dim3 grid((a.M / EF_NC) * a.ny * a.nz * F), block(SP_NT);
#define FQ_SPB(LNV, T) hipLaunchKernelGGL((split_bwd_kernel<LNV, T>), grid, block, 0, s, a, sy)
    switch (F) {
        case 8: if (ln) FQ_SPB(true, 1); else FQ_SPB(false, 1); break;
        case 4: if (ln) FQ_SPB(true, 2); else FQ_SPB(false, 2); break;
        default: FQ_SPB(false, 4); break;  // (the LN backward runs 4 or 8 blocks per tile)
    }
#undef FQ_SPB
}

// Fold the per-tile partials of stream_bwd into the grads (fixed tile order:
// deterministic).  Index layout: stream_bwd_np (kernels.h).
__global__ __launch_bounds__(256) void colsum_reduce_kernel(const ColsumArgs a) {
    const int p = blockIdx.x * 256 + threadIdx.x;
    const int y = blockIdx.y, z = blockIdx.z;
    if (p >= a.NP) return;
    const int slot = a.slots[z];
    const float* __restrict__ src = a.part + (long long)(slot * a.ny + y) * a.tiles * a.NP + p;
    // fixed tile order; 8 loads in flight per batch (one load per iteration waited on each
    // partial separately)
    float s = 0.f;
    int t = 0;
    for (; t + 8 <= a.tiles; t += 8) {
        float v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) v[u] = src[(long long)(t + u) * a.NP];
#pragma unroll
        for (int u = 0; u < 8; ++u) s += v[u];
    }
    for (; t < a.tiles; ++t) s += src[(long long)t * a.NP];
    const int LH = a.L * a.H;
    const int reg = p < LH ? 0 : !a.ln ? 3 : p < 2 * LH ? 1 : p < 3 * LH ? 2 : 3;
    const int pr = reg == 3 ? p - (a.ln ? 3 : 1) * LH : p - reg * LH;
    long long off = a.w5_off + pr;
    if (reg < 3) {
        const int l = pr / a.H, k = pr % a.H;
#pragma unroll
        for (int i = 0; i < EF_MAX_LAYERS; ++i)
            if (i == l) off = (reg == 0 ? a.b_off[i] : reg == 1 ? a.g_off[i] : a.be_off[i]) + k;
    }
    a.grads[(long long)slot * a.P + (long long)y * a.ens + off] = s;
}

void launch_colsum_reduce(const ColsumArgs& a, hipStream_t s) {
    const dim3 grid((a.NP + 255) / 256, a.ny, a.nz);
    hipLaunchKernelGGL(colsum_reduce_kernel, grid, dim3(256), 0, s, a);
}

// W^T copies of the hidden kernels (64 x 64 tiles through LDS).
__global__ __launch_bounds__(256) void transpose_kernel(const TransposeArgs a) {
    __shared__ float t[64][65];
    const int H = a.H, tpr = H / 64;
    const int tr = blockIdx.x / tpr, tc = blockIdx.x % tpr;  // source tile rows k, cols j
    const int mi = blockIdx.y, z = blockIdx.z;
    const int slot = a.slots ? a.slots[z] : z;
    long long so = 0, dof = 0;
#pragma unroll
    for (int i = 0; i < TR_MAX; ++i)
        if (i == mi) { so = a.src_off[i]; dof = a.dst_off[i]; }
    const float* __restrict__ src = a.src + (long long)slot * a.src_ss + so;
    float* __restrict__ dst = a.dst + (long long)slot * a.dst_ss + dof;
    const int k0 = tr * 64, j0 = tc * 64;
#pragma unroll
    for (int p = 0; p < 4; ++p) {
        const int idx = threadIdx.x + 256 * p, r = idx / 16, c4 = idx % 16;
        const float4 v = *reinterpret_cast<const float4*>(src + (long long)(k0 + r) * H + j0 + 4 * c4);
        t[r][4 * c4] = v.x; t[r][4 * c4 + 1] = v.y; t[r][4 * c4 + 2] = v.z; t[r][4 * c4 + 3] = v.w;
    }
    __syncthreads();
#pragma unroll
    for (int p = 0; p < 4; ++p) {
        const int idx = threadIdx.x + 256 * p, r = idx / 16, c4 = idx % 16;  // dst row j0 + r, cols k0 + 4c4..
        *reinterpret_cast<float4*>(dst + (long long)(j0 + r) * H + k0 + 4 * c4) =
            float4{t[4 * c4][r], t[4 * c4 + 1][r], t[4 * c4 + 2][r], t[4 * c4 + 3][r]};
    }
}

void launch_transpose(const TransposeArgs& a, hipStream_t s) {
    if (a.n_mats == 0 || a.nz == 0) return;
    const dim3 grid((a.H / 64) * (a.H / 64), a.n_mats, a.nz);
    hipLaunchKernelGGL(transpose_kernel, grid, dim3(256), 0, s, a);
}

// =============================================================== RNG =======
// Philox4x32-10 (Salmon et al. 2011), counter = (row, step, salt, word).
DEV void philox4x32_10(uint32_t c[4], uint32_t k0, uint32_t k1) {
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        const uint32_t hi0 = __umulhi(0xD2511F53u, c[0]), lo0 = 0xD2511F53u * c[0];
        const uint32_t hi1 = __umulhi(0xCD9E8D57u, c[2]), lo1 = 0xCD9E8D57u * c[2];
        const uint32_t n0 = hi1 ^ c[1] ^ k0, n2 = hi0 ^ c[3] ^ k1;
        c[0] = n0; c[1] = lo1; c[2] = n2; c[3] = lo0;
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
}

DEV float u01_open_closed(uint32_t x) { return ((x >> 8) + 1u) * (1.0f / 16777216.0f); }  // (0,1]
DEV float u01(uint32_t x) { return (x >> 8) * (1.0f / 16777216.0f); }                    // [0,1)

// Normals n[0..cnt) for (row, step, salt), words 1.. of the Philox stream.
DEV void philox_normals(float* n, int cnt, uint64_t seed, uint32_t row, uint32_t step, uint32_t salt) {
    for (int i = 0; i < cnt; i += 2) {
        uint32_t c[4] = {row, step, salt, 1u + (uint32_t)(i >> 1)};
        philox4x32_10(c, (uint32_t)seed, (uint32_t)(seed >> 32));
        const float r = sqrtf(-2.0f * logf(u01_open_closed(c[0])));
        float sv, cv;
        sincosf(6.283185307179586f * u01(c[1]), &sv, &cv);
        n[i] = r * cv;
        if (i + 1 < cnt) n[i + 1] = r * sv;
    }
}

// ============================================================ sampling =====
// Minibatch draw (uniform with replacement, [EXT] Dataset.sample) + noise
// draws + assembly of every network's first-layer input (feature-major
// concatenation = stacking row blocks).  Injected mode reads batch/noise from
// a packed staging buffer instead (parity tests).
// Thread = (minibatch row b, part p of SP): every part draws the row index and
// t (Philox word 0), then part p writes the features k = p mod SP, the Philox
// normal pairs q = p mod SP and action j = p.  Values are identical to a
// one-thread-per-row draw (same counters).
constexpr int SP = 8;
__global__ __launch_bounds__(256) void sample_kernel(const SampleArgs a) {
    constexpr int RPB = 256 / SP;  // rows per block
    const int nbb = (a.B + RPB - 1) / RPB;
    const int bb = blockIdx.x % nbb, z = blockIdx.x / nbb;
    const int slot = a.slots[z];
    const int b = bb * RPB + (int)(threadIdx.x / SP), p = threadIdx.x % SP;
    if (b >= a.B) return;
    const int B = a.B, D = a.D, A = a.A;
    const uint64_t seed = a.seeds[slot];
    const uint32_t step = (uint32_t)(a.count[slot] + a.step_add);
    const long long B2 = 2 * (long long)B, B3 = 3 * (long long)B;
    float* os = at(a.os_in, slot);
    float* bc = at(a.bc_in, slot);
    float* cr = at(a.cr_in, slot);
    float* tg = at(a.tg_in, slot);
    float* eu = at(a.eu_in, slot);
    uint32_t c0[4] = {(uint32_t)b, step, a.stream_salt, 0u};
    philox4x32_10(c0, (uint32_t)seed, (uint32_t)(seed >> 32));
    // minibatch row: injected (packed per active member) or drawn from the dataset
    const float *obs, *nobs, *actp;
    float rew, mask;
    if (a.inj_batch) {
        const long long bs = (long long)B * (2 * D + A + 2);
        const float* pb = a.inj_batch + z * bs;
        obs = pb + (long long)b * D;
        actp = pb + (long long)B * D + (long long)b * A;
        rew = pb[(long long)B * (D + A) + b];
        mask = pb[(long long)B * (D + A + 1) + b];
        nobs = pb + (long long)B * (D + A + 2) + (long long)b * D;
    } else {
        const long long idx = (long long)(((unsigned long long)c0[0] * (unsigned long long)a.n_rows) >> 32);
        actp = a.act + idx * A;
        obs = a.obs + idx * D;
        nobs = a.nobs + idx * D;
        rew = a.rew[idx];
        mask = a.mask[idx];
    }
    const float* pn = a.inj_noise ? a.inj_noise + z * (long long)B * (4 * A + 1) : nullptr;
    const float t = pn ? pn[(long long)B * 2 * A + b] : u01(c0[1]);
    // the row's observation features: the first KQ per thread with every load issued before
    // the first wait (a loop that loads per iteration waits once per iteration; k clamped,
    // stores guarded), any beyond (D > KQ * SP) one by one
    auto put = [&](int k, float o, float n) {
        os[k * B3 + b] = n;
        os[k * B3 + B + b] = o;
        os[k * B3 + 2 * B + b] = o;
        bc[k * B2 + b] = o;
        bc[k * B2 + B + b] = o;
        cr[k * B2 + b] = o;
        cr[k * B2 + B + b] = o;
        tg[(long long)k * B + b] = n;
        eu[(long long)k * B + b] = o;
    };
    constexpr int KQ = 8;
    float ov[KQ], nv0[KQ];
#pragma unroll
    for (int q = 0; q < KQ; ++q) {
        const int k = min(p + SP * q, D - 1);
        ov[q] = obs[k];
        nv0[q] = nobs[k];
    }
#pragma unroll
    for (int q = 0; q < KQ; ++q)
        if (p + SP * q < D) put(p + SP * q, ov[q], nv0[q]);
    for (int k = p + SP * KQ; k < D; k += SP) put(k, obs[k], nobs[k]);
    if (p < A) {
        const float av = actp[p];
        cr[(D + p) * B2 + b] = av;
        at(a.act_t, slot)[(long long)p * B + b] = av;
    }
    // noises: normal i of 4A -> (category i / A: z_next, x0, z_d, z_metric; action j = i % A)
    for (int q = p; 2 * q < 4 * A; q += SP) {
        float nv[2];
        if (pn) {
            for (int h = 0; h < 2; ++h) {
                const int i = 2 * q + h, cat = i / A, j = i % A;
                const long long o = cat == 0 ? (long long)b * A + j
                                  : cat == 1 ? (long long)B * A + b * A + j
                                  : cat == 2 ? (long long)B * (2 * A + 1) + b * A + j
                                             : (long long)B * (3 * A + 1) + b * A + j;
                nv[h] = i < 4 * A ? pn[o] : 0.f;
            }
        } else {
            uint32_t c[4] = {(uint32_t)b, step, a.stream_salt, 1u + (uint32_t)q};
            philox4x32_10(c, (uint32_t)seed, (uint32_t)(seed >> 32));
            const float r = sqrtf(-2.0f * logf(u01_open_closed(c[0])));
            float sv, cv;
            sincosf(6.283185307179586f * u01(c[1]), &sv, &cv);
            nv[0] = r * cv;
            nv[1] = r * sv;
        }
        for (int h = 0; h < 2; ++h) {
            const int i = 2 * q + h;
            if (i >= 4 * A) break;
            const int cat = i / A, j = i % A;
            const long long r = D + j;
            const float v = nv[h];
            if (cat == 0) {
                os[r * B3 + b] = v;
            } else if (cat == 1) {
                at(a.x0_t, slot)[(long long)j * B + b] = v;
                bc[r * B2 + b] = (1.0f - t) * v + t * actp[j];
            } else if (cat == 2) {
                os[r * B3 + B + b] = v;
                bc[r * B2 + B + b] = v;
            } else {
                os[r * B3 + 2 * B + b] = v;
            }
        }
    }
    if (p == 0) {
        bc[(long long)(D + A) * B2 + b] = t;
        bc[(long long)(D + A) * B2 + B + b] = 0.0f;
        at(a.rew_t, slot)[b] = rew;
        at(a.mask_t, slot)[b] = mask;
    }
}

void launch_sample(const SampleArgs& a, hipStream_t s) {
    const int rpb = 256 / SP;
    hipLaunchKernelGGL(sample_kernel, dim3(((a.B + rpb - 1) / rpb) * a.nz), dim3(256), 0, s, a);
}

// =============================================================== losses ====
// [EXT] critic_loss: y = r + gamma*mask*agg_k Qt_k(s',a'); L = mean (Q-y)^2
// over [E,B]; also the Q-term of actor_loss (q = mean_k Q_k(s, clip(a_pi))),
// its gradient seeds, and the mse metric.  One block per member.
__global__ __launch_bounds__(256) void loss_critic_kernel(const LossArgs a) {
    const int z = blockIdx.x, slot = a.slots[z];
    const int B = a.B, E = a.E, A = a.A;
    __shared__ float red[11 * 8];
    const float* q = at(a.q, slot);      // [E][2B] (ens stride = q.sy)
    const float* qt = at(a.qt, slot);    // [E][B]
    const float* rw = at(a.rew, slot);
    const float* mk = at(a.mask, slot);
    float* dq = at(a.dq, slot);
    const float invEB = 1.0f / (float)(E * B);
    float sq = 0.f, qs = 0.f, qmx = -INFINITY, qmn = INFINITY, qpi_s = 0.f, qpi_abs = 0.f;
    float sdq[4] = {0.f, 0.f, 0.f, 0.f};
    for (int b = threadIdx.x; b < B; b += 256) {
        float agg = a.q_min ? INFINITY : 0.f;
        for (int e = 0; e < E; ++e) {
            const float v = qt[e * a.qt.sy + b];
            agg = a.q_min ? fminf(agg, v) : agg + v;
        }
        if (!a.q_min) agg /= (float)E;
        const float y = rw[b] + a.discount * mk[b] * agg;
        float qp = 0.f;
        for (int e = 0; e < E; ++e) {
            const float qv = q[e * a.q.sy + b];
            const float d = qv - y;
            sq += d * d;
            qs += qv;
            qmx = fmaxf(qmx, qv);
            qmn = fminf(qmn, qv);
            const float g = 2.0f * d * invEB;
            dq[e * a.dq.sy + b] = g;
            if (e < 4) sdq[e] += g;
            qp += q[e * a.q.sy + B + b];
        }
        qp /= (float)E;
        qpi_s += qp;
        qpi_abs += fabsf(qp);
    }
    // mse metric of sample_actions(s) against the dataset actions
    const float* am = at(a.amet, slot);
    const float* ac = at(a.act, slot);
    float smse = 0.f;
    for (int i = threadIdx.x; i < A * B; i += 256) {
        const float d = am[i] - ac[i];
        smse += d * d;
    }
    float rv[11] = {sq, qs, qmx, qmn, qpi_s, qpi_abs, smse, sdq[0], sdq[1], sdq[2], sdq[3]};
    block_reduce_n<11>(rv, {0, 0, 1, 2, 0, 0, 0, 0, 0, 0, 0}, red);
    sq = rv[0];
    qs = rv[1];
    qmx = rv[2];
    qmn = rv[3];
    qpi_s = rv[4];
    qpi_abs = rv[5];
    smse = rv[6];
    if (threadIdx.x == 0)
        for (int e = 0; e < E && e < 4; ++e) at(a.g_cb4, slot, e)[0] = rv[7 + e];
    const float qmean_pi = qpi_s / (float)B;
    const float lam = a.normq ? 1.0f / (qpi_abs / (float)B) : 1.0f;
    const float gpi = -lam * invEB;
    for (int b = threadIdx.x; b < B; b += 256)
        for (int e = 0; e < E; ++e) dq[e * a.dq.sy + B + b] = gpi;
    if (threadIdx.x == 0) {
        float* info = at(a.info, slot);
        info[0] = sq * invEB;
        info[1] = qs * invEB;
        info[2] = qmx;
        info[3] = qmn;
        info[7] = -lam * qmean_pi;
        info[8] = qmean_pi;
        info[9] = smse / (float)(A * B);
    }
}

// [EXT] BC flow-matching loss: mean over [B,A] of (v_theta(s,x_t,t) - (a - x0))^2.
__global__ __launch_bounds__(256) void loss_bc_kernel(const LossArgs a) {
    const int z = blockIdx.x, slot = a.slots[z];
    const int B = a.B, A = a.A;
    __shared__ float red[9 * 8];
    const float* vp = at(a.vpred, slot);
    const float* ac = at(a.act, slot);
    const float* x0 = at(a.x0, slot);
    float* dv = at(a.dv, slot);
    const float sc = 2.0f / (float)(A * B);
    float s = 0.f;
    float sdb[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) sdb[j] = 0.f;
    for (int b = threadIdx.x; b < B; b += 256) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            if (j < A) {
                const long long o = (long long)j * B + b;
                const float d = vp[o] - (ac[o] - x0[o]);
                s += d * d;
                const float g = sc * d;
                dv[o] = g;
                sdb[j] += g;
            }
        }
    }
    float rv[9] = {s, sdb[0], sdb[1], sdb[2], sdb[3], sdb[4], sdb[5], sdb[6], sdb[7]};
    block_reduce_n<9>(rv, {0, 0, 0, 0, 0, 0, 0, 0, 0}, red);
    s = rv[0];
    if (threadIdx.x == 0)
        for (int j = 0; j < A; ++j) at(a.g_bcb4, slot)[j] = rv[1 + j];
    if (threadIdx.x == 0) at(a.info, slot)[5] = s / (float)(A * B);
}

// [EXT] actor_loss remainder: distill = mean (a_pi - a_flow)^2; the onestep
// output gradient alpha*d(distill) + 1{-1<a_pi<1} * dq/da (clip passes no
// gradient outside); actor_loss = bc + alpha*distill + q_loss.
__global__ __launch_bounds__(256) void loss_actor_kernel(const LossArgs a) {
    const int z = blockIdx.x, slot = a.slots[z];
    const int B = a.B, A = a.A;
    __shared__ float red[9 * 8];
    const float alpha = a.alpha[slot];
    const float* ap = at(a.apiraw, slot);
    const float* af = at(a.aflow, slot);
    const float* da = at(a.da, slot);
    const long long da_sy = a.da.sy;
    const int da_n = a.da_n;
    float* dout = at(a.dout_os, slot);
    const float sc = 2.0f / (float)(A * B);
    float s = 0.f;
    float sdb[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) sdb[j] = 0.f;
    for (int b = threadIdx.x; b < B; b += 256) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            if (j < A) {
                const long long o = (long long)j * B + b;
                const float x = ap[o];
                const float d = x - af[o];
                s += d * d;
                float dq = da[o];
                for (int e = 1; e < da_n; ++e) dq += da[e * da_sy + o];
                const float g = alpha * (sc * d) + ((x > -1.0f && x < 1.0f) ? dq : 0.0f);
                dout[o] = g;
                sdb[j] += g;
            }
        }
    }
    float rv[9] = {s, sdb[0], sdb[1], sdb[2], sdb[3], sdb[4], sdb[5], sdb[6], sdb[7]};
    block_reduce_n<9>(rv, {0, 0, 0, 0, 0, 0, 0, 0, 0}, red);
    s = rv[0];
    if (threadIdx.x == 0)
        for (int j = 0; j < A; ++j) at(a.g_osb4, slot)[j] = rv[1 + j];
    if (threadIdx.x == 0) {
        float* info = at(a.info, slot);
        const float distill = s / (float)(A * B);
        info[6] = distill;
        info[4] = info[5] + alpha * distill + info[7];
    }
}

void launch_loss_critic(const LossArgs& a, hipStream_t s) {
    hipLaunchKernelGGL(loss_critic_kernel, dim3(a.nz), dim3(256), 0, s, a);
}
void launch_loss_bc(const LossArgs& a, hipStream_t s) {
    hipLaunchKernelGGL(loss_bc_kernel, dim3(a.nz), dim3(256), 0, s, a);
}
void launch_loss_actor(const LossArgs& a, hipStream_t s) {
    hipLaunchKernelGGL(loss_actor_kernel, dim3(a.nz), dim3(256), 0, s, a);
}

// ============================================================ optimiser ====
// optax.adam(lr) (b1 .9, b2 .999, eps 1e-8 outside the sqrt, bias correction
// with count+1) fused with the target-critic EMA (from the PRE-update critic)
// and the per-chunk grad statistics of apply_loss_fn (max, min, sum g^2).
__global__ __launch_bounds__(256) void adam_kernel(const AdamArgs a) { adam_chunk(a, blockIdx.x, blockIdx.y); }

void launch_adam(const AdamArgs& a, hipStream_t s) {
    hipLaunchKernelGGL(adam_kernel, dim3(a.n_chunks, a.nz), dim3(256), 0, s, a);
}

// grad/max, grad/min over every leaf (target-critic leaves contribute zeros),
// grad/norm = sum over leaves of the leaf L2 norm; count += 1.  Wave = leaf
// (leaves w, w + 16, ...): lanes stride its chunks, wave reductions, then thread
// 0 folds the leaves in order -- fixed pattern, deterministic.
constexpr int FIN_WAVES = 16;
__global__ __launch_bounds__(FIN_WAVES * 64) void finalize_kernel(const FinalArgs a) {
    const int z = blockIdx.x, slot = a.slots[z];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const float* st = a.stats + (long long)slot * a.n_total_chunks * 3;
    __shared__ float leaf[3][128];
    for (int l = w; l < a.n_leaves; l += FIN_WAVES) {
        float mx = -INFINITY, mn = INFINITY, ss = 0.f;
        for (int c = a.leaf_first[l] + lane; c < a.leaf_first[l + 1]; c += 64) {
            mx = fmaxf(mx, st[c * 3 + 0]);
            mn = fminf(mn, st[c * 3 + 1]);
            ss += st[c * 3 + 2];
        }
        mx = wave_max(mx);
        mn = wave_min(mn);
        ss = wave_sum(ss);
        if (lane == 0) {
            leaf[0][l] = mx;
            leaf[1][l] = mn;
            leaf[2][l] = sqrtf(ss);
        }
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        float mx = 0.f, mn = 0.f, nrm = 0.f;  // zero target-critic leaves are part of the tree
        for (int l = 0; l < a.n_leaves; ++l) {
            mx = fmaxf(mx, leaf[0][l]);
            mn = fminf(mn, leaf[1][l]);
            nrm += leaf[2][l];
        }
        float* info = at(a.info, slot);
        info[10] = mx;
        info[11] = mn;
        info[12] = nrm;
        a.count[slot] += 1;
    }
}

void launch_finalize(const FinalArgs& a, hipStream_t s) {
    hipLaunchKernelGGL(finalize_kernel, dim3(a.nz), dim3(FIN_WAVES * 64), 0, s, a);
}

// ================================================================= init ====
__global__ __launch_bounds__(256) void init_kernel(const InitArgs a) {
    const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
    if (i >= a.n) return;
    if (a.lim == 0.f) {
        a.p[i] = a.value;
        return;
    }
    uint32_t c[4] = {(uint32_t)i, (uint32_t)(i >> 32), a.salt, 0xF1A5u};
    philox4x32_10(c, (uint32_t)a.seed, (uint32_t)(a.seed >> 32));
    a.p[i] = (2.0f * u01(c[0]) - 1.0f) * a.lim;
}

void launch_init(const InitArgs& a, hipStream_t s) {
    if (a.n <= 0) return;
    hipLaunchKernelGGL(init_kernel, dim3((unsigned)((a.n + 255) / 256)), dim3(256), 0, s, a);
}

// ============================================== world-model rollout eval ==
// (RolloutArgs, kernels.h)  One block = 16 envs (columns) of one member for
// the whole episode; every network runs on LDS-resident activations:
//   actor   - the streamed 512-wide k-loop of stream_fwd (weights from L2),
//             GELU, head -> clip: sample_actions (evaluator/evaluation.py:58-64)
//   s'      - LayerNorm over [s, a] per column, Dense+ReLU..., Dense(D) + s
//   term    - Dense+ReLU..., Dense(1) > 0
// Small Dense layers: 16-feature output tiles round-robin over the 8 waves,
// v_mfma_f32_16x16x4_f32 with W rows from L2 and x from LDS.
bool rollout_supported(int H, int L, int D, int A) {
    return H == EF_H && L >= 1 && L <= EF_MAX_LAYERS && D + A <= EF_K0MAX && A <= 8 && D <= 64;
}

// y[o][c] = act(sum_k W[k][o] x[k][c] + b[o]), o < Wo, k < Wi, c < 16 (LDS in / out,
// row pitch 16); res (optional, LDS [Wo][16]) is added after the activation.  A wave
// issues the W fragments of KS k-steps at once as unguarded buffer loads (k >= Wi reads 0
// past the range; a lane's o >= Wo feeds only its own discarded row), then the MFMAs.
template <bool RELU, int KS>
DEV void ro_dense_t(const float* __restrict__ W, const float* __restrict__ bias, const float* xin, int Wi, int Wo,
                    float* yout, const float* res, int w, int li, int lk) {
    const int ntile = (Wo + 15) / 16, nks = (Wi + 3) / 4;
    const rsrc_t rW = make_rsrc(W, (long long)Wi * Wo);
    for (int t = w; t < ntile; t += EF_NW) {
        const int o = 16 * t + li;
        f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
        for (int s0 = 0; s0 < nks; s0 += KS) {
            float av[KS];
#pragma unroll
            for (int u = 0; u < KS; ++u) av[u] = bload1(rW, ((4 * (s0 + u) + lk) * Wo + o) * 4, 0);
#pragma unroll
            for (int u = 0; u < KS; ++u) {
                if (s0 + u < nks) {
                    const int k = 4 * (s0 + u) + lk;
                    const float xv = xin[min(k, Wi - 1) * EF_NC + li];
                    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(av[u], k < Wi ? xv : 0.f, acc, 0, 0, 0);
                }
            }
        }
        // acc[r]: feature 16t + 4lk + r, column li
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int f = 16 * t + 4 * lk + r;
            if (f < Wo) {
                float v = acc[r] + bias[f];
                if (RELU) v = fmaxf(v, 0.f);
                if (res) v += res[f * EF_NC + li];
                yout[f * EF_NC + li] = v;
            }
        }
    }
}
template <bool RELU>
DEV void ro_dense(const float* W, const float* bias, const float* xin, int Wi, int Wo, float* yout, const float* res,
                  int w, int li, int lk) {
    if (Wi <= 32) ro_dense_t<RELU, 8>(W, bias, xin, Wi, Wo, yout, res, w, li, lk);
    else if (Wi <= 64) ro_dense_t<RELU, 16>(W, bias, xin, Wi, Wo, yout, res, w, li, lk);
    else ro_dense_t<RELU, 32>(W, bias, xin, Wi, Wo, yout, res, w, li, lk);
}

__global__ __launch_bounds__(EF_NW * 64, 1) void rollout_kernel(const RolloutArgs g) {
    constexpr int H = EF_H, NC = EF_NC, NT = EF_NW * 64, PF = EF_PF;
    __shared__ __attribute__((aligned(16))) float slab[H * NC + 64];
    __shared__ __attribute__((aligned(16))) float in0[EF_K0MAX * NC + 64];   // actor input [s; z]
    __shared__ __attribute__((aligned(16))) float bufA[RO_MAX_W * NC];
    __shared__ __attribute__((aligned(16))) float bufB[RO_MAX_W * NC];
    __shared__ float obs_s[64 * NC], obs_n[64 * NC], act_s[8 * NC];
    __shared__ float hred[EF_NW * 8 * NC];
    __shared__ float lnp[2][NC];
    __shared__ int done_s[NC];
    __shared__ float res_s[NC][2];
    __shared__ int all_done;

    const int ntile = (g.n_envs + NC - 1) / NC;
    const int bid = blockIdx.x;
    const int z = bid / ntile, e0 = (bid % ntile) * NC;
    const int slot = g.slots[z];
    const int tid = threadIdx.x, lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int li = lane & 15, lk = lane >> 4;
    const int D = g.D, A = g.A, L = g.L, K0 = D + A;
    const bool tail0 = K0 > 4 * PF && K0 <= 4 * (PF + 1);  // layer 0 as in euler_flow_kernel
    const int NS0 = tail0 ? PF : (K0 + 4 * PF - 1) / (4 * PF) * PF;
    const float* __restrict__ P = g.params + (long long)slot * g.P + g.os_off;
    const uint64_t key = g.seed ^ (g.member_seeds[slot] * 0x9E3779B97F4A7C15ull);

    for (int e = tid; e < EF_K0MAX * NC + 64; e += NT) in0[e] = 0.f;
    for (int e = tid; e < 64 * NC; e += NT) {
        const int k = e / NC, c = e % NC;
        obs_s[e] = (k < D && e0 + c < g.n_envs) ? g.init_obs[(long long)(e0 + c) * D + k] : 0.f;
    }
    if (tid < NC) {
        done_s[tid] = e0 + tid >= g.n_envs;  // padding columns are done from the start
        res_s[tid][0] = 0.f;
        res_s[tid][1] = 0.f;
    }
    const rsrc_t rW = make_rsrc(P, g.P - g.os_off);
    const int lo = lk * H + 64 * w + 4 * li;
    float4 ring[PF];
#pragma unroll
    for (int p = 0; p < PF; ++p) ring[p] = bload4(rW, (int)g.w_off[0] + 4 * p * H + lo);
    float w5r[16];  // head A fragments: W_L[64w + 4s + lk][li], li < A
#pragma unroll
    for (int s = 0; s < 16; ++s) w5r[s] = li < A ? P[g.w_off[L] + (64 * w + 4 * s + lk) * A + li] : 0.f;
    __syncthreads();

    for (int t = 1; t <= g.max_steps; ++t) {
      if (g.actions) {  // env-model step only (fqlpop_envmodel_step): given actions
        if (tid < A * NC) {
            const int j = tid / NC, c = tid % NC;
            act_s[tid] = e0 + c < g.n_envs ? g.actions[(long long)(e0 + c) * A + j] : 0.f;
        }
        __syncthreads();
      } else {
        // ---- actor input [s; z_t] ----------------------------------------
        for (int e = tid; e < K0 * NC; e += NT) {
            const int k = e / NC;
            if (k < D) in0[e] = obs_s[e];
        }
        if (tid < NC * ((A + 1) / 2)) {
            const int c = tid % NC, q = tid / NC;  // normal pair q: actions 2q, 2q+1
            float n0, n1;
            if (g.noise) {
                const float* nz = g.noise + (((long long)z * g.max_steps + (t - 1)) * g.n_envs + e0 + c) * A;
                const bool ok = e0 + c < g.n_envs;
                n0 = ok ? nz[2 * q] : 0.f;
                n1 = (ok && 2 * q + 1 < A) ? nz[2 * q + 1] : 0.f;
            } else {
                uint32_t cc[4] = {(uint32_t)(e0 + c), (uint32_t)t, 0x5E11u, (uint32_t)q};
                philox4x32_10(cc, (uint32_t)key, (uint32_t)(key >> 32));
                const float r = sqrtf(-2.0f * logf(u01_open_closed(cc[0])));
                float sv, cv;
                sincosf(6.283185307179586f * u01(cc[1]), &sv, &cv);
                n0 = r * cv;
                n1 = r * sv;
            }
            in0[(D + 2 * q) * NC + c] = n0;
            if (2 * q + 1 < A) in0[(D + 2 * q + 1) * NC + c] = n1;
        }
        __syncthreads();
        // ---- actor hidden layers (streamed weights, GELU) -----------------
        for (int l = 0; l < L; ++l) {
            const int NS = l == 0 ? NS0 : H / 4;
            const float* xs = l == 0 ? in0 : slab;
            const int nl = l + 1 < L ? l + 1 : 0;
            f32x4 acc[4];
#pragma unroll
            for (int c = 0; c < 4; ++c) acc[c] = f32x4{0.f, 0.f, 0.f, 0.f};
            float4 bias4[4];
#pragma unroll
            for (int r = 0; r < 4; ++r) bias4[r] = bload4(rW, (int)g.b_off[l] + 64 * w + 16 * lk + 4 * r);
            const bool tl = l == 0 && tail0;
            __builtin_amdgcn_s_waitcnt(0x0F74);  // vmcnt(4): as euler_flow_kernel (the bias loads in flight)
            ef_kloop(acc, ring, rW, xs, NS, (int)g.w_off[l], (int)g.w_off[nl], lo, lk, li,
                     tl ? (int)g.w_off[0] + 4 * PF * H : -1);
            if (tl) {
                ef_tail(acc, ring[0], xs, lk, li);
                __builtin_amdgcn_sched_barrier(0);
                ring[0] = bload4(rW, (int)g.w_off[nl] + lo);
            }
            __syncthreads();  // every wave done reading the slab
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const float bb[4] = {bias4[r].x, bias4[r].y, bias4[r].z, bias4[r].w};
#pragma unroll
                for (int c = 0; c < 4; ++c)
                    slab[(64 * w + 16 * lk + 4 * r + c) * NC + li] = gelu_fast(acc[c][r] + bb[c]);
            }
            __syncthreads();
        }
        // ---- head: a = clip(W_L^T h + b_L) ---------------------------------
        {
            f32x4 hacc = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int s = 0; s < 16; ++s)
                hacc = __builtin_amdgcn_mfma_f32_16x16x4f32(w5r[s], slab[(64 * w + 4 * s + lk) * NC + li], hacc, 0, 0, 0);
            if (lk < 2) {
#pragma unroll
                for (int r = 0; r < 4; ++r) hred[w * 8 * NC + (4 * lk + r) * NC + li] = hacc[r];
            }
            __syncthreads();
            if (tid < A * NC) {
                const int j = tid / NC;
                float v = hred[tid];
#pragma unroll
                for (int q = 1; q < EF_NW; ++q) v += hred[q * 8 * NC + tid];
                act_s[tid] = clip1(v + P[g.b_off[L] + j]);
            }
            __syncthreads();
        }
      }
        // ---- state predictor: LayerNorm([s, a]) -> Dense+ReLU ... -> Dense(D) + s
        if (tid < NC) {
            float s1 = 0.f, s2 = 0.f;
            for (int k = 0; k < K0; ++k) {
                const float x = k < D ? obs_s[k * NC + tid] : act_s[(k - D) * NC + tid];
                s1 += x;
                s2 += x * x;
            }
            const float mean = s1 / (float)K0;
            const float var = fmaxf(s2 / (float)K0 - mean * mean, 0.f);
            lnp[0][tid] = mean;
            lnp[1][tid] = 1.0f / sqrtf(var + 1e-6f);
        }
        __syncthreads();
        for (int e = tid; e < K0 * NC; e += NT) {
            const int k = e / NC, c = e % NC;
            const float x = k < D ? obs_s[e] : act_s[(k - D) * NC + c];
            bufA[e] = (x - lnp[0][c]) * lnp[1][c] * g.sp[g.sp_ln_scale + k] + g.sp[g.sp_ln_bias + k];
        }
        __syncthreads();
        {
            float* cur = bufA;
            float* nxt = bufB;
            for (int i = 0; i < g.sp_n; ++i) {
                const bool last = i == g.sp_n - 1;
                if (last)
                    ro_dense<false>(g.sp + g.sp_w[i], g.sp + g.sp_b[i], cur, g.sp_dims[i], g.sp_dims[i + 1], obs_n,
                                    obs_s, w, li, lk);
                else
                    ro_dense<true>(g.sp + g.sp_w[i], g.sp + g.sp_b[i], cur, g.sp_dims[i], g.sp_dims[i + 1], nxt,
                                   nullptr, w, li, lk);
                __syncthreads();
                float* tmp = cur; cur = nxt; nxt = tmp;
            }
        }
        // ---- termination predictor on s' ----------------------------------
        {
            const float* cur = obs_n;
            for (int i = 0; i < g.tp_n; ++i) {
                float* dst = (i & 1) ? bufB : bufA;
                if (i == g.tp_n - 1)
                    ro_dense<false>(g.tp + g.tp_w[i], g.tp + g.tp_b[i], cur, g.tp_dims[i], g.tp_dims[i + 1], dst,
                                    nullptr, w, li, lk);
                else
                    ro_dense<true>(g.tp + g.tp_w[i], g.tp + g.tp_b[i], cur, g.tp_dims[i], g.tp_dims[i + 1], dst,
                                   nullptr, w, li, lk);
                __syncthreads();
                cur = dst;
            }
            if (g.out_logit && tid < NC && e0 + tid < g.n_envs) g.out_logit[(long long)z * g.n_envs + e0 + tid] = cur[tid];
            // ---- bookkeeping (evaluate_actor_fn: first terminated / truncated step)
            if (tid < NC) {
                if (!done_s[tid]) {
                    if (cur[tid] > 0.f) {
                        res_s[tid][0] = 1.f;
                        res_s[tid][1] = (float)t;
                        done_s[tid] = 1;
                    } else if (t >= g.max_steps) {
                        res_s[tid][1] = (float)t;
                        done_s[tid] = 1;
                    }
                }
            }
        }
        for (int e = tid; e < 64 * NC; e += NT) obs_s[e] = obs_n[e];
        __syncthreads();
        if (tid == 0) {
            int a = 1;
            for (int c = 0; c < NC; ++c) a &= done_s[c];
            all_done = a;
        }
        __syncthreads();
        if (all_done) break;
    }
    if (tid < NC && e0 + tid < g.n_envs) {
        float* o = g.out + ((long long)z * g.n_envs + e0 + tid) * 2;
        o[0] = res_s[tid][0];
        o[1] = res_s[tid][1];
    }
    if (g.out_obs) {
        for (int e = tid; e < D * NC; e += NT) {
            const int k = e / NC, c = e % NC;
            if (e0 + c < g.n_envs) g.out_obs[((long long)z * g.n_envs + e0 + c) * D + k] = obs_s[e];
        }
    }
}

void launch_rollout(const RolloutArgs& a, hipStream_t s) {
    const dim3 grid(((a.n_envs + EF_NC - 1) / EF_NC) * a.nz);
    hipLaunchKernelGGL(rollout_kernel, grid, dim3(EF_NW * 64), 0, s, a);
}

}  // namespace fq
