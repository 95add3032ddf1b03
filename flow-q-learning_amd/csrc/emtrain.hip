// Env-model trainer: one training step of the
// reference's world-model trainers on the GPU.
//
//   state predictor       envmodel/state_predictor_trainer.py:67-95 on
//                         BaselineStatePredictor (envmodel/baseline.py:25-37),
//                         state_prediction_loss (envmodel/loss.py:80-111) as bound
//                         by train_env_model.py:37-44 (reconstruction weight 0;
//                         a frozen termination predictor scores the predicted next
//                         observation when termination_weight > 0)
//   termination predictor envmodel/termination_predictor_trainer.py:55-76 on
//                         TerminationPredictor (envmodel/termination_predictor.py:
//                         14-21; input dropout while training), focal_loss
//                         (envmodel/loss.py:33-66; train_env_model.py:79)
//   optimiser             optax.adam(cosine_decay_schedule(init_lr, steps))
//
// The nets are small (obs 28-42 -> 128 -> 256 -> 128 -> obs), so one step is
// two launches: em_grad_kernel (block = 16 minibatch rows: forward, loss,
// backward, per-block partial parameter grads, per-block log sums; activations
// in LDS, feature-major [feature][row]; the weights stream from L2) and
// em_adam_kernel (fixed-order sum of the block partials + Adam, which also
// refreshes the W^T copy the dX products read).  Every Dense product (forward,
// dX, dW) runs on v_mfma_f32_16x16x4_f32 with the block's 16 rows as the MFMA
// width; odd widths (33, 28, 1) are padded by the buffer loads' range check.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <string>
#include <vector>

#include "../../include/fqlpop.h"
#include "kernels.h"

#define DEV __device__ __forceinline__

namespace fq {
namespace em {

constexpr int R = 16;      // minibatch rows per block
constexpr int NT = 512;    // threads per block
constexpr int MAXL = 8;    // Dense layers per net
constexpr int NLOG = 16;   // per-block log sums

struct Net {
    int n;                              // Dense layers (hidden + output)
    int dims[MAXL + 1];                 // dims[0] = input, dims[n] = output
    long long w[MAXL], b[MAXL];         // flat offsets (flax leaf order)
    long long ln_scale, ln_bias;        // state predictor LayerNorm_0 (-1: none)
};

struct StepArgs {
    int kind;                           // FQLPOP_EM_STATE_PREDICTOR / FQLPOP_EM_TERMINATION
    int train;                          // 1: grads + dropout; 0: eval logs only
    Net net, tpn;                       // trained net; frozen termination predictor (kind 0, tw > 0)
    const float* params;
    const float* tp;
    const float *wt, *tpt;              // W^T copies of params / tp (Dense kernels [out][in], same offsets)
    float* part;                        // [blocks][P] partial grads
    long long P;
    float* logs;                        // [blocks][NLOG]
    // rows: injected [B][..] arrays, or gathered from the dataset by Philox indices
    const float *obs, *act, *rew, *nobs;
    long long n_rows;
    int injected;
    const unsigned char* keep;          // injected dropout keep mask [B][obs] or null
    uint64_t seed;
    long long step;                     // update count (sampling counter)
    int B, D, A;
    float tw, ttw, alpha, gamma, rate;
    // multistep (FQLPOP_EM_MULTISTEP): sequence length, rows per dataset episode, and the
    // per-(block, step) activation store of the backpropagation through time
    int T, ep_len;
    float* seq;
    long long seq_stride;
    int tchunks;                        // sweep path: T chunks of the dW GEMM (partials per block)
    unsigned long long* probe;          // diagnostic builds only (FQLPOP_EM_PROBE): sweep phase times
};

// ----------------------------------------------------------------- Philox
DEV void philox(uint32_t c[4], uint32_t k0, uint32_t k1) {
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
// uniform [0, 1) from (seed, a, b, c)
DEV float urand(uint64_t seed, uint32_t a, uint32_t b, uint32_t c) {
    uint32_t x[4] = {a, b, c, 0x3E7u};
    philox(x, (uint32_t)seed, (uint32_t)(seed >> 32));
    return (x[0] >> 8) * (1.0f / 16777216.0f);
}

DEV float softplus(float x) { return fmaxf(x, 0.f) + log1pf(expf(-fabsf(x))); }

// Dense layers on v_mfma_f32_16x16x4_f32: out[m][c] = act(sum_k A[k][m] x[k][c] + bias[m])
// for m < M, c < R = 16 (LDS, feature-major [m][R]); A is k-major [Kr][M] (m contiguous).
// A block's 8 waves take 16-feature output tiles round-robin; a wave loads the A
// fragments of KS k-steps (4 k each, up to 32) into registers at once (all in flight: the loop is
// L2-latency bound otherwise), then runs the MFMAs with x from LDS.  Forward: A = W
// [K][N]; dX: A = W^T [N][K] with mask = relu'(the layer input).
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __amdgpu_buffer_rsrc_t rsrc_t;
// An LDS activation pointer that went through a runtime-indexed pointer array (acts[i]) is
// generic again: its accesses compile to flat instructions, which count in both vmcnt and
// lgkmcnt, so every LDS read behind them also waited for the global loads and stores in
// flight.  The assumption lets the compiler address LDS directly.
template <typename T>
DEV T* lds_ptr(T* p) {
#if __HIP_DEVICE_COMPILE__  // (the builtin exists for the device pass only)
    __builtin_assume(__builtin_amdgcn_is_shared((const void*)p));
#endif
    return p;
}
template <int KS>
DEV void em_mfma_t(const float* __restrict__ A, const float* __restrict__ bias, const float* x, int Kr, int M,
                   float* y, bool relu, const float* mask) {
    x = lds_ptr(x);
    y = lds_ptr(y);
    if (mask) mask = lds_ptr(mask);
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, li = lane & 15, lk = lane >> 4;
    const int ntile = (M + 15) / 16, nks = (Kr + 3) / 4;
    // unguarded buffer loads (a guarded load compiles to a branch + vmcnt(0) wait): k >= Kr
    // falls past the range and reads 0; a lane's o >= M only feeds its own discarded row
    const rsrc_t rA = __builtin_amdgcn_make_buffer_rsrc((void*)A, (short)0, Kr * M * 4, 0x00020000);
    for (int t = w; t < ntile; t += NT / 64) {
        const int o = 16 * t + li;
        f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
        for (int s0 = 0; s0 < nks; s0 += KS) {
            float av[KS];
#pragma unroll
            for (int u = 0; u < KS; ++u)
                av[u] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
                                                      rA, ((4 * (s0 + u) + lk) * M + o) * 4, 0, 0));
#pragma unroll
            for (int u = 0; u < KS; ++u) {
                if (s0 + u < nks) {
                    const int k = 4 * (s0 + u) + lk;
                    const float xv = x[min(k, Kr - 1) * R + li];
                    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(av[u], k < Kr ? xv : 0.f, acc, 0, 0, 0);
                }
            }
        }
        // acc[r]: output m = 16t + 4lk + r, column li
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int m = 16 * t + 4 * lk + r;
            if (m < M) {
                float v = acc[r] + (bias ? bias[m] : 0.f);
                if (relu) v = fmaxf(v, 0.f);
                if (mask && !(mask[m * R + li] > 0.f)) v = 0.f;  // relu' (0 at 0)
                y[m * R + li] = v;
            }
        }
    }
    __syncthreads();
}
// KSMAX: the most k-steps a wave keeps in flight (32 = 32 VGPRs of fragments; the multistep
// kernel, at its register limit, takes 16)
template <int KSMAX = 32>
DEV void em_mfma(const float* A, const float* bias, const float* x, int Kr, int M, float* y, bool relu,
                 const float* mask) {
    if (Kr <= 32) em_mfma_t<8>(A, bias, x, Kr, M, y, relu, mask);
    else if (Kr <= 64 || KSMAX < 32) em_mfma_t<16>(A, bias, x, Kr, M, y, relu, mask);
    else em_mfma_t<32>(A, bias, x, Kr, M, y, relu, mask);
}
// out[f][r] = act(sum_k W[k][f] in[k][r] + b[f])
template <int KSMAX = 32>
DEV void dense_fwd(const float* W, const float* b, const float* in, int K, int N, float* out, bool relu) {
    em_mfma<KSMAX>(W, b, in, K, N, out, relu, nullptr);
}
// g_in[k][r] = sum_f W[k][f] g[f][r] (times relu'(in) when mask_in), from WT = W^T [N][K]
// (the transposed copy the optimiser keeps)
template <int KSMAX = 32>
DEV void dense_dx(const float* WT, const float* g, int K, int N, float* g_in, const float* mask_in) {
    em_mfma<KSMAX>(WT, nullptr, g, N, K, g_in, false, mask_in);
}

// Partial parameter grads of one Dense over the block's rows (MFMA over the 16 rows):
// dW[k][f] = sum_r in[k][r] g[f][r], db[f] = sum_r g[f][r]
// (acc: added to the partials already there -- the sum over the steps of a sequence).
// A wave's tiles go in batches of DW_MT: with acc, the batch's old partials are loaded
// first, all in flight together (one dependent read per tile cost one L2 round trip each,
// 16 of them per wave in a 128 x 256 layer, at every step of a multistep sequence)
constexpr int DW_MT = 8;
DEV void dense_dw(const float* in, const float* g, int K, int N, float* __restrict__ pW, float* __restrict__ pb,
                  bool acc = false) {
    in = lds_ptr(in);
    g = lds_ptr(g);
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, li = lane & 15, lk = lane >> 4;
    const int tf = (N + 15) / 16, nt = (K + 15) / 16 * tf;
    constexpr int NW = NT / 64;
    for (int t0 = w; t0 < nt; t0 += NW * DW_MT) {
        float old[DW_MT][4];
        if (acc) {
#pragma unroll
            for (int j = 0; j < DW_MT; ++j) {
                const int t = min(t0 + NW * j, nt - 1);  // past the wave's last tile: a re-read
                const int k0 = 16 * (t / tf), f0 = 16 * (t % tf);
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const int k = min(k0 + 4 * lk + q, K - 1), f = min(f0 + li, N - 1);  // in range
                    old[j][q] = pW[(long long)k * N + f];
                }
            }
        }
#pragma unroll
        for (int j = 0; j < DW_MT; ++j) {
            const int t = t0 + NW * j;
            if (t >= nt) break;
            const int k0 = 16 * (t / tf), f0 = 16 * (t % tf);
            f32x4 d = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int s = 0; s < R / 4; ++s) {
                const float av = k0 + li < K ? in[(k0 + li) * R + 4 * s + lk] : 0.f;  // A[k][r]
                const float bv = f0 + li < N ? g[(f0 + li) * R + 4 * s + lk] : 0.f;   // B[r][f]
                d = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bv, d, 0, 0, 0);
            }
            // d[q]: k = k0 + 4lk + q, f = f0 + li
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int k = k0 + 4 * lk + q, f = f0 + li;
                if (k < K && f < N) pW[(long long)k * N + f] = acc ? old[j][q] + d[q] : d[q];
            }
        }
    }
    for (int f = threadIdx.x; f < N; f += NT) {
        const float* b = g + f * R;
        float s = 0.f;
#pragma unroll
        for (int r = 0; r < R; ++r) s += b[r];
        pb[f] = acc ? pb[f] + s : s;
    }
}

// Frozen termination predictor on pred = tacts[0] [D][R]: weighted BCE of its logit
// (envmodel/loss.py:14-30) into the log sums 1..5, and its input gradient, scaled by
// tw / norm, added to gA [D][R].  inv_n: 1 / (number of scored predictions).
template <int KSMAX = 32>
DEV void tp_score(const StepArgs& a, float* const* tacts, float* gA, float* gB, float* gC, const float* lab,
                  float (*lsum)[R], float inv_n, float norm) {
    const Net& T = a.tpn;
    const int tid = threadIdx.x;
    for (int i = 0; i < T.n; ++i)
        dense_fwd<KSMAX>(a.tp + T.w[i], a.tp + T.b[i], tacts[i], T.dims[i], T.dims[i + 1], tacts[i + 1], i < T.n - 1);
    if (tid < R) {
        const float x = lds_ptr(tacts[T.n])[tid], z = lab[tid], w = a.ttw;
        const float ce = softplus(x) - x * z;
        lsum[1][tid] += (z > 0.f ? w * ce : ce) / (w + 1.f);
        lsum[2][tid] += z > 0.f ? ce : 0.f;
        lsum[3][tid] += z > 0.f ? 0.f : ce;
        lsum[4][tid] += z;
        lsum[5][tid] += 1.f - z;
        const float p = 1.0f / (1.0f + expf(-x));
        gB[tid] = (z > 0.f ? w : 1.f) / (w + 1.f) * (p - z) * inv_n;  // d bce / d logit
    }
    __syncthreads();
    // dX down the frozen stack (relu' of each hidden input), gB <-> gC
    float* src = gB;
    float* dst = gC;
    for (int i = T.n - 1; i >= 0; --i) {
        dense_dx<KSMAX>(a.tpt + T.w[i], src, T.dims[i], T.dims[i + 1], dst, i > 0 ? tacts[i] : nullptr);
        float* tmp = src;
        src = dst;
        dst = tmp;
    }
    src = lds_ptr(src);
    for (int t = tid; t < a.D * R; t += NT) gA[t] += a.tw / norm * src[t];
    __syncthreads();
}

__global__ __launch_bounds__(NT) void em_grad_kernel(const StepArgs a) {
    extern __shared__ __attribute__((aligned(16))) float lds[];
    __shared__ float lsum[NLOG][R];
    __shared__ float lab[R];
    __shared__ long long rowid[R];
    const int tid = threadIdx.x, blk = blockIdx.x;
    const Net& N = a.net;
    const int D = a.D, A = a.A;
    const int K0 = N.dims[0];
    // LDS: x0 [K0][R] | xhat [K0][R] | acts[i] [dims[i]][R] i = 0..n (acts[n] = output) |
    //      gA, gB, gC [maxd][R] | nobs [D][R] | tp acts [dims][R]
    int maxd = 0;
    for (int i = 0; i <= N.n; ++i) maxd = max(maxd, N.dims[i]);
    for (int i = 0; i <= a.tpn.n; ++i) maxd = max(maxd, a.tpn.dims[i]);
    float* x0 = lds;
    float* xhat = x0 + K0 * R;
    float* acts[MAXL + 1];
    acts[0] = xhat + K0 * R;
    for (int i = 1; i <= N.n; ++i) acts[i] = acts[i - 1] + N.dims[i - 1] * R;
    float* gA = acts[N.n] + N.dims[N.n] * R;
    float* gB = gA + maxd * R;
    float* gC = gB + maxd * R;
    float* nobs = gC + maxd * R;
    float* tacts[MAXL + 1];
    tacts[0] = nobs + D * R;
    for (int i = 1; i <= a.tpn.n; ++i) tacts[i] = tacts[i - 1] + a.tpn.dims[i - 1] * R;

    // ---- rows: injected batch rows, or Philox-drawn dataset rows ([EXT] Dataset.sample)
    if (tid < R) {
        const int gr = blk * R + tid;
        long long id = gr;
        if (!a.injected) {
            uint32_t c[4] = {(uint32_t)gr, (uint32_t)a.step, 0xE7u, 0u};
            philox(c, (uint32_t)a.seed, (uint32_t)(a.seed >> 32));
            id = (long long)((((uint64_t)c[1] << 32) | c[0]) % (uint64_t)a.n_rows);
        }
        rowid[tid] = id;
        lab[tid] = a.rew[id] == 0.f ? 1.f : 0.f;
    }
    for (int q = tid; q < NLOG * R; q += NT) lsum[q / R][q % R] = 0.f;
    __syncthreads();
    for (int t = tid; t < D * R; t += NT) {
        const int k = t / R, r = t % R;
        nobs[t] = a.nobs[rowid[r] * D + k];
    }
    if (a.kind == FQLPOP_EM_STATE_PREDICTOR) {
        for (int t = tid; t < K0 * R; t += NT) {
            const int k = t / R, r = t % R;
            x0[t] = k < D ? a.obs[rowid[r] * D + k] : a.act[rowid[r] * A + (k - D)];
        }
    } else {
        // termination predictor: dropout on the input while training; the keep mask is fixed
        // per (batch position, feature), as the reference's constant dropout rng
        for (int t = tid; t < K0 * R; t += NT) {
            const int k = t / R, r = t % R;
            float v = a.nobs[rowid[r] * D + k];
            if (a.train) {
                const int pos = blk * R + r;
                const bool keep = a.keep ? a.keep[(long long)pos * D + k] != 0
                                         : urand(a.seed, (uint32_t)pos, (uint32_t)k, 0xD20u) >= a.rate;
                v = keep ? v / (1.0f - a.rate) : 0.f;
            }
            x0[t] = v;
        }
    }
    __syncthreads();

    // ---- forward
    const float* P = a.params;
    if (N.ln_scale >= 0) {
        // flax LayerNorm over the K0 input features of each row (eps 1e-6, E[x^2] - mu^2 clipped)
        __shared__ float mu_s[R], rs_s[R];
        if (tid < R) {
            float s1 = 0.f, s2 = 0.f;
            for (int k = 0; k < K0; ++k) {
                const float v = x0[k * R + tid];
                s1 += v;
                s2 += v * v;
            }
            const float mu = s1 / K0;
            mu_s[tid] = mu;
            rs_s[tid] = 1.0f / sqrtf(fmaxf(s2 / K0 - mu * mu, 0.f) + 1e-6f);
        }
        __syncthreads();
        for (int t = tid; t < K0 * R; t += NT) {
            const int k = t / R, r = t % R;
            const float xh = (x0[t] - mu_s[r]) * rs_s[r];
            xhat[t] = xh;
            lds_ptr(acts[0])[t] = xh * P[N.ln_scale + k] + P[N.ln_bias + k];
        }
    } else {
        for (int t = tid; t < K0 * R; t += NT) lds_ptr(acts[0])[t] = x0[t];
    }
    __syncthreads();
    for (int i = 0; i < N.n; ++i)
        dense_fwd(P + N.w[i], P + N.b[i], acts[i], N.dims[i], N.dims[i + 1], acts[i + 1], i < N.n - 1);
    const float* out = lds_ptr(acts[N.n]);

    // ---- loss, output gradient (gA [dout][R]) and log sums
    const float invB = 1.0f / (float)a.B;
    if (a.kind == FQLPOP_EM_STATE_PREDICTOR) {
        // pred = out + obs; MSE(pred, next) over B x D; grads / (1 + tw)
        const float norm = 1.0f + a.tw;
        const float gscale = 2.0f / ((float)a.B * D) / norm;
        float* pred = lds_ptr(tacts[0]);  // pred [D][R]: the frozen termination predictor's input
        for (int t = tid; t < D * R; t += NT) {
            const float p = out[t] + x0[t];  // x0 rows k < D are the observations
            const float d = p - nobs[t];
            pred[t] = p;
            gA[t] = gscale * d;
            atomicAdd(&lsum[0][t % R], d * d);
        }
        __syncthreads();
        if (a.tw > 0.f) tp_score(a, tacts, gA, gB, gC, lab, lsum, invB, norm);
    } else {
        // focal loss (alpha, gamma) on the logit
        if (tid < R) {
            const float x = out[tid], z = lab[tid];
            const float p = 1.0f / (1.0f + expf(-x));
            const float ce = softplus(x) - x * z;
            const float pt = z > 0.f ? p : 1.f - p;
            const float af = z > 0.f ? a.alpha : 1.f - a.alpha;
            const float li = af * powf(1.f - pt, a.gamma) * ce;
            const float logp = -softplus(-x), log1mp = -softplus(x);
            const float d = z > 0.f ? powf(1.f - p, a.gamma) * (a.gamma * p * logp - (1.f - p))
                                    : powf(p, a.gamma) * (-a.gamma * (1.f - p) * log1mp + p);
            gA[tid] = af * d * invB;
            lsum[1][tid] = li;
            lsum[2][tid] = z > 0.f ? li : 0.f;
            lsum[3][tid] = z > 0.f ? 0.f : li;
            lsum[4][tid] = z;
            lsum[5][tid] = 1.f - z;
            const bool pr = x > 0.f;
            lsum[6][tid] = (pr == (z > 0.f)) ? 1.f : 0.f;
            lsum[7][tid] = (pr && z > 0.f) ? 1.f : 0.f;
            lsum[8][tid] = pr ? 1.f : 0.f;
        }
        __syncthreads();
    }

    // ---- block log sums
    if (tid < NLOG) {
        float s = 0.f;
        for (int r = 0; r < R; ++r) s += lsum[tid][r];
        a.logs[(long long)blk * NLOG + tid] = s;
    }
    if (!a.train) return;

    // ---- backward: partial grads of every Dense (and LayerNorm_0)
    float* pg = a.part + (long long)blk * a.P;
    float* g = gA;
    float* gn = gB;
    for (int i = N.n - 1; i >= 0; --i) {
        dense_dw(acts[i], g, N.dims[i], N.dims[i + 1], pg + N.w[i], pg + N.b[i]);
        if (i > 0 || N.ln_scale >= 0) dense_dx(a.wt + N.w[i], g, N.dims[i], N.dims[i + 1], gn, i > 0 ? acts[i] : nullptr);
        else __syncthreads();
        float* tmp = g;
        g = gn;
        gn = tmp;
    }
    if (N.ln_scale >= 0) {
        // g = grad wrt the LayerNorm output [K0][R]
        g = lds_ptr(g);
        for (int k = tid; k < K0; k += NT) {
            float ss = 0.f, sb = 0.f;
            for (int r = 0; r < R; ++r) {
                ss += g[k * R + r] * xhat[k * R + r];
                sb += g[k * R + r];
            }
            pg[N.ln_scale + k] = ss;
            pg[N.ln_bias + k] = sb;
        }
    }
}

// Multistep state predictor (envmodel/multistep.py:31-54): block = 16 sequences, the
// baseline cell stepped T times from observations[:, 0] (each step's prediction is the
// next step's observation), the loss of every step as in em_grad_kernel (normalised over
// B x T), then backpropagation through time: the step's activations go to a per-block
// store in HBM on the way forward and come back in reverse; the gradient w.r.t. the
// carried observation (the residual plus the LayerNorm input gradient of its D
// features) flows from step t + 1 into step t.  Partial grads accumulate over the steps.
#ifndef EM_SEQ_KS
#define EM_SEQ_KS 16
#endif
__global__ __launch_bounds__(NT) void em_seq_grad_kernel(const StepArgs a) {
    extern __shared__ __attribute__((aligned(16))) float lds[];
    __shared__ float lsum[NLOG][R];
    __shared__ float lab[R];
    __shared__ long long rowbase[R];
    __shared__ float mu_s[R], rs_s[R], cs[2][R];
    const int tid = threadIdx.x, blk = blockIdx.x;
    const Net& N = a.net;
    const int D = a.D, A = a.A, T = a.T;
    const int K0 = N.dims[0];
    int maxd = 0;
    for (int i = 0; i <= N.n; ++i) maxd = max(maxd, N.dims[i]);
    for (int i = 0; i <= a.tpn.n; ++i) maxd = max(maxd, a.tpn.dims[i]);
    // LDS as em_grad_kernel, + carry [D][R] (the gradient w.r.t. the carried observation)
    float* x0 = lds;
    float* xhat = x0 + K0 * R;
    float* acts[MAXL + 1];
    acts[0] = xhat + K0 * R;
    for (int i = 1; i <= N.n; ++i) acts[i] = acts[i - 1] + N.dims[i - 1] * R;
    float* gA = acts[N.n] + N.dims[N.n] * R;
    float* gB = gA + maxd * R;
    float* gC = gB + maxd * R;
    float* nobs = gC + maxd * R;
    float* tacts[MAXL + 1];
    tacts[0] = nobs + D * R;
    for (int i = 1; i <= a.tpn.n; ++i) tacts[i] = tacts[i - 1] + a.tpn.dims[i - 1] * R;
    float* carry = tacts[a.tpn.n > 0 ? a.tpn.n : 0] + (a.tpn.n > 0 ? a.tpn.dims[a.tpn.n] * R : D * R);

    // ---- sequences: injected [B][T] rows, or MultistepLoader windows drawn by Philox
    if (tid < R) {
        const int gr = blk * R + tid;
        long long base = (long long)gr * T;
        if (!a.injected) {
            uint32_t c[4] = {(uint32_t)gr, (uint32_t)a.step, 0xE5u, 0u};
            philox(c, (uint32_t)a.seed, (uint32_t)(a.seed >> 32));
            const long long n_ep = a.n_rows / a.ep_len;
            const long long ep = (long long)((((uint64_t)c[1] << 32) | c[0]) % (uint64_t)n_ep);
            const long long st = (long long)(c[2] % (uint32_t)(a.ep_len - T));
            base = ep * a.ep_len + st;
        }
        rowbase[tid] = base;
    }
    for (int q = tid; q < NLOG * R; q += NT) lsum[q / R][q % R] = 0.f;
    __syncthreads();

    const float* P = a.params;
    const float norm = 1.0f + a.tw;
    const float inv_n = 1.0f / ((float)a.B * (float)T);
    const float gscale = 2.0f / ((float)a.B * (float)T * D) / norm;
    float* const sq = a.seq + (long long)blk * T * a.seq_stride;  // this block's store
    // store layout per step: xhat [K0][R] | rstd [R] | acts[0..n-1] | direct output grad [D][R]
    int act_floats = 0;
    for (int i = 0; i < N.n; ++i) act_floats += N.dims[i] * R;

    // ---- forward through the sequence
    for (int t = 0; t < T; ++t) {
        for (int q = tid; q < K0 * R; q += NT) {
            const int k = q / R, r = q % R;
            const long long row = rowbase[r] + t;
            if (k >= D) x0[q] = a.act[row * A + (k - D)];
            else if (t == 0) x0[q] = a.obs[row * D + k];  // later steps: the previous prediction
        }
        for (int q = tid; q < D * R; q += NT) {
            const int k = q / R, r = q % R;
            nobs[q] = a.nobs[(rowbase[r] + t) * D + k];
        }
        if (tid < R) lab[tid] = a.rew[rowbase[tid] + t] == 0.f ? 1.f : 0.f;
        __syncthreads();
        if (tid < R) {
            float s1 = 0.f, s2 = 0.f;
            for (int k = 0; k < K0; ++k) {
                const float v = x0[k * R + tid];
                s1 += v;
                s2 += v * v;
            }
            const float mu = s1 / K0;
            mu_s[tid] = mu;
            rs_s[tid] = 1.0f / sqrtf(fmaxf(s2 / K0 - mu * mu, 0.f) + 1e-6f);
        }
        __syncthreads();
        for (int q = tid; q < K0 * R; q += NT) {
            const int k = q / R, r = q % R;
            const float xh = (x0[q] - mu_s[r]) * rs_s[r];
            xhat[q] = xh;
            lds_ptr(acts[0])[q] = xh * P[N.ln_scale + k] + P[N.ln_bias + k];
        }
        __syncthreads();
        for (int i = 0; i < N.n; ++i)
            dense_fwd<EM_SEQ_KS>(P + N.w[i], P + N.b[i], acts[i], N.dims[i], N.dims[i + 1], acts[i + 1], i < N.n - 1);
        const float* out = lds_ptr(acts[N.n]);
        float* pred = lds_ptr(tacts[0]);
        for (int q = tid; q < D * R; q += NT) {
            const float p = out[q] + x0[q];
            const float d = p - nobs[q];
            pred[q] = p;
            gA[q] = gscale * d;
            atomicAdd(&lsum[0][q % R], d * d);
        }
        __syncthreads();
        if (a.tw > 0.f) tp_score<EM_SEQ_KS>(a, tacts, gA, gB, gC, lab, lsum, inv_n, norm);
        if (a.train) {
            float* st = sq + (long long)t * a.seq_stride;
            for (int q = tid; q < K0 * R; q += NT) st[q] = xhat[q];
            if (tid < R) st[K0 * R + tid] = rs_s[tid];
            float* sa = st + K0 * R + R;
            for (int q = tid; q < act_floats; q += NT) sa[q] = lds_ptr(acts[0])[q];  // acts[0..n-1] are contiguous
            float* sg = sa + act_floats;
            for (int q = tid; q < D * R; q += NT) sg[q] = gA[q];
        }
        for (int q = tid; q < D * R; q += NT) x0[q] = pred[q];  // the next step's observation
        __syncthreads();
    }
    if (tid < NLOG) {
        float s = 0.f;
        for (int r = 0; r < R; ++r) s += lsum[tid][r];
        a.logs[(long long)blk * NLOG + tid] = s;
    }
    if (!a.train) return;

    // ---- backward through time
    float* pg = a.part + (long long)blk * a.P;
    for (int t = T - 1; t >= 0; --t) {
        const bool acc = t < T - 1;
        const float* st = sq + (long long)t * a.seq_stride;
        {
            // the step's record (xhat | rstd | acts[0..n-1]) in batches of 8 loads per thread,
            // all in flight before their LDS stores (one HBM round trip per element otherwise)
            constexpr int BQ = 8;
            const int n1 = K0 * R, n2 = n1 + R, n3 = n2 + act_floats;
            float* const a0 = lds_ptr(acts[0]);
            for (int q0 = tid; q0 < n3; q0 += BQ * NT) {
                float v[BQ];
#pragma unroll
                for (int j = 0; j < BQ; ++j) v[j] = st[min(q0 + j * NT, n3 - 1)];  // unguarded
#pragma unroll
                for (int j = 0; j < BQ; ++j) {
                    const int q = q0 + j * NT;
                    if (q < n1) xhat[q] = v[j];
                    else if (q < n2) rs_s[q - n1] = v[j];
                    else if (q < n3) a0[q - n2] = v[j];
                }
            }
        }
        const float* sg = st + K0 * R + R + act_floats;
        // total gradient w.r.t. this step's prediction: its own loss terms + the next step's
        for (int q = tid; q < D * R; q += NT) {
            const float gv = sg[q] + (acc ? carry[q] : 0.f);
            gA[q] = gv;
            carry[q] = gv;  // the residual path: pred_t = out_t + obs_t
        }
        __syncthreads();
        float* g = gA;
        float* gn = gB;
        for (int i = N.n - 1; i >= 0; --i) {
            dense_dw(acts[i], g, N.dims[i], N.dims[i + 1], pg + N.w[i], pg + N.b[i], acc);
            dense_dx<EM_SEQ_KS>(a.wt + N.w[i], g, N.dims[i], N.dims[i + 1], gn, i > 0 ? acts[i] : nullptr);
            float* tmp = g;
            g = gn;
            gn = tmp;
        }
        // g = grad w.r.t. the LayerNorm output [K0][R]
        g = lds_ptr(g);
        for (int k = tid; k < K0; k += NT) {
            float ss = 0.f, sb = 0.f;
            for (int r = 0; r < R; ++r) {
                ss += g[k * R + r] * xhat[k * R + r];
                sb += g[k * R + r];
            }
            pg[N.ln_scale + k] = acc ? pg[N.ln_scale + k] + ss : ss;
            pg[N.ln_bias + k] = acc ? pg[N.ln_bias + k] + sb : sb;
        }
        if (tid < R) {
            float c1 = 0.f, c2 = 0.f;
            for (int k = 0; k < K0; ++k) {
                const float gy = g[k * R + tid] * P[N.ln_scale + k];
                c1 += gy;
                c2 += gy * xhat[k * R + tid];
            }
            cs[0][tid] = c1 / K0;
            cs[1][tid] = c2 / K0;
        }
        __syncthreads();
        // LayerNorm input gradient of the observation features: into the carry
        for (int q = tid; q < D * R; q += NT) {
            const int k = q / R, r = q % R;
            carry[q] += rs_s[r] * (g[q] * P[N.ln_scale + k] - cs[0][r] - xhat[q] * cs[1][r]);
        }
        __syncthreads();
    }
}

// ====================================== multistep BPTT as sweeps (round 6, 1024 threads) ==
// em_seq_grad_kernel at the reference defaults (B = 256, T = 256) is 16 blocks of 512 threads
// whose every Dense product is a chain of L2 round trips (A fragments in batches of 16
// k-steps, up to 8 batches per wave and layer), and whose backward read-modify-writes the
// block's partial dW in L2 at every one of the T steps: 18 ms per train step (VERDICT r5
// item 6).  This path splits the work where the dependencies allow:
//   * em_sweep_kernel (16 waves per block, the same 16 sequences per block): every Dense op
//     of a step is at most ONE unit per wave, a 16-wide output tile x a chunk of <= 32
//     k-steps (split-K partials summed in a fixed order through LDS), and the A fragments of
//     the NEXT op are loaded while the current op's MFMAs run (weights do not depend on the
//     data; the barriers wait for LDS only), so an op costs about one MFMA chain and one or
//     two barriers instead of 2-8 dependent L2 round trips;
//   * its backward sweep runs only what is sequential in t: the dX chain, the LayerNorm
//     backward and the carried observation gradient; it stores each layer's output gradient
//     g_i beside the forward record, and sums the LayerNorm grads over t in LDS;
//   * em_seq_dw_kernel: dW_i = sum over the (t, row) pairs of acts_i g_i^T and db_i, one GEMM
//     per (block, T chunk, 64 x 64 tile) over the stored records, into the per-chunk partials
//     that em_adam_kernel folds in a fixed order.
// Taken when every op fits one unit per wave (fqlpop_emtrain_create: sw_fits); otherwise, and
// under engine option em_seq_sweep = 0, em_seq_grad_kernel runs.
constexpr int SW_NT = 1024, SW_NW = SW_NT / 64, SW_FM = 32, SW_SCR = SW_NW * 16 * R;
constexpr int SW_RQ = 10;    // a step's record, loaded a step ahead: <= SW_RQ floats per thread
// diagnostic phase slots (FQ_DIAG, FQLPOP_EM_PROBE): 0 inputs, 26 LayerNorm statistics, 1
// normalise, 2-5 forward ops, 6-13 termination-predictor ops, 27 record stores, 14 next
// observation; backward: 28 record to LDS, 29 next record's loads, 15 barrier, 16 carry,
// 17-20 dX ops, 30 LayerNorm backward sums, 25 carry update
constexpr int EM_PH_N = 32;

struct SwOp {
    const float* A;  // k-major [Kc][No] (No contiguous): W for a forward op, W^T for a dX op
    int Kc, No;      // contracted rows, outputs
};
// units of an op: ntile output tiles x S k-chunks of cks k-steps (4 rows each), at most one per wave
DEV void sw_plan(int Kc, int No, int& ntile, int& S, int& cks) {
    ntile = (No + 15) >> 4;
    const int nks = (Kc + 3) >> 2;
    S = 1;
    while (S < SW_NW && ntile * S * 2 <= SW_NW && S * 2 <= nks) S *= 2;
    cks = (nks + S - 1) / S;
}
bool sw_op_fits(int Kc, int No) {
    const int ntile = (No + 15) >> 4, nks = (Kc + 3) >> 2;
    int S = 1;
    while (S < SW_NW && ntile * S * 2 <= SW_NW && S * 2 <= nks) S *= 2;
    return ntile * S <= SW_NW && (nks + S - 1) / S <= SW_FM;
}
// the wave's A fragments of op o: fr[j] = A[4 (ch cks + j) + lk][16 tile + li] (unguarded buffer
// loads: rows >= Kc read 0, a lane's column >= No feeds only its own discarded output row)
// wave-uniform values through readfirstlane: an op descriptor picked by run-time branches is
// not known to be uniform, and a buffer resource built from VGPRs puts every load of the
// chain in a waterfall loop
DEV int sw_uni(int v) { return __builtin_amdgcn_readfirstlane(v); }
DEV const float* sw_uniptr(const float* p) {
    const unsigned long long v = (unsigned long long)p;
    const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)v), hi = __builtin_amdgcn_readfirstlane((unsigned)(v >> 32));
    return (const float*)(((unsigned long long)hi << 32) | lo);
}
DEV void sw_load(SwOp o, float (&fr)[SW_FM]) {
    o.A = sw_uniptr(o.A);
    o.Kc = sw_uni(o.Kc);
    o.No = sw_uni(o.No);
    int ntile, S, cks;
    sw_plan(o.Kc, o.No, ntile, S, cks);
    const int w = sw_uni(threadIdx.x >> 6), lane = threadIdx.x & 63, li = lane & 15, lk = lane >> 4;
    if (w >= ntile * S) return;  // (a wave without a unit loads nothing: see sw_chain)
    const int tile = w % ntile, ch = w / ntile;
    const rsrc_t rA = __builtin_amdgcn_make_buffer_rsrc((void*)o.A, (short)0, o.Kc * o.No * 4, 0x00020000);
    const int voff = ((4 * ch * cks + lk) * o.No + 16 * tile + li) * 4, sstep = 16 * o.No;
#pragma unroll
    for (int j = 0; j < SW_FM; ++j)
        fr[j] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rA, voff, j < cks ? j * sstep : 0x40000000, 0));
}
// One unit's MFMA chain (C) over all SW_FM slots, with slot j refilled with the next op's
// fragment right behind the MFMA that consumed it (L).  All or nothing, on both sides: a wave
// with a unit in the next op loads every slot and then reads every slot, a wave without one
// does neither.  (A load whose result is never read leaves its register free for the
// allocator while the load is in flight, and the next value put there must first wait for it
// (vmcnt counts in order): with per-op slot counts the chain ran at L2 latency per few MFMAs,
// and per-count code paths were merged by the compiler into one with the slots in scratch.)
// No branch around a load: slots j >= ck2 of the next op are loaded from past the buffer's
// range (an SGPR offset beyond num_records: they read exact zeros) and then read by an empty
// asm instead of an MFMA; rows >= Kc read zeros the same way, and x is read unconditionally
// (past the operand: other, initialised LDS buffers, times a zero fragment).  Even and odd
// slots are two independent chains, summed at the end.
template <bool C, bool L>
DEV void sw_chain(float (&fr)[SW_FM], f32x4& acc, const float* xl, int cks, rsrc_t rN, int voff, int sstep, int ck2) {
    f32x4 odd = f32x4{0.f, 0.f, 0.f, 0.f};
    // groups of 4 slots: one wave-uniform branch per group (past the chunk: no MFMA), the group's
    // 4 x reads issued together (a branch per slot kept every x read in front of its own MFMA,
    // one exposed LDS latency each); slots j >= cks inside a live group hold zero fragments
#pragma unroll
    for (int g = 0; g < SW_FM / 4; ++g) {
        if (C) {
            if (4 * g < cks) {
                float xv[4];
#pragma unroll
                for (int q = 0; q < 4; ++q) xv[q] = xl[4 * (4 * g + q) * R];
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    if (q & 1) odd = __builtin_amdgcn_mfma_f32_16x16x4f32(fr[4 * g + q], xv[q], odd, 0, 0, 0);
                    else acc = __builtin_amdgcn_mfma_f32_16x16x4f32(fr[4 * g + q], xv[q], acc, 0, 0, 0);
                }
            } else {  // the slots' (zero) loads are read: see above
                asm volatile("" ::"v"(fr[4 * g]), "v"(fr[4 * g + 1]), "v"(fr[4 * g + 2]), "v"(fr[4 * g + 3]));
            }
        }
        if (L) {
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int j = 4 * g + q;
                fr[j] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
                                                      rN, voff, j < ck2 ? j * sstep : 0x40000000, 0));
            }
        }
    }
    if (C) acc = acc + odd;
}
// y[m][c] = act(sum_k A[k][m] x[k][c] + bias[m]), m < No, c < R; mode 0 linear, 1 ReLU, 2 zero
// where mask[m][c] <= 0 (relu' of a hidden layer's output); x, y, mask, scr in LDS.  fr holds
// this op's fragments on entry and the next op's (nx) on exit, so the next op's L2 latency
// hides under this op's chain
DEV void sw_compute(SwOp o, SwOp nx, float (&fr)[SW_FM], const float* bias, const float* x, float* y, int mode,
                    const float* mask, float* scr) {
    o.A = sw_uniptr(o.A);
    o.Kc = sw_uni(o.Kc);
    o.No = sw_uni(o.No);
    nx.A = sw_uniptr(nx.A);
    nx.Kc = sw_uni(nx.Kc);
    nx.No = sw_uni(nx.No);
    if (bias) bias = sw_uniptr(bias);
    x = lds_ptr(x);
    y = lds_ptr(y);
    scr = lds_ptr(scr);
    if (mask) mask = lds_ptr(mask);
    int ntile, S, cks, nt2, S2, ck2;
    sw_plan(o.Kc, o.No, ntile, S, cks);
    sw_plan(nx.Kc, nx.No, nt2, S2, ck2);
    const int tid = threadIdx.x, w = sw_uni(tid >> 6), lane = tid & 63, li = lane & 15, lk = lane >> 4;
    const bool mine = w < ntile * S;
    const int tile = mine ? w % ntile : 0, ch = mine ? w / ntile : 0;
    const int u2 = w < nt2 * S2 ? w : 0;
    const int tile2 = u2 % nt2, chn = u2 / nt2;
    const rsrc_t rN = __builtin_amdgcn_make_buffer_rsrc((void*)nx.A, (short)0, nx.Kc * nx.No * 4, 0x00020000);
    // the bias values this thread adds, loaded before the refills: a wait for a load issued
    // after them would also wait for every refill in flight (vmcnt counts in order)
    // (S == 1: the lane's 4 outputs 16 tile + 4 lk + r; S > 1: output (tid + i SW_NT) / R of the
    // reduction pass; outputs >= No read 0)
    float bq[4] = {0.f, 0.f, 0.f, 0.f};
    if (bias) {
        const rsrc_t rB = __builtin_amdgcn_make_buffer_rsrc((void*)bias, (short)0, o.No * 4, 0x00020000);
#pragma unroll
        for (int i = 0; i < 4; ++i)
            bq[i] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
                                                  rB, (S == 1 ? 16 * tile + 4 * lk + i : (tid + i * SW_NT) / R) * 4, 0, 0));
    }
    // one address VGPR per operand: the k-step part of every offset is wave-uniform (the load's
    // SGPR offset; the LDS read's immediate)
    const int voff = ((4 * chn * ck2 + lk) * nx.No + 16 * tile2 + li) * 4, sstep = 16 * nx.No;
    const float* xl = x + (4 * ch * cks + lk) * R + li;
    f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
    const bool mine2 = w < nt2 * S2;
    if (mine && mine2) sw_chain<true, true>(fr, acc, xl, cks, rN, voff, sstep, ck2);
    else if (mine) sw_chain<true, false>(fr, acc, xl, cks, rN, voff, sstep, ck2);
    else if (mine2) sw_chain<false, true>(fr, acc, xl, cks, rN, voff, sstep, ck2);
    if (mine) {
        // acc[r]: output m = 16 tile + 4 lk + r, column li
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int m = 16 * tile + 4 * lk + r;
            if (S == 1) {
                if (m < o.No) {
                    float v = acc[r] + bq[r];
                    if (mode == 1) v = fmaxf(v, 0.f);
                    if (mode == 2 && !(mask[m * R + li] > 0.f)) v = 0.f;
                    y[m * R + li] = v;
                }
            } else {
                scr[(ch * ntile * 16 + m) * R + li] = acc[r];
            }
        }
    }
    __syncthreads();
    if (S > 1) {  // (No <= 128 here: ntile S <= 16 with S >= 2; q < 4 SW_NT)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int q = tid + i * SW_NT;
            if (q < o.No * R) {
                const int m = q / R, c = q % R;
                float v = scr[m * R + c];
                for (int c2 = 1; c2 < S; ++c2) v += scr[(c2 * ntile * 16 + m) * R + c];
                v += bq[i];
                if (mode == 1) v = fmaxf(v, 0.f);
                if (mode == 2 && !(mask[q] > 0.f)) v = 0.f;
                y[q] = v;
            }
        }
        __syncthreads();
    }
    // every bias value is read (no load result left dead in flight: see sw_chain)
    asm volatile("" ::"v"(bq[0]), "v"(bq[1]), "v"(bq[2]), "v"(bq[3]));
}

// threadIdx.x through an opaque copy: per-thread addresses derived from it inside a time loop
// are recomputed where used instead of hoisted out of the loop and spilled (each spill reload
// was a vmcnt(0) that also waited for the next op's fragment refills)
DEV int opaque_tid() {
    int v;
    asm volatile("v_mov_b32 %0, %1" : "=v"(v) : "v"((int)threadIdx.x));
    return v;
}

// record of one (block, step) in a.seq: xhat [K0][R] | rstd [R] | acts[0..n-1] | the step's own
// output gradient [D][R] | (sweep path) g_i [dims[i + 1]][R], i = 0..n-1 (each layer's output
// gradient after the ReLU mask: the dW operands)
__global__ __launch_bounds__(SW_NT) void em_sweep_kernel(const StepArgs a) {
    extern __shared__ __attribute__((aligned(16))) float lds[];
    __shared__ float lsum[NLOG][R];
    __shared__ float lab[R];
    __shared__ long long rowbase[R];
    __shared__ float mu_s[R], rs_s[R], cs[2][R];
    const int tid = threadIdx.x, blk = blockIdx.x;
#ifdef FQ_DIAG  // phase times of block 0 (s_memrealtime, 100 MHz), summed over the steps
    __shared__ unsigned long long ph[EM_PH_N];
    unsigned long long ph_prev = 0;
    const bool ph_on = a.probe != nullptr && blk == 0;
    if (ph_on && tid < EM_PH_N) ph[tid] = 0;
    auto stamp = [&](int i) {
        if (ph_on && threadIdx.x == 0) {
            const unsigned long long now = __builtin_amdgcn_s_memrealtime();
            if (i >= 0) ph[i] += now - ph_prev;
            ph_prev = now;
        }
    };
#else
    auto stamp = [](int) {};
#endif
    const Net& N = a.net;
    const Net& TP = a.tpn;
    const int D = a.D, A = a.A, T = a.T, n = N.n, m = a.tw > 0.f ? TP.n : 0;
    const int K0 = N.dims[0];
    int maxd = 0;
    for (int i = 0; i <= n; ++i) maxd = max(maxd, N.dims[i]);
    for (int i = 0; i <= m; ++i) maxd = max(maxd, TP.dims[i]);
    // LDS: x0, xhat [K0][R] | acts[0..n] | gA, gB, gC [maxd][R] | nobs [D][R] | tp acts (or pred
    // [D][R]) | carry [D][R] | scr [SW_SCR] | ln grad sums [2][K0]
    float* x0 = lds;
    float* xhat = x0 + K0 * R;
    // (layer buffers by computed offset: a runtime-indexed array of LDS pointers went to scratch)
    float* const acts0 = xhat + K0 * R;
    auto acts = [&](int i) {
        float* p = acts0;
        for (int j = 0; j < i; ++j) p += N.dims[j] * R;
        return lds_ptr(p);
    };
    float* gA = acts(n) + N.dims[n] * R;
    float* gB = gA + maxd * R;
    float* gC = gB + maxd * R;
    float* nobs = gC + maxd * R;
    float* const tacts0 = nobs + D * R;
    auto tacts = [&](int i) {
        float* p = tacts0;
        for (int j = 0; j < i; ++j) p += TP.dims[j] * R;
        return lds_ptr(p);
    };
    float* carry = tacts(m) + (m > 0 ? TP.dims[m] * R : D * R);
    float* scr = carry + D * R;
    float* lnacc = scr + SW_SCR;   // [2][K0] LayerNorm grad sums over t
    float* lnp = lnacc + 2 * K0;   // [2][K0] LayerNorm scale, bias (no global load inside the sweeps)

    if (tid < R) {
        const int gr = blk * R + tid;
        long long base = (long long)gr * T;
        if (!a.injected) {  // MultistepLoader windows, as em_seq_grad_kernel
            uint32_t c[4] = {(uint32_t)gr, (uint32_t)a.step, 0xE5u, 0u};
            philox(c, (uint32_t)a.seed, (uint32_t)(a.seed >> 32));
            const long long n_ep = a.n_rows / a.ep_len;
            const long long ep = (long long)((((uint64_t)c[1] << 32) | c[0]) % (uint64_t)n_ep);
            const long long st = (long long)(c[2] % (uint32_t)(a.ep_len - T));
            base = ep * a.ep_len + st;
        }
        rowbase[tid] = base;
    }
    // every LDS float finite before the first op: a chain reads x past its operand (times zeros)
    for (int q = tid; q < (int)(lnp - lds); q += SW_NT) lds[q] = 0.f;
    for (int q = tid; q < NLOG * R; q += SW_NT) lsum[q / R][q % R] = 0.f;
    for (int q = tid; q < 2 * K0; q += SW_NT) {
        lnacc[q] = 0.f;
        lnp[q] = q < K0 ? a.params[a.net.ln_scale + q] : a.params[a.net.ln_bias + q - K0];
    }
    __syncthreads();

    const float* P = a.params;
    const float norm = 1.0f + a.tw;
    const float inv_n = 1.0f / ((float)a.B * (float)T);
    const float gscale = 2.0f / ((float)a.B * (float)T * D) / norm;
    float* const sq = a.seq + (long long)blk * T * a.seq_stride;
    int act_floats = 0;
    for (int i = 0; i < n; ++i) act_floats += N.dims[i] * R;
    const int off_g0 = K0 * R + R + act_floats + D * R;  // g_i from here (g_{n-1} first)

    // ---- the forward sweep's op program: n layers, then (tw > 0) the frozen termination
    // predictor's m layers and its m dX ops
    const int nfw = n + 2 * m;
    auto fw_op = [&](int j) -> SwOp {
        if (j < n) return SwOp{P + N.w[j], N.dims[j], N.dims[j + 1]};
        if (j < n + m) return SwOp{a.tp + TP.w[j - n], TP.dims[j - n], TP.dims[j - n + 1]};
        const int i = m - 1 - (j - n - m);
        return SwOp{a.tpt + TP.w[i], TP.dims[i + 1], TP.dims[i]};
    };
    float fr[SW_FM];
    sw_load(fw_op(0), fr);
    // the next step's input rows (actions; observations at t = 0 only; next observations; rewards),
    // one value per thread, loaded a step ahead
    const int nin = (A + D + 1) * R;
    auto in_load = [&](int t, int tid) -> float {
        if (tid >= nin || t >= T) return 0.f;
        const int r = tid % R, f = tid / R;
        const long long row = rowbase[r] + t;
        if (f < A) return a.act[row * A + f];
        if (f < A + D) return a.nobs[row * D + (f - A)];
        return a.rew[row];
    };
    float inx = in_load(0, tid);
    for (int q = tid; q < D * R; q += SW_NT) x0[q] = a.obs[rowbase[q % R] * D + q / R];  // observations[:, 0]

    stamp(-1);
    for (int t = 0; t < T; ++t) {
        const int tid = opaque_tid();
        if (tid < nin) {
            const int r = tid % R, f = tid / R;
            if (f < A) x0[(D + f) * R + r] = inx;
            else if (f < A + D) nobs[(f - A) * R + r] = inx;
            else lab[r] = inx == 0.f ? 1.f : 0.f;
        }
        inx = in_load(t + 1, tid);
        __syncthreads();
        stamp(0);
        if (tid < R) {
            float s1 = 0.f, s2 = 0.f;
            for (int k = 0; k < K0; ++k) {
                const float v = x0[k * R + tid];
                s1 += v;
                s2 += v * v;
            }
            const float mu = s1 / K0;
            mu_s[tid] = mu;
            rs_s[tid] = 1.0f / sqrtf(fmaxf(s2 / K0 - mu * mu, 0.f) + 1e-6f);
        }
        __syncthreads();
        stamp(26);
        for (int q = tid; q < K0 * R; q += SW_NT) {
            const int k = q / R, r = q % R;
            const float xh = (x0[q] - mu_s[r]) * rs_s[r];
            xhat[q] = xh;
            acts0[q] = xh * lnp[k] + lnp[K0 + k];
        }
        __syncthreads();
        stamp(1);
        float* src = gB;  // the termination predictor's backward ping-pong
        float* dst = gC;
        for (int j = 0; j < nfw; ++j) {
            const SwOp o = fw_op(j), on = fw_op(j + 1 < nfw ? j + 1 : 0);  // (past the last op: the next step's first)
            if (j < n) {
                sw_compute(o, on, fr, P + N.b[j], acts(j), acts(j + 1), j < n - 1 ? 1 : 0, nullptr, scr);
                if (j == n - 1) {
                    // pred = out + obs; MSE; d loss / d pred (gA); the termination predictor's input
                    const float* out = acts(n);
                    float* pred = tacts(0);
                    for (int q = tid; q < D * R; q += SW_NT) {
                        const float p = out[q] + x0[q];
                        const float d = p - nobs[q];
                        pred[q] = p;
                        gA[q] = gscale * d;
                        atomicAdd(&lsum[0][q % R], d * d);
                    }
                    __syncthreads();
                }
            } else if (j < n + m) {
                const int i = j - n;
                sw_compute(o, on, fr, a.tp + TP.b[i], tacts(i), tacts(i + 1), i < m - 1 ? 1 : 0, nullptr, scr);
                if (i == m - 1) {  // weighted BCE of the logit (tp_score)
                    if (tid < R) {
                        const float x = tacts(m)[tid], z = lab[tid], w = a.ttw;
                        const float ce = softplus(x) - x * z;
                        lsum[1][tid] += (z > 0.f ? w * ce : ce) / (w + 1.f);
                        lsum[2][tid] += z > 0.f ? ce : 0.f;
                        lsum[3][tid] += z > 0.f ? 0.f : ce;
                        lsum[4][tid] += z;
                        lsum[5][tid] += 1.f - z;
                        const float p = 1.0f / (1.0f + expf(-x));
                        src[tid] = (z > 0.f ? w : 1.f) / (w + 1.f) * (p - z) * inv_n;
                    }
                    __syncthreads();
                }
            } else {
                const int i = m - 1 - (j - n - m);
                sw_compute(o, on, fr, nullptr, src, dst, i > 0 ? 2 : 0, i > 0 ? tacts(i) : nullptr, scr);
                float* tmp = src;
                src = dst;
                dst = tmp;
                if (i == 0) {
                    const float* sp = lds_ptr(src);
                    for (int q = tid; q < D * R; q += SW_NT) gA[q] += a.tw / norm * sp[q];
                    __syncthreads();
                }
            }
            stamp(2 + min(j, 11));
        }
        if (a.train) {
            float* st = sq + (long long)t * a.seq_stride;
            for (int q = tid; q < K0 * R; q += SW_NT) st[q] = xhat[q];
            if (tid < R) st[K0 * R + tid] = rs_s[tid];
            float* sa = st + K0 * R + R;
            for (int q = tid; q < act_floats; q += SW_NT) sa[q] = acts0[q];  // acts[0..n-1] contiguous
            float* sg = sa + act_floats;
            for (int q = tid; q < D * R; q += SW_NT) sg[q] = gA[q];
        }
        stamp(27);
        const float* pred = tacts(0);
        for (int q = tid; q < D * R; q += SW_NT) x0[q] = pred[q];  // the next step's observation
        __syncthreads();
        stamp(14);
    }
    if (tid < NLOG) {
        float s = 0.f;
        for (int r = 0; r < R; ++r) s += lsum[tid][r];
        a.logs[(long long)blk * NLOG + tid] = s;
    }
    if (!a.train) return;
    // the backward reads records other threads stored (the last one just now): every store of
    // the forward sweep complete before any wave goes on (__syncthreads waits for LDS only)
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();

    // ---- the backward sweep: dX chain, LayerNorm backward and carry, t = T-1 .. 0
    auto bw_op = [&](int j) -> SwOp {  // j = 0..n-1: layer n-1-j's dX from W^T
        const int i = n - 1 - j;
        return SwOp{a.wt + N.w[i], N.dims[i + 1], N.dims[i]};
    };
    sw_load(bw_op(0), fr);
    // the step's record (xhat | rstd | acts[1..n-1] for the masks | own output gradient), a step
    // ahead in registers (RQ per thread), then into LDS at the step's start
    constexpr int RQ = SW_RQ;
    const int n_rec = K0 * R + R + act_floats + D * R;
    float rec[RQ];
    auto rec_load = [&](int t, int tid) {
        const float* st = sq + (long long)max(t, 0) * a.seq_stride;
#pragma unroll
        for (int j = 0; j < RQ; ++j) rec[j] = st[min(tid + j * SW_NT, n_rec - 1)];
    };
    rec_load(T - 1, tid);
    for (int t = T - 1; t >= 0; --t) {
        const int tid = opaque_tid();
        float* st = sq + (long long)t * a.seq_stride;
        {
            float* const a0 = acts0;
            const int n1 = K0 * R, n2 = n1 + R, n3 = n2 + act_floats;
#pragma unroll
            for (int j = 0; j < RQ; ++j) {
                const int q = tid + j * SW_NT;
                if (q < n1) xhat[q] = rec[j];
                else if (q < n2) rs_s[q - n1] = rec[j];
                else if (q < n3) a0[q - n2] = rec[j];
                else if (q < n_rec) gA[q - n3] = rec[j];
            }
        }
        stamp(28);
        rec_load(t - 1, tid);
        stamp(29);
        __syncthreads();
        stamp(15);
        for (int q = tid; q < D * R; q += SW_NT) {
            const float gv = gA[q] + (t < T - 1 ? carry[q] : 0.f);
            gA[q] = gv;
            carry[q] = gv;  // the residual path: pred_t = out_t + obs_t
        }
        __syncthreads();
        stamp(16);
        float* g = gA;
        float* gn = gB;
        float* sgi = st + off_g0;
        for (int j = 0; j < n; ++j) {
            const int i = n - 1 - j;
            for (int q = tid; q < N.dims[i + 1] * R; q += SW_NT) sgi[q] = lds_ptr(g)[q];  // g_i for dW
            sgi += N.dims[i + 1] * R;
            sw_compute(bw_op(j), bw_op(j + 1 < n ? j + 1 : 0), fr, nullptr, g, gn, i > 0 ? 2 : 0,
                       i > 0 ? acts(i) : nullptr, scr);
            float* tmp = g;
            g = gn;
            gn = tmp;
            stamp(17 + min(j, 7));
        }
        // g = grad w.r.t. the LayerNorm output [K0][R]
        g = lds_ptr(g);
        if (tid < K0) {
            float ss = 0.f, sb = 0.f;
            for (int r = 0; r < R; ++r) {
                ss += g[tid * R + r] * xhat[tid * R + r];
                sb += g[tid * R + r];
            }
            lnacc[tid] += ss;
            lnacc[K0 + tid] += sb;
        }
        if (tid < R) {
            float c1 = 0.f, c2 = 0.f;
            for (int k = 0; k < K0; ++k) {
                const float gy = g[k * R + tid] * lnp[k];
                c1 += gy;
                c2 += gy * xhat[k * R + tid];
            }
            cs[0][tid] = c1 / K0;
            cs[1][tid] = c2 / K0;
        }
        __syncthreads();
        stamp(30);
        for (int q = tid; q < D * R; q += SW_NT) {
            const int k = q / R, r = q % R;
            carry[q] += rs_s[r] * (g[q] * lnp[k] - cs[0][r] - xhat[q] * cs[1][r]);
        }
        __syncthreads();
        stamp(25);
    }
#ifdef FQ_DIAG
    if (ph_on && tid < EM_PH_N) a.probe[tid] += ph[tid];
#endif
    // LayerNorm grads into T chunk 0's partials (the other chunks' are zero: em_seq_dw_kernel
    // writes the Dense leaves of every chunk)
    for (int c = 0; c < a.tchunks; ++c) {
        float* pg = a.part + (long long)(blk * a.tchunks + c) * a.P;
        for (int k = tid; k < K0; k += SW_NT) {
            pg[N.ln_scale + k] = c == 0 ? lnacc[k] : 0.f;
            pg[N.ln_bias + k] = c == 0 ? lnacc[K0 + k] : 0.f;
        }
    }
}

// dW_i[k][f] = sum over the chunk's steps t and rows r of acts_i[t][k][r] g_i[t][f][r], db_i[f] =
// sum of g_i[t][f][r]; block = (sequence block b, T chunk c, layer i, 64 x 64 tile); 4 waves of
// 2 x 2 16 x 16 tiles (v_mfma_f32_16x16x4_f32, the contraction over the 16 rows of a step);
// each step's [64][R] operand slices staged through LDS, double-buffered
struct SeqDwArgs {
    const float* seq;
    long long seq_stride;
    float* part;
    long long P;
    Net net;
    int T, tchunks, K0, D;
    int first[MAXL + 1];  // prefix of per-layer tile counts
};
__global__ __launch_bounds__(256) void em_seq_dw_kernel(const SeqDwArgs a) {
    __shared__ __attribute__((aligned(16))) float As[2][64 * R], Bs[2][64 * R];
    const int per = a.first[a.net.n];
    const int bc = blockIdx.x / per, tl = blockIdx.x % per;  // bc = b tchunks + c
    const int b = bc / a.tchunks, c = bc % a.tchunks;
    int i = 0;
    while (i + 1 < a.net.n && tl >= a.first[i + 1]) ++i;
    const int K = a.net.dims[i], Nn = a.net.dims[i + 1];
    const int tf = (Nn + 63) / 64, lt = tl - a.first[i];
    const int k0 = 64 * (lt / tf), f0 = 64 * (lt % tf);
    // offsets of acts_i and g_i inside a record
    int oa = a.K0 * R + R, og = 0;
    for (int j = 0; j < i; ++j) oa += a.net.dims[j] * R;
    int act_floats = 0;
    for (int j = 0; j < a.net.n; ++j) act_floats += a.net.dims[j] * R;
    og = a.K0 * R + R + act_floats + a.D * R;
    for (int j = a.net.n - 1; j > i; --j) og += a.net.dims[j + 1] * R;  // g_{n-1} first
    const int t0 = a.T * c / a.tchunks, t1 = a.T * (c + 1) / a.tchunks;
    const float* sq = a.seq + (long long)b * a.T * a.seq_stride;
    const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63, li = lane & 15, lk = lane >> 4;
    const int wk = (w >> 1) * 32, wf = (w & 1) * 32;
    // staging: thread -> one float4 of each slice ([64][R] = 256 float4); rows past K / N read as 0
    const int sr = tid >> 2, sc = (tid & 3) * 4;
    auto ld = [&](int t, float4& va, float4& vb) {
        const float* st = sq + (long long)t * a.seq_stride;
        va = k0 + sr < K ? *reinterpret_cast<const float4*>(st + oa + (k0 + sr) * R + sc) : float4{0.f, 0.f, 0.f, 0.f};
        vb = f0 + sr < Nn ? *reinterpret_cast<const float4*>(st + og + (f0 + sr) * R + sc) : float4{0.f, 0.f, 0.f, 0.f};
    };
    f32x4 acc[2][2];
#pragma unroll
    for (int x = 0; x < 2; ++x)
#pragma unroll
        for (int y = 0; y < 2; ++y) acc[x][y] = f32x4{0.f, 0.f, 0.f, 0.f};
    float bsum = 0.f;
    float4 va, vb;
    ld(t0, va, vb);
    *reinterpret_cast<float4*>(&As[0][sr * R + sc]) = va;
    *reinterpret_cast<float4*>(&Bs[0][sr * R + sc]) = vb;
    __syncthreads();
    for (int t = t0; t < t1; ++t) {
        const int cur = (t - t0) & 1;
        if (t + 1 < t1) ld(t + 1, va, vb);
        const float* Ac = As[cur];
        const float* Bc = Bs[cur];
#pragma unroll
        for (int s = 0; s < R / 4; ++s) {
            float av[2], bv[2];
#pragma unroll
            for (int x = 0; x < 2; ++x) av[x] = Ac[(wk + 16 * x + li) * R + 4 * s + lk];
#pragma unroll
            for (int y = 0; y < 2; ++y) bv[y] = Bc[(wf + 16 * y + li) * R + 4 * s + lk];
#pragma unroll
            for (int x = 0; x < 2; ++x)
#pragma unroll
                for (int y = 0; y < 2; ++y) acc[x][y] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[x], bv[y], acc[x][y], 0, 0, 0);
        }
        if (k0 == 0 && tid < 64) {
            const float4* row = reinterpret_cast<const float4*>(&Bc[tid * R]);
            float s = 0.f;
#pragma unroll
            for (int q = 0; q < R / 4; ++q) s += row[q].x + row[q].y + row[q].z + row[q].w;
            bsum += s;
        }
        if (t + 1 < t1) {
            *reinterpret_cast<float4*>(&As[cur ^ 1][sr * R + sc]) = va;
            *reinterpret_cast<float4*>(&Bs[cur ^ 1][sr * R + sc]) = vb;
        }
        __syncthreads();
    }
    float* pg = a.part + (long long)bc * a.P;
    // acc[x][y][r]: k = k0 + wk + 16 x + 4 lk + r, f = f0 + wf + 16 y + li
#pragma unroll
    for (int x = 0; x < 2; ++x)
#pragma unroll
        for (int y = 0; y < 2; ++y)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int k = k0 + wk + 16 * x + 4 * lk + r, f = f0 + wf + 16 * y + li;
                if (k < K && f < Nn) pg[a.net.w[i] + (long long)k * Nn + f] = acc[x][y][r];
            }
    if (k0 == 0 && tid < 64 && f0 + tid < Nn) pg[a.net.b[i] + f0 + tid] = bsum;
}

struct AdamArgsEm {
    float* params;
    float* wt;                          // W^T copy, refreshed with the update
    Net net;
    float *m, *v;
    const float* part;
    long long P;
    int blocks;
    float lr, bc1, bc2;
};

// Fixed-order sum of the block partials + optax.adam
__global__ __launch_bounds__(256) void em_adam_kernel(const AdamArgsEm a) {
    const long long p = (long long)blockIdx.x * 256 + threadIdx.x;
    if (p >= a.P) return;
    float g = 0.f;
    for (int b = 0; b < a.blocks; ++b) g += a.part[(long long)b * a.P + p];
    const float m = 0.1f * g + 0.9f * a.m[p];
    const float v = 0.001f * (g * g) + 0.999f * a.v[p];
    a.m[p] = m;
    a.v[p] = v;
    const float np = a.params[p] + (-a.lr) * ((m / a.bc1) / (sqrtf(v / a.bc2) + 1e-8f));
    a.params[p] = np;
    for (int i = 0; i < a.net.n; ++i) {
        const long long o = p - a.net.w[i];
        const int K = a.net.dims[i], N = a.net.dims[i + 1];
        if (o >= 0 && o < (long long)K * N) a.wt[a.net.w[i] + (o % N) * K + o / N] = np;
    }
}

}  // namespace em
}  // namespace fq

// ===================================================================== ABI ==
using namespace fq::em;

namespace {
thread_local std::string em_err;
struct EmErr {
    int code;
    std::string msg;
};
#define EMCHK(x)                                                                          \
    do {                                                                                  \
        hipError_t e_ = (x);                                                              \
        if (e_ != hipSuccess) throw EmErr{FQLPOP_E_HIP, std::string(#x) + ": " + hipGetErrorString(e_)}; \
    } while (0)
#define EMARG(c, m)                                          \
    do {                                                     \
        if (!(c)) throw EmErr{FQLPOP_E_ARG, std::string(m)}; \
    } while (0)
template <class F>
int em_guard(F&& f) {
    try {
        f();
        em_err.clear();
        return FQLPOP_OK;
    } catch (const EmErr& e) {
        em_err = e.msg;
        fq::set_last_error(e.msg.c_str());
        return e.code;
    }
}

// flax leaf order (path-sorted): Dense_i/bias, Dense_i/kernel ..., LayerNorm_0/bias, LayerNorm_0/scale
Net layout(int in, int nh, const int* hid, int out, bool ln, long long* total) {
    Net n{};
    n.n = nh + 1;
    EMARG(n.n <= MAXL, "too many layers");
    n.dims[0] = in;
    for (int i = 0; i < nh; ++i) n.dims[i + 1] = hid[i];
    n.dims[nh + 1] = out;
    long long o = 0;
    for (int i = 0; i < n.n; ++i) {
        n.b[i] = o;
        o += n.dims[i + 1];
        n.w[i] = o;
        o += (long long)n.dims[i] * n.dims[i + 1];
    }
    n.ln_scale = n.ln_bias = -1;
    if (ln) {
        n.ln_bias = o;
        o += in;
        n.ln_scale = o;
        o += in;
    }
    *total = o;
    return n;
}

// Flat params with every Dense kernel [in][out] replaced by its transpose [out][in]
std::vector<float> transposed(const Net& n, const float* p, long long P) {
    std::vector<float> t(p, p + P);
    for (int i = 0; i < n.n; ++i) {
        const int K = n.dims[i], N = n.dims[i + 1];
        for (int k = 0; k < K; ++k)
            for (int f = 0; f < N; ++f) t[n.w[i] + (long long)f * K + k] = p[n.w[i] + (long long)k * N + f];
    }
    return t;
}
}  // namespace

struct fqlpop_emtrain {
    fqlpop_emtrain_config cfg{};
    int device = 0;
    Net net{}, tpn{};
    long long P = 0, PT = 0;
    float *params = nullptr, *m = nullptr, *v = nullptr, *part = nullptr, *logs = nullptr, *tp = nullptr;
    float *wt = nullptr, *tpt = nullptr;  // W^T copies (the backward's dX reads)
    float *d_obs = nullptr, *d_act = nullptr, *d_rew = nullptr, *d_nobs = nullptr;
    long long n_rows = 0;
    float *i_obs = nullptr, *i_act = nullptr, *i_rew = nullptr, *i_nobs = nullptr;
    unsigned char* i_keep = nullptr;
    long long count = 0;
    int blocks = 0;
    int lds_bytes = 0;
    int T = 1;                   // rows per sequence of a batch (FQLPOP_EM_MULTISTEP: sequence_length)
    float* seq = nullptr;        // multistep: per-(block, step) activation store
    long long seq_stride = 0;
    unsigned long long* probe = nullptr;  // diagnostic builds: sweep phase sums (mapped host memory)
    long long probe_launches = 0;
    bool sweep = false;          // multistep through em_sweep_kernel + em_seq_dw_kernel (sw_fits)
    int tchunks = 1;             // sweep: T chunks of the dW GEMM (partial sets per block)
    int sweep_lds = 0;
    hipStream_t s = nullptr;
};

static void em_free(fqlpop_emtrain* h) {
    for (void* p : {(void*)h->params, (void*)h->m, (void*)h->v, (void*)h->part, (void*)h->logs, (void*)h->tp,
                    (void*)h->d_obs, (void*)h->d_act, (void*)h->d_rew, (void*)h->d_nobs, (void*)h->i_obs,
                    (void*)h->i_act, (void*)h->i_rew, (void*)h->i_nobs, (void*)h->i_keep, (void*)h->seq,
                    (void*)h->wt, (void*)h->tpt})
        if (p) (void)hipFree(p);
    if (h->s) (void)hipStreamDestroy(h->s);
}

static void em_layouts(const fqlpop_emtrain_config* c, Net* net, long long* P, Net* tpn, long long* PT) {
    EMARG(c->obs_dim > 0 && c->action_dim >= 0, "bad obs/action dims");
    EMARG(c->num_hidden >= 0 && c->num_hidden < MAXL, "bad num_hidden");
    for (int i = 0; i < c->num_hidden; ++i) EMARG(c->hidden_dims[i] > 0 && c->hidden_dims[i] <= 1024, "bad hidden dim");
    if (c->kind == FQLPOP_EM_STATE_PREDICTOR || c->kind == FQLPOP_EM_MULTISTEP) {
        *net = layout(c->obs_dim + c->action_dim, c->num_hidden, c->hidden_dims, c->obs_dim, true, P);
        *PT = 0;
        if (c->termination_weight > 0.f) {
            EMARG(c->tp_num_hidden >= 0 && c->tp_num_hidden < MAXL, "bad tp_num_hidden");
            *tpn = layout(c->obs_dim, c->tp_num_hidden, c->tp_hidden_dims, 1, false, PT);
        } else {
            *tpn = Net{};
            tpn->ln_scale = tpn->ln_bias = -1;
        }
    } else {
        EMARG(c->kind == FQLPOP_EM_TERMINATION,
              "kind must be FQLPOP_EM_STATE_PREDICTOR, FQLPOP_EM_TERMINATION or FQLPOP_EM_MULTISTEP");
        *net = layout(c->obs_dim, c->num_hidden, c->hidden_dims, 1, false, P);
        *tpn = Net{};
        tpn->ln_scale = tpn->ln_bias = -1;
        *PT = 0;
    }
}

// the sweep path takes every Dense op (both directions, the frozen termination predictor's
// too) as one unit per wave, and a step's record in 16 loads per thread
static bool sw_fits(const Net& n, const Net& tpn, bool tp, int D) {
    for (int i = 0; i < n.n; ++i)
        if (!sw_op_fits(n.dims[i], n.dims[i + 1]) || !sw_op_fits(n.dims[i + 1], n.dims[i])) return false;
    if (tp)
        for (int i = 0; i < tpn.n; ++i)
            if (!sw_op_fits(tpn.dims[i], tpn.dims[i + 1]) || !sw_op_fits(tpn.dims[i + 1], tpn.dims[i])) return false;
    long long act = 0;
    for (int i = 0; i < n.n; ++i) act += n.dims[i];
    return (long long)R * (n.dims[0] + 1 + act + D) <= (long long)SW_RQ * SW_NT;
}

extern "C" {

int fqlpop_emtrain_param_count(const fqlpop_emtrain_config* cfg, int64_t* n_params) {
    return em_guard([&] {
        EMARG(cfg && n_params, "null argument");
        Net a, b;
        long long P, PT;
        em_layouts(cfg, &a, &P, &b, &PT);
        *n_params = P;
    });
}

int fqlpop_emtrain_create(const fqlpop_emtrain_config* cfg, const float* params, int64_t n_params, int device,
                          fqlpop_emtrain_t** out) {
    return em_guard([&] {
        EMARG(cfg && params && out, "null argument");
        EMARG(cfg->batch_size > 0 && cfg->batch_size % R == 0, "batch_size must be a positive multiple of 16");
        EMARG(cfg->steps > 0, "steps must be > 0");
        auto h = std::make_unique<fqlpop_emtrain>();
        h->cfg = *cfg;
        h->device = device;
        em_layouts(cfg, &h->net, &h->P, &h->tpn, &h->PT);
        EMARG(n_params == h->P, "params size mismatch");
        EMCHK(hipSetDevice(device));
        // LDS: x0, xhat [K0][R], acts [sum dims][R], gA, gB [maxd][R], nobs [D][R], tp acts
        int maxd = 0, sum = 0, tsum = 0;
        for (int i = 0; i <= h->net.n; ++i) { maxd = std::max(maxd, h->net.dims[i]); sum += h->net.dims[i]; }
        for (int i = 0; i <= h->tpn.n && h->tpn.n > 0; ++i) { maxd = std::max(maxd, h->tpn.dims[i]); tsum += h->tpn.dims[i]; }
        const bool ms = cfg->kind == FQLPOP_EM_MULTISTEP;
        if (ms) {
            EMARG(cfg->sequence_length >= 1, "sequence_length must be >= 1");
            EMARG(cfg->episode_length > cfg->sequence_length, "episode_length must exceed sequence_length");
            h->T = cfg->sequence_length;
        }
        // multistep: + the carried-gradient buffer, + the prediction buffer when no frozen
        // termination predictor owns one
        const long long fl = (long long)R * (2 * h->net.dims[0] + sum + 3 * maxd + cfg->obs_dim + tsum +
                                             (ms ? cfg->obs_dim * (h->tpn.n > 0 ? 1 : 2) : 0));
        EMARG(fl * 4 <= 150 * 1024, "env-model layer widths exceed the LDS budget of the fused step");
        h->lds_bytes = (int)(fl * 4);
        h->blocks = cfg->batch_size / R;
        if (ms && fq::engine_option_em_seq_sweep() && sw_fits(h->net, h->tpn, h->tpn.n > 0, cfg->obs_dim)) {
            const long long sl = fl + SW_SCR + 4 * h->net.dims[0];
            if (sl * 4 <= 160 * 1024) {
                h->sweep = true;
                h->sweep_lds = (int)(sl * 4);
                // dW GEMM blocks: 16-step chunks at least, at most 4 chunks per sequence block
                h->tchunks = std::max(1, std::min(4, h->T / 16));
            }
        }
        const long long P = h->P;
        EMCHK(hipStreamCreateWithFlags(&h->s, hipStreamNonBlocking));
        EMCHK(hipMalloc(&h->params, 4 * P));
        EMCHK(hipMalloc(&h->m, 4 * P));
        EMCHK(hipMalloc(&h->v, 4 * P));
        EMCHK(hipMalloc(&h->part, 4 * P * h->blocks * h->tchunks));
        EMCHK(hipMalloc(&h->logs, 4 * (long long)NLOG * h->blocks));
        EMCHK(hipMemcpy(h->params, params, 4 * P, hipMemcpyHostToDevice));
        EMCHK(hipMalloc(&h->wt, 4 * P));
        const std::vector<float> wt = transposed(h->net, params, P);
        EMCHK(hipMemcpy(h->wt, wt.data(), 4 * P, hipMemcpyHostToDevice));
        EMCHK(hipMemset(h->m, 0, 4 * P));
        EMCHK(hipMemset(h->v, 0, 4 * P));
        EMCHK(hipMemset(h->logs, 0, 4 * (long long)NLOG * h->blocks));
        const long long B = cfg->batch_size * (long long)h->T, D = cfg->obs_dim, A = cfg->action_dim;
        if (ms) {
            long long act = 0;
            for (int i = 0; i < h->net.n; ++i) act += h->net.dims[i];
            long long gfl = 0;  // sweep: each layer's output gradient g_i (the dW operands)
            if (h->sweep)
                for (int i = 0; i < h->net.n; ++i) gfl += h->net.dims[i + 1];
            h->seq_stride = (long long)R * (h->net.dims[0] + 1 + act + D + gfl);
            EMCHK(hipMalloc(&h->seq, 4 * h->seq_stride * h->T * h->blocks));
        }
        EMCHK(hipMalloc(&h->i_obs, 4 * B * D));
        EMCHK(hipMalloc(&h->i_act, 4 * std::max(1LL, B * A)));
        EMCHK(hipMalloc(&h->i_rew, 4 * B));
        EMCHK(hipMalloc(&h->i_nobs, 4 * B * D));
        EMCHK(hipMalloc(&h->i_keep, B * D));
        EMCHK(hipFuncSetAttribute((const void*)em_grad_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, h->lds_bytes));
        EMCHK(hipFuncSetAttribute((const void*)em_seq_grad_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  h->lds_bytes));
        if (h->sweep)
            EMCHK(hipFuncSetAttribute((const void*)em_sweep_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                      h->sweep_lds));
#ifdef FQ_DIAG
        if (h->sweep && std::getenv("FQLPOP_EM_PROBE")) {
            EMCHK(hipHostMalloc((void**)&h->probe, 8 * EM_PH_N, hipHostMallocMapped | hipHostMallocCoherent));
            std::memset(h->probe, 0, 8 * EM_PH_N);
        }
#endif
        *out = h.release();
    });
}

int fqlpop_emtrain_destroy(fqlpop_emtrain_t* h) {
    return em_guard([&] {
        if (!h) return;
        (void)hipSetDevice(h->device);
        (void)hipDeviceSynchronize();
        if (h->probe) {  // diagnostic builds: mean phase times per step of the sweep (block 0)
            std::fprintf(stderr, "[em sweep phases, us per step, %lld launches, T %d]", h->probe_launches, h->T);
            for (int i = 0; i < EM_PH_N; ++i)
                if (h->probe[i])
                    std::fprintf(stderr, " %d:%.2f", i, h->probe[i] * 0.01 / ((double)h->probe_launches * h->T));
            std::fprintf(stderr, "\n");
            (void)hipHostFree(h->probe);
        }
        em_free(h);
        delete h;
    });
}

int fqlpop_emtrain_set_frozen_termination(fqlpop_emtrain_t* h, const float* tp_params, int64_t n) {
    return em_guard([&] {
        EMARG(h && tp_params, "null argument");
        EMARG(h->PT > 0, "no frozen termination predictor in this config (termination_weight == 0)");
        EMARG(n == h->PT, "termination predictor size mismatch");
        EMCHK(hipSetDevice(h->device));
        if (!h->tp) EMCHK(hipMalloc(&h->tp, 4 * h->PT));
        if (!h->tpt) EMCHK(hipMalloc(&h->tpt, 4 * h->PT));
        EMCHK(hipMemcpy(h->tp, tp_params, 4 * h->PT, hipMemcpyHostToDevice));
        const std::vector<float> tt = transposed(h->tpn, tp_params, h->PT);
        EMCHK(hipMemcpy(h->tpt, tt.data(), 4 * h->PT, hipMemcpyHostToDevice));
    });
}

int fqlpop_emtrain_set_dataset(fqlpop_emtrain_t* h, const float* obs, const float* act, const float* rew,
                               const float* next_obs, int64_t n_rows) {
    return em_guard([&] {
        EMARG(h && obs && rew && next_obs && (act || h->cfg.action_dim == 0), "null argument");
        EMARG(n_rows > 0, "n_rows must be > 0");
        if (h->cfg.kind == FQLPOP_EM_MULTISTEP)  // MultistepLoader reshapes to [n / episode_length][episode_length]
            EMARG(n_rows % h->cfg.episode_length == 0, "multistep: n_rows must be a multiple of episode_length");
        EMCHK(hipSetDevice(h->device));
        for (float* p : {h->d_obs, h->d_act, h->d_rew, h->d_nobs})
            if (p) EMCHK(hipFree(p));
        const long long D = h->cfg.obs_dim, A = h->cfg.action_dim;
        EMCHK(hipMalloc(&h->d_obs, 4 * n_rows * D));
        EMCHK(hipMalloc(&h->d_act, 4 * std::max(1LL, n_rows * A)));
        EMCHK(hipMalloc(&h->d_rew, 4 * n_rows));
        EMCHK(hipMalloc(&h->d_nobs, 4 * n_rows * D));
        EMCHK(hipMemcpy(h->d_obs, obs, 4 * n_rows * D, hipMemcpyHostToDevice));
        if (A) EMCHK(hipMemcpy(h->d_act, act, 4 * n_rows * A, hipMemcpyHostToDevice));
        EMCHK(hipMemcpy(h->d_rew, rew, 4 * n_rows, hipMemcpyHostToDevice));
        EMCHK(hipMemcpy(h->d_nobs, next_obs, 4 * n_rows * D, hipMemcpyHostToDevice));
        h->n_rows = n_rows;
    });
}

static StepArgs em_args(fqlpop_emtrain* h, bool train, bool injected) {
    const auto& c = h->cfg;
    StepArgs a{};
    a.kind = c.kind;
    a.train = train ? 1 : 0;
    a.net = h->net;
    a.tpn = h->tpn;
    a.params = h->params;
    a.tp = h->tp;
    a.wt = h->wt;
    a.tpt = h->tpt;
    a.part = h->part;
    a.P = h->P;
    a.logs = h->logs;
    a.injected = injected ? 1 : 0;
    if (injected) {
        a.obs = h->i_obs; a.act = h->i_act; a.rew = h->i_rew; a.nobs = h->i_nobs;
        a.n_rows = (long long)c.batch_size * h->T;
    } else {
        a.obs = h->d_obs; a.act = h->d_act; a.rew = h->d_rew; a.nobs = h->d_nobs;
        a.n_rows = h->n_rows;
    }
    a.seed = c.seed;
    a.step = h->count;
    a.B = c.batch_size; a.D = c.obs_dim; a.A = c.action_dim;
    a.tw = c.kind != FQLPOP_EM_TERMINATION ? c.termination_weight : 0.f;
    a.T = h->T;
    a.ep_len = c.episode_length;
    a.seq = h->seq;
    a.seq_stride = h->seq_stride;
    a.tchunks = h->tchunks;
    if (h->probe && train) {
        unsigned long long* dp = nullptr;
        EMCHK(hipHostGetDevicePointer((void**)&dp, h->probe, 0));
        a.probe = dp;
        ++h->probe_launches;
    }
    a.ttw = c.true_termination_weight;
    a.alpha = c.focal_alpha; a.gamma = c.focal_gamma; a.rate = c.dropout_rate;
    return a;
}

static void em_launch_step(fqlpop_emtrain* h, const StepArgs& a) {
    if (h->sweep) {
        hipLaunchKernelGGL(em_sweep_kernel, dim3(h->blocks), dim3(SW_NT), h->sweep_lds, h->s, a);
        EMCHK(hipGetLastError());
        if (a.train) {
            SeqDwArgs d{};
            d.seq = h->seq; d.seq_stride = h->seq_stride; d.part = h->part; d.P = h->P; d.net = h->net;
            d.T = h->T; d.tchunks = h->tchunks; d.K0 = h->net.dims[0]; d.D = h->cfg.obs_dim;
            int tot = 0;
            for (int i = 0; i < h->net.n; ++i) {
                d.first[i] = tot;
                tot += ((h->net.dims[i] + 63) / 64) * ((h->net.dims[i + 1] + 63) / 64);
            }
            d.first[h->net.n] = tot;
            hipLaunchKernelGGL(em_seq_dw_kernel, dim3(h->blocks * h->tchunks * tot), dim3(256), 0, h->s, d);
        }
    } else if (h->cfg.kind == FQLPOP_EM_MULTISTEP) {
        hipLaunchKernelGGL(em_seq_grad_kernel, dim3(h->blocks), dim3(NT), h->lds_bytes, h->s, a);
    } else {
        hipLaunchKernelGGL(em_grad_kernel, dim3(h->blocks), dim3(NT), h->lds_bytes, h->s, a);
    }
    EMCHK(hipGetLastError());
    if (!a.train) return;
    // optax.cosine_decay_schedule(init, steps)(count), adam bias correction with count + 1
    const auto& c = h->cfg;
    const double cc = (double)std::min<long long>(h->count, c.steps);
    AdamArgsEm ad{};
    ad.params = h->params; ad.wt = h->wt; ad.net = h->net; ad.m = h->m; ad.v = h->v; ad.part = h->part;
    ad.P = h->P; ad.blocks = h->blocks * h->tchunks;
    ad.lr = (float)(c.init_lr * 0.5 * (1.0 + std::cos(3.14159265358979323846 * cc / c.steps)));
    ad.bc1 = (float)(1.0 - std::pow(0.9, (double)(h->count + 1)));
    ad.bc2 = (float)(1.0 - std::pow(0.999, (double)(h->count + 1)));
    hipLaunchKernelGGL(em_adam_kernel, dim3((unsigned)((h->P + 255) / 256)), dim3(256), 0, h->s, ad);
    EMCHK(hipGetLastError());
    ++h->count;
}

static void em_check_ready(fqlpop_emtrain* h) {
    if (h->cfg.kind != FQLPOP_EM_TERMINATION && h->cfg.termination_weight > 0.f && !h->tp)
        throw EmErr{FQLPOP_E_STATE, "termination_weight > 0 needs fqlpop_emtrain_set_frozen_termination"};
}

int fqlpop_emtrain_step(fqlpop_emtrain_t* h, int n_steps) {
    return em_guard([&] {
        EMARG(h && n_steps >= 0, "bad argument");
        EMARG(h->n_rows > 0, "no dataset: call fqlpop_emtrain_set_dataset");
        em_check_ready(h);
        EMCHK(hipSetDevice(h->device));
        for (int i = 0; i < n_steps; ++i) em_launch_step(h, em_args(h, true, false));
    });
}

static void em_upload_batch(fqlpop_emtrain* h, const float* obs, const float* act, const float* rew,
                            const float* next_obs) {
    EMARG(obs && rew && next_obs && (act || h->cfg.action_dim == 0), "null batch array");
    const long long B = (long long)h->cfg.batch_size * h->T, D = h->cfg.obs_dim, A = h->cfg.action_dim;
    EMCHK(hipMemcpyAsync(h->i_obs, obs, 4 * B * D, hipMemcpyHostToDevice, h->s));
    if (A) EMCHK(hipMemcpyAsync(h->i_act, act, 4 * B * A, hipMemcpyHostToDevice, h->s));
    EMCHK(hipMemcpyAsync(h->i_rew, rew, 4 * B, hipMemcpyHostToDevice, h->s));
    EMCHK(hipMemcpyAsync(h->i_nobs, next_obs, 4 * B * D, hipMemcpyHostToDevice, h->s));
}

int fqlpop_emtrain_step_injected(fqlpop_emtrain_t* h, const float* obs, const float* act, const float* rew,
                                 const float* next_obs, const uint8_t* keep_mask) {
    return em_guard([&] {
        EMARG(h, "null handle");
        em_check_ready(h);
        EMCHK(hipSetDevice(h->device));
        em_upload_batch(h, obs, act, rew, next_obs);
        StepArgs a = em_args(h, true, true);
        if (keep_mask) {
            EMCHK(hipMemcpyAsync(h->i_keep, keep_mask, (size_t)h->cfg.batch_size * h->cfg.obs_dim,
                                 hipMemcpyHostToDevice, h->s));
            a.keep = h->i_keep;
        }
        em_launch_step(h, a);
        EMCHK(hipStreamSynchronize(h->s));  // host batch buffers are reused
    });
}

// logs [FQLPOP_EM_LOG_STRIDE] from the per-block sums (layout: include/fqlpop.h)
static void em_logs(fqlpop_emtrain* h, float* out) {
    std::vector<float> lg((size_t)NLOG * h->blocks);
    EMCHK(hipMemcpyAsync(lg.data(), h->logs, 4 * lg.size(), hipMemcpyDeviceToHost, h->s));
    EMCHK(hipStreamSynchronize(h->s));
    double s[NLOG] = {0};
    for (int b = 0; b < h->blocks; ++b)
        for (int k = 0; k < NLOG; ++k) s[k] += lg[(size_t)b * NLOG + k];
    const double B = (double)h->cfg.batch_size * h->T, D = h->cfg.obs_dim;  // scored predictions
    for (int k = 0; k < FQLPOP_EM_LOG_STRIDE; ++k) out[k] = 0.f;
    if (h->cfg.kind != FQLPOP_EM_TERMINATION) {
        const double mse = s[0] / (B * D), tw = h->cfg.termination_weight;
        const double tl = tw > 0 ? s[1] / B : 0.0;
        out[0] = (float)((mse + tw * tl) / (1.0 + tw));
        out[1] = (float)mse;
        out[2] = (float)tl;
        out[3] = (float)(s[4] > 0 ? s[2] / s[4] : NAN);
        out[4] = (float)(s[5] > 0 ? s[3] / s[5] : NAN);
    } else {
        out[0] = (float)(s[1] / B);
        out[1] = (float)(s[2] / (s[4] + 1e-8));
        out[2] = (float)(s[3] / (s[5] + 1e-8));
        out[3] = (float)(s[6] / B);
        out[4] = (float)(s[8] > 0 ? s[7] / s[8] : 1.0);
        out[5] = (float)(s[4] > 0 ? s[7] / s[4] : 1.0);
    }
}

int fqlpop_emtrain_read_logs(fqlpop_emtrain_t* h, float* logs) {
    return em_guard([&] {
        EMARG(h && logs, "null argument");
        EMCHK(hipSetDevice(h->device));
        em_logs(h, logs);
    });
}

int fqlpop_emtrain_eval(fqlpop_emtrain_t* h, const float* obs, const float* act, const float* rew,
                        const float* next_obs, float* logs) {
    return em_guard([&] {
        EMARG(h && logs, "null argument");
        em_check_ready(h);
        EMCHK(hipSetDevice(h->device));
        em_upload_batch(h, obs, act, rew, next_obs);
        em_launch_step(h, em_args(h, false, true));
        em_logs(h, logs);
    });
}

int fqlpop_emtrain_get_params(fqlpop_emtrain_t* h, int which, float* out, int64_t n) {
    return em_guard([&] {
        EMARG(h && out, "null argument");
        EMARG(n == h->P, "params size mismatch");
        EMARG(which >= 0 && which <= 2, "which must be FQLPOP_STATE_PARAMS/ADAM_M/ADAM_V");
        EMCHK(hipSetDevice(h->device));
        const float* src = which == 0 ? h->params : which == 1 ? h->m : h->v;
        EMCHK(hipMemcpyAsync(out, src, 4 * n, hipMemcpyDeviceToHost, h->s));
        EMCHK(hipStreamSynchronize(h->s));
    });
}

int fqlpop_emtrain_get_count(fqlpop_emtrain_t* h, int64_t* count) {
    return em_guard([&] {
        EMARG(h && count, "null argument");
        *count = h->count;
    });
}

int fqlpop_emtrain_sync(fqlpop_emtrain_t* h) {
    return em_guard([&] {
        EMARG(h, "null handle");
        EMCHK(hipSetDevice(h->device));
        EMCHK(hipStreamSynchronize(h->s));
    });
}

}  // extern "C"
