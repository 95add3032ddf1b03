// Internal interface between the HIP kernels (kernels.hip) and the host
// runtime (runtime.cpp).  Not part of the C ABI.
//
// Data layout in HBM: every activation is stored
// FEATURE-MAJOR, x'[feature][row] (row = minibatch element, contiguous), so
// the forward Dense layer  y = x W + b  is computed as  y' = W^T x'  with both
// MFMA operands read straight from memory (W is [in][out] row-major, the flax
// layout).  Every per-member tensor lives at base + slot * slot_stride
// (+ e * ens_stride for the critic ensemble).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace fq {

// Tensor reference: pointer + element stride per population slot and per
// sub-batch index (critic ensemble member).
struct TRef {
    float* p;
    long long ss;  // slot stride
    long long sy;  // ensemble (y) stride
};

inline TRef tref(float* p, long long ss, long long sy = 0) { return TRef{p, ss, sy}; }

// ---------------------------------------------------------------- GEMM ----
// C[i][j] = sum_r A(i,r) B(r,j)   (fp32 in, fp32 accumulate, MFMA 32x32x2)
//   A(i,r) = A_RC ? A[i*lda + r] : A[r*lda + i]
//   B(r,j) = B_RC ? B[j*ldb + r] : B[r*ldb + j]
enum GemmLayout { LAYOUT_FWD = 0, LAYOUT_DX = 1, LAYOUT_DW = 2 };
enum GemmEpi { EPI_STORE = 0, EPI_BIAS = 1, EPI_BIAS_GELU2 = 2, EPI_BIAS_GELU = 3, EPI_ADAM = 4 };

struct GemmArgs {
    TRef A, B, C, C2, bias;
    int M, N, K;
    int lda, ldb, ldc;
    int ny, nz;
    const int* slots;
    // optional timing probe (dominant kernel only): per block {start, end}
    // s_memrealtime stamps (100 MHz), [2 * blockIdx.x + 0/1]
    unsigned long long* probe;
};
// tile: 0 = 64x64, 1 = 128x64 (i x j), 2 = 64x128, 3 = 128x128
void launch_gemm(int layout, int epi, int tile, const GemmArgs& a, hipStream_t s);
// The dominant kernel of the step: Euler-flow hidden layer, forward GEMM with
// bias+GELU epilogue on the 4-stage LDS-DMA ring (its own kernel symbol).
// Requires M % 64 == 0 and N % 64 == 0.
void launch_gemm_euler_hidden(const GemmArgs& a, hipStream_t s);
// variant: bit 0 = K slice 64 (else 32), bit 1 = two accumulator chains
void launch_gemm_variant(int layout, int epi, int tile, int variant, const GemmArgs& a, hipStream_t s);
// Up to GEMM_GROUP_MAX independent dW-layout problems (A and B both
// r-contiguous, EPI_STORE) in one launch; N % BN == 0 for every problem.
constexpr int GEMM_GROUP_MAX = 8;
struct Chunk { long long off; int len; int leaf; };  // element offset into a net's param block
struct AdamArgs {
    const float* p_in;            // parameters read (current buffer, slot stride P)
    float* p_out;                 // parameters written (the other buffer of the pair)
    float *g, *m, *v;             // arenas (slot stride P)
    float* target;                // target arena (slot stride PT) or null
    long long P, PT;
    long long net_off;            // offset of this net inside the params arena
    const Chunk* chunks;          // chunk table of ALL nets (index = stats chunk id)
    const int* ids;               // chunk ids to process (block = ids[blockIdx.x]), or null:
    int n_chunks, chunk_base;     //   chunk ids chunk_base .. chunk_base + n_chunks - 1
    float* stats;                 // [slots][n_total_chunks][3] (max, min, sumsq)
    int n_total_chunks;
    const int* count;
    float lr, tau;
    int nz;
    const int* slots;
};
// Fused optimiser epilogue of the grouped dW launch: problem gi is the kernel
// leaf W_l of one net; its output tile is the gradient, and the epilogue runs
// optax.adam on it (reading p from p_in, writing p_out, m, v in place), the
// target-critic EMA from the pre-update value (critic only), the W_l^T copy
// the streamed backward reads (hidden layers), and the tile's grad stats
// (max, min, sum g^2) at chunk id stat_base[gi] + y * tiles_per_problem + tile.
struct AdamEpi {
    const float* p_in;
    float *p_out, *m, *v, *target, *wt_out;
    long long P, PT, PTT;             // slot strides of params / target / W^T arenas
    long long ens, wt_sy;             // ensemble strides in params and W^T
    long long w_off[GEMM_GROUP_MAX];  // leaf offset inside a params slot (net offset included)
    long long wt_off[GEMM_GROUP_MAX]; // offset inside a W^T slot, -1 = no copy
    int stat_base[GEMM_GROUP_MAX];
    float* stats;                     // [slots][n_total_chunks][3]
    int n_total_chunks;
    const int* count;
    float lr, tau;
    int mode;                         // 0; timing probes (FQLPOP_DW_MODE): 1 = no optimiser pass, 2 = one k-slice,
                                      // 3 = no W^T pass
    int nt;                           // non-temporal optimiser streams: 1 m/v, 2 target, 4 p_in, 8 p_out/W^T
    // the net's small leaves (biases, LN, head) ride in the same launch: blocks past the
    // GEMM tiles run the adam_kernel body on small.ids chunks (small_blocks = chunks x nz)
    AdamArgs small;
    int small_blocks;
};
struct GemmGroupArgs {
    GemmArgs g[GEMM_GROUP_MAX];
    int first[GEMM_GROUP_MAX + 1];   // prefix of per-problem block counts
    int ng;
    AdamEpi adam;                    // used by the fused-Adam launch only
};
// tile: 2 = 64x128, 3 = 128x128 (others 64x64 / 128x64); adam != null: fused
// optimiser epilogue (tile 2 or 3 only), else plain stores into g[i].C; with adam: 6 / 10 =
// 64x128 at BK 16 (3 / 4 blocks per CU)
void launch_gemm_group_dw(int tile, const GemmArgs* gs, int ng, hipStream_t s, const AdamEpi* adam = nullptr);
// tiles per problem of the grouped dW launch (stats chunks of a fused W leaf)
int gemm_group_tiles(int tile, int M, int N);

// --------------------------------------------------- persistent Euler flow --
// Euler steps first..S-1 of the BC flow (compute_flow_actions) for every active
// member in ONE launch.  A block owns 16 minibatch columns of one member for
// the whole chain: the activation slab x'[H][16] stays in LDS across layers
// and steps, the weights stream from L2 into MFMA fragments.  H = 512 only
// (euler_flow_supported); the caller falls back to per-layer launches.
constexpr int EF_MAX_LAYERS = 8;
struct EulerArgs {
    const float* params;                  // params arena (slot stride P)
    long long P;
    long long w_off[EF_MAX_LAYERS + 1];   // Dense_l kernel offset inside a slot (l = 0..L, L = head)
    long long b_off[EF_MAX_LAYERS + 1];   // Dense_l bias offset
    TRef eu;                              // [D+A+1][B] state after step first-1 (s rows, x rows)
    TRef aflow;                           // out [A][B]: clip(x) after the last step
    int D, A, H, L, B, S, first;
    float steps_f;
    int nz;
    const int* slots;
    unsigned long long* probe;            // optional per-block {start, end} stamps
    unsigned long long* phase;            // diagnostics (FQLPOP_PHASE_PROBE): [EF_PHASE_STRIDE] per block
};
// per block: [0] start, then per (step, layer) k-loop start / k-loop end / epilogue end / barrier out
constexpr int EF_PHASE_STRIDE = 4 * 10 * (EF_MAX_LAYERS + 1) + 8;
bool euler_flow_supported(int H, int L, int D, int A, int B);
void launch_euler_flow(const EulerArgs& a, hipStream_t s);

// ------------------------------------------------------- row-wise kernels --
struct LnArgs {           // h = LN(gelu(u)) * gamma + beta, per column
    TRef u, h, mu, rstd, gamma, beta;
    int H, M, ld;         // features, columns, leading dim (columns of buffer)
    int ny, nz;
    const int* slots;
};
void launch_ln_gelu_fwd(const LnArgs& a, hipStream_t s);

enum HeadMode { HEAD_STORE = 0, HEAD_BC_FUSED = 1, HEAD_EULER = 2, HEAD_OS = 3, HEAD_ACT = 4 };
struct HeadArgs {         // out'[j][m] = sum_k W[k][j] h'[k][m] + b[j]
    TRef h, W, b;
    TRef o0, o1, o2, o3;  // mode-dependent outputs (see kernels.hip)
    int H, M, ld, nout;
    int ld0, ld1, ld2, ld3;
    int B, D;             // batch size, obs dim (row offsets into input buffers)
    int last;             // HEAD_EULER: final step (write clipped actions)
    float steps_f;        // flow_steps as float (divisor of the Euler update)
    float t_next;         // HEAD_EULER/BC_FUSED: time row value of the next step
    int ny, nz;
    const int* slots;
};
void launch_head_fwd(int mode, const HeadArgs& a, hipStream_t s);

// ------------------------------------------------ streamed MLP forward ----
// One launch = the whole forward pass of one network (every hidden layer with
// its GELU / LayerNorm, and the head) for all active members and ensemble
// members: a block owns 16 columns for all H = 512 features (slab in LDS),
// weights stream from L2 (same k-loop as the Euler flow).  Stores the
// activations the backward pass needs for columns [st_lo, st_hi), then calls
// the head-mode epilogue of HeadArgs (head_write).
struct StreamArgs {
    const float* params;                  // arena + net offset (slot stride P, ensemble stride ens)
    long long P, ens;
    long long w_off[EF_MAX_LAYERS + 1], b_off[EF_MAX_LAYERS + 1];
    long long g_off[EF_MAX_LAYERS], be_off[EF_MAX_LAYERS];  // LN scale / bias
    const float* x0;                      // input [K0][ld_x] (+ slot * x0_ss), shared by ensemble members
    long long x0_ss;
    int ld_x, K0, L, M;
    float* U[EF_MAX_LAYERS];              // pre-activation [H][ld_s] (+ slot*s_ss + y*s_sy), or null
    float* G[EF_MAX_LAYERS];              // layer output (post GELU / LN) [H][ld_s], or null
    float* MU[EF_MAX_LAYERS];             // LN mean [ld_s] (+ slot*st_ss + y*st_sy)
    float* RS[EF_MAX_LAYERS];             // LN 1/sigma
    long long s_ss, s_sy, st_ss, st_sy;
    int ld_s, st_lo, st_hi;
    int g_hi;                             // G is stored for columns [st_lo, g_hi) only (<= st_hi)
    HeadArgs head;                        // head outputs (head.M/.ld unused)
    int ny, nz;
    const int* slots;
};
bool stream_fwd_supported(int H, int L, int K0, int nout, int M);
void launch_stream_fwd(int head_mode, bool ln, const StreamArgs& a, hipStream_t s);

// --------------------------------- split streamed forward (small populations) --
// The streamed forward / persistent Euler flow with each 16-column tile computed by a
// cluster of F = 2, 4 or 8 blocks that exchange every hidden layer's output through
// L2 / MALL (kernels.hip, "split streamed forward"): bit-identical to the unsplit
// kernels, and F times as many blocks, so that 1-4 members fill the chip.
struct SplitSync {
    unsigned long long* xch;  // exchange words {value, tag}, split_cluster_bytes() per cluster
    unsigned* cnt;            // counters split_counter_stride() apart: [clusters] last-arriver, then the
                              // ticket and the exit counter; zero at launch (the last block of every
                              // launch zeroes them)
    unsigned* gen;            // the site's launch generation (never zeroed; the tags' high bits)
    unsigned* err;            // set to nonzero when a hand-off wait gives up (results then invalid)
};
struct SplitFwdArgs {
    StreamArgs s;           // as launch_stream_fwd (Euler: params, w_off, b_off, x0 = state after step
                            // first - 1 [D+A+1][B], K0 = D+A+1, L, M = B, ny = 1, head.nout = A)
    TRef aflow;             // Euler: out [A][B]
    int D, A, S, first;     // Euler: obs / action dims, flow steps, first step
    float steps_f;
    unsigned long long* probe;   // optional per-block {start, end} stamps
    SplitSync sync;
    unsigned long long* phase;   // diagnostics (FQLPOP_PHASE_PROBE, Euler): [EF_PHASE_STRIDE] per block
    float* pre0;                 // Euler: layer-0 accumulators, split_euler_pre0_floats() per block
};
long long split_cluster_bytes();
constexpr long long split_euler_pre0_floats() { return 2LL * 256 * 16; }  // [h][thread][16]
// the Euler flow's layer-0 form: its observation rows once per launch (split_fwd_kernel PRE0)
bool split_euler_pre0(int K0, int D);
int split_counter_stride();
bool split_fwd_supported(int H, int L, int K0, int nout, int M);
// F = 8, 4 or 2 blocks per 16-column tile; grid = tiles x ny x nz x F blocks of 256 threads
void launch_split_fwd(int head_mode, bool ln, bool euler, int F, const SplitFwdArgs& a, hipStream_t s);

// ----------------------------------------------- streamed MLP backward ----
// One launch = the whole dX chain of one network for all active members and
// ensemble members: from the head-output gradient dout through every hidden
// layer (GELU', LayerNorm backward) down to du_0.  A block owns 16 columns and
// all H = 512 features; du_l stays in LDS as the A operand of the next
// layer's dh = W du (weights streamed from L2).  Writes du_l [H][ld_d] for the
// dW GEMMs and, for columns < Mg, per-block column sums of du (bias grads), of
// dh * xhat and dh (LN scale / bias grads) and of G_{L-1} dout (head kernel
// grad) into `part` [tile][NP]; colsum_reduce folds the tiles into the grads.
struct StreamBwdArgs {
    const float* params;                  // arena + net offset (slot stride P, ensemble stride ens)
    long long P, ens;
    const float* paramsT;                 // transposed hidden kernels W_l^T [out][in] (slot stride PT, ens stride ensT)
    long long PT, ensT;
    long long wt_off[EF_MAX_LAYERS];      // offset of W_l^T (l >= 1) inside one ensemble member's T block
    long long w_off[EF_MAX_LAYERS + 1], b_off[EF_MAX_LAYERS + 1];
    long long g_off[EF_MAX_LAYERS], be_off[EF_MAX_LAYERS];
    const float* dout;                    // [nout][ld_o] (+ slot * dout_ss + y * dout_sy)
    long long dout_ss, dout_sy;
    int ld_o;
    const float* U[EF_MAX_LAYERS];        // pre-activations [H][ld_s] (+ slot*s_ss + y*s_sy), column coff + m
    const float* Ghead;                   // G_{L-1} (head input), same addressing as U
    const float* MU[EF_MAX_LAYERS];       // LN stats [.] (+ slot*st_ss + y*st_sy), column coff + m
    const float* RS[EF_MAX_LAYERS];
    long long s_ss, s_sy, st_ss, st_sy;
    int ld_s, coff;
    float* DU[EF_MAX_LAYERS];             // du_l out [H][ld_d] (+ slot*d_ss + y*d_sy)
    long long d_ss, d_sy;
    int ld_d;
    float* part;                          // [slot][y][tile < Mg/16][NP]
    int NP;
    int L, M, Mg, nout;
    // optional (critic): dQ/da of the actor's action inputs for the columns [Mg, M),
    // da[slot][y][j][m - Mg] = sum_f W_0[D0 + j][f] du_0[f][m], one partial per ensemble member
    float* da;
    long long da_ss, da_sy;
    int ld_da, D0, na;
    int ny, nz;
    const int* slots;
    // optional diagnostics (FQLPOP_PHASE_PROBE): per block [SB_PHASE_STRIDE] s_memrealtime stamps:
    // [0] start, [1] end, then per layer pass (L-1-l): top, stats barrier in/out, slab barrier out,
    // product done
    unsigned long long* phase;
};
constexpr int SB_PHASE_STRIDE = 48;
bool stream_bwd_supported(int H, int L, int nout, int M, int Mg);
void launch_stream_bwd(bool ln, const StreamBwdArgs& a, hipStream_t s);
// Partial index layout of StreamBwdArgs::part (per tile):
//   [0, L*H) bias of layer l;  LN: [L*H, 2L*H) scale, [2L*H, 3L*H) bias;
//   then H*nout head kernel W_L[k][j] at k*nout + j.
inline int stream_bwd_np(int L, int H, int nout, bool ln) { return (ln ? 3 : 1) * L * H + H * nout; }

// Split form of launch_stream_bwd for small populations (F = 8, 4 or 2 blocks per 16-column
// tile, bit-identical; the SplitSync of the launch site, counters zeroed before the launch).
bool split_bwd_supported(int H, int L, int nout, int M, int Mg);
void launch_split_bwd(bool ln, int F, const StreamBwdArgs& a, const SplitSync& sy, hipStream_t s);

struct ColsumArgs {                      // grads[off(p)] = sum over tiles of part[t][p]
    const float* part;
    int NP, tiles;                        // tiles that hold partials (Mg / 16)
    float* grads;                         // arena + net offset (slot stride P, ensemble stride ens)
    long long P, ens;
    long long b_off[EF_MAX_LAYERS], g_off[EF_MAX_LAYERS], be_off[EF_MAX_LAYERS], w5_off;
    int L, H, ln;
    int ny, nz;
    const int* slots;
};
void launch_colsum_reduce(const ColsumArgs& a, hipStream_t s);

// W_l^T copies of the hidden Dense kernels (H x H) for the streamed backward:
// dst[dst_off[i] + j*H + k] = src[src_off[i] + k*H + j] for every matrix i.
constexpr int TR_MAX = 32;
struct TransposeArgs {
    const float* src;
    long long src_ss;             // slot stride of src
    float* dst;
    long long dst_ss;
    long long src_off[TR_MAX], dst_off[TR_MAX];
    int n_mats, H;
    int nz;
    const int* slots;             // null: slot = z
};
void launch_transpose(const TransposeArgs& a, hipStream_t s);


struct BwdArgs {
    TRef dh;              // [H][ld_d] gradient w.r.t. layer output (non-head mode)
    TRef dout, W5;        // head mode: dout'[nout][ld_o], W5[H][nout]
    TRef u, x_head;       // u'[H][ld] pre-activation; x_head'[H][ld] head input (LN output)
    TRef mu, rstd, gamma; // LN
    TRef c1, c2;          // LN row statistics of the backward pass [ld]
    TRef du;              // [H][ld_d] output
    TRef g_b, g_gamma, g_beta, g_W5;  // grads (written, not accumulated)
    int H, M, Mg, ld, ld_d, ld_o, nout;
    int ny, nz;
    const int* slots;
};
void launch_bwd_rowstats(bool head, const BwdArgs& a, hipStream_t s);
void launch_bwd_cols(bool head, bool ln, const BwdArgs& a, hipStream_t s);

struct InGradArgs {       // da'[j][m] = sum_e sum_n W0_e[(D+j)][n] du0_e'[n][off+m]
    TRef W0, du0, da;
    int H, D, A, E, ld, off, M;
    int nz;
    const int* slots;
};
void launch_input_grad(const InGradArgs& a, hipStream_t s);

// --------------------------------------------------------------- batch ----
struct SampleArgs {
    // dataset (row-major) or injected staging (per active member, packed)
    const float *obs, *act, *rew, *mask, *nobs;
    long long n_rows;
    const float* inj_batch;   // non-null => injected mode
    const float* inj_noise;
    const uint64_t* seeds;    // per slot
    const int* count;         // per slot (Adam count == update index)
    int step_add;             // added to count (cross-step groups: a snapshot of count at the group's
                              // start + the step's position in the group)
    unsigned stream_salt;     // distinguishes train / val draws
    int B, D, A;
    // outputs (feature-major)
    TRef os_in;   // [D+A][3B]
    TRef bc_in;   // [D+A+1][2B]
    TRef cr_in;   // [D+A][2B]
    TRef tg_in;   // [D+A][B]
    TRef eu_in;   // [D+A+1][B]
    TRef act_t, x0_t, rew_t, mask_t;  // [A][B], [A][B], [B], [B]
    int nz;
    const int* slots;
};
void launch_sample(const SampleArgs& a, hipStream_t s);

// ---------------------------------------------------------------- loss ----
struct LossArgs {
    TRef q, qt, rew, mask;        // q'[E][2B], qt'[E][B]
    TRef vpred, act, x0, amet;    // [A][B]
    TRef apiraw, aflow, da;       // [A][B]; da: da_n partials at ensemble stride da.sy, summed
    TRef dq;                      // out [E][2B]
    TRef dv;                      // out [A][B]
    TRef dout_os;                 // out [A][B]
    TRef g_cb4, g_bcb4, g_osb4;   // head-bias grads: critic [E] (ens stride), bc [A], os [A]
    TRef info;                    // [16]
    const float* alpha;           // per slot
    int B, A, E, da_n;
    int q_min, normq;
    float discount;
    int nz;
    const int* slots;
};
void launch_loss_critic(const LossArgs& a, hipStream_t s);
void launch_loss_bc(const LossArgs& a, hipStream_t s);
void launch_loss_actor(const LossArgs& a, hipStream_t s);

// ---------------------------------------------------------- optimiser ----
void launch_adam(const AdamArgs& a, hipStream_t s);

struct FinalArgs {
    const float* stats;           // [slots][n_total_chunks][3]
    const int* chunk_leaf;        // leaf id of every chunk
    const int* leaf_first;        // [n_leaves + 1]: a leaf's chunks are [leaf_first[l], leaf_first[l+1])
    int n_total_chunks, n_leaves;
    TRef info;
    int* count;
    int nz;
    const int* slots;
};
void launch_finalize(const FinalArgs& a, hipStream_t s);

// ---------------------------------------------------------------- init ----
struct InitArgs {                 // uniform(-lim, lim) fill of one tensor of one slot
    float* p;
    long long n;
    float lim;                    // 0 => constant fill with `value`
    float value;
    uint64_t seed;
    unsigned salt;
};
void launch_init(const InitArgs& a, hipStream_t s);

// ------------------------------------------- world-model rollout eval ----
// evaluator/evaluation.py:75-114 on task/offline_task_simulated.py:85-107 for
// every active member in ONE launch: per step a = clip(onestep(s, z)),
// s' = BaselineStatePredictor(s, a) (envmodel/baseline.py:25-37: LayerNorm of
// [s, a], Dense+ReLU hidden layers, Dense(obs) + s), terminated =
// TerminationPredictor(s') > 0 (envmodel/termination_predictor.py:14-21),
// until every env has terminated or max_steps.  Block = 16 envs of one member.
constexpr int RO_MAX_LAYERS = 8;   // env-model Dense layers (hidden + output)
constexpr int RO_MAX_W = 512;      // widest env-model layer
struct RolloutArgs {
    const float* params;           // population arena (slot stride P), one-step actor at os_off
    long long P, os_off;
    long long w_off[EF_MAX_LAYERS + 1], b_off[EF_MAX_LAYERS + 1];
    int D, A, L;                   // actor hidden width 512
    const float* sp;               // state predictor params (flat, flax order)
    int sp_n;                      // Dense layers (hidden + output)
    int sp_dims[RO_MAX_LAYERS + 1];
    long long sp_w[RO_MAX_LAYERS], sp_b[RO_MAX_LAYERS], sp_ln_scale, sp_ln_bias;
    const float* tp;               // termination predictor params
    int tp_n;
    int tp_dims[RO_MAX_LAYERS + 1];
    long long tp_w[RO_MAX_LAYERS], tp_b[RO_MAX_LAYERS];
    const float* init_obs;         // [n_envs][D]
    int n_envs, max_steps;
    uint64_t seed;
    const uint64_t* member_seeds;  // per slot: the member key sample_key(seed, alpha) (runtime.cpp)
    const float* noise;            // null or [nz][max_steps][n_envs][A]
    float* out;                    // [nz][n_envs][2]: success, episode length
    float* out_obs;                // null or [nz][n_envs][D]: observation after the last step
    const float* actions;          // non-null: env-model step only, a = actions [n_envs][A] (no actor)
    float* out_logit;              // null or [nz][n_envs]: termination logit of the last step
    int nz;
    const int* slots;
};
bool rollout_supported(int H, int L, int D, int A);
void launch_rollout(const RolloutArgs& a, hipStream_t s);

// The C ABI's thread-local last-error message (runtime.cpp), for entry points
// defined in other translation units (emtrain.hip).
void set_last_error(const char* msg);
// engine option em_seq_sweep (runtime.cpp), read by fqlpop_emtrain_create
int engine_option_em_seq_sweep();

}  // namespace fq
