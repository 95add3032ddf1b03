// Host runtime of libfqlpop.so: the C ABI of include/fqlpop.h.
//
// One handle = one population on one GPU.  The handle owns every device
// buffer (params / grads / Adam moments / target critic arenas, activations,
// datasets) and three HIP streams that carry the update DAG of one population
// step:
//   sF  flow chain : BC-flow forward fused with Euler step 0, Euler steps 1..S-1
//   sB  BC branch  : BC loss, BC backward, BC Adam (after the flow chain)
//   sM  main chain : sampling, one-step actor forward, critic/target forward,
//                    critic loss + backward + Adam/EMA, actor loss (joins sF),
//                    one-step backward + Adam, grad stats (joins sB)
// The whole DAG is captured once into a hipGraph and replayed per step.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <map>
#include <set>
#include <memory>
#include <string>
#include <vector>

#include "../../include/fqlpop.h"
#include "kernels.h"

using namespace fq;

namespace {

thread_local std::string g_err;

struct FqErr {
    int code;
    std::string msg;
};

#define HIPCHK(x)                                                                                 \
    do {                                                                                          \
        hipError_t e_ = (x);                                                                      \
        if (e_ != hipSuccess)                                                                     \
            throw FqErr{FQLPOP_E_HIP, std::string(#x) + " failed: " + hipGetErrorString(e_)};     \
    } while (0)

#define ARGCHK(c, m)                                         \
    do {                                                     \
        if (!(c)) throw FqErr{FQLPOP_E_ARG, std::string(m)}; \
    } while (0)

constexpr long long kAlign = 64;  // floats (256 B)
long long align_up(long long x) { return (x + kAlign - 1) / kAlign * kAlign; }

// Timing-only switches that change or corrupt results (launches left out, phases of the
// fused optimiser switched off, cross-step pipelining without the step's joins, per-block
// phase stamps) exist only in the diagnostic builds (make DIAG=1 / PHASE=1, -DFQ_DIAG).
// The production library reads no environment variable at all: diag_env is nullptr.
#ifdef FQ_DIAG
const char* diag_env(const char* name) { return std::getenv(name); }
#else
const char* diag_env(const char*) { return nullptr; }
#endif

// Engine options (fqlpop_set_engine_option): alternate code paths and stream schedules
// that give the same results (bit-identical, or the per-layer / unfused paths within the
// parity tolerance), read by fqlpop_create.  Test and profiling hooks; the defaults are the
// measured-fastest configuration (DESIGN.md sections 4-5).
struct EngineOptions {
    int euler_fused = 1;   // persistent Euler launch (0: per-layer GEMMs)
    int stream_fwd = 1;    // whole-network forward launches
    int stream_bwd = 1;    // whole-network dX chains
    int fused_adam = 1;    // optimiser in the grouped dW epilogue
    int serial = 0;        // every launch on one stream (uncontended kernel traces)
    int dw_tile_critic = 10, dw_tile_actor = 10;  // grouped dW tile ids (launch_gemm_group_dw)
    int adam_nt = 3;       // non-temporal optimiser streams (AdamEpi::nt bit mask)
    int split = 1;         // small populations: streamed forwards / Euler flow as clusters of 2-8 blocks per
                           // 16-column tile (bit-identical); 0 off, 1 auto, 2 / 4 / 8 blocks where they fit
    int small_sched = 1;   // the 4th-stream schedule: target critic and the critic's TD-column backward on
                           // a 4th stream sX beside the main chain (bit-identical); 0 = three streams
    int split_blocks = 256;  // the most blocks of a split forward / Euler launch (F shrinks to fit)
    int split_sites = 0;   // per-site override of split: 3 bits per launch site (SITE_*: bits 3 site ..),
                           // 0 auto, 1 unsplit, 2 / 3 / 4 = 2 / 4 / 8 blocks per tile (A/B runs)
    int hw_queues = 4;     // the HIP runtime's hardware queues per process (GPU_MAX_HW_QUEUES, which the
                           // caller sets; the Python layer passes it): below 4 the step is captured on
                           // one stream (graph launch and hardware queues)
    int em_seq_sweep = 1;  // env-model multistep training: the 1024-thread BPTT sweep with dW as a separate
                           // GEMM (emtrain.hip); 0 = the round-5 kernel (dW inside the time loop)
};
// (Schedule experiments that measured slower were removed in round 4 and stay in git history
// and DESIGN.md section 5: a 4th stream, stream priorities, the critic optimiser on the main
// chain's queue, first-wave staggering of the fused dW launch, the cross-step critic tail,
// the BC update late in the step, the critic-loss seeds in the critic forward's head, and the
// main chain's early joins.)
EngineOptions g_engine_opts;

// Streams (= parallel branches of the step's graph) the step is captured on.  The HIP
// runtime's graph launch is only safe for branches <= hardware queues (DESIGN.md section 4,
// graph launch and hardware queues), so below kStepBranches queues the step runs on one
// stream.  Any schedule change that adds a stream raises kStepBranches and, through the
// check in graph_for, can never be captured beside fewer queues than it has branches.
constexpr int kStepBranches = 4;  // sM, sF, sB, sX
int step_streams(const EngineOptions& eo) {
    return (eo.serial || eo.hw_queues < kStepBranches) ? 1 : kStepBranches;
}

struct EngineOptionRef {
    const char* name;
    int EngineOptions::*field;
    int lo, hi;
};
const EngineOptionRef kEngineOptions[] = {
    {"euler_fused", &EngineOptions::euler_fused, 0, 1}, {"stream_fwd", &EngineOptions::stream_fwd, 0, 1},
    {"stream_bwd", &EngineOptions::stream_bwd, 0, 1},   {"fused_adam", &EngineOptions::fused_adam, 0, 1},
    {"serial", &EngineOptions::serial, 0, 1},
    {"dw_tile_critic", &EngineOptions::dw_tile_critic, 0, 10},
    {"dw_tile_actor", &EngineOptions::dw_tile_actor, 0, 10},
    {"adam_nt", &EngineOptions::adam_nt, 0, 3},
    {"split", &EngineOptions::split, 0, 8},
    {"small_sched", &EngineOptions::small_sched, 0, 1},
    {"hw_queues", &EngineOptions::hw_queues, 1, 1024},
    {"split_sites", &EngineOptions::split_sites, 0, (1 << 24) - 1},
    {"split_blocks", &EngineOptions::split_blocks, 64, 1024},
    {"em_seq_sweep", &EngineOptions::em_seq_sweep, 0, 1},
};

// ---------------------------------------------------------------- host Philox
void philox_host(uint32_t c[4], uint32_t k0, uint32_t k1) {
    for (int r = 0; r < 10; ++r) {
        const uint64_t p0 = (uint64_t)0xD2511F53u * c[0], p1 = (uint64_t)0xCD9E8D57u * c[2];
        const uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
        const uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
        const uint32_t n0 = hi1 ^ c[1] ^ k0, n2 = hi0 ^ c[3] ^ k1;
        c[0] = n0; c[1] = lo1; c[2] = n2; c[3] = lo0;
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
}

// Sampler key of a member: its seed mixed with the bits of its alpha (splitmix64
// finaliser).  The reference draws every experiment's batches from the global
// np.random stream (trainer/trainer.py:76-81, [EXT] Dataset.sample), so two members
// that share a seed but not an alpha see different batches there; keying the device
// sampler by the seed alone would give them identical minibatches, flow times and
// noises.  Independent of the slot, so a resumed or re-slotted member draws the same
// stream.
uint64_t sample_key(uint64_t seed, float alpha) {
    uint32_t ab;
    std::memcpy(&ab, &alpha, sizeof(ab));
    uint64_t z = seed ^ ((uint64_t)ab << 32 | 0x9E3779B9u);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

// ---------------------------------------------------------------- layout
// Parameter block of one network, flax MLP naming: Dense_l (kernel [in][out],
// bias [out]) and LayerNorm_l (scale, bias) after every hidden Dense.
struct NetLayout {
    std::string name;
    int in_dim = 0, out_dim = 0, L = 0, H = 0, E = 1;
    bool ln = false;
    long long off = 0;        // offset of the net inside its arena
    long long ens_size = 0;   // floats of one ensemble member (aligned)
    std::vector<long long> W, b, gam, bet;  // offsets inside one ensemble member
    int kdim(int l) const { return l == 0 ? in_dim : H; }
    int ndim(int l) const { return l == L ? out_dim : H; }

    void build(const std::string& nm, int in, int out, int nh, int h, int e, bool use_ln) {
        name = nm; in_dim = in; out_dim = out; L = nh; H = h; E = e; ln = use_ln;
        long long o = 0;
        for (int l = 0; l <= L; ++l) {
            W.push_back(o); o = align_up(o + (long long)kdim(l) * ndim(l));
            b.push_back(o); o = align_up(o + ndim(l));
            if (l < L && ln) {
                gam.push_back(o); o = align_up(o + H);
                bet.push_back(o); o = align_up(o + H);
            }
        }
        ens_size = o;
    }
    long long size() const { return ens_size * E; }
};

// Leaf of the flax-ordered flat state.
struct Leaf {
    std::string name;
    int net;          // 0 critic, 1 target, 2 bc, 3 os  (internal ids)
    int kind;         // 0 kernel, 1 bias, 2 LN scale, 3 LN bias
    int layer;
    int ndim;
    long long shape[3];
    long long flat_off;
    long long size;
};

struct Graphs {
    hipGraphExec_t exec = nullptr;
    int nz = -1;
};

}  // namespace

struct fqlpop {
    fqlpop_config cfg{};
    EngineOptions opt{};  // g_engine_opts at create
    int n = 0;          // slots
    int device = 0;
    int D = 0, A = 0, H = 0, L = 0, B = 0, E = 0, S = 0;
    NetLayout critic, bc, os;   // critic at arena offset 0 (target arena mirrors it)
    long long P = 0, PT = 0;    // per-slot arena sizes
    std::vector<Leaf> leaves;
    long long state_size = 0;

    // device state
    // Parameters are double-buffered: a step reads every parameter from
    // `params` and its optimiser writes `params_nx`; the host swaps the pair
    // after enqueueing a train step (flip_params).  So no kernel of a step has
    // to wait for another's last read of a parameter before updating it.
    float* params_buf[2] = {nullptr, nullptr};
    float* paramsT_buf[2] = {nullptr, nullptr};
    int cur = 0;
    float *params = nullptr, *params_nx = nullptr;
    float *grads = nullptr, *adam_m = nullptr, *adam_v = nullptr, *target = nullptr;
    int* count = nullptr;
    uint64_t* seeds = nullptr;
    uint64_t* skeys = nullptr;  // per-member sampler key: sample_key(seed, alpha)
    float* alpha = nullptr;
    int* slots = nullptr;
    float* stats = nullptr;
    Chunk* chunks = nullptr;
    int* chunk_leaf = nullptr;
    int* leaf_first = nullptr;
    int n_chunks_net[3] = {0, 0, 0}, chunk_base_net[3] = {0, 0, 0}, n_chunks_total = 0;
    // fused optimiser (Adam in the dW epilogue): stats chunk id of each net's
    // W_l tiles, and the remaining (small-leaf) chunks the adam kernel runs
    bool fused_adam = false;
    int w_stat_base[3][EF_MAX_LAYERS] = {};
    int* res_ids = nullptr;
    int res_base[3] = {0, 0, 0}, res_n[3] = {0, 0, 0};
    int n_train_leaves = 0;

    // host mirror
    std::vector<float> h_alpha;
    std::vector<uint64_t> h_seeds;
    std::vector<uint8_t> active;
    std::vector<int> h_slots;
    int nz = 0;

    // datasets
    struct Dataset {
        float *obs = nullptr, *act = nullptr, *rew = nullptr, *mask = nullptr, *nobs = nullptr;
        long long rows = 0;
    } ds[2];

    // activations (slot-strided)
    std::vector<float*> allocs;
    float *os_in, *bc_in, *eu_in, *cr_in, *tg_in;
    float* cr_in_buf[2] = {nullptr, nullptr};  // cr_in per parameter buffer (cr_in = cr_in_buf[cur])
    std::vector<float*> os_u, os_g, bc_u, bc_g, eu_g, cr_u, cr_h, cr_mu, cr_rs, tg_u, tg_h, tg_mu, tg_rs;
    std::vector<float*> cr_du, bc_du, os_du;
    float *cr_dh, *bc_dh, *os_dh, *cr_c1, *cr_c2;
    float *q, *qt, *dq, *vpred, *dv, *act_t, *x0_t, *rew_t, *mask_t, *apiraw, *aflow, *amet, *da, *dout_os;
    float *info, *vinfo;
    float *inj_batch = nullptr, *inj_noise = nullptr;
    long long inj_bs = 0, inj_ns = 0;

    hipStream_t sM = nullptr, sF = nullptr, sB = nullptr, sX = nullptr;  // sX: small-population schedule
    hipEvent_t ev_sample, ev_bcfwd, ev_bcloss, ev_flow, ev_bdone;
    hipEvent_t ev_t0 = nullptr, ev_t1 = nullptr;  // fqlpop_time_dominant_kernel
    std::vector<hipEvent_t> ev_pool;
    int ev_next = 0;
    // in-step timing probe of the dominant kernel (Euler hidden-layer GEMM):
    // its blocks stamp s_memrealtime into per-launch slots; two slot sets are
    // used by alternate steps so the host reads step i-2 while step i runs
    bool euler_fused = false;      // Euler steps 1..S-1 as one persistent launch (euler_flow_kernel)
    // split launches (engine option split): per launch site an exchange area and a block of
    // arrival counters (zeroed by a memset node before every launch), and one error word
    struct SplitSite {
        unsigned long long* xch = nullptr;
        unsigned* cnt = nullptr;
        unsigned* gen = nullptr;
        long long clusters = 0;    // capacity
    } split_site[8];
    unsigned* split_err = nullptr;       // device pointer of split_err_host (mapped, coherent host memory)
    unsigned* split_err_host = nullptr;  // the host reads it without a copy or a synchronisation
    // members whose state a failed split launch may have written (sticky until restored): bit
    // w of restored[i] is set by fqlpop_set_state(i, w); all three restore the member, and so
    // does fqlpop_set_member(i, ..., reinit = 1)
    std::vector<unsigned char> poisoned, restored;
    float* euler_pre0 = nullptr;        // the split Euler flow's layer-0 accumulators (SplitFwdArgs::pre0)
    long long euler_pre0_blocks = 0;     // its capacity in blocks
    bool split_ok = false;
    bool stream_fwd = false;       // whole-network forward launches (stream_fwd_kernel)
    bool stream_bwd = false;       // whole-network dX chains (stream_bwd_kernel)
    float *part_cr = nullptr, *part_bc = nullptr, *part_os = nullptr;  // stream_bwd column-sum partials
    // W_l^T copies of the hidden kernels (l = 1..L-1) for stream_bwd, per slot:
    // [critic e=0..E-1 | bc | os] x (L-1) x H x H; refreshed after each Adam
    float *paramsT = nullptr, *paramsT_nx = nullptr;   // current / next buffer (see params)
    long long PTT = 0, wt_net_off[3] = {0, 0, 0};
    bool wt_dirty = true;          // params changed on the host side: re-transpose before the next step
    // world-model rollout evaluator (fqlpop_set_env_model / fqlpop_rollout)
    fqlpop_envmodel_config em{};
    float *sp_params = nullptr, *tp_params = nullptr;
    RolloutArgs em_args{};
    bool em_set = false;
    bool probe = false;
    int probe_set = -1;            // set used by the step being enqueued (-1: none)
    int probe_idx = 0;             // next launch slot of that set
    long long probe_step = 0;
    unsigned long long* probe_slots = nullptr;   // [2 sets][pairs][probe_blocks][2] (device view)
    unsigned long long* probe_host = nullptr;    // the same slots: mapped coherent host memory
    // FQLPOP_PHASE_PROBE=1 (diagnostics): the critic backward's per-block phase stamps (mapped
    // host memory, overwritten by every launch; summarised on stderr at destroy)
    unsigned long long* phase_host = nullptr;
    unsigned long long* phase_dev = nullptr;
    long long phase_blocks = 0;
    unsigned long long* ephase_host = nullptr;  // the same for the persistent Euler launch
    unsigned long long* ephase_dev = nullptr;
    long long ephase_blocks = 0;
    int probe_pairs = 0;
    long long probe_blocks = 0;                  // max blocks of one dominant-kernel launch
    long long probe_nb[2] = {0, 0};              // blocks of the dominant launch of the step that used each set
    hipEvent_t probe_done[2] = {nullptr, nullptr};
    hipStream_t probe_stream = nullptr;
    bool probe_pending[2] = {false, false};
    double probe_total_ms = 0.0;
    long long probe_launches = 0;
    long long probe_blocks_seen = 0, probe_blocks_expected = 0;  // stamped / launched blocks (coverage)
    double clock_check_event_us = 0.0, clock_check_stamp_us = 0.0;
    std::map<long long, Graphs> graphs;  // key: mode, active count, probe set, current buffer

    float* alloc(long long per_slot) {
        float* p = nullptr;
        HIPCHK(hipMalloc(&p, sizeof(float) * std::max<long long>(1, per_slot * n)));
        HIPCHK(hipMemset(p, 0, sizeof(float) * std::max<long long>(1, per_slot * n)));
        allocs.push_back(p);
        return p;
    }
};

namespace {

// ------------------------------------------------------------- leaves/chunks
void build_leaves(fqlpop* h) {
    // flax ModuleDict order: modules_actor_bc_flow, modules_actor_onestep_flow,
    // modules_critic, modules_target_critic; leaves sorted by path.
    struct NetRef { const char* name; int id; const NetLayout* lay; };
    const NetRef order[4] = {{"actor_bc_flow", 2, &h->bc}, {"actor_onestep_flow", 3, &h->os},
                             {"critic", 0, &h->critic}, {"target_critic", 1, &h->critic}};
    long long off = 0;
    for (const auto& nr : order) {
        const NetLayout& N = *nr.lay;
        std::vector<Leaf> ls;
        for (int l = 0; l <= N.L; ++l) {
            for (int kind = 0; kind < 2; ++kind) {
                Leaf lf{};
                lf.net = nr.id; lf.kind = kind; lf.layer = l;
                lf.name = std::string(nr.name) + "/Dense_" + std::to_string(l) + (kind == 0 ? "/kernel" : "/bias");
                std::vector<long long> shp;
                if (N.E > 1) shp.push_back(N.E);
                if (kind == 0) shp.push_back(N.kdim(l));
                shp.push_back(N.ndim(l));
                lf.ndim = (int)shp.size();
                lf.size = 1;
                for (int i = 0; i < lf.ndim; ++i) { lf.shape[i] = shp[i]; lf.size *= shp[i]; }
                ls.push_back(lf);
            }
            if (l < N.L && N.ln) {
                for (int kind = 2; kind < 4; ++kind) {
                    Leaf lf{};
                    lf.net = nr.id; lf.kind = kind; lf.layer = l;
                    lf.name = std::string(nr.name) + "/LayerNorm_" + std::to_string(l) + (kind == 2 ? "/scale" : "/bias");
                    lf.ndim = N.E > 1 ? 2 : 1;
                    lf.shape[0] = N.E > 1 ? N.E : N.H;
                    if (N.E > 1) lf.shape[1] = N.H;
                    lf.size = (long long)N.E * N.H;
                    ls.push_back(lf);
                }
            }
        }
        std::sort(ls.begin(), ls.end(), [](const Leaf& a, const Leaf& b) { return a.name < b.name; });
        for (auto& lf : ls) { lf.flat_off = off; off += lf.size; h->leaves.push_back(lf); }
    }
    h->state_size = off;
}

long long leaf_internal_off(const NetLayout& N, int kind, int layer) {
    switch (kind) {
        case 0: return N.W[layer];
        case 1: return N.b[layer];
        case 2: return N.gam[layer];
        default: return N.bet[layer];
    }
}

// per-ensemble-member element count of a leaf
long long leaf_member_size(const NetLayout& N, int kind, int layer) {
    if (kind == 0) return (long long)N.kdim(layer) * N.ndim(layer);
    if (kind == 1) return N.ndim(layer);
    return N.H;
}

// dW group tile of a net (stream_bwd_net; 0 = 64x64, 1 = 128x64, 2 = 64x128, 3 = 128x128,
// + 4: k-slices of 16 instead of 32 in the fused-optimiser launch)
// (64 x 128 for every net: with the fused optimiser epilogue, more co-resident blocks
// overlap one block's HBM-bound epilogue with the others' k-loops better than
// 2 blocks of 128 x 128.  BK = 16: 33 KB of LDS and 129 VGPRs instead of 51 KB and
// 146, +0.6 % same-box; 10 = the same at <= 128 VGPRs, 4 blocks per CU instead of 3,
// +0.4 % same-box; engine options dw_tile_critic / dw_tile_actor override, for measurements)
int dw_tile(const fqlpop* h, const NetLayout& N) {
    return N.E > 1 ? h->opt.dw_tile_critic : h->opt.dw_tile_actor;
}

void build_chunks(fqlpop* h) {
    constexpr int CH = 16384;
    std::vector<Chunk> all;
    std::vector<int> all_leaf, res;
    const NetLayout* nets[3] = {&h->critic, &h->bc, &h->os};
    int leaf_id = 0;
    for (int ni = 0; ni < 3; ++ni) {
        const NetLayout& N = *nets[ni];
        h->chunk_base_net[ni] = (int)all.size();
        h->res_base[ni] = (int)res.size();
        for (int l = 0; l <= N.L; ++l) {
            for (int kind = 0; kind < 4; ++kind) {
                if (kind >= 2 && (l == N.L || !N.ln)) continue;
                if (h->fused_adam && kind == 0 && l < N.L) {
                    // W_l: the fused dW epilogue writes one stats chunk per tile
                    h->w_stat_base[ni][l] = (int)all.size();
                    const int nt = gemm_group_tiles(dw_tile(h, N), N.kdim(l), N.H) * N.E;
                    for (int t = 0; t < nt; ++t) {
                        all.push_back(Chunk{0, 0, leaf_id});
                        all_leaf.push_back(leaf_id);
                    }
                    ++leaf_id;
                    continue;
                }
                const long long len = leaf_member_size(N, kind, l);
                for (int e = 0; e < N.E; ++e) {
                    const long long base = e * N.ens_size + leaf_internal_off(N, kind, l);
                    for (long long s = 0; s < len; s += CH) {
                        Chunk c;
                        c.off = base + s;
                        c.len = (int)std::min<long long>(CH, len - s);
                        c.leaf = leaf_id;
                        res.push_back((int)all.size());
                        all.push_back(c);
                        all_leaf.push_back(leaf_id);
                    }
                }
                ++leaf_id;
            }
        }
        h->n_chunks_net[ni] = (int)all.size() - h->chunk_base_net[ni];
        h->res_n[ni] = (int)res.size() - h->res_base[ni];
    }
    HIPCHK(hipMalloc(&h->res_ids, sizeof(int) * std::max<size_t>(1, res.size())));
    if (!res.empty()) HIPCHK(hipMemcpy(h->res_ids, res.data(), sizeof(int) * res.size(), hipMemcpyHostToDevice));
    h->n_chunks_total = (int)all.size();
    h->n_train_leaves = leaf_id;
    ARGCHK(leaf_id <= 128, "too many leaves");
    HIPCHK(hipMalloc(&h->chunks, sizeof(Chunk) * all.size()));
    HIPCHK(hipMemcpy(h->chunks, all.data(), sizeof(Chunk) * all.size(), hipMemcpyHostToDevice));
    std::vector<int> first(leaf_id + 1, 0);
    for (size_t c = all_leaf.size(); c-- > 0;) first[all_leaf[c]] = (int)c;
    first[leaf_id] = (int)all_leaf.size();
    for (size_t c = 1; c < all_leaf.size(); ++c)
        ARGCHK(all_leaf[c] >= all_leaf[c - 1], "chunks of a leaf must be contiguous");
    HIPCHK(hipMalloc(&h->leaf_first, sizeof(int) * first.size()));
    HIPCHK(hipMemcpy(h->leaf_first, first.data(), sizeof(int) * first.size(), hipMemcpyHostToDevice));
    HIPCHK(hipMalloc(&h->chunk_leaf, sizeof(int) * all_leaf.size()));
    HIPCHK(hipMemcpy(h->chunk_leaf, all_leaf.data(), sizeof(int) * all_leaf.size(), hipMemcpyHostToDevice));
    HIPCHK(hipMalloc(&h->stats, sizeof(float) * 3 * all.size() * h->n));
    HIPCHK(hipMemset(h->stats, 0, sizeof(float) * 3 * all.size() * h->n));
}

// ------------------------------------------------------------- params init
// Copy a slot's current parameters into the other buffer of the pair (after a
// host-side write, or for a member that stops stepping: both buffers must hold
// its parameters whichever one is current when it steps again).
void mirror_params(fqlpop* h, int slot, hipStream_t s) {
    HIPCHK(hipMemcpyAsync(h->params_nx + (long long)slot * h->P, h->params + (long long)slot * h->P,
                          sizeof(float) * h->P, hipMemcpyDeviceToDevice, s));
}

void upload_skey(fqlpop* h, int member) {
    const uint64_t k = sample_key(h->h_seeds[member], h->h_alpha[member]);
    HIPCHK(hipMemcpy(h->skeys + member, &k, sizeof(k), hipMemcpyHostToDevice));
}

void init_member(fqlpop* h, int slot, uint64_t seed) {
    unsigned salt = 1;
    auto init_net = [&](const NetLayout& N) {
        for (int e = 0; e < N.E; ++e) {
            float* base = h->params + (long long)slot * h->P + N.off + e * N.ens_size;
            for (int l = 0; l <= N.L; ++l) {
                const int fi = N.kdim(l), fo = N.ndim(l);
                InitArgs a{base + N.W[l], (long long)fi * fo, std::sqrt(6.0f / (float)(fi + fo)), 0.f, seed, salt++};
                launch_init(a, h->sM);
                InitArgs ab{base + N.b[l], fo, 0.f, 0.f, seed, salt++};
                launch_init(ab, h->sM);
                if (l < N.L && N.ln) {
                    InitArgs ag{base + N.gam[l], N.H, 0.f, 1.f, seed, salt++};
                    launch_init(ag, h->sM);
                    InitArgs abt{base + N.bet[l], N.H, 0.f, 0.f, seed, salt++};
                    launch_init(abt, h->sM);
                }
            }
        }
    };
    init_net(h->critic);
    init_net(h->bc);
    init_net(h->os);
    HIPCHK(hipGetLastError());
    HIPCHK(hipMemsetAsync(h->adam_m + (long long)slot * h->P, 0, sizeof(float) * h->P, h->sM));
    HIPCHK(hipMemsetAsync(h->adam_v + (long long)slot * h->P, 0, sizeof(float) * h->P, h->sM));
    HIPCHK(hipMemcpyAsync(h->target + (long long)slot * h->PT, h->params + (long long)slot * h->P,
                          sizeof(float) * h->PT, hipMemcpyDeviceToDevice, h->sM));
    HIPCHK(hipMemsetAsync(h->count + slot, 0, sizeof(int), h->sM));
    mirror_params(h, slot, h->sM);
    HIPCHK(hipStreamSynchronize(h->sM));
    h->wt_dirty = true;
}

// ------------------------------------------------------------- DAG helpers
// the network whose backward the phase probe stamps (diagnostic builds): FQLPOP_PHASE_NET =
// bc / os, else the critic
const NetLayout* phase_net(const fqlpop* h) {
    const char* v = diag_env("FQLPOP_PHASE_NET");
    if (v != nullptr && std::strcmp(v, "bc") == 0) return &h->bc;
    if (v != nullptr && std::strcmp(v, "os") == 0) return &h->os;
    return &h->critic;
}

struct Ctx {
    fqlpop* h;
    int nz;
};

TRef pref(fqlpop* h, float* arena, const NetLayout& N, long long off) {
    return tref(arena + N.off + off, h->P, N.ens_size);
}

// Fork/join events of one enqueued step come from a pool (a distinct event per
// record keeps graph capture dependencies unambiguous).
hipEvent_t next_event(fqlpop* h) {
    if (h->ev_next >= (int)h->ev_pool.size()) throw FqErr{FQLPOP_E_STATE, "event pool exhausted"};
    return h->ev_pool[h->ev_next++];
}

// Tile / pipeline choice per GEMM family, from build/gemm_bench on MI355X
// (profiles/ records the measurements): forward GEMMs use the LDS-DMA ring
// (variant 4 = 3 stages, 5 = 4 stages), dX/dW the register-staged kernel.
struct TileChoice {
    int tile, variant;
};
TileChoice pick_gemm(int layout, int M, int N, int nyz) {
    const long long t64 = (long long)((M + 63) / 64) * (N / 64) * nyz;
    if (layout == LAYOUT_FWD) {
        if (M % 64 != 0) return {0, 0};
        if (t64 <= 512) return {0, 5};
        if (N % 128 == 0 && N < 768) return {2, 4};
        return {0, 4};
    }
    if (M < 64) return {0, 0};
    if (N % 128 != 0) return {0, 0};
    return {t64 >= 2048 ? 3 : 2, 0};
}

void gemm(int layout, int epi, const GemmArgs& g, hipStream_t s) {
    const TileChoice t = pick_gemm(layout, g.M, g.N, g.ny * g.nz);
    launch_gemm_variant(layout, epi, t.tile, t.variant, g, s);
}

// Split launch sites (fqlpop::split_site): BC forward, Euler flow (sF); one-step, target
// critic, critic forwards, critic and one-step backwards (sM); in the 4th-stream schedule
// the target critic and the critic's TD-column backward (SITE_CRB2) run on sX.  The
// BC backward (sB) stays unsplit.
// the 4th-stream schedule runs up to this many 16-column tiles per step (B / 16 x members):
// cube 16 members (256) neutral, ant 4 (256) +2.1 %, ant 16 (1 024) -1.1 %
constexpr long long kSmallSchedTiles = 256;
enum { SITE_BCF = 0, SITE_EULER = 1, SITE_OSF = 2, SITE_TGT = 3, SITE_CRF = 4, SITE_CRB = 5, SITE_OSB = 6, SITE_CRB2 = 7,
       SITE_N = 8 };
// a site with more 16-column tiles than its cap runs unsplit (same-box A/B, DESIGN.md section 5,
// round 5): 128 for the Euler flow, the one-step forward (the chain's first launch) and the
// critic's LN backward, 64 for the BC forward, the target critic, the critic forward and the
// one-step backward (at 96-128 tiles their unsplit kernels were 3-5 % faster in the step)
constexpr long long kSplitMaxClusters = 128;
constexpr long long kSplitMaxClustersSide = 64;
constexpr long long split_cap(int site) {
    return (site == SITE_BCF || site == SITE_TGT || site == SITE_CRF || site == SITE_OSB) ? kSplitMaxClustersSide
                                                                                        : kSplitMaxClusters;
}
constexpr long long kSplitMaxBlocks = 256;       // one block per CU (see split_factor)

// Blocks per 16-column tile of a split launch (1 = the unsplit kernel).  Only where the
// unsplit kernel leaves CUs idle (<= split_cap tiles); the most of
// 8, 4, 2 blocks that keeps the launch within 256 blocks (forced values shrink to fit).  The
// Euler flow and the LN backward use 4 or 8 blocks (their 2-block forms would spill).
// Residency: a split kernel takes 200-256 VGPRs (2 waves per SIMD) for its 4 waves, so the
// chip holds 512 split blocks at once, and up to three split launches (sF, sM, sX) can be in
// flight together, more blocks than fit.  Progress does not depend on a budget: every launch's
// blocks take their clusters by ticket in the order they become resident (kernels.hip,
// sp_begin), so each launch has at most one partly resident cluster (<= 7 blocks) and all its
// other clusters can finish and free their CUs, whatever else runs (the hand-off waits give
// up after ~2 s and set the error word otherwise).  The budgets are for speed: same-box A/B
//  put the critic's LN backward at 256 blocks (F = 4 at 2 members, 8 at
// 1), the one-step backward unsplit from 128 tiles (8 members) and the side forwards from 96.
int split_factor_opts(const EngineOptions& o, bool split_ok, int site, long long clusters, bool min4,
                      long long max_blocks) {
    int opt = o.split;
    const int code = (o.split_sites >> (3 * site)) & 7;
    if (code == 1) return 1;
    if (code >= 2 && code <= 4) {
        opt = 1 << (code - 1);
        max_blocks = std::max<long long>(max_blocks, clusters * opt);  // (a forced F is not shrunk)
    }
    if (!split_ok || opt == 0 || clusters > split_cap(site)) return 1;
    for (int F = std::max(opt >= 2 ? opt : 8, min4 ? 4 : 2); F >= 2; F /= 2) {
        if (min4 && F < 4) break;
        if (clusters * F <= max_blocks) return F;
    }
    return 1;
}
int split_factor(const fqlpop* h, int site, long long clusters, bool min4, long long max_blocks = kSplitMaxBlocks) {
    return split_factor_opts(h->opt, h->split_ok, site, clusters, min4, max_blocks);
}

// The split plan of a step over nz members: F per launch site (1 = unsplit) and whether the
// 4th-stream schedule runs, from the shapes and engine options alone (no GPU).  The
// launches compute their F at the call sites (stream_fwd, euler_split, bwd_split) and check it
// against this plan, so the plan that fqlpop_split_plan reports is the one that runs.
struct SplitShape {
    int H, L, A, B, E, K0bc, K0os, K0cr;
    bool critic_ln, stream_fwd, stream_bwd, fused_adam, euler_fused, multi_stream;
};
void split_plan(const EngineOptions& o, const SplitShape& d, int nz, int F[SITE_N], bool* small) {
    const bool ok = d.stream_fwd && o.split != 0;
    const int B = d.B, B2 = 2 * B, B3 = 3 * B, T = B / 16;
    auto fwd = [&](int site, int K0, int nout, int M, long long clusters, bool min4) {
        F[site] = d.stream_fwd && split_fwd_supported(d.H, d.L, K0, nout, M)
                      ? split_factor_opts(o, ok, site, clusters, min4, o.split_blocks) : 1;
    };
    fwd(SITE_EULER, d.K0bc, d.A, B, (long long)T * nz, true);
    if (!d.euler_fused) F[SITE_EULER] = 1;
    *small = o.small_sched && d.multi_stream && d.stream_fwd && d.stream_bwd && d.fused_adam &&
             (long long)T * nz <= kSmallSchedTiles;
    fwd(SITE_BCF, d.K0bc, d.A, B2, (long long)(B2 / 16) * nz, false);
    fwd(SITE_OSF, d.K0os, d.A, B3, (long long)(B3 / 16) * nz, false);
    fwd(SITE_TGT, d.K0cr, 1, B, (long long)T * d.E * nz, false);
    fwd(SITE_CRF, d.K0cr, 1, B2, (long long)(B2 / 16) * d.E * nz, false);
    auto bwd = [&](int site, int nout, int M, int Mg, long long clusters, bool min4) {
        F[site] = d.stream_bwd && split_bwd_supported(d.H, d.L, nout, M, Mg)
                      ? split_factor_opts(o, ok, site, clusters, min4, kSplitMaxBlocks) : 1;
    };
    if (*small) {
        bwd(SITE_CRB, 1, B, 0, (long long)T * d.E * nz, d.critic_ln);  // the Q-loss columns
        bwd(SITE_CRB2, 1, B, B, (long long)T * d.E * nz, d.critic_ln);  // the TD columns (sX)
    } else {
        bwd(SITE_CRB, 1, B2, B, (long long)(B2 / 16) * d.E * nz, d.critic_ln);
        F[SITE_CRB2] = 1;
    }
    bwd(SITE_OSB, d.A, B, B, (long long)T * nz, false);
}
SplitShape split_shape(const fqlpop* h) {
    return SplitShape{h->H, h->L, h->A, h->B, h->E, h->bc.in_dim, h->os.in_dim, h->critic.in_dim, h->critic.ln,
                      h->stream_fwd, h->stream_bwd, h->fused_adam, h->euler_fused, h->sX != h->sM};
}
// the call site's F against the plan (a divergence would make fqlpop_split_plan report a
// schedule that does not run)
void check_plan(const fqlpop* h, int site, int nz, int F) {
    int plan[SITE_N];
    bool small = false;
    split_plan(h->opt, split_shape(h), nz, plan, &small);
    ARGCHK(plan[site] == F, "split launch differs from the split plan");
}

// The site's synchronisation state for one launch over `clusters` tiles.  Its counters (per
// cluster, then the ticket and the exit counter) are zero at every launch: zeroed at
// allocation, by the last block of every launch, and by check_split_error after a failed one
// (no memset node in the step: at 2 members the seven 5-8 us fills were on the chains).
SplitSync split_prep(fqlpop* h, int site, long long clusters, hipStream_t) {
    fqlpop::SplitSite& st = h->split_site[site];
    ARGCHK(clusters <= st.clusters, "split launch larger than its site");
    return SplitSync{st.xch, st.cnt, st.gen, h->split_err};
}

// Blocks per tile of a streamed backward launch (1 = unsplit): the critic (LN: its 2-block
// form would spill, so 4 or 8, up to 2 blocks per CU: 4 x 128 tiles for a 2-member
// population) and the one-step actor on sM; never the BC actor on sB.
int bwd_split(const fqlpop* h, int site, const NetLayout& N, int M, int Mg, int nz) {
    if (&N == &h->bc || !split_bwd_supported(N.H, N.L, N.out_dim, M, Mg)) return 1;
    return split_factor(h, site, (long long)(M / 16) * N.E * nz, N.ln, kSplitMaxBlocks);
}

// Forward of the hidden stack of `N` over `M` columns of input X (ld = ldx).
// U[l]/G[l]: pre-activation and layer output buffers (ld = ldx).  store_u:
// keep u (needed by backward / LN); otherwise G[l] = gelu(u) directly.
void fwd_hidden(const Ctx& c, hipStream_t s, const NetLayout& N, TRef X, int ldx, int M,
                const std::vector<float*>& U, const std::vector<float*>& G, long long act_sy,
                const std::vector<float*>* MU, const std::vector<float*>* RS, long long st_sy,
                bool store_u, bool euler = false) {
    fqlpop* h = c.h;
    for (int l = 0; l < N.L; ++l) {
        GemmArgs g{};
        g.A = pref(h, h->params, N, N.W[l]);
        g.B = l == 0 ? X : tref(G[l - 1], (long long)N.H * ldx * N.E, act_sy);
        if (N.ln) {
            g.C = tref(U[l], (long long)N.H * ldx * N.E, act_sy);
        } else {
            g.C = tref(store_u ? U[l] : G[l], (long long)N.H * ldx * N.E, act_sy);
            g.C2 = tref(G[l], (long long)N.H * ldx * N.E, act_sy);
        }
        g.bias = pref(h, h->params, N, N.b[l]);
        g.M = N.H; g.N = M; g.K = N.kdim(l);
        g.lda = N.H; g.ldb = ldx; g.ldc = ldx;
        g.ny = N.E; g.nz = c.nz; g.slots = h->slots;
        const int epi = N.ln ? EPI_BIAS : (store_u ? EPI_BIAS_GELU2 : EPI_BIAS_GELU);
        if (euler && l >= 1 && epi == EPI_BIAS_GELU && g.M % 64 == 0 && g.N % 64 == 0) {
            // the dominant kernel: its own symbol, optionally with in-kernel timing stamps
            if (h->probe_set >= 0 && h->probe_idx < h->probe_pairs)
                g.probe = h->probe_slots + 2 * h->probe_blocks * ((long long)h->probe_set * h->probe_pairs + h->probe_idx++);
            launch_gemm_euler_hidden(g, s);
        } else {
            gemm(LAYOUT_FWD, epi, g, s);
        }
        if (N.ln) {
            LnArgs a{};
            a.u = tref(U[l], (long long)N.H * ldx * N.E, act_sy);
            a.h = tref(G[l], (long long)N.H * ldx * N.E, act_sy);
            a.mu = tref((*MU)[l], (long long)ldx * N.E, st_sy);
            a.rstd = tref((*RS)[l], (long long)ldx * N.E, st_sy);
            a.gamma = pref(h, h->params, N, N.gam[l]);
            a.beta = pref(h, h->params, N, N.bet[l]);
            a.H = N.H; a.M = M; a.ld = ldx; a.ny = N.E; a.nz = c.nz; a.slots = h->slots;
            launch_ln_gelu_fwd(a, s);
        }
    }
}

HeadArgs head_args(const Ctx& c, const NetLayout& N, float* Glast, int ldx, int M, long long act_sy) {
    fqlpop* h = c.h;
    HeadArgs a{};
    a.h = tref(Glast, (long long)N.H * ldx * N.E, act_sy);
    a.W = pref(h, h->params, N, N.W[N.L]);
    a.b = pref(h, h->params, N, N.b[N.L]);
    a.H = N.H; a.M = M; a.ld = ldx; a.nout = N.out_dim;
    a.B = h->B; a.D = h->D;
    a.steps_f = (float)h->S;
    a.ny = N.E; a.nz = c.nz; a.slots = h->slots;
    return a;
}

// Backward of one network from its head-output gradient `dout` ([nout][ld_o]).
// Activations (U, G, X0) are read at column offset `coff` with leading dim
// `ld`; M columns are back-propagated, of which the first Mg feed the
// parameter gradients.
void bwd_net(const Ctx& c, hipStream_t s, const NetLayout& N, TRef dout, int ld_o, TRef X0, int ld,
             long long coff, int M, int Mg, const std::vector<float*>& U, const std::vector<float*>& G,
             long long act_sy, const std::vector<float*>* MU, const std::vector<float*>* RS, long long st_sy,
             const std::vector<float*>& DU, float* DH, float* C1, float* C2, int ld_d, hipStream_t sw) {
    fqlpop* h = c.h;
    const long long act_ss = (long long)N.H * ld * N.E;
    const long long d_ss = (long long)N.H * ld_d * N.E, d_sy = (long long)N.H * ld_d;
    auto act = [&](float* p) { return tref(p + coff, act_ss, act_sy); };
    for (int l = N.L - 1; l >= 0; --l) {
        const bool head = (l == N.L - 1);
        BwdArgs b{};
        if (head) {
            b.dout = dout;
            b.W5 = pref(h, h->params, N, N.W[N.L]);
            b.x_head = act(G[l]);
            b.g_W5 = pref(h, h->grads, N, N.W[N.L]);
        } else {
            b.dh = tref(DH, d_ss, d_sy);
        }
        b.u = act(U[l]);
        if (N.ln) {
            b.mu = tref((*MU)[l] + coff, (long long)ld * N.E, st_sy);
            b.rstd = tref((*RS)[l] + coff, (long long)ld * N.E, st_sy);
            b.gamma = pref(h, h->params, N, N.gam[l]);
            b.c1 = tref(C1, (long long)ld_d * N.E, ld_d);
            b.c2 = tref(C2, (long long)ld_d * N.E, ld_d);
            b.g_gamma = pref(h, h->grads, N, N.gam[l]);
            b.g_beta = pref(h, h->grads, N, N.bet[l]);
        }
        b.du = tref(DU[l], d_ss, d_sy);
        b.g_b = pref(h, h->grads, N, N.b[l]);
        b.H = N.H; b.M = M; b.Mg = Mg; b.ld = ld; b.ld_d = ld_d; b.ld_o = ld_o; b.nout = N.out_dim;
        b.ny = N.E; b.nz = c.nz; b.slots = h->slots;
        if (N.ln) launch_bwd_rowstats(head, b, s);
        launch_bwd_cols(head, N.ln, b, s);

        // dW_l = X_l^T du_l over the first Mg columns, on the dW stream `sw`
        // (off the dX chain's critical path)
        if (sw != s) {
            hipEvent_t ev = next_event(h);
            HIPCHK(hipEventRecord(ev, s));
            HIPCHK(hipStreamWaitEvent(sw, ev, 0));
        }
        GemmArgs gw{};
        gw.A = l == 0 ? X0 : act(G[l - 1]);
        gw.B = tref(DU[l], d_ss, d_sy);
        gw.C = pref(h, h->grads, N, N.W[l]);
        gw.M = N.kdim(l); gw.N = N.H; gw.K = Mg;
        gw.lda = ld; gw.ldb = ld_d; gw.ldc = N.H;
        gw.ny = N.E; gw.nz = c.nz; gw.slots = h->slots;
        gemm(LAYOUT_DW, EPI_STORE, gw, sw);
        if (l > 0) {
            // dh_{l-1} = W_l du_l  (all M columns)
            GemmArgs gx{};
            gx.A = pref(h, h->params, N, N.W[l]);
            gx.B = tref(DU[l], d_ss, d_sy);
            gx.C = tref(DH, d_ss, d_sy);
            gx.M = N.H; gx.N = M; gx.K = N.H;
            gx.lda = N.H; gx.ldb = ld_d; gx.ldc = ld_d;
            gx.ny = N.E; gx.nz = c.nz; gx.slots = h->slots;
            gemm(LAYOUT_DX, EPI_STORE, gx, s);
        }
    }
}

AdamArgs adam_args(const Ctx& c, int ni);

// Whole-network backward of `N` (stream_bwd_kernel) on `s`: dX chain from the
// head gradient `dout` ([nout][ld_o]) down to du_0, LayerNorm / GELU' fused,
// parameter-grad column sums as per-tile partials.  Then, on `sw`, the
// partial reduction (bias / LN / head-kernel grads) and the dW_l GEMMs.
// Activations are read at column offset `coff` (ld `ld`), du_l written with
// ld `ld_d`; M columns are back-propagated, the first Mg feed the grads.
int skip_mask();

void stream_bwd_net(const Ctx& c, hipStream_t s, const NetLayout& N, TRef dout, int ld_o, TRef X0, int ld,
                    long long coff, int M, int Mg, const std::vector<float*>& U, const std::vector<float*>& G,
                    long long act_sy, const std::vector<float*>* MU, const std::vector<float*>* RS, long long st_sy,
                    const std::vector<float*>& DU, int ld_d, float* part, hipStream_t sw,
                    const InGradArgs* ig = nullptr, std::function<void()>* defer = nullptr) {
    fqlpop* h = c.h;
    const long long act_ss = (long long)N.H * ld * N.E;
    const long long d_ss = (long long)N.H * ld_d * N.E, d_sy = (long long)N.H * ld_d;
    StreamBwdArgs a{};
    a.params = h->params + N.off;
    a.P = h->P; a.ens = N.ens_size;
    const int ni = &N == &h->critic ? 0 : &N == &h->bc ? 1 : 2;
    a.paramsT = h->paramsT + h->wt_net_off[ni];
    a.PT = h->PTT; a.ensT = (long long)(N.L - 1) * N.H * N.H;
    for (int l = 1; l < N.L; ++l) a.wt_off[l] = (long long)(l - 1) * N.H * N.H;
    for (int l = 0; l <= N.L; ++l) {
        a.w_off[l] = N.W[l];
        a.b_off[l] = N.b[l];
        if (l < N.L) {
            if (N.ln) {
                a.g_off[l] = N.gam[l];
                a.be_off[l] = N.bet[l];
                a.MU[l] = (*MU)[l];
                a.RS[l] = (*RS)[l];
            }
            a.U[l] = U[l];
            a.DU[l] = DU[l];
        }
    }
    a.dout = dout.p; a.dout_ss = dout.ss; a.dout_sy = dout.sy; a.ld_o = ld_o;
    a.Ghead = G[N.L - 1];
    a.s_ss = act_ss; a.s_sy = act_sy; a.st_ss = (long long)ld * N.E; a.st_sy = st_sy;
    a.ld_s = ld; a.coff = (int)coff;
    a.d_ss = d_ss; a.d_sy = d_sy; a.ld_d = ld_d;
    a.part = part; a.NP = stream_bwd_np(N.L, N.H, N.out_dim, N.ln);
    a.L = N.L; a.M = M; a.Mg = Mg; a.nout = N.out_dim;
    a.ny = N.E; a.nz = c.nz; a.slots = h->slots;
    if (ig) {
        // the critic's dQ/da, computed by the backward's layer-0 epilogue (per-ensemble partials)
        ARGCHK(ig->off == Mg && ig->M == M - Mg, "input-grad columns must follow the grad columns");
        ARGCHK(ig->A >= 1 && ig->A <= 8, "fused dQ/da: at most 8 action inputs");
        a.da = ig->da.p; a.da_ss = ig->da.ss; a.da_sy = (long long)ig->A * ig->M;
        a.ld_da = ig->M; a.D0 = ig->D; a.na = ig->A;
    }
    if (h->phase_dev != nullptr && &N == phase_net(h)) {
        ARGCHK((long long)(M / 16) * N.E * c.nz <= h->phase_blocks, "phase probe: too many blocks");
        a.phase = h->phase_dev;
    }
    if (!(skip_mask() & (&N == &h->critic ? 32 : &N == &h->bc ? 64 : 128))) {
        const int site = &N != &h->critic ? SITE_OSB : (s == h->sX && h->sX != h->sM) ? SITE_CRB2 : SITE_CRB;
        const int F = bwd_split(h, site, N, M, Mg, c.nz);
        if (&N != &h->bc) check_plan(h, site, c.nz, F);
        if (F > 1) {
            const long long clusters = (long long)(M / 16) * N.E * c.nz;
            launch_split_bwd(N.ln, F, a, split_prep(h, site, clusters, s), s);
        } else {
            launch_stream_bwd(N.ln, a, s);
        }
    }
    if (Mg == 0) return;  // (the critic's Q-loss columns alone: no parameter grads)
    hipEvent_t ev = nullptr;
    if (sw != s) {
        ev = next_event(h);
        HIPCHK(hipEventRecord(ev, s));
    }
    // the parameter-grad half (partial reduction + dW, fused optimiser): now,
    // or by the caller later (`defer`), so that the step's critical chain is
    // captured ahead of it
    const int NP = a.NP;
    auto dw_half = [=, &N]() {
    if (ev) HIPCHK(hipStreamWaitEvent(sw, ev, 0));
    ColsumArgs r{};
    r.part = part; r.NP = NP; r.tiles = Mg / 16;
    r.grads = h->grads + N.off; r.P = h->P; r.ens = N.ens_size;
    for (int l = 0; l < N.L; ++l) {
        r.b_off[l] = N.b[l];
        if (N.ln) { r.g_off[l] = N.gam[l]; r.be_off[l] = N.bet[l]; }
    }
    r.w5_off = N.W[N.L];
    r.L = N.L; r.H = N.H; r.ln = N.ln ? 1 : 0;
    r.ny = N.E; r.nz = c.nz; r.slots = h->slots;
    if (!(skip_mask() & 512)) launch_colsum_reduce(r, sw);
    // dW_l = X_l^T du_l over the first Mg columns, every layer in one grouped launch
    auto act = [&](float* p) { return tref(p + coff, act_ss, act_sy); };
    std::vector<GemmArgs> gs;
    for (int l = N.L - 1; l >= 0; --l) {
        GemmArgs gw{};
        gw.A = l == 0 ? X0 : act(G[l - 1]);
        gw.B = tref(DU[l], d_ss, d_sy);
        gw.C = pref(h, h->grads, N, N.W[l]);
        gw.M = N.kdim(l); gw.N = N.H; gw.K = Mg;
        gw.lda = ld; gw.ldb = ld_d; gw.ldc = N.H;
        gw.ny = N.E; gw.nz = c.nz; gw.slots = h->slots;
        gs.push_back(gw);
    }
    if (h->fused_adam) {
        // dW of every layer with Adam / EMA / W^T / grad stats in the epilogue
        AdamEpi ae{};
        ae.p_in = h->params; ae.p_out = h->params_nx; ae.m = h->adam_m; ae.v = h->adam_v;
        ae.target = ni == 0 ? h->target : nullptr;
        ae.wt_out = h->paramsT_nx;
        ae.P = h->P; ae.PT = h->PT; ae.PTT = h->PTT;
        ae.ens = N.ens_size;
        ae.wt_sy = (long long)(N.L - 1) * N.H * N.H;
        for (int gi = 0; gi < (int)gs.size(); ++gi) {
            const int l = N.L - 1 - gi;
            ae.w_off[gi] = N.off + N.W[l];
            ae.wt_off[gi] = l >= 1 ? h->wt_net_off[ni] + (long long)(l - 1) * N.H * N.H : -1;
            ae.stat_base[gi] = h->w_stat_base[ni][l];
        }
        ae.stats = h->stats; ae.n_total_chunks = h->n_chunks_total;
        ae.count = h->count;
        ae.lr = h->cfg.lr; ae.tau = h->cfg.tau;
        {
            // FQLPOP_DW_MODE (diagnostic builds only, timing probes with wrong results):
            // 1 / 2 one phase of the launch, 3 no W^T pass, 4 no W^T pass for the actor nets
            const char* dm = diag_env("FQLPOP_DW_MODE");
            ae.mode = dm ? std::atoi(dm) : 0;
            if (ae.mode == 4) ae.mode = ni == 0 ? 0 : 3;
            // m, v and the target stream non-temporally: read and written once per step, they
            // need not displace the weights the streamed kernels re-read from L2 / MALL
            // (+1.0 % same-box; engine option adam_nt: bit mask, see AdamEpi::nt)
            ae.nt = h->opt.adam_nt;
        }
        ae.small = adam_args(c, ni);
        ae.small_blocks = ae.small.n_chunks * c.nz;
        launch_gemm_group_dw(dw_tile(h, N), gs.data(), (int)gs.size(), sw, &ae);
    } else if (N.L <= GEMM_GROUP_MAX && N.H % 128 == 0) {
        launch_gemm_group_dw(dw_tile(h, N), gs.data(), (int)gs.size(), sw);
    } else {
        for (const GemmArgs& gw : gs) gemm(LAYOUT_DW, EPI_STORE, gw, sw);
    }
    };
    if (defer) *defer = dw_half;
    else dw_half();
}

// W^T copies (dst, a paramsT buffer) of the hidden kernels of the nets in
// `mask` (bit ni: 0 critic, 1 bc, 2 os) from src (a params buffer), for the
// active slots (all slots when all_slots).
void transpose_nets(fqlpop* h, hipStream_t s, int mask, bool all_slots, const float* src, float* dst) {
    TransposeArgs t{};
    t.src = src; t.src_ss = h->P;
    t.dst = dst; t.dst_ss = h->PTT;
    t.H = h->H;
    const NetLayout* nets[3] = {&h->critic, &h->bc, &h->os};
    const long long HH = (long long)h->H * h->H;
    int n = 0;
    for (int ni = 0; ni < 3; ++ni) {
        if (!(mask & (1 << ni))) continue;
        const NetLayout& N = *nets[ni];
        for (int e = 0; e < N.E; ++e)
            for (int l = 1; l < N.L; ++l) {
                ARGCHK(n < TR_MAX, "too many transposed matrices");
                t.src_off[n] = N.off + e * N.ens_size + N.W[l];
                t.dst_off[n] = h->wt_net_off[ni] + ((long long)e * (N.L - 1) + (l - 1)) * HH;
                ++n;
            }
    }
    t.n_mats = n;
    if (all_slots) { t.slots = nullptr; t.nz = h->n; }
    else { t.slots = h->slots; t.nz = h->nz; }
    launch_transpose(t, s);
}

AdamArgs adam_args(const Ctx& c, int ni) {
    fqlpop* h = c.h;
    const NetLayout* nets[3] = {&h->critic, &h->bc, &h->os};
    AdamArgs a{};
    a.p_in = h->params; a.p_out = h->params_nx;
    a.g = h->grads; a.m = h->adam_m; a.v = h->adam_v;
    a.target = ni == 0 ? h->target : nullptr;
    a.P = h->P; a.PT = h->PT;
    a.net_off = nets[ni]->off;
    a.chunks = h->chunks;
    if (h->fused_adam) {
        a.ids = h->res_ids + h->res_base[ni];
        a.n_chunks = h->res_n[ni];
    } else {
        a.ids = nullptr;
        a.n_chunks = h->n_chunks_net[ni];
        a.chunk_base = h->chunk_base_net[ni];
    }
    a.stats = h->stats; a.n_total_chunks = h->n_chunks_total;
    a.count = h->count;
    a.lr = h->cfg.lr; a.tau = h->cfg.tau;
    a.nz = c.nz; a.slots = h->slots;
    return a;
}

// Adam (+ EMA, grad stats) of net ni from params to params_nx: every leaf, or
// with the fused optimiser only the leaves the dW epilogue does not cover
// (those normally ride in the fused launch itself, see stream_bwd_net).
void adam_net(const Ctx& c, hipStream_t s, int ni) {
    const AdamArgs a = adam_args(c, ni);
    if (a.n_chunks > 0) launch_adam(a, s);
}

// One whole-network forward launch (stream_fwd_kernel).  `arena` + N.off is the
// net's parameter block (slot stride P); activations for the backward pass are
// stored for columns [st_lo, st_hi) into U/G (slot stride s_ss, ensemble
// stride s_sy, leading dim ld_s) and MU/RS (st_ss, st_sy) when given.
void stream_fwd(const Ctx& c, hipStream_t s, const NetLayout& N, const float* arena, long long P, TRef X, int ldx,
                int M, const std::vector<float*>* U, const std::vector<float*>* G, const std::vector<float*>* MU,
                const std::vector<float*>* RS, long long s_ss, long long s_sy, long long st_ss, long long st_sy,
                int st_lo, int st_hi, int mode, const HeadArgs& head, int g_hi = -1) {
    fqlpop* h = c.h;
    StreamArgs a{};
    a.params = arena + N.off;
    a.P = P;
    a.ens = N.ens_size;
    for (int l = 0; l <= N.L; ++l) {
        a.w_off[l] = N.W[l];
        a.b_off[l] = N.b[l];
        if (l < N.L && N.ln) {
            a.g_off[l] = N.gam[l];
            a.be_off[l] = N.bet[l];
        }
        if (l < N.L) {
            a.U[l] = U ? (*U)[l] : nullptr;
            a.G[l] = G ? (*G)[l] : nullptr;
            a.MU[l] = MU ? (*MU)[l] : nullptr;
            a.RS[l] = RS ? (*RS)[l] : nullptr;
        }
    }
    a.x0 = X.p;
    a.x0_ss = X.ss;
    a.ld_x = ldx; a.K0 = N.in_dim; a.L = N.L; a.M = M;
    a.s_ss = s_ss; a.s_sy = s_sy; a.st_ss = st_ss; a.st_sy = st_sy;
    a.ld_s = ldx; a.st_lo = st_lo; a.st_hi = st_hi;
    a.g_hi = g_hi < 0 ? st_hi : g_hi;
    a.head = head;
    a.head.nout = N.out_dim;
    a.ny = N.E; a.nz = c.nz; a.slots = h->slots;
    const int sk = skip_mask();
    const int bit = &N == &h->bc ? 16 : &N == &h->os ? 8 : arena == h->target ? 2 : 4;
    if (sk & bit) return;
    const int site = &N == &h->bc ? SITE_BCF : &N == &h->os ? SITE_OSF : arena == h->target ? SITE_TGT : SITE_CRF;
    const long long clusters = (long long)(M / 16) * N.E * c.nz;
    const int F = split_fwd_supported(N.H, N.L, N.in_dim, N.out_dim, M) ? split_factor(h, site, clusters, false, h->opt.split_blocks) : 1;
    check_plan(h, site, c.nz, F);
    if (F > 1) {
        SplitFwdArgs sa{};
        sa.s = a;
        sa.sync = split_prep(h, site, clusters, s);
        launch_split_fwd(mode, N.ln, false, F, sa, s);
    } else {
        launch_stream_fwd(mode, N.ln, a, s);
    }
}

// The split form of the persistent Euler flow (euler_args' launch), or F = 1.
int euler_split(const fqlpop* h, int nz) {
    const NetLayout& N = h->bc;
    if (!h->euler_fused || !split_fwd_supported(N.H, N.L, N.in_dim, N.out_dim, h->B)) return 1;
    return split_factor(h, SITE_EULER, (long long)(h->B / 16) * nz, true, h->opt.split_blocks);
}
SplitFwdArgs euler_split_args(fqlpop* h, const EulerArgs& ea, hipStream_t s) {
    const NetLayout& N = h->bc;
    SplitFwdArgs sa{};
    StreamArgs& a = sa.s;
    a.params = ea.params; a.P = ea.P; a.ens = 0;
    for (int l = 0; l <= N.L; ++l) { a.w_off[l] = ea.w_off[l]; a.b_off[l] = ea.b_off[l]; }
    a.x0 = ea.eu.p; a.x0_ss = ea.eu.ss; a.ld_x = ea.B; a.K0 = ea.D + ea.A + 1; a.L = ea.L; a.M = ea.B;
    a.head.nout = ea.A;
    a.ny = 1; a.nz = ea.nz; a.slots = ea.slots;
    sa.aflow = ea.aflow;
    sa.D = ea.D; sa.A = ea.A; sa.S = ea.S; sa.first = ea.first; sa.steps_f = ea.steps_f;
    sa.probe = ea.probe;
    sa.phase = ea.phase;
    sa.sync = split_prep(h, SITE_EULER, (long long)(ea.B / 16) * ea.nz, s);
    // the layer-0 scratch when it covers the launch (else the kernel's full layer-0 chain)
    const long long blocks = (long long)(ea.B / 16) * ea.nz * euler_split(h, ea.nz);
    sa.pre0 = h->euler_pre0 && blocks <= h->euler_pre0_blocks ? h->euler_pre0 : nullptr;
    return sa;
}
long long euler_blocks(const fqlpop* h, int nz) { return (long long)(h->B / 16) * nz * euler_split(h, nz); }
void launch_euler(fqlpop* h, const EulerArgs& ea, hipStream_t s) {
    const int F = euler_split(h, ea.nz);
    // every block of the launch writes its two probe stamps and its phase stamps
    ARGCHK(ea.probe == nullptr || euler_blocks(h, ea.nz) <= h->probe_blocks, "Euler probe: too many blocks");
    ARGCHK(ea.phase == nullptr || euler_blocks(h, ea.nz) <= h->ephase_blocks, "Euler phase probe: too many blocks");
    if (F > 1) launch_split_fwd(HEAD_EULER, false, true, F, euler_split_args(h, ea, s), s);
    else launch_euler_flow(ea, s);
}

// FQLPOP_SKIP (diagnostic builds only; TIMING EXPERIMENT, results are garbage): bit mask
// of launches left out of the step, to measure each one's marginal cost in the concurrent
// step: 1 Euler flow, 2 target-critic fwd, 4 critic fwd, 8 one-step fwd, 16 BC fwd,
// 32 critic bwd (dX chain), 64 BC bwd, 128 one-step bwd, 256 actor loss, 512 the three
// colsum reductions.  Always 0 in the production build.
int skip_mask() {
    static const int m = [] { const char* v = diag_env("FQLPOP_SKIP"); return v ? std::atoi(v) : 0; }();
    return m;
}

// Arguments of the persistent Euler-flow launch: steps 1..S-1 from eu_in (the
// state the BC head left after step 0) to aflow.
EulerArgs euler_args(fqlpop* h, int nz) {
    const NetLayout& N = h->bc;
    EulerArgs ea{};
    ea.params = h->params + N.off;
    ea.P = h->P;
    for (int l = 0; l <= N.L; ++l) {
        ea.w_off[l] = N.W[l];
        ea.b_off[l] = N.b[l];
    }
    ea.eu = tref(h->eu_in, (long long)(h->D + h->A + 1) * h->B);
    ea.aflow = tref(h->aflow, (long long)h->A * h->B);
    ea.D = h->D; ea.A = h->A; ea.H = h->H; ea.L = h->L; ea.B = h->B; ea.S = h->S; ea.first = 1;
    ea.steps_f = (float)h->S;
    ea.nz = nz; ea.slots = h->slots;
    ea.phase = h->ephase_dev;
    return ea;
}

// Algorithmic FLOPs of one dominant launch over the active members.
double dominant_flops(const fqlpop* h) {
    const double B = h->B, H = h->H, K0 = h->D + h->A + 1, A = h->A;
    if (h->euler_fused)
        return (h->S - 1) * 2.0 * B * (K0 * H + (h->L - 1) * H * H + H * A) * h->nz;
    return 2.0 * H * B * H * h->nz;
}

// FQLPOP_PHASE_PROBE: mean phase durations (us) of the probed backward's last launch (the
// critic's, or FQLPOP_PHASE_NET=bc / os), from wave 0's stamps of every block (s_memrealtime,
// 100 MHz).  The actor variant (no LayerNorm) stamps only the layer start, the slab barrier
// exit and the product end.
void phase_report(const unsigned long long* ph, long long nb, int L, bool ln, const char* name) {
    long long t0 = -1, t1 = 0, n = 0;
    double blk = 0, pro = 0, tail = 0, pass1[8] = {}, wait2[8] = {}, p2[8] = {}, prod[8] = {}, hp[4] = {};
    for (long long b = 0; b < nb; ++b) {
        const unsigned long long* p = ph + b * SB_PHASE_STRIDE;
        if (p[0] == 0 || p[1] < p[0]) continue;
        ++n;
        t0 = t0 < 0 ? (long long)p[0] : std::min(t0, (long long)p[0]);
        t1 = std::max(t1, (long long)p[1]);
        blk += (double)(p[1] - p[0]);
        pro += (double)(p[2] - p[0]);
        tail += (double)(p[1] - p[2 + 5 * (L - 1) + 3]);
        if (p[40] != 0)  // the general head's prologue (nout > 1): W_L / dout staged, barrier, head grads, barrier
            for (int i = 0; i < 4; ++i) hp[i] += (double)(p[40 + i] - (i == 0 ? p[0] : p[39 + i]));
        for (int i = 0; i < L && i < 8; ++i) {
            const unsigned long long* q = p + 2 + 5 * i;
            if (ln) {
                pass1[i] += (double)(q[1] - q[0]);
                wait2[i] += (double)(q[2] - q[1]);
                p2[i] += (double)(q[3] - q[2]);
            } else {
                p2[i] += (double)(q[3] - q[0]);
            }
            if (i + 1 < L) prod[i] += (double)(q[4] - q[3]);
        }
    }
    if (n == 0) return;
    const double us = 0.01 / (double)n;  // 100 MHz ticks -> us, averaged over blocks
    std::fprintf(stderr,
                 "phase probe (%s backward, last launch): %lld blocks, span %.1f us, block %.2f us "
                 "(prologue %.2f, after the last slab barrier %.2f)\n",
                 name, n, (double)(t1 - t0) * 0.01, blk * us, pro * us, tail * us);
    if (hp[0] > 0)
        std::fprintf(stderr, "  prologue: head operands staged %.2f | barrier %.2f | head grads %.2f | dh + barrier %.2f\n",
                     hp[0] * us, hp[1] * us, hp[2] * us, hp[3] * us);
    for (int i = 0; i < L && i < 8; ++i)
        if (ln)
            std::fprintf(stderr, "  pass %d: LN pass 1 %.2f | stats barrier %.2f | pass 2 + du + slab barrier %.2f | dX product %.2f\n",
                         i, pass1[i] * us, wait2[i] * us, p2[i] * us, prod[i] * us);
        else
            std::fprintf(stderr, "  pass %d: GELU' + du + slab barrier (+ dQ/da at pass %d) %.2f | dX product %.2f\n",
                         i, L - 1, p2[i] * us, prod[i] * us);
}

// FQLPOP_PHASE_PROBE: the persistent Euler launch's mean per-layer phases (us) over its steps
// and blocks (wave 0's stamps of the last launch)
void euler_phase_report(const unsigned long long* ph, long long nb, int L, int steps) {
    double kl[9] = {}, ep[9] = {}, br[9] = {}, gap[9] = {}, pro = 0, blk = 0;
    long long n = 0;
    for (long long b = 0; b < nb; ++b) {
        const unsigned long long* p = ph + b * EF_PHASE_STRIDE;
        if (p[0] == 0) continue;
        ++n;
        pro += (double)(p[1] - p[0]);
        blk += (double)(p[1 + 4 * ((steps - 1) * (L + 1) + L) + 3] - p[0]);
        for (int st = 0; st < steps; ++st)
            for (int l = 0; l <= L; ++l) {
                const unsigned long long* q = p + 1 + 4 * (st * (L + 1) + l);
                if (l < L) {
                    kl[l] += (double)(q[1] - q[0]);
                    ep[l] += (double)(q[2] - q[1]);
                    br[l] += (double)(q[3] - q[2]);
                    gap[l] += (double)(q[0] - (l > 0 ? q[-1] : st > 0 ? q[-1] : q[0]));
                } else {
                    kl[l] += (double)(q[3] - q[0]);  // head: MFMAs, reduction, state update
                }
            }
    }
    if (n == 0) return;
    const double us = 0.01 / (double)n, per = us / (double)steps;
    std::fprintf(stderr, "phase probe (Euler flow, last launch): %lld blocks, %d steps, block %.1f us, prologue %.2f us\n",
                 n, steps, blk * us, pro * us);
    for (int l = 0; l < L; ++l)
        std::fprintf(stderr, "  layer %d per step: k-loop %.3f | epilogue %.3f | barrier %.3f | gap before %.3f\n", l,
                     kl[l] * per, ep[l] * per, br[l] * per, gap[l] * per);
    std::fprintf(stderr, "  head per step: %.3f\n", kl[L] * per);
}

// FQLPOP_PHASE_PROBE, split Euler launch: mean per-step phases (us) over blocks and steps:
// per hidden layer the wait for the previous layer's words (stage), the k-loop, the epilogue
// + publish; the head's wait for the 8 partials; and the spread of the blocks' start times
void split_euler_phase_report(const unsigned long long* ph, long long nb, int L, int steps) {
    double stg[9] = {}, kl[9] = {}, ep[9] = {}, head = 0, pro = 0, blk = 0, l0 = 0;
    long long n = 0, t0 = -1, t1 = 0, tl = 0;
    int xcc[8] = {};
    for (long long b = 0; b < nb; ++b) {
        const unsigned long long* p = ph + b * EF_PHASE_STRIDE;
        if (p[0] == 0) continue;
        ++n;
        t0 = t0 < 0 ? (long long)p[0] : std::min(t0, (long long)p[0]);
        tl = std::max(tl, (long long)p[0]);
        const unsigned long long* e = p + 1 + 4 * ((steps - 1) * (L + 1) + L);
        t1 = std::max(t1, (long long)e[3]);
        pro += (double)(p[1] - p[0]);
        blk += (double)(e[3] - p[0]);
        ++xcc[p[EF_PHASE_STRIDE - 1] & 7];
        for (int st = 0; st < steps; ++st) {
            const unsigned long long* q0 = p + 1 + 4 * (st * (L + 1));
            l0 += (double)(q0[3] - q0[0]);
            for (int l = 1; l < L; ++l) {
                const unsigned long long* q = q0 + 4 * l;
                stg[l] += (double)(q[1] - q[0]);
                kl[l] += (double)(q[2] - q[1]);
                ep[l] += (double)(q[3] - q[2]);
            }
            const unsigned long long* qh = q0 + 4 * L;
            head += (double)(qh[3] - qh[0]);
        }
    }
    if (n == 0) return;
    const double us = 0.01 / (double)n, per = us / (double)steps;
    std::fprintf(stderr, "phase probe (split Euler flow, last launch): %lld blocks, %d steps, span %.1f us, block %.1f us, "
                 "start spread %.2f us, prologue %.2f us; blocks per XCC %d %d %d %d %d %d %d %d\n",
                 n, steps, (double)(t1 - t0) * 0.01, blk * us, (double)(tl - t0) * 0.01, pro * us, xcc[0], xcc[1],
                 xcc[2], xcc[3], xcc[4], xcc[5], xcc[6], xcc[7]);
    std::fprintf(stderr, "  layer 0 per step (redundant, no hand-off): %.3f\n", l0 * per);
    for (int l = 1; l < L; ++l)
        std::fprintf(stderr, "  layer %d per step: stage (wait + copy) %.3f | k-loop %.3f | epilogue + publish %.3f\n", l,
                     stg[l] * per, kl[l] * per, ep[l] * per);
    std::fprintf(stderr, "  head per step (wait for the 8 partials + update): %.3f\n", head * per);
}

void flip_params(fqlpop* h);

// Enqueue one population update (train) or one total_loss pass (!train).
//
// Capture rule (the HIP runtime's stream capture, ROCm 7.2): a side stream that waits on an
// event joins the capture under the stream that recorded it, and hipStreamEndCapture resets
// the joined streams recursively along those links.  A side stream that waited on another
// side stream's event which itself (transitively) waited on the first would close a cycle
// there and recurse without end (round 3's crash inside libamdhip64).  So the waits between
// side streams form a chain: sF and sB fork from sM, sB waits on sF (the BC forward), and sF
// never waits on sB; everything joins back into sM.
void enqueue(fqlpop* h, bool train, bool inj_batch, bool inj_noise) {
    const Ctx c{h, h->nz};
    const int B = h->B, D = h->D, A = h->A, H = h->H, E = h->E, L = h->L, S = h->S;
    const int Kc = D + A, Kb = D + A + 1;
    const int B2 = 2 * B, B3 = 3 * B;
    hipStream_t sM = h->sM, sF = h->sF, sB = h->sB, sX = h->sX;
    h->ev_next = 0;
    h->probe_idx = 0;
    h->cr_in = h->cr_in_buf[h->cur];
    // the persistent Euler launch writes both stamps of every block it launches, and the
    // reduction reads only those (probe_nb): no per-step clearing node at the step's head
    if (h->probe_set >= 0 && !h->euler_fused)
        HIPCHK(hipMemsetAsync(h->probe_slots + 2LL * h->probe_blocks * h->probe_set * h->probe_pairs, 0,
                              sizeof(unsigned long long) * 2 * h->probe_blocks * h->probe_pairs, sM));

    // Fork / join helper: `to` waits for everything enqueued on `from` so far.
    auto dep = [&](hipStream_t from, hipStream_t to) {
        if (from == to) return;
        hipEvent_t ev = next_event(h);
        HIPCHK(hipEventRecord(ev, from));
        HIPCHK(hipStreamWaitEvent(to, ev, 0));
    };

    // ---- sampling / assembly ------------------------------------------
    const auto& dset = (!train && h->ds[1].rows > 0) ? h->ds[1] : h->ds[0];
    SampleArgs sa{};
    sa.obs = dset.obs; sa.act = dset.act; sa.rew = dset.rew; sa.mask = dset.mask; sa.nobs = dset.nobs;
    sa.n_rows = dset.rows;
    sa.inj_batch = inj_batch ? h->inj_batch : nullptr;
    sa.inj_noise = inj_noise ? h->inj_noise : nullptr;
    sa.seeds = h->skeys; sa.count = h->count;
    sa.step_add = 0;
    sa.stream_salt = train ? 0x51A7u : 0x5A1Du;
    sa.B = B; sa.D = D; sa.A = A;
    sa.os_in = tref(h->os_in, (long long)Kc * B3);
    sa.bc_in = tref(h->bc_in, (long long)Kb * B2);
    sa.cr_in = tref(h->cr_in, (long long)Kc * B2);
    sa.tg_in = tref(h->tg_in, (long long)Kc * B);
    sa.eu_in = tref(h->eu_in, (long long)Kb * B);
    sa.act_t = tref(h->act_t, (long long)A * B);
    sa.x0_t = tref(h->x0_t, (long long)A * B);
    sa.rew_t = tref(h->rew_t, B);
    sa.mask_t = tref(h->mask_t, B);
    sa.nz = c.nz; sa.slots = h->slots;
    // one-step actor forward on [s'; s; s] (z_next; z_d; z_metric), on sM
    auto os_forward = [&]() {
        const NetLayout& N = h->os;
        HeadArgs ha = head_args(c, N, h->os_g[L - 1], B3, B3, 0);
        ha.o0 = tref(h->apiraw, (long long)A * B); ha.ld0 = B;
        ha.o1 = tref(h->tg_in, (long long)Kc * B); ha.ld1 = B;
        ha.o2 = tref(h->cr_in, (long long)Kc * B2); ha.ld2 = B2;
        ha.o3 = tref(h->amet, (long long)A * B); ha.ld3 = B;
        if (h->stream_fwd) {
            // only the z_d rows [B, 2B) are back-propagated (distill + Q loss)
            stream_fwd(c, sM, N, h->params, h->P, tref(h->os_in, (long long)Kc * B3), B3, B3, &h->os_u, &h->os_g,
                       nullptr, nullptr, (long long)H * B3, 0, 0, 0, B, 2 * B, HEAD_OS, ha);
        } else {
            fwd_hidden(c, sM, N, tref(h->os_in, (long long)Kc * B3), B3, B3, h->os_u, h->os_g, 0,
                       nullptr, nullptr, 0, true);
            launch_head_fwd(HEAD_OS, ha, sM);
        }
    };
    launch_sample(sa, sM);
    HIPCHK(hipEventRecord(h->ev_sample, sM));
    if (sF != sM) HIPCHK(hipStreamWaitEvent(sF, h->ev_sample, 0));
    if (sB != sM) HIPCHK(hipStreamWaitEvent(sB, h->ev_sample, 0));

    float* info = train ? h->info : h->vinfo;
    LossArgs la{};
    la.q = tref(h->q, (long long)E * B2, B2);
    la.qt = tref(h->qt, (long long)E * B, B);
    la.rew = tref(h->rew_t, B);
    la.mask = tref(h->mask_t, B);
    la.vpred = tref(h->vpred, (long long)A * B);
    la.act = tref(h->act_t, (long long)A * B);
    la.x0 = tref(h->x0_t, (long long)A * B);
    la.amet = tref(h->amet, (long long)A * B);
    la.apiraw = tref(h->apiraw, (long long)A * B);
    la.aflow = tref(h->aflow, (long long)A * B);
    la.da = tref(h->da, (long long)E * A * B, (long long)A * B);
    la.da_n = h->stream_bwd ? E : 1;  // per-ensemble partials of the streamed backward, else one sum
    la.dq = tref(h->dq, (long long)E * B2, B2);
    la.dv = tref(h->dv, (long long)A * B);
    la.dout_os = tref(h->dout_os, (long long)A * B);
    la.g_cb4 = pref(h, h->grads, h->critic, h->critic.b[L]);
    la.g_bcb4 = pref(h, h->grads, h->bc, h->bc.b[L]);
    la.g_osb4 = pref(h, h->grads, h->os, h->os.b[L]);
    la.info = tref(info, FQLPOP_INFO_STRIDE);
    la.alpha = h->alpha;
    la.B = B; la.A = A; la.E = E;
    la.q_min = h->cfg.q_agg_min; la.normq = h->cfg.normalize_q_loss;
    la.discount = h->cfg.discount;
    la.nz = c.nz; la.slots = h->slots;

    // ---- sF: BC-flow forward (train rows) fused with Euler step 0 --------
    {
        const NetLayout& N = h->bc;
        HeadArgs ha = head_args(c, N, h->bc_g[L - 1], B2, B2, 0);
        ha.o0 = tref(h->vpred, (long long)A * B); ha.ld0 = B;
        ha.o1 = tref(h->bc_in, (long long)Kb * B2); ha.ld1 = B2;
        ha.o2 = tref(h->eu_in, (long long)Kb * B); ha.ld2 = B;
        ha.t_next = (float)(1.0 / (double)S);
        if (h->stream_fwd) {
            // train rows [0, B) feed the BC backward; rows [B, 2B) are Euler step 0
            stream_fwd(c, sF, N, h->params, h->P, tref(h->bc_in, (long long)Kb * B2), B2, B2, &h->bc_u, &h->bc_g,
                       nullptr, nullptr, (long long)H * B2, 0, 0, 0, 0, B, HEAD_BC_FUSED, ha);
        } else {
            fwd_hidden(c, sF, N, tref(h->bc_in, (long long)Kb * B2), B2, B2, h->bc_u, h->bc_g, 0,
                       nullptr, nullptr, 0, true);
            launch_head_fwd(HEAD_BC_FUSED, ha, sF);
        }
        HIPCHK(hipEventRecord(h->ev_bcfwd, sF));
        if (h->euler_fused) {
            EulerArgs ea = euler_args(h, c.nz);
            if (h->probe_set >= 0 && h->probe_idx < h->probe_pairs)
                ea.probe = h->probe_slots + 2 * h->probe_blocks * ((long long)h->probe_set * h->probe_pairs + h->probe_idx++);
            if (!(skip_mask() & 1)) launch_euler(h, ea, sF);
        }
        for (int i = 1; !h->euler_fused && i < S + (S == 1 ? 1 : 0); ++i) {
            // S == 1: one zero-cost pass that only clips (not used by the configs here)
            fwd_hidden(c, sF, N, tref(h->eu_in, (long long)Kb * B), B, B, h->eu_g, h->eu_g, 0,
                       nullptr, nullptr, 0, false, /*euler=*/true);
            HeadArgs he = head_args(c, N, h->eu_g[L - 1], B, B, 0);
            he.o0 = tref(h->aflow, (long long)A * B); he.ld0 = B;
            he.o2 = tref(h->eu_in, (long long)Kb * B); he.ld2 = B;
            he.last = (i == S - 1) ? 1 : 0;
            he.t_next = (float)((double)(i + 1) / (double)S);
            launch_head_fwd(HEAD_EULER, he, sF);
        }
        HIPCHK(hipEventRecord(h->ev_flow, sF));
    }

    // ---- sB: BC loss + backward + Adam ------------------------------------
    // (Adam writes params_nx, so it need not wait for the flow's reads)
    if (sB != sF) HIPCHK(hipStreamWaitEvent(sB, h->ev_bcfwd, 0));
    launch_loss_bc(la, sB);
    HIPCHK(hipEventRecord(h->ev_bcloss, sB));
    if (train) {
        const NetLayout& N = h->bc;
        if (h->stream_bwd)
            stream_bwd_net(c, sB, N, tref(h->dv, (long long)A * B), B, tref(h->bc_in, (long long)Kb * B2), B2, 0, B,
                           B, h->bc_u, h->bc_g, 0, nullptr, nullptr, 0, h->bc_du, B, h->part_bc, sB);
        else
            bwd_net(c, sB, N, tref(h->dv, (long long)A * B), B, tref(h->bc_in, (long long)Kb * B2), B2, 0, B, B,
                    h->bc_u, h->bc_g, 0, nullptr, nullptr, 0, h->bc_du, h->bc_dh, nullptr, nullptr, B, sB);
        if (!h->fused_adam) {
            adam_net(c, sB, 1);
            if (h->stream_bwd) transpose_nets(h, sB, 2, false, h->params_nx, h->paramsT_nx);
        }
    }
    HIPCHK(hipEventRecord(h->ev_bdone, sB));

    // ---- sM: one-step actor forward on [s'; s; s] (z_next; z_d; z_metric) --
    os_forward();
    const NetLayout& NC = h->critic;
    const long long sy2 = (long long)H * B2, sy1 = (long long)H * B;
    // The 4th-stream schedule ("small-population schedule", since round 5
    // at every population size): the target critic and, later, the critic's TD-column backward
    // run on a 4th stream sX beside the main chain, which then carries the critic forward, the
    // Q-loss columns' backward (dQ/da) and the actor chain only.  sX forks from sM and joins
    // sM / sB; it never waits on sB or sF (capture rule above).  Same box against three
    // streams: +3.7 % at 6 members, +3.3 % at 8, +0.9 % at 12, +1.6 / +2.1 % at ant 2 / 4,
    // neutral at 4 and 16 (round 4's -12-14 % at 4 members was under the old split plan),
    // -1.1 % at ant 16 (1 024 tiles): on up to kSmallSchedTiles 16-column tiles
    const bool small = h->opt.small_sched && h->sX != h->sM && h->stream_fwd && h->stream_bwd && h->fused_adam &&
                       (long long)(h->B / 16) * c.nz <= kSmallSchedTiles;
    {
        int plan[SITE_N];
        bool plan_small = false;
        split_plan(h->opt, split_shape(h), c.nz, plan, &plan_small);
        ARGCHK(plan_small == small && plan[SITE_EULER] == euler_split(h, c.nz), "step differs from the split plan");
    }
    hipStream_t sT = small ? h->sX : sM;
    dep(sM, sT);  // a' is in the target-critic input
    // ---- sM (sX): target critic on [s', a'] (params from the target arena) -----
    if (h->stream_fwd) {
        HeadArgs ht{};
        ht.B = B; ht.D = D; ht.steps_f = (float)S;
        ht.o0 = tref(h->qt, (long long)E * B, B); ht.ld0 = B;
        stream_fwd(c, sT, NC, h->target, h->PT, tref(h->tg_in, (long long)Kc * B), B, B, nullptr, nullptr, nullptr,
                   nullptr, 0, 0, 0, 0, 0, 0, HEAD_STORE, ht);
    } else {
        const NetLayout& N = NC;
        for (int l = 0; l < L; ++l) {
            GemmArgs g{};
            g.A = tref(h->target + N.W[l], h->PT, N.ens_size);
            g.B = l == 0 ? tref(h->tg_in, (long long)Kc * B, 0) : tref(h->tg_h[l - 1], (long long)H * B * E, sy1);
            g.C = tref(N.ln ? h->tg_u[l] : h->tg_h[l], (long long)H * B * E, sy1);
            g.bias = tref(h->target + N.b[l], h->PT, N.ens_size);
            g.M = H; g.N = B; g.K = N.kdim(l);
            g.lda = H; g.ldb = B; g.ldc = B;
            g.ny = E; g.nz = c.nz; g.slots = h->slots;
            gemm(LAYOUT_FWD, N.ln ? EPI_BIAS : EPI_BIAS_GELU, g, sM);
            if (N.ln) {
                LnArgs a{};
                a.u = tref(h->tg_u[l], (long long)H * B * E, sy1);
                a.h = tref(h->tg_h[l], (long long)H * B * E, sy1);
                a.mu = tref(h->tg_mu[l], (long long)B * E, B);
                a.rstd = tref(h->tg_rs[l], (long long)B * E, B);
                a.gamma = tref(h->target + N.gam[l], h->PT, N.ens_size);
                a.beta = tref(h->target + N.bet[l], h->PT, N.ens_size);
                a.H = H; a.M = B; a.ld = B; a.ny = E; a.nz = c.nz; a.slots = h->slots;
                launch_ln_gelu_fwd(a, sM);
            }
        }
        HeadArgs ht{};
        ht.h = tref(h->tg_h[L - 1], (long long)H * B * E, sy1);
        ht.W = tref(h->target + N.W[L], h->PT, N.ens_size);
        ht.b = tref(h->target + N.b[L], h->PT, N.ens_size);
        ht.H = H; ht.M = B; ht.ld = B; ht.nout = 1; ht.B = B; ht.D = D; ht.steps_f = (float)S;
        ht.o0 = tref(h->qt, (long long)E * B, B); ht.ld0 = B;
        ht.ny = E; ht.nz = c.nz; ht.slots = h->slots;
        launch_head_fwd(HEAD_STORE, ht, sM);
    }
    // ---- sM: critic on [s,a ; s,clip(a_pi)] -------------------------------
    {
        const NetLayout& N = NC;
        HeadArgs hc = head_args(c, N, h->cr_h[L - 1], B2, B2, sy2);
        hc.o0 = tref(h->q, (long long)E * B2, B2); hc.ld0 = B2;
        if (h->stream_fwd) {
            // the a_pi columns [B, 2B) are back-propagated for dQ/da only: their layer outputs
            // (the dW GEMMs' operand) are not needed by the streamed backward
            stream_fwd(c, sM, N, h->params, h->P, tref(h->cr_in, (long long)Kc * B2, 0), B2, B2, &h->cr_u, &h->cr_h,
                       N.ln ? &h->cr_mu : nullptr, N.ln ? &h->cr_rs : nullptr, (long long)H * B2 * E, sy2,
                       (long long)B2 * E, B2, 0, B2, HEAD_STORE, hc, h->stream_bwd ? B : B2);
        } else {
            fwd_hidden(c, sM, N, tref(h->cr_in, (long long)Kc * B2, 0), B2, B2, h->cr_u, h->cr_h, sy2,
                       &h->cr_mu, &h->cr_rs, B2, true);
            launch_head_fwd(HEAD_STORE, hc, sM);
        }
    }
    dep(sT, sM);  // Q_target
    launch_loss_critic(la, sM);
    // the fused optimiser: the critic's dW + Adam is captured after the actor's dX chain, on
    // sB (idle by then), so that it runs beside that chain instead of ahead of it on a shared
    // queue (+0.5-0.9 %)
    std::function<void()> critic_dw;
    if (train) {
        // critic backward: the dX chain on sM
        InGradArgs ig{};
        ig.W0 = pref(h, h->params, NC, NC.W[0]);
        ig.du0 = tref(h->cr_du[0], (long long)H * B2 * E, sy2);
        ig.da = tref(h->da, (long long)E * A * B);
        ig.H = H; ig.D = D; ig.A = A; ig.E = E; ig.ld = B2; ig.off = B; ig.M = B;
        ig.nz = c.nz; ig.slots = h->slots;
        if (small) {
            // the Q-loss columns [B, 2B) on sM (dQ/da: the actor chain waits for it), the TD columns
            // [0, B) (parameter grads) on sX; the same per-column arithmetic as one launch
            dep(sM, sX);
            InGradArgs ig0 = ig;
            ig0.off = 0;  // (relative to the launch's columns)
            stream_bwd_net(c, sM, NC, tref(h->dq + B, (long long)E * B2, B2), B2, tref(h->cr_in, (long long)Kc * B2, 0),
                           B2, B, B, 0, h->cr_u, h->cr_h, sy2, &h->cr_mu, &h->cr_rs, B2, h->cr_du, B2, h->part_cr, sM,
                           &ig0, nullptr);
            stream_bwd_net(c, sX, NC, tref(h->dq, (long long)E * B2, B2), B2, tref(h->cr_in, (long long)Kc * B2, 0),
                           B2, 0, B, B, h->cr_u, h->cr_h, sy2, &h->cr_mu, &h->cr_rs, B2, h->cr_du, B2, h->part_cr, sB,
                           nullptr, &critic_dw);
        } else if (h->stream_bwd) {
            stream_bwd_net(c, sM, NC, tref(h->dq, (long long)E * B2, B2), B2, tref(h->cr_in, (long long)Kc * B2, 0),
                           B2, 0, B2, B, h->cr_u, h->cr_h, sy2, &h->cr_mu, &h->cr_rs, B2, h->cr_du, B2, h->part_cr,
                           h->fused_adam ? sB : sM, &ig, h->fused_adam ? &critic_dw : nullptr);
        } else {
            bwd_net(c, sM, NC, tref(h->dq, (long long)E * B2, B2), B2, tref(h->cr_in, (long long)Kc * B2, 0), B2, 0,
                    B2, B, h->cr_u, h->cr_h, sy2, &h->cr_mu, &h->cr_rs, B2, h->cr_du, h->cr_dh, h->cr_c1, h->cr_c2,
                    B2, sM);
            launch_input_grad(ig, sM);
        }
        // critic Adam + target EMA (the unfused paths)
        if (!h->fused_adam) {
            adam_net(c, sM, 0);
            if (h->stream_bwd) transpose_nets(h, sM, 1, false, h->params_nx, h->paramsT_nx);
        }
    }
    if (sF != sM) HIPCHK(hipStreamWaitEvent(sM, h->ev_flow, 0));
    if (sB != sM) HIPCHK(hipStreamWaitEvent(sM, h->ev_bcloss, 0));
    if (!(skip_mask() & 256)) launch_loss_actor(la, sM);
    if (train) {
        const NetLayout& N = h->os;
        if (h->fused_adam) {
            // the critic's dW launch waits for the actor loss too, so that the actor backward
            // (the critical chain) is dispatched first: a dW launch dispatched ahead of it
            // takes every CU's LDS (3 blocks of 51 KB) and starves it
            dep(sM, sB);
            if (small) dep(sX, sB);  // (and for the TD-column backward on sX)
            // actor dX chain, then the critic's grads + Adam (sB) beside the actor's (sM), then
            // the join
            std::function<void()> os_dw;
            stream_bwd_net(c, sM, N, tref(h->dout_os, (long long)A * B), B, tref(h->os_in + B, (long long)Kc * B3), B3,
                           B, B, B, h->os_u, h->os_g, 0, nullptr, nullptr, 0, h->os_du, B, h->part_os, sM, nullptr,
                           &os_dw);
            critic_dw();  // the fused launches include each net's small-leaf Adam
            os_dw();
            dep(sB, sM);
        } else {
            if (h->stream_bwd)
                stream_bwd_net(c, sM, N, tref(h->dout_os, (long long)A * B), B, tref(h->os_in + B, (long long)Kc * B3),
                               B3, B, B, B, h->os_u, h->os_g, 0, nullptr, nullptr, 0, h->os_du, B, h->part_os, sM);
            else
                bwd_net(c, sM, N, tref(h->dout_os, (long long)A * B), B, tref(h->os_in + B, (long long)Kc * B3), B3, B,
                        B, B, h->os_u, h->os_g, 0, nullptr, nullptr, 0, h->os_du, h->os_dh, nullptr, nullptr, B, sM);
            adam_net(c, sM, 2);
            if (h->stream_bwd) transpose_nets(h, sM, 4, false, h->params_nx, h->paramsT_nx);
        }
        if (sB != sM) HIPCHK(hipStreamWaitEvent(sM, h->ev_bdone, 0));
        FinalArgs fa{};
        fa.stats = h->stats; fa.chunk_leaf = h->chunk_leaf; fa.leaf_first = h->leaf_first;
        fa.n_total_chunks = h->n_chunks_total; fa.n_leaves = h->n_train_leaves;
        fa.info = tref(h->info, FQLPOP_INFO_STRIDE);
        fa.count = h->count;
        fa.nz = c.nz; fa.slots = h->slots;
        launch_finalize(fa, sM);
    } else if (sB != sM) {
        HIPCHK(hipStreamWaitEvent(sM, h->ev_bdone, 0));
    }
    HIPCHK(hipGetLastError());
}

// Swap the parameter buffer pairs after a train step was enqueued.
void flip_params(fqlpop* h) {
    h->cur ^= 1;
    h->params = h->params_buf[h->cur];
    h->params_nx = h->params_buf[h->cur ^ 1];
    h->paramsT = h->paramsT_buf[h->cur];
    h->paramsT_nx = h->paramsT_buf[h->cur ^ 1];
}

Graphs& graph_for(fqlpop* h, bool train, bool inj_batch, bool inj_noise, bool recapture);

void run(fqlpop* h, bool train, bool inj_batch, bool inj_noise) {
    if (h->nz == 0) return;
    if (h->stream_bwd && h->wt_dirty) {  // params set on the host side since the last step
        transpose_nets(h, h->sM, 7, true, h->params, h->paramsT);
        transpose_nets(h, h->sM, 7, true, h->params, h->paramsT_nx);
        h->wt_dirty = false;
    }
    if (!h->cfg.use_graph) {
        enqueue(h, train, inj_batch, inj_noise);
        if (train) flip_params(h);
        return;
    }
    Graphs& gr = graph_for(h, train, inj_batch, inj_noise, false);
    HIPCHK(hipGraphLaunch(gr.exec, h->sM));
    if (train) flip_params(h);
}

// The graph of one step for the current (mode, active count, probe set, parameter buffer),
// captured if missing (or always, with `recapture`).
Graphs& graph_for(fqlpop* h, bool train, bool inj_batch, bool inj_noise, bool recapture) {
    // one graph per (mode, active-member count): kernels read the active slot ids
    // from device memory, so any active set of the same size replays the graph
    const long long key = ((train ? 4 : 0) + (inj_batch ? 2 : 0) + (inj_noise ? 1 : 0)) + 8LL * h->nz +
                          (1LL << 32) * (h->probe_set + 1) + (1LL << 36) * h->cur;
    Graphs& gr = h->graphs[key];
    if (recapture || gr.exec == nullptr || gr.nz != h->nz) {
        if (gr.exec) HIPCHK(hipGraphExecDestroy(gr.exec));
        gr.exec = nullptr;
        hipGraph_t graph;
        {   // the hardware-queue invariant: no more branches than the runtime has queues
            std::vector<hipStream_t> ss;
            for (hipStream_t s : {h->sM, h->sF, h->sB, h->sX})
                if (std::find(ss.begin(), ss.end(), s) == ss.end()) ss.push_back(s);
            if ((int)ss.size() > 1 && (int)ss.size() > h->opt.hw_queues)
                throw FqErr{FQLPOP_E_STATE, "step graph would have " + std::to_string(ss.size()) +
                                                " parallel branches on " + std::to_string(h->opt.hw_queues) +
                                                " hardware queues (hipGraphLaunch is unsafe then)"};
        }
        HIPCHK(hipStreamBeginCapture(h->sM, hipStreamCaptureModeRelaxed));
        try {
            enqueue(h, train, inj_batch, inj_noise);
        } catch (...) {
            (void)hipStreamEndCapture(h->sM, &graph);
            throw;
        }
        HIPCHK(hipStreamEndCapture(h->sM, &graph));
        HIPCHK(hipGraphInstantiate(&gr.exec, graph, nullptr, nullptr, 0));
        HIPCHK(hipGraphUpload(gr.exec, h->sM));  // (else the first launch uploads it)
        HIPCHK(hipGraphDestroy(graph));
        gr.nz = h->nz;
    }
    return gr;
}

// Launch duration from per-block stamps: max(end) - min(start) over the blocks
// that ran (0 = slot not written).  s_memrealtime counts at 100 MHz.
double probe_launch_us(const unsigned long long* v, long long blocks) {
    unsigned long long lo = ~0ULL, hi = 0;
    for (long long b = 0; b < blocks; ++b) {
        if (v[2 * b] == 0 || v[2 * b + 1] == 0) continue;
        lo = std::min(lo, v[2 * b]);
        hi = std::max(hi, v[2 * b + 1]);
    }
    return hi > lo ? (double)(hi - lo) * 0.01 : -1.0;
}

// Accumulate the timing stamps of one probe set (waits for its step to finish).
void probe_consume(fqlpop* h, int set) {
    HIPCHK(hipEventSynchronize(h->probe_done[set]));
    const long long per = 2 * h->probe_blocks;
    std::vector<unsigned long long> v(per * h->probe_pairs);
    std::memcpy(v.data(), h->probe_host + per * set * h->probe_pairs, sizeof(unsigned long long) * v.size());
    for (int p = 0; p < h->probe_pairs; ++p) {
        const long long nb = h->euler_fused ? h->probe_nb[set] : h->probe_blocks;
        const double us = probe_launch_us(v.data() + per * p, nb);
        if (us < 0) continue;  // launch not probed
        h->probe_total_ms += us * 1e-3;
        ++h->probe_launches;
        for (long long b = 0; b < nb; ++b) h->probe_blocks_seen += v[per * p + 2 * b] && v[per * p + 2 * b + 1];
        h->probe_blocks_expected += nb;
    }
    // cleared after reading, so every launch's coverage counts only its own stamps (the set's
    // next launch is enqueued after this: fqlpop_step consumes a set before reusing it)
    std::memset(h->probe_host + per * set * h->probe_pairs, 0, sizeof(unsigned long long) * v.size());
    h->probe_pending[set] = false;
}

void sync_all_streams(fqlpop* h) {
    for (hipStream_t s : {h->sM, h->sF, h->sB, h->sX})
        if (s) HIPCHK(hipStreamSynchronize(s));
}

void update_slots(fqlpop* h) {
    const int prev = h->nz;
    h->h_slots.clear();
    for (int i = 0; i < h->n; ++i)
        if (h->active[i]) h->h_slots.push_back(i);
    h->nz = (int)h->h_slots.size();
    HIPCHK(hipStreamSynchronize(h->sM));
    if (h->nz != prev) {
        // a changed active count changes the cluster count of every split site: exchange words
        // of clusters the next launches do not rewrite would keep old tags, and the 24-bit
        // generation in a tag repeats after 2^24 launches.  Tag 0 matches no hand-off.
        bool any = false;
        for (auto& st : h->split_site) any |= st.xch != nullptr;
        if (any) {
            sync_all_streams(h);
            for (auto& st : h->split_site)
                if (st.xch) HIPCHK(hipMemset(st.xch, 0, split_cluster_bytes() * st.clusters));
            HIPCHK(hipDeviceSynchronize());
        }
    }
    if (h->nz) HIPCHK(hipMemcpy(h->slots, h->h_slots.data(), sizeof(int) * h->nz, hipMemcpyHostToDevice));
}

template <typename F>
int guard(F&& f) {
    try {
        f();
        g_err.clear();
        return FQLPOP_OK;
    } catch (const FqErr& e) {
        g_err = e.msg;
        return e.code;
    } catch (const std::exception& e) {
        g_err = e.what();
        return FQLPOP_E_STATE;
    }
}

bool split_error_pending(const fqlpop* h) {
    return h->split_err_host && __atomic_load_n(h->split_err_host, __ATOMIC_ACQUIRE) != 0;
}

// A split launch whose hand-off wait gave up (kernels.hip, sp_fail) left invalid results.
// The failure is sticky per member: every member that was active poisons, and each entry
// point that would train on or export a poisoned member's state keeps refusing until the
// caller restores it (set_state of params, Adam m and Adam v, or set_member with reinit).
// member < 0: any poisoned member refuses (whole-population calls).  The caller has
// synchronised the streams.
// The pending error word, if set, becomes the poison flags of the active members (returns true).
bool absorb_split_error(fqlpop* h) {
    if (!split_error_pending(h)) return false;
    __atomic_store_n(h->split_err_host, 0u, __ATOMIC_RELEASE);
    for (auto& st : h->split_site)  // a launch that gave up may have left its counters set
        if (st.cnt) HIPCHK(hipMemset(st.cnt, 0, sizeof(unsigned) * split_counter_stride() * (st.clusters + 2)));
    for (int i = 0; i < h->n; ++i)
        if (h->active[i]) {
            h->poisoned[i] = 1;
            h->restored[i] = 0;
        }
    return true;
}
const char* const kSplitFailMsg =
    "a split launch's hand-off wait timed out (blocks of a cluster not resident together); the state of every "
    "member it stepped is invalid until restored (fqlpop_set_state of params, Adam m and v, or fqlpop_set_member "
    "with reinit)";
// only_active: whole-population training calls refuse for poisoned ACTIVE members only (a
// pruned member does not step)
void check_split_error(fqlpop* h, int member = -1, bool only_active = false) {
    if (absorb_split_error(h)) throw FqErr{FQLPOP_E_STATE, kSplitFailMsg};
    for (int i = member < 0 ? 0 : member; i < (member < 0 ? h->n : member + 1); ++i)
        if (h->poisoned[i] && (!only_active || h->active[i]))
            throw FqErr{FQLPOP_E_STATE, "member " + std::to_string(i) + "'s state was written by a failed split "
                                        "launch; restore it first (fqlpop_set_state of params, Adam m and v, or "
                                        "fqlpop_set_member with reinit)"};
}
void note_restored(fqlpop* h, int member, int which) {
    if (!h->poisoned[member]) return;
    h->restored[member] |= (unsigned char)(1u << which);
    if (h->restored[member] == 7) h->poisoned[member] = 0;
}

void check_member(fqlpop* h, int member) {
    ARGCHK(h != nullptr, "null handle");
    ARGCHK(member >= 0 && member < h->n, "member index out of range");
}

}  // namespace

void fq::set_last_error(const char* msg) { g_err = msg ? msg : ""; }
int fq::engine_option_em_seq_sweep() { return g_engine_opts.em_seq_sweep; }

// =================================================================== C ABI ==
extern "C" {

const char* fqlpop_last_error(void) { return g_err.c_str(); }

int fqlpop_set_engine_option(const char* name, int value) {
    return guard([&] {
        ARGCHK(name != nullptr, "null option name");
        for (const EngineOptionRef& o : kEngineOptions)
            if (std::strcmp(o.name, name) == 0) {
                ARGCHK(value >= o.lo && value <= o.hi, std::string("engine option ") + name + " out of range");
                ARGCHK(o.field != &EngineOptions::split || value <= 2 || value == 4 || value == 8,
                       "engine option split: 0, 1, 2, 4 or 8");
                g_engine_opts.*o.field = value;
                return;
            }
        throw FqErr{FQLPOP_E_ARG, std::string("unknown engine option ") + name};
    });
}

int fqlpop_get_engine_option(const char* name, int* value) {
    return guard([&] {
        ARGCHK(name != nullptr && value != nullptr, "null argument");
        for (const EngineOptionRef& o : kEngineOptions)
            if (std::strcmp(o.name, name) == 0) {
                *value = g_engine_opts.*o.field;
                return;
            }
        throw FqErr{FQLPOP_E_ARG, std::string("unknown engine option ") + name};
    });
}

int fqlpop_reset_engine_options(void) {
    return guard([&] { g_engine_opts = EngineOptions{}; });
}

int fqlpop_split_plan(const fqlpop_config* cfg, int n_members, int* blocks_per_tile, int* small_sched) {
    return guard([&] {
        ARGCHK(cfg && blocks_per_tile && small_sched && n_members >= 1, "bad argument");
        const EngineOptions& eo = g_engine_opts;
        const int D = cfg->obs_dim, A = cfg->action_dim, B = cfg->batch_size, H = cfg->hidden_dim, L = cfg->num_hidden;
        SplitShape d{H, L, A, B, cfg->num_qs, D + A + 1, D + A, D + A, cfg->layer_norm != 0,
                     stream_fwd_supported(H, L, D + A + 1, A, B) && eo.stream_fwd != 0,
                     stream_bwd_supported(H, L, A, B, B) && eo.stream_bwd != 0, false,
                     euler_flow_supported(H, L, D, A, B) && !cfg->actor_layer_norm && eo.euler_fused != 0,
                     step_streams(eo) > 1};
        d.fused_adam = d.stream_bwd && H % 128 == 0 && L <= GEMM_GROUP_MAX && eo.fused_adam;
        int F[SITE_N];
        bool small = false;
        split_plan(eo, d, n_members, F, &small);
        for (int i = 0; i < SITE_N; ++i) blocks_per_tile[i] = F[i];
        *small_sched = small ? 1 : 0;
    });
}

int fqlpop_step_streams(int* n_streams) {
    return guard([&] {
        ARGCHK(n_streams != nullptr, "null argument");
        *n_streams = step_streams(g_engine_opts);
    });
}

int fqlpop_diagnostic_build(void) {
#ifdef FQ_DIAG
    return 1;
#else
    return 0;
#endif
}

double fqlpop_flops_per_member_step(const fqlpop_config* c) {
    // F(i,o) = 2B(iH + (L-1)H^2 + Ho) per forward; dX without
    // the first layer = 2B((L-1)H^2 + Ho).
    const double B = c->batch_size, H = c->hidden_dim, L = c->num_hidden, D = c->obs_dim, A = c->action_dim;
    const double E = c->num_qs, S = c->flow_steps;
    auto F = [&](double i, double o) { return 2.0 * B * (i * H + (L - 1) * H * H + H * o); };
    auto dX = [&](double o) { return 2.0 * B * ((L - 1) * H * H + H * o); };
    const double Fc = F(D + A, 1), Fbc = F(D + A + 1, A), Fos = F(D + A, A);
    return Fos + E * Fc + E * Fc + E * Fc + E * dX(1) + Fbc + Fbc + dX(A) + S * Fbc + Fos + Fos + dX(A) +
           E * Fc + E * Fc + Fos;
}

int fqlpop_create(const fqlpop_config* cfg, int n_members, const float* alphas, const uint64_t* seeds_in,
                  int device, fqlpop_t** out) {
    return guard([&] {
        ARGCHK(cfg && out && alphas && seeds_in, "null argument");
        ARGCHK(n_members > 0, "n_members must be > 0");
        ARGCHK(cfg->action_dim >= 1 && cfg->action_dim <= 8, "action_dim must be in [1, 8]");
        ARGCHK(cfg->obs_dim >= 1, "obs_dim must be >= 1");
        {
            const int hd = cfg->hidden_dim;
            ARGCHK(hd == 64 || hd == 128 || hd == 256 || hd == 512 || hd == 1024,
                   "hidden_dim must be one of 64, 128, 256, 512, 1024");
        }
        ARGCHK(cfg->num_hidden >= 1, "num_hidden must be >= 1");
        ARGCHK(cfg->batch_size >= 64 && cfg->batch_size % 64 == 0, "batch_size must be a multiple of 64");
        ARGCHK(cfg->num_qs >= 1 && cfg->num_qs <= 4, "num_qs must be in [1, 4]");
        ARGCHK(cfg->flow_steps >= 2, "flow_steps must be >= 2");
        if (cfg->actor_layer_norm)
            throw FqErr{FQLPOP_E_UNSUPPORTED, "actor_layer_norm is not supported yet (reference default False)"};
        auto h = std::make_unique<fqlpop>();
        h->cfg = *cfg;
        h->n = n_members;
        h->device = device;
        HIPCHK(hipSetDevice(device));
        h->D = cfg->obs_dim; h->A = cfg->action_dim; h->H = cfg->hidden_dim; h->L = cfg->num_hidden;
        h->B = cfg->batch_size; h->E = cfg->num_qs; h->S = cfg->flow_steps;
        const int D = h->D, A = h->A, H = h->H, L = h->L, B = h->B, E = h->E;
        h->critic.build("critic", D + A, 1, L, H, E, cfg->layer_norm != 0);
        h->bc.build("actor_bc_flow", D + A + 1, A, L, H, 1, cfg->actor_layer_norm != 0);
        h->os.build("actor_onestep_flow", D + A, A, L, H, 1, cfg->actor_layer_norm != 0);
        h->critic.off = 0;
        h->bc.off = align_up(h->critic.size());
        h->os.off = align_up(h->bc.off + h->bc.size());
        h->P = align_up(h->os.off + h->os.size());
        h->PT = align_up(h->critic.size());
        build_leaves(h.get());

        h->opt = g_engine_opts;
        const EngineOptions& eo = h->opt;
        // three or four streams; serial (profiling option): every kernel
        // of the step on sM, so a kernel trace shows uncontended durations.  With fewer than 4
        // hardware queues the step is captured on one stream too: the HIP runtime's graph launch
        // hands a graph's parallel branches to a pool of streams and can index past that pool
        // when more than one of them shares the launch stream's hardware queue (a crash inside
        // hipGraphLaunch)
        HIPCHK(hipStreamCreateWithFlags(&h->sM, hipStreamNonBlocking));
        if (step_streams(eo) == 1) {
            h->sF = h->sB = h->sX = h->sM;
        } else {
            HIPCHK(hipStreamCreateWithFlags(&h->sF, hipStreamNonBlocking));
            HIPCHK(hipStreamCreateWithFlags(&h->sB, hipStreamNonBlocking));
            HIPCHK(hipStreamCreateWithFlags(&h->sX, hipStreamNonBlocking));
        }
        h->ev_pool.resize(64);
        h->euler_fused = euler_flow_supported(H, L, D, A, B) && !h->bc.ln && eo.euler_fused;
        h->stream_fwd = stream_fwd_supported(H, L, D + A + 1, A, B) && eo.stream_fwd;
        h->stream_bwd = stream_bwd_supported(H, L, A, B, B) && eo.stream_bwd;
        // Adam / EMA / W^T / grad stats fused into the grouped dW epilogue
        h->fused_adam = h->stream_bwd && H % 128 == 0 && L <= GEMM_GROUP_MAX && h->critic.off == 0 && eo.fused_adam;
        if (h->euler_fused) {  // dominant kernel: one persistent Euler launch per step
            h->probe_pairs = 1;
            // (the split Euler launch: up to 8 blocks per 16-column tile)
            h->probe_blocks = std::max<long long>((long long)(cfg->batch_size / 16) * n_members * 8, kSplitMaxBlocks);
        } else {               // dominant kernel: the Euler hidden-layer GEMMs
            h->probe_pairs = std::max(1, (cfg->flow_steps - 1) * (cfg->num_hidden - 1));
            h->probe_blocks = (long long)((cfg->hidden_dim + 63) / 64) * ((cfg->batch_size + 63) / 64) * n_members;
        }
        // the stamps go straight to mapped host memory: the host reads them after the step's
        // event, with no device-to-host copy (a copy kernel) interleaved with the steps
        const size_t pb = sizeof(unsigned long long) * 4 * h->probe_blocks * h->probe_pairs;
        HIPCHK(hipHostMalloc((void**)&h->probe_host, pb, hipHostMallocMapped | hipHostMallocCoherent));
#ifdef FQ_PHASE_PROBE  // the kernels write the phase stamps only in this build (make PHASE=1)
        if (const char* e = diag_env("FQLPOP_PHASE_PROBE"); e != nullptr && e[0] == '1') {
            // the critic backward's blocks: 2B columns in 16-column tiles per ensemble member
            h->phase_blocks = (long long)(2 * cfg->batch_size / 16) * E * n_members;
            const size_t phb = sizeof(unsigned long long) * SB_PHASE_STRIDE * h->phase_blocks;
            HIPCHK(hipHostMalloc((void**)&h->phase_host, phb, hipHostMallocMapped | hipHostMallocCoherent));
            std::memset(h->phase_host, 0, phb);
            HIPCHK(hipHostGetDevicePointer((void**)&h->phase_dev, h->phase_host, 0));
            if (h->euler_fused && cfg->flow_steps <= 11) {
                h->ephase_blocks = (long long)(cfg->batch_size / 16) * n_members * 8;  // (split: up to 8 per tile)
                const size_t eb = sizeof(unsigned long long) * EF_PHASE_STRIDE * h->ephase_blocks;
                HIPCHK(hipHostMalloc((void**)&h->ephase_host, eb, hipHostMallocMapped | hipHostMallocCoherent));
                std::memset(h->ephase_host, 0, eb);
                HIPCHK(hipHostGetDevicePointer((void**)&h->ephase_dev, h->ephase_host, 0));
            }
        }
#endif
        std::memset(h->probe_host, 0, pb);
        HIPCHK(hipHostGetDevicePointer((void**)&h->probe_slots, h->probe_host, 0));
        for (auto& e : h->probe_done) HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
        HIPCHK(hipStreamCreateWithFlags(&h->probe_stream, hipStreamNonBlocking));
        for (auto& e : h->ev_pool) HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
        for (hipEvent_t* e : {&h->ev_sample, &h->ev_bcfwd, &h->ev_bcloss, &h->ev_flow, &h->ev_bdone})
            HIPCHK(hipEventCreateWithFlags(e, hipEventDisableTiming));
        HIPCHK(hipEventCreate(&h->ev_t0));
        HIPCHK(hipEventCreate(&h->ev_t1));

        const int n = h->n;
        for (float*& pb : h->params_buf) {
            HIPCHK(hipMalloc(&pb, sizeof(float) * h->P * n));
            HIPCHK(hipMemset(pb, 0, sizeof(float) * h->P * n));
        }
        h->params = h->params_buf[0];
        h->params_nx = h->params_buf[1];
        HIPCHK(hipMalloc(&h->grads, sizeof(float) * h->P * n));
        HIPCHK(hipMalloc(&h->adam_m, sizeof(float) * h->P * n));
        HIPCHK(hipMalloc(&h->adam_v, sizeof(float) * h->P * n));
        HIPCHK(hipMalloc(&h->target, sizeof(float) * h->PT * n));
        HIPCHK(hipMemset(h->grads, 0, sizeof(float) * h->P * n));
        HIPCHK(hipMalloc(&h->count, sizeof(int) * n));
        HIPCHK(hipMalloc(&h->seeds, sizeof(uint64_t) * n));
        HIPCHK(hipMalloc(&h->skeys, sizeof(uint64_t) * n));
        HIPCHK(hipMalloc(&h->alpha, sizeof(float) * n));
        HIPCHK(hipMalloc(&h->slots, sizeof(int) * n));
        build_chunks(h.get());

        const int Kc = D + A, Kb = D + A + 1, B2 = 2 * B, B3 = 3 * B;
        h->os_in = h->alloc(align_up((long long)Kc * B3));
        h->bc_in = h->alloc(align_up((long long)Kb * B2));
        h->eu_in = h->alloc(align_up((long long)Kb * B));
        for (float*& cb : h->cr_in_buf) cb = h->alloc(align_up((long long)Kc * B2));
        h->cr_in = h->cr_in_buf[0];
        h->tg_in = h->alloc(align_up((long long)Kc * B));
        for (int l = 0; l < L; ++l) {
            h->os_u.push_back(h->alloc((long long)H * B3));
            h->os_g.push_back(h->alloc((long long)H * B3));
            h->bc_u.push_back(h->alloc((long long)H * B2));
            h->bc_g.push_back(h->alloc((long long)H * B2));
            h->eu_g.push_back(h->alloc((long long)H * B));
            h->cr_u.push_back(h->alloc((long long)H * B2 * E));
            h->cr_h.push_back(h->alloc((long long)H * B2 * E));
            h->cr_mu.push_back(h->alloc((long long)B2 * E));
            h->cr_rs.push_back(h->alloc((long long)B2 * E));
            h->tg_u.push_back(h->alloc((long long)H * B * E));
            h->tg_h.push_back(h->alloc((long long)H * B * E));
            h->tg_mu.push_back(h->alloc((long long)B * E));
            h->tg_rs.push_back(h->alloc((long long)B * E));
            h->cr_du.push_back(h->alloc((long long)H * B2 * E));
            h->bc_du.push_back(h->alloc((long long)H * B));
            h->os_du.push_back(h->alloc((long long)H * B));
        }
        if (h->stream_bwd) {
            const int T = B / 16;  // tiles with partials (Mg = B for every net)
            h->part_cr = h->alloc((long long)E * T * stream_bwd_np(L, H, 1, h->critic.ln));
            h->part_bc = h->alloc((long long)T * stream_bwd_np(L, H, A, h->bc.ln));
            h->part_os = h->alloc((long long)T * stream_bwd_np(L, H, A, h->os.ln));
            const long long HH = (long long)H * H;
            h->wt_net_off[0] = 0;
            h->wt_net_off[1] = (long long)E * (L - 1) * HH;
            h->wt_net_off[2] = (long long)(E + 1) * (L - 1) * HH;
            h->PTT = (long long)(E + 2) * (L - 1) * HH;
            h->paramsT_buf[0] = h->paramsT = h->alloc(std::max<long long>(1, h->PTT));
            h->paramsT_buf[1] = h->paramsT_nx = h->alloc(std::max<long long>(1, h->PTT));
        }
        // split launch sites: exchange and counters for up to kSplitMaxClusters tiles each
        h->split_ok = h->stream_fwd && eo.split != 0;
        if (h->split_ok) {
            const long long tiles_per_member[SITE_N] = {B2 / 16, B / 16, B3 / 16, (long long)E * B / 16,
                                                        (long long)E * B2 / 16, (long long)E * B2 / 16, B / 16,
                                                        (long long)E * B / 16};
            for (int si = 0; si < SITE_N; ++si) {
                auto& st = h->split_site[si];
                st.clusters = std::min(kSplitMaxClusters, tiles_per_member[si] * n);
                HIPCHK(hipMalloc(&st.xch, split_cluster_bytes() * st.clusters));
                HIPCHK(hipMemset(st.xch, 0, split_cluster_bytes() * st.clusters));  // tag 0 matches no hand-off
                HIPCHK(hipMalloc(&st.cnt, sizeof(unsigned) * split_counter_stride() * (st.clusters + 2)));
                HIPCHK(hipMemset(st.cnt, 0, sizeof(unsigned) * split_counter_stride() * (st.clusters + 2)));
                HIPCHK(hipMalloc(&st.gen, 64));
                HIPCHK(hipMemset(st.gen, 0, 64));
            }
            // the split Euler flow's layer-0 accumulators: 32 KB per block, for the largest split
            // Euler launch (up to 128 tiles at 8 blocks each)
            if (split_euler_pre0(D + A + 1, D)) {
                h->euler_pre0_blocks = std::min<long long>(h->split_site[SITE_EULER].clusters, 128) * 8;
                HIPCHK(hipMalloc(&h->euler_pre0, sizeof(float) * split_euler_pre0_floats() * h->euler_pre0_blocks));
            }
            // the error word lives in host memory so that every entry point can test it without a
            // device-to-host copy (fqlpop_step does, before it enqueues more steps)
            HIPCHK(hipHostMalloc((void**)&h->split_err_host, 64, hipHostMallocMapped | hipHostMallocCoherent));
            std::memset(h->split_err_host, 0, 64);
            HIPCHK(hipHostGetDevicePointer((void**)&h->split_err, h->split_err_host, 0));
        }
        h->cr_dh = h->alloc((long long)H * B2 * E);
        h->bc_dh = h->alloc((long long)H * B);
        h->os_dh = h->alloc((long long)H * B);
        h->cr_c1 = h->alloc((long long)B2 * E);
        h->cr_c2 = h->alloc((long long)B2 * E);
        h->q = h->alloc((long long)E * B2);
        h->dq = h->alloc((long long)E * B2);
        h->qt = h->alloc((long long)E * B);
        for (float** p : {&h->vpred, &h->dv, &h->act_t, &h->x0_t, &h->apiraw, &h->aflow, &h->amet, &h->dout_os})
            *p = h->alloc((long long)A * B);
        h->da = h->alloc((long long)E * A * B);  // dQ/da, one partial per critic ensemble member
        h->rew_t = h->alloc(B);
        h->mask_t = h->alloc(B);
        h->info = h->alloc(FQLPOP_INFO_STRIDE);
        h->vinfo = h->alloc(FQLPOP_INFO_STRIDE);
        h->inj_bs = (long long)B * (2 * D + A + 2);
        h->inj_ns = (long long)B * (4 * A + 1);
        h->inj_batch = h->alloc(h->inj_bs);
        h->inj_noise = h->alloc(h->inj_ns);

        h->h_alpha.assign(alphas, alphas + n);
        h->h_seeds.assign(seeds_in, seeds_in + n);
        HIPCHK(hipMemcpy(h->alpha, alphas, sizeof(float) * n, hipMemcpyHostToDevice));
        HIPCHK(hipMemcpy(h->seeds, seeds_in, sizeof(uint64_t) * n, hipMemcpyHostToDevice));
        for (int i = 0; i < n; ++i) upload_skey(h.get(), i);
        for (int i = 0; i < n; ++i) init_member(h.get(), i, seeds_in[i]);
        h->active.assign(n, 1);
        h->poisoned.assign(n, 0);
        h->restored.assign(n, 0);
        update_slots(h.get());
        HIPCHK(hipDeviceSynchronize());
        *out = h.release();
    });
}

int fqlpop_destroy(fqlpop_t* h) {
    return guard([&] {
        if (!h) return;
        (void)hipSetDevice(h->device);
        (void)hipDeviceSynchronize();
        for (auto& kv : h->graphs)
            if (kv.second.exec) (void)hipGraphExecDestroy(kv.second.exec);
        for (float* p : h->allocs) (void)hipFree(p);
        for (void* p : {(void*)h->params_buf[0], (void*)h->params_buf[1], (void*)h->res_ids, (void*)h->grads, (void*)h->adam_m, (void*)h->adam_v, (void*)h->target,
                        (void*)h->count, (void*)h->seeds, (void*)h->skeys, (void*)h->alpha, (void*)h->slots, (void*)h->stats,
                        (void*)h->chunks, (void*)h->chunk_leaf, (void*)h->leaf_first, (void*)h->sp_params,
                        (void*)h->tp_params})
            if (p) (void)hipFree(p);
        for (auto& d : h->ds)
            for (float* p : {d.obs, d.act, d.rew, d.mask, d.nobs})
                if (p) (void)hipFree(p);
        for (auto& st : h->split_site) {
            if (st.xch) (void)hipFree(st.xch);
            if (st.cnt) (void)hipFree(st.cnt);
            if (st.gen) (void)hipFree(st.gen);
        }
        if (h->euler_pre0) (void)hipFree(h->euler_pre0);
        if (h->split_err_host) (void)hipHostFree(h->split_err_host);
        for (hipEvent_t e : {h->ev_sample, h->ev_bcfwd, h->ev_bcloss, h->ev_flow, h->ev_bdone, h->ev_t0, h->ev_t1})
            if (e) (void)hipEventDestroy(e);
        for (hipEvent_t e : h->ev_pool) (void)hipEventDestroy(e);
        for (hipEvent_t e : h->probe_done)
            if (e) (void)hipEventDestroy(e);
        if (h->probe_stream) (void)hipStreamDestroy(h->probe_stream);
        if (h->probe_host) (void)hipHostFree(h->probe_host);
        if (h->phase_host) {
            (void)hipDeviceSynchronize();
            if (const char* f = diag_env("FQLPOP_PHASE_DUMP")) {  // raw stamps for offline analysis
                if (FILE* fp = std::fopen(f, "wb")) {
                    std::fwrite(h->phase_host, sizeof(unsigned long long), (size_t)SB_PHASE_STRIDE * h->phase_blocks, fp);
                    std::fclose(fp);
                }
            }
            const NetLayout* pn = phase_net(h);
            phase_report(h->phase_host, h->phase_blocks, h->L, pn->ln,
                         pn == &h->critic ? "critic" : pn == &h->bc ? "BC" : "one-step");
            (void)hipHostFree(h->phase_host);
        }
        if (h->ephase_host) {
            if (euler_split(h, h->nz) > 1)
                split_euler_phase_report(h->ephase_host, h->ephase_blocks, h->L, h->S - 1);
            else
                euler_phase_report(h->ephase_host, h->ephase_blocks, h->L, h->S - 1);
            (void)hipHostFree(h->ephase_host);
        }
        if (h->sX && h->sX != h->sM) (void)hipStreamDestroy(h->sX);
        if (h->sF && h->sF != h->sM) (void)hipStreamDestroy(h->sF);
        if (h->sB && h->sB != h->sM) (void)hipStreamDestroy(h->sB);
        if (h->sM) (void)hipStreamDestroy(h->sM);
        delete h;
    });
}

int fqlpop_set_dataset(fqlpop_t* h, int which, const float* obs, const float* act, const float* rew,
                       const float* mask, const float* next_obs, int64_t n_rows, int on_device) {
    return guard([&] {
        ARGCHK(h && obs && act && rew && mask && next_obs, "null argument");
        ARGCHK(which == 0 || which == 1, "which must be 0 (train) or 1 (val)");
        ARGCHK(n_rows > 0 && n_rows < (1LL << 32), "n_rows out of range");
        HIPCHK(hipSetDevice(h->device));
        HIPCHK(hipDeviceSynchronize());
        auto& d = h->ds[which];
        for (float* p : {d.obs, d.act, d.rew, d.mask, d.nobs})
            if (p) HIPCHK(hipFree(p));
        const long long n = n_rows;
        const hipMemcpyKind kind = on_device ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice;
        auto up = [&](float** dst, const float* src, long long cnt) {
            HIPCHK(hipMalloc(dst, sizeof(float) * cnt));
            HIPCHK(hipMemcpy(*dst, src, sizeof(float) * cnt, kind));
        };
        up(&d.obs, obs, n * h->D);
        up(&d.act, act, n * h->A);
        up(&d.rew, rew, n);
        up(&d.mask, mask, n);
        up(&d.nobs, next_obs, n * h->D);
        d.rows = n;
        // graphs bake dataset pointers in: drop them
        for (auto& kv : h->graphs)
            if (kv.second.exec) { HIPCHK(hipGraphExecDestroy(kv.second.exec)); kv.second.exec = nullptr; }
    });
}

int fqlpop_set_active(fqlpop_t* h, const uint8_t* mask) {
    return guard([&] {
        ARGCHK(h && mask, "null argument");
        for (int i = 0; i < h->n; ++i) h->active[i] = mask[i] ? 1 : 0;
        update_slots(h);
        // a member that does not step keeps its parameters in both buffers
        for (int i = 0; i < h->n; ++i)
            if (!h->active[i]) mirror_params(h, i, h->sM);
        HIPCHK(hipStreamSynchronize(h->sM));
        h->wt_dirty = true;
    });
}

int fqlpop_step(fqlpop_t* h, int n_steps) {
    return guard([&] {
        ARGCHK(h, "null handle");
        ARGCHK(n_steps >= 0, "n_steps must be >= 0");
        if (split_error_pending(h)) sync_all_streams(h);  // (no copy, no sync when clear)
        check_split_error(h, -1, true);  // a failed split launch stops training until restored
        if (h->ds[0].rows == 0) throw FqErr{FQLPOP_E_STATE, "no training dataset set (fqlpop_set_dataset)"};
        HIPCHK(hipSetDevice(h->device));
        for (int i = 0; i < n_steps; ++i) {
            if (h->probe) {
                const int set = (int)(h->probe_step & 1);
                if (h->probe_pending[set]) probe_consume(h, set);  // the step i-2 that used this set
                h->probe_set = set;
                h->probe_nb[set] = euler_blocks(h, h->nz);
                run(h, true, false, false);
                h->probe_set = -1;
                HIPCHK(hipEventRecord(h->probe_done[set], h->sM));
                h->probe_pending[set] = true;
                ++h->probe_step;
            } else {
                run(h, true, false, false);
            }
        }
    });
}

// stage the injected batch / noise of every active member on sM
static void stage_injected(fqlpop* h, const float* batch, const float* noise) {
    if (batch)
        HIPCHK(hipMemcpyAsync(h->inj_batch, batch, sizeof(float) * h->inj_bs * h->nz, hipMemcpyHostToDevice, h->sM));
    if (noise)
        HIPCHK(hipMemcpyAsync(h->inj_noise, noise, sizeof(float) * h->inj_ns * h->nz, hipMemcpyHostToDevice, h->sM));
}

int fqlpop_step_injected(fqlpop_t* h, const float* batch, const float* noise) {
    return guard([&] {
        ARGCHK(h && batch, "null argument");
        HIPCHK(hipSetDevice(h->device));
        if (split_error_pending(h)) sync_all_streams(h);
        check_split_error(h, -1, true);
        if (h->nz == 0) return;
        stage_injected(h, batch, noise);
        run(h, true, true, noise != nullptr);
        HIPCHK(hipStreamSynchronize(h->sM));  // host buffers are borrowed only for the call
    });
}

int fqlpop_total_loss(fqlpop_t* h, const float* batch, const float* noise) {
    return guard([&] {
        ARGCHK(h, "null handle");
        ARGCHK(batch != nullptr || noise == nullptr, "noise without batch is not supported");
        HIPCHK(hipSetDevice(h->device));
        if (h->nz == 0) return;
        if (!batch && h->ds[0].rows == 0 && h->ds[1].rows == 0) throw FqErr{FQLPOP_E_STATE, "no dataset set"};
        stage_injected(h, batch, noise);
        run(h, false, batch != nullptr, noise != nullptr);
        if (batch) HIPCHK(hipStreamSynchronize(h->sM));
    });
}

int fqlpop_read_info(fqlpop_t* h, int which, float* out) {
    return guard([&] {
        ARGCHK(h && out, "null argument");
        HIPCHK(hipSetDevice(h->device));
        HIPCHK(hipStreamSynchronize(h->sM));
        check_split_error(h);
        HIPCHK(hipMemcpy(out, which ? h->vinfo : h->info, sizeof(float) * FQLPOP_INFO_STRIDE * h->n,
                         hipMemcpyDeviceToHost));
    });
}

int fqlpop_sample_actions(fqlpop_t* h, int member, const float* obs, int64_t n, const float* noise, uint64_t seed,
                          float* out) {
    return guard([&] {
        check_member(h, member);
        ARGCHK(obs && out && n > 0, "bad argument");
        HIPCHK(hipSetDevice(h->device));
        HIPCHK(hipStreamSynchronize(h->sM));
        const int D = h->D, A = h->A, H = h->H, L = h->L, Kc = D + A;
        const long long M = (n + 63) / 64 * 64;
        // feature-major input [s; z] built on the host
        std::vector<float> x((size_t)Kc * M, 0.f);
        for (long long r = 0; r < n; ++r) {
            for (int k = 0; k < D; ++k) x[(size_t)k * M + r] = obs[r * D + k];
            for (int j = 0; j < A; j += 2) {
                float z0, z1;
                if (noise) {
                    z0 = noise[r * A + j];
                    z1 = (j + 1 < A) ? noise[r * A + j + 1] : 0.f;
                } else {
                    uint32_t c[4] = {(uint32_t)r, (uint32_t)(r >> 32), 0xAC7u, (uint32_t)j};
                    philox_host(c, (uint32_t)seed, (uint32_t)(seed >> 32));
                    const float u1 = ((c[0] >> 8) + 1u) * (1.0f / 16777216.0f);
                    const float u2 = (c[1] >> 8) * (1.0f / 16777216.0f);
                    const float rr = std::sqrt(-2.0f * std::log(u1));
                    z0 = rr * std::cos(6.283185307179586f * u2);
                    z1 = rr * std::sin(6.283185307179586f * u2);
                }
                x[(size_t)(D + j) * M + r] = z0;
                if (j + 1 < A) x[(size_t)(D + j + 1) * M + r] = z1;
            }
        }
        float *dx = nullptr, *dout = nullptr, *dg = nullptr;
        int* dslot = nullptr;
        HIPCHK(hipMalloc(&dx, sizeof(float) * x.size()));
        HIPCHK(hipMalloc(&dout, sizeof(float) * A * M));
        HIPCHK(hipMalloc(&dg, sizeof(float) * 2 * H * M));
        HIPCHK(hipMalloc(&dslot, sizeof(int)));
        HIPCHK(hipMemcpy(dx, x.data(), sizeof(float) * x.size(), hipMemcpyHostToDevice));
        HIPCHK(hipMemcpy(dslot, &member, sizeof(int), hipMemcpyHostToDevice));
        const NetLayout& N = h->os;
        float* buf[2] = {dg, dg + (long long)H * M};
        for (int l = 0; l < L; ++l) {
            GemmArgs g{};
            g.A = tref(h->params + N.off + N.W[l], h->P);
            g.B = l == 0 ? tref(dx, 0) : tref(buf[(l - 1) & 1], 0);
            g.C = tref(buf[l & 1], 0);
            g.bias = tref(h->params + N.off + N.b[l], h->P);
            g.M = H; g.N = (int)M; g.K = N.kdim(l);
            g.lda = H; g.ldb = (int)M; g.ldc = (int)M;
            g.ny = 1; g.nz = 1; g.slots = dslot;
            if (N.ln) {
                throw FqErr{FQLPOP_E_UNSUPPORTED, "sample_actions with actor_layer_norm is not supported"};
            }
            gemm(LAYOUT_FWD, EPI_BIAS_GELU, g, h->sM);
        }
        HeadArgs ha{};
        ha.h = tref(buf[(L - 1) & 1], 0);
        ha.W = tref(h->params + N.off + N.W[L], h->P);
        ha.b = tref(h->params + N.off + N.b[L], h->P);
        ha.H = H; ha.M = (int)M; ha.ld = (int)M; ha.nout = A; ha.B = h->B; ha.D = D; ha.steps_f = 1.f;
        ha.o0 = tref(dout, 0); ha.ld0 = (int)M;
        ha.ny = 1; ha.nz = 1; ha.slots = dslot;
        launch_head_fwd(HEAD_ACT, ha, h->sM);
        HIPCHK(hipGetLastError());
        std::vector<float> o((size_t)A * M);
        HIPCHK(hipStreamSynchronize(h->sM));
        HIPCHK(hipMemcpy(o.data(), dout, sizeof(float) * o.size(), hipMemcpyDeviceToHost));
        for (long long r = 0; r < n; ++r)
            for (int j = 0; j < A; ++j) out[r * A + j] = o[(size_t)j * M + r];
        (void)hipFree(dx); (void)hipFree(dout); (void)hipFree(dg); (void)hipFree(dslot);
    });
}

int fqlpop_state_size(fqlpop_t* h, int64_t* n_floats) {
    return guard([&] {
        ARGCHK(h && n_floats, "null argument");
        *n_floats = h->state_size;
    });
}

static void state_copy(fqlpop* h, int member, int which, float* flat, const float* in, bool get) {
    ARGCHK(which >= 0 && which <= 2, "which must be FQLPOP_STATE_PARAMS/ADAM_M/ADAM_V");
    float* arena = which == 0 ? h->params : which == 1 ? h->adam_m : h->adam_v;
    std::vector<float> blk((size_t)h->P), tblk((size_t)h->PT, 0.f);
    HIPCHK(hipSetDevice(h->device));
    HIPCHK(hipDeviceSynchronize());
    // never export (checkpoint, member copy) state a failed launch wrote; a write restores it
    if (get) check_split_error(h, member);
    else (void)absorb_split_error(h);
    HIPCHK(hipMemcpy(blk.data(), arena + (long long)member * h->P, sizeof(float) * h->P, hipMemcpyDeviceToHost));
    if (which == 0)
        HIPCHK(hipMemcpy(tblk.data(), h->target + (long long)member * h->PT, sizeof(float) * h->PT,
                         hipMemcpyDeviceToHost));
    for (const Leaf& lf : h->leaves) {
        const NetLayout& N = lf.net == 2 ? h->bc : lf.net == 3 ? h->os : h->critic;
        const bool is_target = lf.net == 1;
        float* src = is_target ? tblk.data() : blk.data() + N.off;
        const long long per = leaf_member_size(N, lf.kind, lf.layer);
        for (int e = 0; e < N.E; ++e) {
            float* p = src + e * N.ens_size + leaf_internal_off(N, lf.kind, lf.layer);
            const long long fo = lf.flat_off + e * per;
            if (get) {
                if (is_target && which != 0) std::fill(flat + fo, flat + fo + per, 0.f);
                else std::memcpy(flat + fo, p, sizeof(float) * per);
            } else {
                std::memcpy(p, in + fo, sizeof(float) * per);
            }
        }
    }
    if (!get) {
        if (which == 0) h->wt_dirty = true;
        HIPCHK(hipMemcpy(arena + (long long)member * h->P, blk.data(), sizeof(float) * h->P, hipMemcpyHostToDevice));
        if (which == 0) {
            HIPCHK(hipMemcpy(h->target + (long long)member * h->PT, tblk.data(), sizeof(float) * h->PT,
                             hipMemcpyHostToDevice));
            mirror_params(h, member, h->sM);
            HIPCHK(hipStreamSynchronize(h->sM));
        }
        note_restored(h, member, which);
    }
}

int fqlpop_get_state(fqlpop_t* h, int member, int which, float* flat, int64_t n) {
    return guard([&] {
        check_member(h, member);
        ARGCHK(flat && n == h->state_size, "flat buffer size mismatch");
        state_copy(h, member, which, flat, nullptr, true);
    });
}

int fqlpop_set_state(fqlpop_t* h, int member, int which, const float* flat, int64_t n) {
    return guard([&] {
        check_member(h, member);
        ARGCHK(flat && n == h->state_size, "flat buffer size mismatch");
        state_copy(h, member, which, nullptr, flat, false);
    });
}

int fqlpop_get_count(fqlpop_t* h, int member, int32_t* count) {
    return guard([&] {
        check_member(h, member);
        ARGCHK(count, "null argument");
        HIPCHK(hipSetDevice(h->device));
        HIPCHK(hipDeviceSynchronize());
        check_split_error(h, member);
        HIPCHK(hipMemcpy(count, h->count + member, sizeof(int), hipMemcpyDeviceToHost));
    });
}

int fqlpop_set_count(fqlpop_t* h, int member, int32_t count) {
    return guard([&] {
        check_member(h, member);
        ARGCHK(count >= 0, "count must be >= 0");
        HIPCHK(hipSetDevice(h->device));
        HIPCHK(hipDeviceSynchronize());
        HIPCHK(hipMemcpy(h->count + member, &count, sizeof(int), hipMemcpyHostToDevice));
    });
}

int fqlpop_set_member(fqlpop_t* h, int member, float alpha, uint64_t seed, int reinit) {
    return guard([&] {
        check_member(h, member);
        HIPCHK(hipSetDevice(h->device));
        HIPCHK(hipDeviceSynchronize());
        h->h_alpha[member] = alpha;
        h->h_seeds[member] = seed;
        HIPCHK(hipMemcpy(h->alpha + member, &alpha, sizeof(float), hipMemcpyHostToDevice));
        HIPCHK(hipMemcpy(h->seeds + member, &seed, sizeof(uint64_t), hipMemcpyHostToDevice));
        upload_skey(h, member);
        if (reinit) {
            (void)absorb_split_error(h);
            init_member(h, member, seed);
            h->poisoned[member] = 0;  // a fresh member: nothing a failed launch wrote is left
        }
    });
}

int fqlpop_num_leaves(fqlpop_t* h, int* n) {
    return guard([&] {
        ARGCHK(h && n, "null argument");
        *n = (int)h->leaves.size();
    });
}

int fqlpop_leaf_info(fqlpop_t* h, int i, char* name, int name_cap, int64_t* offset, int* ndim, int64_t* shape3) {
    return guard([&] {
        ARGCHK(h && name && offset && ndim && shape3 && name_cap > 0, "null argument");
        ARGCHK(i >= 0 && i < (int)h->leaves.size(), "leaf index out of range");
        const Leaf& lf = h->leaves[i];
        std::snprintf(name, name_cap, "%s", lf.name.c_str());
        *offset = lf.flat_off;
        *ndim = lf.ndim;
        for (int k = 0; k < 3; ++k) shape3[k] = k < lf.ndim ? lf.shape[k] : 0;
    });
}

int fqlpop_sync(fqlpop_t* h) {
    return guard([&] {
        ARGCHK(h, "null handle");
        HIPCHK(hipSetDevice(h->device));
        sync_all_streams(h);
        // reported once here; the members stay poisoned for step / get_state / get_count / read_info
        if (absorb_split_error(h)) throw FqErr{FQLPOP_E_STATE, kSplitFailMsg};
    });
}

int fqlpop_debug_fail_split(fqlpop_t* h) {
    return guard([&] {
        ARGCHK(h, "null handle");
        HIPCHK(hipSetDevice(h->device));
        if (!h->split_err_host) throw FqErr{FQLPOP_E_STATE, "this population runs no split launch"};
        sync_all_streams(h);
        __atomic_store_n(h->split_err_host, 1u, __ATOMIC_RELEASE);
    });
}

int fqlpop_time_dominant_kernel(fqlpop_t* h, int iters, double* avg_us, double* flops) {
    return guard([&] {
        ARGCHK(h && avg_us && flops && iters > 0, "bad argument");
        HIPCHK(hipSetDevice(h->device));
        HIPCHK(hipDeviceSynchronize());
        const NetLayout& N = h->bc;
        const int B = h->B, H = h->H;
        // the dominant launch, replayed alone on sF with the buffers of the last step:
        // the persistent Euler flow (reads eu_in, writes aflow: idempotent), or
        // Euler hidden layer 1: eu_g[1] = gelu(W1^T eu_g[0] + b1)
        EulerArgs ea = euler_args(h, h->nz);
        GemmArgs g{};
        g.A = pref(h, h->params, N, N.W[1]);
        g.B = tref(h->eu_g[0], (long long)H * B);
        g.C = tref(h->eu_g[1], (long long)H * B);
        g.bias = pref(h, h->params, N, N.b[1]);
        g.M = H; g.N = B; g.K = H; g.lda = H; g.ldb = B; g.ldc = B;
        g.ny = 1; g.nz = h->nz; g.slots = h->slots;
        auto launch = [&](unsigned long long* probe) {
            if (h->euler_fused) {
                ea.probe = probe;
                launch_euler(h, ea, h->sF);
            } else {
                g.probe = probe;
                launch_gemm_euler_hidden(g, h->sF);
            }
        };
        launch(nullptr);  // warm-up
        HIPCHK(hipEventRecord(h->ev_t0, h->sF));
        for (int i = 0; i < iters; ++i) launch(nullptr);
        HIPCHK(hipEventRecord(h->ev_t1, h->sF));
        HIPCHK(hipEventSynchronize(h->ev_t1));
        float ms = 0.f;
        HIPCHK(hipEventElapsedTime(&ms, h->ev_t0, h->ev_t1));
        *avg_us = 1000.0 * ms / iters;
        *flops = dominant_flops(h);
        // clock cross-check of the in-kernel stamps: the same launch timed by
        // HIP events and by its blocks' s_memrealtime stamps (slot set 0)
        HIPCHK(hipMemsetAsync(h->probe_slots, 0, sizeof(unsigned long long) * 2 * h->probe_blocks, h->sF));
        HIPCHK(hipEventRecord(h->ev_t0, h->sF));
        launch(h->probe_slots);
        HIPCHK(hipEventRecord(h->ev_t1, h->sF));
        HIPCHK(hipEventSynchronize(h->ev_t1));
        HIPCHK(hipEventElapsedTime(&ms, h->ev_t0, h->ev_t1));
        std::vector<unsigned long long> v(2 * h->probe_blocks);
        std::memcpy(v.data(), h->probe_host, sizeof(unsigned long long) * v.size());
        h->clock_check_event_us = 1000.0 * ms;
        h->clock_check_stamp_us = probe_launch_us(v.data(), h->euler_fused ? euler_blocks(h, h->nz) : h->probe_blocks);
    });
}

int fqlpop_dominant_kernel_info(fqlpop_t* h, char* name, int name_cap, double* flops, double* bytes) {
    return guard([&] {
        ARGCHK(h && name && name_cap > 0 && flops && bytes, "null argument");
        const double B = h->B, H = h->H, K0 = h->D + h->A + 1, A = h->A, L = h->L, nz = h->nz;
        std::string nm;
        if (h->euler_fused) {
            const int F = euler_split(h, h->nz);
            nm = F > 1 ? "split_fwd_kernel<HEAD_EULER> F=" + std::to_string(F) : "euler_flow_kernel";
            // unique bytes: the bc net's Dense kernels + biases, the state in, a_flow out
            *bytes = 4.0 * nz * (K0 * H + (L - 1) * H * H + H * A + L * H + A + K0 * B + A * B);
        } else {
            nm = "gemm_fwd_dma_kernel<64, 64, 4, 3, 1>";
            *bytes = 4.0 * nz * (H * H + H * B + H + H * B);
        }
        *flops = dominant_flops(h);
        std::snprintf(name, name_cap, "%s", nm.c_str());
    });
}

int fqlpop_set_probe(fqlpop_t* h, int enable) {
    return guard([&] {
        ARGCHK(h, "null handle");
        HIPCHK(hipSetDevice(h->device));
        for (int st = 0; st < 2; ++st)
            if (h->probe_pending[st]) probe_consume(h, st);
        h->probe = enable != 0;
        h->probe_total_ms = 0.0;
        h->probe_launches = 0;
        h->probe_blocks_seen = h->probe_blocks_expected = 0;
    });
}

int fqlpop_probe_coverage(fqlpop_t* h, int64_t* blocks_seen, int64_t* blocks_expected) {
    return guard([&] {
        ARGCHK(h && blocks_seen && blocks_expected, "null argument");
        HIPCHK(hipSetDevice(h->device));
        for (int st = 0; st < 2; ++st)
            if (h->probe_pending[st]) probe_consume(h, st);
        *blocks_seen = h->probe_blocks_seen;
        *blocks_expected = h->probe_blocks_expected;
    });
}

int fqlpop_read_probe(fqlpop_t* h, double* total_us, int64_t* launches, double* clock_check) {
    return guard([&] {
        ARGCHK(h && total_us && launches, "null argument");
        HIPCHK(hipSetDevice(h->device));
        for (int st = 0; st < 2; ++st)
            if (h->probe_pending[st]) probe_consume(h, st);
        *total_us = 1000.0 * h->probe_total_ms;
        *launches = h->probe_launches;
        if (clock_check) {
            clock_check[0] = h->clock_check_event_us;
            clock_check[1] = h->clock_check_stamp_us;
        }
    });
}

}  // extern "C"

// ------------------------------------------------------------ env model
namespace {
// Offsets of the flax-ordered env-model leaves; returns the float count.
// dims: in, hidden..., out.  ln: BaselineStatePredictor (LayerNorm_0 after the Dense leaves).
long long envmodel_layout(const std::vector<int>& dims, bool ln, long long* w, long long* b, long long* ln_bias,
                          long long* ln_scale) {
    long long o = 0;
    for (size_t i = 0; i + 1 < dims.size(); ++i) {
        b[i] = o; o += dims[i + 1];                          // Dense_i/bias
        w[i] = o; o += (long long)dims[i] * dims[i + 1];     // Dense_i/kernel
    }
    if (ln) {
        *ln_bias = o; o += dims[0];                          // LayerNorm_0/bias
        *ln_scale = o; o += dims[0];                         // LayerNorm_0/scale
    }
    return o;
}

void envmodel_dims(const fqlpop_envmodel_config* c, std::vector<int>& sp, std::vector<int>& tp) {
    ARGCHK(c->obs_dim > 0 && c->action_dim > 0, "bad env-model dims");
    ARGCHK(c->sp_num_hidden >= 0 && c->sp_num_hidden < RO_MAX_LAYERS && c->tp_num_hidden >= 0 &&
               c->tp_num_hidden < RO_MAX_LAYERS, "too many env-model layers");
    sp = {c->obs_dim + c->action_dim};
    for (int i = 0; i < c->sp_num_hidden; ++i) sp.push_back(c->sp_hidden[i]);
    sp.push_back(c->obs_dim);
    tp = {c->obs_dim};
    for (int i = 0; i < c->tp_num_hidden; ++i) tp.push_back(c->tp_hidden[i]);
    tp.push_back(1);
    for (int d : sp) ARGCHK(d > 0 && d <= RO_MAX_W, "env-model layer width must be in 1..512");
    for (int d : tp) ARGCHK(d > 0 && d <= RO_MAX_W, "env-model layer width must be in 1..512");
}
}  // namespace

int fqlpop_envmodel_param_count(const fqlpop_envmodel_config* cfg, int64_t* n_sp, int64_t* n_tp) {
    return guard([&] {
        ARGCHK(cfg && n_sp && n_tp, "null argument");
        std::vector<int> sp, tp;
        envmodel_dims(cfg, sp, tp);
        long long w[RO_MAX_LAYERS], b[RO_MAX_LAYERS], lb = 0, ls = 0;
        *n_sp = envmodel_layout(sp, true, w, b, &lb, &ls);
        *n_tp = envmodel_layout(tp, false, w, b, &lb, &ls);
    });
}

int fqlpop_set_env_model(fqlpop_t* h, const fqlpop_envmodel_config* cfg, const float* sp_params, int64_t n_sp,
                         const float* tp_params, int64_t n_tp) {
    return guard([&] {
        ARGCHK(h && cfg && sp_params && tp_params, "null argument");
        ARGCHK(cfg->obs_dim == h->D && cfg->action_dim == h->A, "env-model obs/action dims differ from the agent's");
        std::vector<int> sp, tp;
        envmodel_dims(cfg, sp, tp);
        RolloutArgs& r = h->em_args;
        r = RolloutArgs{};
        const long long nsp = envmodel_layout(sp, true, r.sp_w, r.sp_b, &r.sp_ln_bias, &r.sp_ln_scale);
        long long lb = 0, ls = 0;
        const long long ntp = envmodel_layout(tp, false, r.tp_w, r.tp_b, &lb, &ls);
        ARGCHK(n_sp == nsp && n_tp == ntp, "env-model parameter count mismatch (fqlpop_envmodel_param_count)");
        r.sp_n = (int)sp.size() - 1;
        r.tp_n = (int)tp.size() - 1;
        for (size_t i = 0; i < sp.size(); ++i) r.sp_dims[i] = sp[i];
        for (size_t i = 0; i < tp.size(); ++i) r.tp_dims[i] = tp[i];
        HIPCHK(hipSetDevice(h->device));
        HIPCHK(hipDeviceSynchronize());
        if (h->sp_params) (void)hipFree(h->sp_params);
        if (h->tp_params) (void)hipFree(h->tp_params);
        h->sp_params = h->tp_params = nullptr;
        HIPCHK(hipMalloc(&h->sp_params, sizeof(float) * nsp));
        HIPCHK(hipMalloc(&h->tp_params, sizeof(float) * ntp));
        HIPCHK(hipMemcpy(h->sp_params, sp_params, sizeof(float) * nsp, hipMemcpyHostToDevice));
        HIPCHK(hipMemcpy(h->tp_params, tp_params, sizeof(float) * ntp, hipMemcpyHostToDevice));
        h->em = *cfg;
        h->em_set = true;
    });
}

int fqlpop_rollout(fqlpop_t* h, const float* init_obs, int n_envs, int max_steps, uint64_t seed, const float* noise,
                   float* out, float* out_obs) {
    return guard([&] {
        ARGCHK(h && init_obs && out, "null argument");
        ARGCHK(n_envs > 0 && max_steps > 0, "n_envs and max_steps must be positive");
        if (!h->em_set) throw FqErr{FQLPOP_E_STATE, "no env model set (fqlpop_set_env_model)"};
        if (!rollout_supported(h->H, h->L, h->D, h->A))
            throw FqErr{FQLPOP_E_UNSUPPORTED, "rollout needs hidden_dim 512, obs_dim + action_dim <= 64"};
        if (h->os.ln) throw FqErr{FQLPOP_E_UNSUPPORTED, "rollout with actor_layer_norm is not supported"};
        HIPCHK(hipSetDevice(h->device));
        HIPCHK(hipStreamSynchronize(h->sM));
        const int nz = h->nz, D = h->D, A = h->A;
        if (nz == 0) return;
        RolloutArgs r = h->em_args;
        r.params = h->params; r.P = h->P; r.os_off = h->os.off;
        for (int l = 0; l <= h->L; ++l) { r.w_off[l] = h->os.W[l]; r.b_off[l] = h->os.b[l]; }
        r.D = D; r.A = A; r.L = h->L;
        r.sp = h->sp_params; r.tp = h->tp_params;
        r.n_envs = n_envs; r.max_steps = max_steps; r.seed = seed; r.member_seeds = h->skeys;
        r.nz = nz; r.slots = h->slots;
        float *d_obs = nullptr, *d_noise = nullptr, *d_out = nullptr, *d_oobs = nullptr;
        const size_t n_noise = (size_t)nz * max_steps * n_envs * A;
        HIPCHK(hipMalloc(&d_obs, sizeof(float) * n_envs * D));
        HIPCHK(hipMalloc(&d_out, sizeof(float) * nz * n_envs * 2));
        HIPCHK(hipMemcpy(d_obs, init_obs, sizeof(float) * n_envs * D, hipMemcpyHostToDevice));
        if (noise) {
            HIPCHK(hipMalloc(&d_noise, sizeof(float) * n_noise));
            HIPCHK(hipMemcpy(d_noise, noise, sizeof(float) * n_noise, hipMemcpyHostToDevice));
        }
        if (out_obs) HIPCHK(hipMalloc(&d_oobs, sizeof(float) * nz * n_envs * D));
        r.init_obs = d_obs; r.noise = d_noise; r.out = d_out; r.out_obs = d_oobs;
        launch_rollout(r, h->sM);
        HIPCHK(hipGetLastError());
        HIPCHK(hipStreamSynchronize(h->sM));
        HIPCHK(hipMemcpy(out, d_out, sizeof(float) * nz * n_envs * 2, hipMemcpyDeviceToHost));
        if (out_obs) HIPCHK(hipMemcpy(out_obs, d_oobs, sizeof(float) * nz * n_envs * D, hipMemcpyDeviceToHost));
        for (float* p : {d_obs, d_noise, d_out, d_oobs})
            if (p) (void)hipFree(p);
    });
}

int fqlpop_envmodel_step(fqlpop_t* h, const float* obs, const float* actions, int n, float* next_obs, float* logits) {
    return guard([&] {
        ARGCHK(h && obs && actions && next_obs && logits && n > 0, "bad argument");
        if (!h->em_set) throw FqErr{FQLPOP_E_STATE, "no env model set (fqlpop_set_env_model)"};
        ARGCHK(h->D + h->A <= 64 && h->D <= 64 && h->A <= 8, "obs_dim + action_dim must be <= 64");
        HIPCHK(hipSetDevice(h->device));
        HIPCHK(hipStreamSynchronize(h->sM));
        const int D = h->D, A = h->A;
        RolloutArgs r = h->em_args;
        r.params = h->params; r.P = h->P; r.os_off = h->os.off;
        r.D = D; r.A = A; r.L = h->L;
        r.sp = h->sp_params; r.tp = h->tp_params;
        r.n_envs = n; r.max_steps = 1; r.seed = 0; r.member_seeds = h->skeys;
        r.nz = 1; r.slots = h->slots;  // any slot: the actor is not run
        float *d_obs = nullptr, *d_act = nullptr, *d_out = nullptr, *d_oobs = nullptr, *d_logit = nullptr;
        HIPCHK(hipMalloc(&d_obs, sizeof(float) * n * D));
        HIPCHK(hipMalloc(&d_act, sizeof(float) * n * A));
        HIPCHK(hipMalloc(&d_out, sizeof(float) * n * 2));
        HIPCHK(hipMalloc(&d_oobs, sizeof(float) * n * D));
        HIPCHK(hipMalloc(&d_logit, sizeof(float) * n));
        HIPCHK(hipMemcpy(d_obs, obs, sizeof(float) * n * D, hipMemcpyHostToDevice));
        HIPCHK(hipMemcpy(d_act, actions, sizeof(float) * n * A, hipMemcpyHostToDevice));
        r.init_obs = d_obs; r.actions = d_act; r.out = d_out; r.out_obs = d_oobs; r.out_logit = d_logit;
        launch_rollout(r, h->sM);
        HIPCHK(hipGetLastError());
        HIPCHK(hipStreamSynchronize(h->sM));
        HIPCHK(hipMemcpy(next_obs, d_oobs, sizeof(float) * n * D, hipMemcpyDeviceToHost));
        HIPCHK(hipMemcpy(logits, d_logit, sizeof(float) * n, hipMemcpyDeviceToHost));
        for (float* p : {d_obs, d_act, d_out, d_oobs, d_logit}) (void)hipFree(p);
    });
}
