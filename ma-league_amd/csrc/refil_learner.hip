// refil_learner.hip -- REFILLearner.train (src/marl/learners/refil_learner.py:102-218) as one device pipeline.
//
//   pack        online/target agent + 4 hypernets -> kernel layouts; transposes for the backward
//   mask_sum    mask = filled[:, :-1] * (1 - terminated shifted) and its sum              (:106-108, :197-201)
//   ein         entity inputs [entities | last-action one-hot of agent entities] per (b, t)  (_build_inputs,
//               entity_controller.py:11-30, _get_mixer_ins :81-100)
//   ent_fwd     per item pair: fc1 -> in_trans -> attention for the three agent copies (plain, within,
//               interact; entity_rnn_agent.py:88-126) -> out_trans -> fc2 -> W_ih x; target net: plain copy only
//   rec         GRU recurrence over t for all online (3 copies) and target rows, gates saved
//   q           fc3 for every (t, row), masked agents -> 0 (entity_rnn_agent.py:58-61)
//   hyper_fwd   per (item, hypernet, net): AttentionHyperNet forward (flex_qmix.py:20-53); hyper_w_1 online with
//               the plain / W / I attention masks (imagine groups)
//   mix_td      per item: chosen Q gather, double-Q target (refil_learner.py:147-164), FlexQMixer mixing of the
//               plain and the imagined Q (:166-190, flex_qmix.py:73-117), targets, TD, the lambda-mixed loss
//               (:193-208), and the mixing backward -> dX of every hypernet output and dQ of every agent copy
//   hyper_bwd   per (item, hypernet): fc2 / out_trans / attention / in_trans / fc1 backward (deltas for wgrad)
//   rec_bwd     reverse-time GRU backward of the online rows
//   ent_bwd     per item pair: W_ih^T, fc2, out_trans, attention (3 copies, accumulated), in_trans, fc1 backward
//   wgrad       23 weight-gradient jobs (wgrad_device.h), deterministic
//   finish      clip_grad_norm_ (10), RMSprop, stats (:211-231)
// Agent rows: r = (c * B + b) * NA + n for copy c (0 plain, 1 within, 2 interact); target rows r = b * NA + n.
// Items i = b * T + t. Mixer items use t < T - 1 (the other kernels write zeros for t = T - 1).
#include "mlg_host.h"
#include "batch_mask_device.h"
#include "gru4_device.h"
#include "refil_device.h"
#include "wgrad_device.h"

using namespace refil;

namespace {

constexpr int MJ = 24;
using RJobs = mlg::BJobsT<MJ>;

struct RCfg {
    int B, T, T1, NA, NE, ED, D0, K1, A, Ap, I, Ron, Rtg;
    int double_q, softmax;
    float gamma, lmbda;
};

constexpr int REFIL_HYPER_JOBS = 16;  // weight-gradient jobs of the 4 hypernets (make_jobs)
constexpr int64_t REFIL_HSP = 12 * 2 * 3 * 64 * 4;  // split hypernet in_trans (hyper_split_kernel)
struct WsR {
    int64_t pa_on, pa_tg, ph_on[4], ph_tg[4];
    int64_t a_winT, a_woutT, a_w2T, a_wihT, h_winT[4], h_woutT[4], h_w2T[4];
    int64_t h_wsp[10], h_wspT[5];  // + in_trans^T split for hyper_bwd (hypernet k) / ent_bwd (agent: [4])  // in_trans as split-bf16 A operands: hypernet k of net at [k + 4 net], agent net at [8 + net]
    int64_t ein, x1, qkv, P, o, x2, x3, gi_on, gi_tg, hs_on, hs_tg, gr, gz, gn, ghn, mac, tmac;
    int64_t x1m[4], qkvm[4], Pm[4], om[4], x2m[4], X[4], Xtg[4], dX[4], doutm[4], dqkvm[4], dfc1m[4];
    int64_t dq, d2, part, msum, dgi, dgh, dfc2, dout, dqkv, dfc1, rows;
    int64_t slab, nrm, total;
};

struct Plan {
    RCfg c;
    RAgent La;
    RHyper Lh;
    WsR w;
    int64_t n_agent, n_mixer;
};

__host__ __device__ inline int nvar(int k) { return k == 0 ? 3 : 1; }

int check_cfg(const MlgRefilLearnerCfg* c) {
    MLG_REQUIRE(c != nullptr, "null refil learner cfg");
    MLG_REQUIRE(c->B >= 1 && c->T >= 2, "refil learner: B=%d T=%d", c->B, c->T);
    MLG_REQUIRE(c->n_agents >= 1 && c->n_agents <= NAS && c->n_entities >= c->n_agents && c->n_entities <= NE,
                "refil learner: n_agents=%d n_entities=%d unsupported (<= 8, <= 16)", c->n_agents, c->n_entities);
    MLG_REQUIRE(c->attn_embed_dim == EMB && c->rnn_hidden_dim == EMB && c->hypernet_embed == EMB && c->attn_n_heads == NH &&
                    c->mixing_embed_dim == EM,
                "refil learner: attn_embed_dim/rnn_hidden_dim/hypernet_embed 64, 4 heads, mixing_embed_dim 32 supported");
    const int D0 = c->entity_shape + (c->entity_last_action ? c->n_actions : 0);
    MLG_REQUIRE(D0 <= KMAX && c->n_actions >= 1 && c->n_actions <= 32, "refil learner: entity input %d / actions %d",
                D0, c->n_actions);
    MLG_REQUIRE(c->imagine == 1, "refil learner: the imagine agent (REFIL) is the built path");
    // the recurrences store hs / gates / dGI / dGH through buffer resources (32-bit byte offsets): the largest of
    // them, (T + 1) x 3B*NA rows x 3*EMB floats, must stay under 2 GiB or its stores would be silently dropped
    MLG_REQUIRE((int64_t)(c->T + 1) * 3 * c->B * c->n_agents * 3 * EMB < (int64_t)1 << 29,
                "refil learner: (T+1)*3B*NA*3*EMB=%lld floats exceeds the 2 GB buffer-store range",
                (long long)(c->T + 1) * 3 * c->B * c->n_agents * 3 * EMB);
    return 0;
}

Plan make_plan(const MlgRefilLearnerCfg* cfg, int T1) {
    Plan p;
    RCfg& c = p.c;
    c.B = cfg->B;
    c.T = cfg->T;
    c.T1 = T1;
    c.NA = cfg->n_agents;
    c.NE = cfg->n_entities;
    c.ED = cfg->entity_shape;
    c.A = cfg->n_actions;
    c.D0 = cfg->entity_shape + (cfg->entity_last_action ? cfg->n_actions : 0);
    c.K1 = (c.D0 + 15) / 16 * 16;
    c.Ap = (c.A + 15) / 16 * 16;
    c.I = c.B * c.T;
    c.Ron = 3 * c.B * c.NA;
    c.Rtg = c.B * c.NA;
    c.double_q = cfg->double_q;
    c.softmax = cfg->softmax_mixing_weights;
    c.gamma = cfg->gamma;
    c.lmbda = cfg->lmbda;
    p.La = make_ragent(c.D0, c.A);
    p.Lh = make_rhyper(c.D0);
    p.n_agent = p.La.c_total;
    p.n_mixer = 4 * p.Lh.c_total;
    WsR& w = p.w;
    int64_t o = 0;
    auto take = [&](int64_t n) { int64_t r = o; o += mlg_align4(n); return r; };
    const int64_t I = c.I, T = c.T, Ron = c.Ron, Rtg = c.Rtg;
    w.pa_on = take(p.La.total);
    w.pa_tg = take(p.La.total);
    for (int k = 0; k < 4; ++k) w.ph_on[k] = take(p.Lh.total);
    for (int k = 0; k < 4; ++k) w.ph_tg[k] = take(p.Lh.total);
    w.a_winT = take(EMB * 3 * EMB);
    w.a_woutT = take(EMB * EMB);
    w.a_w2T = take(EMB * EMB);
    w.a_wihT = take(EMB * 3 * EMB);
    for (int k = 0; k < 4; ++k) {
        w.h_winT[k] = take(EMB * 3 * EMB);
        w.h_woutT[k] = take(EMB * EMB);
        w.h_w2T[k] = take(EMB * EM);
    }
    for (int k = 0; k < 10; ++k) w.h_wsp[k] = take(REFIL_HSP);
    for (int k = 0; k < 5; ++k) w.h_wspT[k] = take(REFIL_HSP);
    w.ein = take(I * NE * c.K1);
    w.x1 = take(I * NE * EMB);
    w.qkv = take(I * NE * 3 * EMB);
    w.P = take(3 * I * 1024);
    w.o = take(T * Ron * EMB);
    w.x2 = take(T * Ron * EMB);
    w.x3 = take(T * Ron * EMB);
    w.gi_on = take(T * Ron * 3 * EMB);
    w.gi_tg = take(T * Rtg * 3 * EMB);
    w.hs_on = take((T + 1) * Ron * EMB);
    w.hs_tg = take((T + 1) * Rtg * EMB);
    w.gr = take(T * Ron * EMB);
    w.gz = take(T * Ron * EMB);
    w.gn = take(T * Ron * EMB);
    w.ghn = take(T * Ron * EMB);
    w.mac = take(T * Ron * c.A);
    w.tmac = take(T * Rtg * c.A);
    for (int k = 0; k < 4; ++k) {
        const int V = nvar(k);
        w.x1m[k] = take(I * NE * EMB);
        w.qkvm[k] = take(I * NE * 3 * EMB);
        w.Pm[k] = take((int64_t)V * I * 1024);
        w.om[k] = take((int64_t)V * I * NAS * EMB);
        w.x2m[k] = take((int64_t)V * I * NAS * EMB);
        w.X[k] = take((int64_t)V * I * NAS * EM);
        w.Xtg[k] = take(I * NAS * EM);
        w.dX[k] = take((int64_t)V * I * NAS * EM);
        w.doutm[k] = take((int64_t)V * I * NAS * EMB);
        w.dqkvm[k] = take(I * NE * 3 * EMB);
        w.dfc1m[k] = take(I * NE * EMB);
    }
    w.dq = take(T * Ron);
    w.d2 = take(T * Ron * c.A);
    w.part = take(I * 8);
    w.msum = take(4 + c.B);  // [mask sum, max_t_filled, -, -, live mixer items of episode b ...]
    w.dgi = take(T * Ron * 3 * EMB);
    w.dgh = take(T * Ron * 3 * EMB);
    w.dfc2 = take(T * Ron * EMB);
    w.dout = take(T * Ron * EMB);
    w.dqkv = take(I * NE * 3 * EMB);
    w.dfc1 = take(I * NE * EMB);
    w.rows = take(MLG_INLINE_ROWS);  // int32 slot map (host_rows)
    w.slab = o;
    w.nrm = 0;
    w.total = o;
    return p;
}

// The refil_8 shape (8 agent slots, 16 entities, entity width 8 + the 21-action last-action one-hot, 21 actions) as
// a static instantiation of the per-item kernels (S8 = 1): their dims and the packed-block offsets become
// immediates (loops over agents / entities unrolled, no kernel-argument SGPRs held across them). Other shapes run
// S8 = 0 with the same code.
struct S8Dims {
    static constexpr int NA = 8, NE = 16, ED = 8, A = 21, D0 = 29, K1 = 32, Ap = 32;
};
template <int S8>
__device__ __forceinline__ RCfg static_cfg(RCfg c) {
    if constexpr (S8 != 0) {
        c.NA = S8Dims::NA;
        c.NE = S8Dims::NE;
        c.ED = S8Dims::ED;
        c.A = S8Dims::A;
        c.D0 = S8Dims::D0;
        c.K1 = S8Dims::K1;
        c.Ap = S8Dims::Ap;
    }
    return c;
}
inline bool is_s8(const RCfg& c) {
    return c.NA == S8Dims::NA && c.NE == S8Dims::NE && c.ED == S8Dims::ED && c.A == S8Dims::A && c.D0 == S8Dims::D0 &&
           getenv("MLG_REFIL_GENERIC") == nullptr;
}

// ---- small kernels ---------------------------------------------------------------------------------------
struct CopyJob {
    int64_t src, src2, dst;
    int rows_dst, cols_dst, rows_src, cols_src;
};
struct CopyJobs {
    static constexpr int kCap = 16;
    CopyJob j[kCap];
    int n;
    int64_t total;
    bool overflow;
};

// One launch packs several parameter blocks with the same layout: blockIdx.y selects the (src, dst) pair.
struct CopyPairs {
    static constexpr int kCap = 8;  // agent: online + target; hypernets: 4 x (online + target)
    const float* src[kCap];
    float* dst[kCap];
};
__device__ void copy_jobs_body(const CopyJobs& J, const CopyPairs& pp, int bx, int by) {
    const float* __restrict__ src = pp.src[by];
    float* __restrict__ dst = pp.dst[by];
    const int64_t i = (int64_t)bx * blockDim.x + threadIdx.x;
    if (i >= J.total) return;
    float v = 0.f;
    for (int q = 0; q < J.n; ++q) {
        const CopyJob& c = J.j[q];
        const int64_t n = (int64_t)c.rows_dst * c.cols_dst;
        if (i >= c.dst && i < c.dst + n) {
            const int64_t l = i - c.dst;
            const int r = (int)(l / c.cols_dst), col = (int)(l % c.cols_dst);
            if (r < c.rows_src && col < c.cols_src) {
                v = src[c.src + (int64_t)r * c.cols_src + col];
                if (c.src2 >= 0) v += src[c.src2 + (int64_t)r * c.cols_src + col];
            }
            break;
        }
    }
    dst[i] = v;
}

CopyJob cj(int64_t src, int64_t dst, int rd, int cd, int rs, int cs, int64_t src2 = -1) {
    return CopyJob{src, src2, dst, rd, cd, rs, cs};
}
// bounded append: a table filled past its capacity is reported by run_train instead of overrunning
void push(CopyJobs& J, const CopyJob& c) {
    if (J.n < CopyJobs::kCap) J.j[J.n++] = c;
    else J.overflow = true;
}

CopyJobs agent_jobs(const RAgent& L) {
    CopyJobs J{};
    push(J, cj(L.c_w1, L.w1, EMB, L.K1, EMB, L.D0));
    push(J, cj(L.c_b1, L.b1, 1, EMB, 1, EMB));
    push(J, cj(L.c_win, L.win, 3 * EMB, EMB, 3 * EMB, EMB));
    push(J, cj(L.c_wout, L.wout, EMB, EMB, EMB, EMB));
    push(J, cj(L.c_bout, L.bout, 1, EMB, 1, EMB));
    push(J, cj(L.c_w2, L.w2, EMB, EMB, EMB, EMB));
    push(J, cj(L.c_b2, L.b2, 1, EMB, 1, EMB));
    push(J, cj(L.c_wih, L.wih, 3 * EMB, EMB, 3 * EMB, EMB));
    push(J, cj(L.c_whh, L.whh, 3 * EMB, EMB, 3 * EMB, EMB));
    push(J, cj(L.c_bih, L.bih, 1, 3 * EMB, 1, 3 * EMB));
    push(J, cj(L.c_bhh, L.bhh, 1, 3 * EMB, 1, 3 * EMB));
    push(J, cj(L.c_bih, L.brz, 1, 2 * EMB, 1, 2 * EMB, L.c_bhh));
    push(J, cj(L.c_w3, L.w3, L.Ap, EMB, L.A, EMB));
    push(J, cj(L.c_b3, L.b3, 1, L.Ap, 1, L.A));
    J.total = L.gsp;  // the rollout's pre-split sections (gsp, wsp) are not read by the learner
    return J;
}

CopyJobs hyper_jobs(const RHyper& L) {
    CopyJobs J{};
    push(J, cj(L.c_w1, L.w1, EMB, L.K1, EMB, L.D0));
    push(J, cj(L.c_b1, L.b1, 1, EMB, 1, EMB));
    push(J, cj(L.c_win, L.win, 3 * EMB, EMB, 3 * EMB, EMB));
    push(J, cj(L.c_wout, L.wout, EMB, EMB, EMB, EMB));
    push(J, cj(L.c_bout, L.bout, 1, EMB, 1, EMB));
    push(J, cj(L.c_w2, L.w2, EM, EMB, EM, EMB));
    push(J, cj(L.c_b2, L.b2, 1, EM, 1, EM));
    J.total = L.total;
    return J;
}

// Hypernet in_trans [192][64] as split-bf16 MFMA A operands for hyper_fwd (the rollout's wsp tiles 0-11 layout:
// element ((reg * 64 + lane) * 4 + q), reg = (tile * 2 + kk) * 3 + piece), blockIdx.y = (hypernet, net) block.
struct HSplit {
    static constexpr int kCap = 10;  // 4 hypernets + the agent, online + target
    const float* src[kCap];
    float* dst[kCap];
};
__device__ void hyper_split_body(const HSplit& J, int bx, int by) {
    const int64_t k = (int64_t)bx * blockDim.x + threadIdx.x;
    if (k >= REFIL_HSP) return;
    const int q = (int)(k & 3), lane = (int)((k >> 2) & 63), reg = (int)(k >> 8);
    const int pc = reg % 3, kk = (reg / 3) % 2, mt = reg / 6;
    const int i0 = 2 * q, f0 = (2 * kk + i0 / 4) * 16 + 4 * (lane >> 4) + i0 % 4;
    const float* W = J.src[by] + (int64_t)(mt * 16 + (lane & 15)) * EMB;
    J.dst[by][k] = split_bf16_pair(W[f0], W[f0 + 1], pc);
}

// in_trans^T [64][192] (the dX1 = W_in^T dQKV operand of the backward kernels) as split-bf16 A operands, from the
// canonical in_trans [192][64]: element ((reg * 64 + lane) * 4 + q), reg = (tile * 6 + kk) * 3 + piece, tile < 4,
// kk < 6 (K = 192). blockIdx.y = block (src[y] canonical in_trans, dst[y]).
__device__ void hyper_splitT_body(const HSplit& J, int bx, int by) {
    const int64_t k = (int64_t)bx * blockDim.x + threadIdx.x;
    if (k >= REFIL_HSP) return;
    const int q = (int)(k & 3), lane = (int)((k >> 2) & 63), reg = (int)(k >> 8);
    const int pc = reg % 3, kk = (reg / 3) % 6, mt = reg / 18;
    const int i0 = 2 * q, f0 = (2 * kk + i0 / 4) * 16 + 4 * (lane >> 4) + i0 % 4;
    const int row = mt * 16 + (lane & 15);
    const float* W = J.src[by];
    J.dst[by][k] = split_bf16_pair(W[(int64_t)f0 * EMB + row], W[(int64_t)(f0 + 1) * EMB + row], pc);
}

// acc[mt] += in_trans^T . X over one 16-row tile (X = dQKV rows in LDS, K = 192) as split-bf16 fp32 emulation;
// replaces mm_lds<4>(acc, winT, 3 * EMB, 0, X, LDQ, 12, lane). Weights streamed per output tile (18 loads).
__device__ inline void in_transT_lds_b16(floatx4 (&acc)[4], const float* __restrict__ wspT, const float* X, int lane) {
    const int col = lane & 15, g = lane >> 4;
    Split3 xs[6];
#pragma unroll
    for (int kk = 0; kk < 6; ++kk)
        xs[kk] = split3(ld4(X + col * LDQ + 2 * kk * 16 + 4 * g), ld4(X + col * LDQ + (2 * kk + 1) * 16 + 4 * g));
    const u32x4* ws = reinterpret_cast<const u32x4*>(wspT) + lane;
    bf16x8 wb[2][18];
    auto load = [&](int mt, bf16x8 (&w)[18]) {
#pragma unroll
        for (int i = 0; i < 18; ++i) w[i] = __builtin_bit_cast(bf16x8, ws[(mt * 18 + i) * 64]);
    };
    load(0, wb[0]);
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) {
        if (mt + 1 < 4) load(mt + 1, wb[(mt + 1) & 1]);
        __builtin_amdgcn_sched_barrier(0);
        const bf16x8(&w)[18] = wb[mt & 1];
#pragma unroll
        for (int kk = 0; kk < 6; ++kk) {
            Split3 a;
            a.p[0] = w[kk * 3];
            a.p[1] = w[kk * 3 + 1];
            a.p[2] = w[kk * 3 + 2];
            acc[mt] = mfma_x6(a, xs[kk], acc[mt]);
        }
        __builtin_amdgcn_sched_barrier(0);
    }
}

// Y = in_trans(X) over one 16-row tile (X, Y in LDS) as split-bf16 fp32 emulation (six partial products; the
// rollout's entity_block_reg scheme): X rows split once per 32-wide K step in the wsp K order, weights streamed in
// 3-tile stages. Replaces dense_lds<false>(win, ...) -- 144 bf16 MFMAs instead of 192 f32 MFMAs.
__device__ inline void in_trans_lds_b16(const float* __restrict__ wsp, const float* X, float* Y, int ldy, int lane) {
    const int col = lane & 15, g = lane >> 4;
    Split3 xs[2];
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
        xs[kk] = split3(ld4(X + col * LDX + 2 * kk * 16 + 4 * g), ld4(X + col * LDX + (2 * kk + 1) * 16 + 4 * g));
    const u32x4* ws = reinterpret_cast<const u32x4*>(wsp) + lane;
    bf16x8 wb[2][18];
    auto load = [&](int stg, bf16x8 (&w)[18]) {
#pragma unroll
        for (int i = 0; i < 18; ++i) w[i] = __builtin_bit_cast(bf16x8, ws[(stg * 18 + i) * 64]);
    };
    load(0, wb[0]);
#pragma unroll
    for (int stg = 0; stg < 4; ++stg) {
        if (stg + 1 < 4) load(stg + 1, wb[(stg + 1) & 1]);
        __builtin_amdgcn_sched_barrier(0);
        const bf16x8(&w)[18] = wb[stg & 1];
#pragma unroll
        for (int ti = 0; ti < 3; ++ti) {
            floatx4 acc = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int kk = 0; kk < 2; ++kk) {
                Split3 a;
                a.p[0] = w[ti * 6 + kk * 3];
                a.p[1] = w[ti * 6 + kk * 3 + 1];
                a.p[2] = w[ti * 6 + kk * 3 + 2];
                acc = mfma_x6(a, xs[kk], acc);
            }
            st_row(Y, ldy, stg * 3 + ti, acc, lane);
        }
        __builtin_amdgcn_sched_barrier(0);
    }
}

// All the prologue's weight transposes in one launch: blockIdx.y = job.
struct TrJob {
    const float* src;
    float* dst;
    int rows, cols;
};
struct TrJobs {
    static constexpr int kCap = 16;
    TrJob j[kCap];
    int n;
};
__device__ void transpose_body(const TrJobs& J, int bx, int by) {
    const TrJob& t = J.j[by];
    const int64_t i = (int64_t)bx * blockDim.x + threadIdx.x;
    if (i >= (int64_t)t.rows * t.cols) return;
    const int r = (int)(i / t.cols), c = (int)(i % t.cols);
    t.dst[(int64_t)c * t.rows + r] = t.src[i];
}

__device__ __forceinline__ int64_t eslot(const MlgEntityBatch& bt, int b) {
    return bt.rows ? (int64_t)bt.rows[b] : (int64_t)b;
}

__device__ __forceinline__ float emask_at(const MlgEntityBatch& bt, int b, int t) {
    const int64_t base = eslot(bt, b) * bt.T1;
    float m = (float)bt.filled[base + t];
    if (t > 0) m *= 1.f - (float)bt.terminated[base + t - 1];
    return m;
}

__device__ void mask_sum_body(const MlgEntityBatch& bt, int B, int T, float* __restrict__ msum, float* red) {
    // msum[1] = max_t_filled (the reference's truncation, ma_experiment.py:235-239): the learner uses transitions
    // t < max_t_filled - 1 only; the sequential kernels stop there and the per-t kernels skip the steps beyond
    int mx = 0;  // a wave per episode: filled steps counted with ballots
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
    for (int b = wave; b < B; b += nw) {
        const int64_t base = eslot(bt, b) * bt.T1;
        int n = 0;
        for (int t0 = 0; t0 < T; t0 += 64) {
            const int t = t0 + lane;
            n += __popcll(__ballot(t < T && bt.filled[base + t] != 0));
        }
        mx = n > mx ? n : mx;
    }
    red[threadIdx.x] = (float)mx;
    __syncthreads();
    for (int w = blockDim.x / 2; w > 0; w >>= 1) {
        if (threadIdx.x < w) red[threadIdx.x] = fmaxf(red[threadIdx.x], red[threadIdx.x + w]);
        __syncthreads();
    }
    const int Te = (int)fminf(fmaxf(red[0], 2.f), (float)T);
    __syncthreads();
    float s = 0.f;
    for (int i = threadIdx.x; i < B * (Te - 1); i += blockDim.x) s += emask_at(bt, i / (Te - 1), i % (Te - 1));
    red[threadIdx.x] = s;
    __syncthreads();
    for (int w = blockDim.x / 2; w > 0; w >>= 1) {
        if (threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        msum[0] = red[0];
        msum[1] = (float)Te;
    }
    // msum[4 + b]: the episode's live mixer items = 1 + the last t < Te - 1 with mask(b, t) != 0 (0: none). Every item
    // t >= it has mask 0 (its loss, its deltas and every gradient through it are exactly zero), so the per-item kernels
    // skip items t >= mix_len (mixer, agent backward) and t > mix_len (agent forward: Q at mix_len is the last step's
    // target): at the bench's sampled batches (max_t_filled 101, episodes ~47 steps) about half of all items.
    for (int b = wave; b < B; b += nw) {
        const int64_t base = eslot(bt, b) * bt.T1;
        int last = -1;
        for (int t0 = 0; t0 < Te - 1; t0 += 64) {
            const int t = t0 + lane;
            bool live = false;
            if (t < Te - 1) {
                live = bt.filled[base + t] != 0 && (t == 0 || bt.terminated[base + t - 1] == 0);
            }
            const uint64_t m = __ballot(live);
            if (m) last = t0 + 63 - __builtin_clzll(m);
        }
        if (lane == 0) msum[4 + b] = (float)(last + 1);
    }
}

__device__ __forceinline__ int t_eff(const float* msum) { return (int)msum[1]; }
// live mixer items of episode b (mask(b, t) == 0 for every t >= it; see mask_sum_body)
__device__ __forceinline__ int mix_len(const float* msum, int b) { return (int)msum[4 + b]; }

// entity inputs ein[i][j][c] (K1 columns, zero padded)
__device__ void ein_body(const RCfg& c, const MlgEntityBatch& bt, float* __restrict__ ein, int bx) {
    const int64_t idx = (int64_t)bx * blockDim.x + threadIdx.x;
    if (idx >= (int64_t)c.I * NE * c.K1) return;
    const int col = (int)(idx % c.K1);
    const int j = (int)((idx / c.K1) % NE);
    const int i = (int)(idx / ((int64_t)c.K1 * NE));
    const int b = i / c.T, t = i % c.T;
    const int64_t row = eslot(bt, b) * bt.T1 + t;
    float v = 0.f;
    if (j < c.NE) {
        if (col < c.ED) v = bt.entities[(row * c.NE + j) * c.ED + col];
        else if (col < c.D0 && j < c.NA && t > 0) v = bt.actions_onehot[((row - 1) * c.NA + j) * c.A + (col - c.ED)];
    }
    ein[idx] = v;
}

// The whole prologue in one launch of 256-thread blocks (was seven launches, each a few microseconds of mostly
// launch / drain latency): block ranges in this order -- the mask sum (one block, the longest single-block task,
// dispatched first), the agent packs (online + target), the hypernet packs (4 x 2), the in_trans splits (10), the
// in_trans^T splits (5), the weight transposes, the entity inputs. The tasks are independent: each reads only the
// parameters / the batch and writes its own workspace region.
struct Prologue {
    CopyJobs aj, hj;
    CopyPairs ap, hp;
    HSplit hs, hsT;
    TrJobs tj;
    RCfg c;
    MlgEntityBatch bt;
    float *ein, *msum;
    int nb_a, nb_h, nb_s, nb_t, nb_e;  // blocks per agent pack, hypernet pack, split block, transpose job; ein blocks
    int n_rows_in;                     // > 0: the slot map travels here (host_rows); block 0 stores it to rows_dst
    int32_t* rows_dst;
    int32_t rows_in[MLG_INLINE_ROWS];
};
static_assert(sizeof(Prologue) <= 4096, "prologue kernel arguments over 4 KB");
inline int prologue_blocks(const Prologue& P) {
    return 1 + 2 * P.nb_a + 8 * P.nb_h + 15 * P.nb_s + P.tj.n * P.nb_t + P.nb_e;
}
__global__ void __launch_bounds__(256) prologue_kernel(Prologue P) {
    __shared__ float red[256];
    __shared__ int32_t srows[MLG_INLINE_ROWS];
    MlgEntityBatch bt = P.bt;
    if (P.n_rows_in > 0) {  // this launch reads the slot map from LDS, the later launches from rows_dst
        if ((int)threadIdx.x < P.n_rows_in) {
            srows[threadIdx.x] = P.rows_in[threadIdx.x];
            if (blockIdx.x == 0) P.rows_dst[threadIdx.x] = P.rows_in[threadIdx.x];
        }
        __syncthreads();
        bt.rows = srows;
    }
    int blk = blockIdx.x;
    if (blk == 0) {
        __shared__ mlg::MaskStatsLds ms;
        constexpr int EPW = 8;  // episodes per wave: 4 waves cover the bench's 32-episode batches
        if (mlg::mask_stats_fits<EPW>(P.c.B, P.c.T, blockDim.x / 64))  // one round trip (batch_mask_device.h)
            mlg::batch_mask_stats<EPW>(bt.filled, bt.terminated, bt.T1, [&](int b) { return eslot(bt, b); }, P.c.B,
                                       P.c.T, P.msum, P.msum + 4, ms);
        else
            mask_sum_body(bt, P.c.B, P.c.T, P.msum, red);
        return;
    }
    blk -= 1;
    if (blk < 2 * P.nb_a) return copy_jobs_body(P.aj, P.ap, blk % P.nb_a, blk / P.nb_a);
    blk -= 2 * P.nb_a;
    if (blk < 8 * P.nb_h) return copy_jobs_body(P.hj, P.hp, blk % P.nb_h, blk / P.nb_h);
    blk -= 8 * P.nb_h;
    if (blk < 10 * P.nb_s) return hyper_split_body(P.hs, blk % P.nb_s, blk / P.nb_s);
    blk -= 10 * P.nb_s;
    if (blk < 5 * P.nb_s) return hyper_splitT_body(P.hsT, blk % P.nb_s, blk / P.nb_s);
    blk -= 5 * P.nb_s;
    if (blk < P.tj.n * P.nb_t) return transpose_body(P.tj, blk % P.nb_t, blk / P.nb_t);
    blk -= P.tj.n * P.nb_t;
    ein_body(P.c, bt, P.ein, blk);
}

// ---- masks -----------------------------------------------------------------------------------------------
// a mask row of n <= NE bytes as bits (bit j = byte j != 0), bits >= n set: the NE loads are unrolled and issued
// back to back (a loop over the runtime n waited for each byte in turn; these sit on every per-item kernel's
// critical path)
__device__ __forceinline__ uint32_t mask_row_bits(const uint8_t* row, int n) {
    uint32_t m = ~((1u << n) - 1u) & 0xFFFFu;
    uint8_t v[NE];
#pragma unroll
    for (int j = 0; j < NE; ++j) v[j] = row[j < n ? j : 0];
#pragma unroll
    for (int j = 0; j < NE; ++j) m |= (uint32_t)(j < n && v[j] != 0) << j;
    return m;
}
// entity mask bits of (b, t); bits >= NE set (absent)
__device__ __forceinline__ uint32_t em_bits(const RCfg& c, const MlgEntityBatch& bt, int b, int t) {
    return mask_row_bits(bt.entity_mask + (eslot(bt, b) * bt.T1 + t) * c.NE, c.NE);
}
__device__ __forceinline__ uint32_t om_row(const RCfg& c, const MlgEntityBatch& bt, int b, int t, int q) {
    if (q >= c.NE) return 0xFFFFu;
    return mask_row_bits(bt.obs_mask + ((eslot(bt, b) * bt.T1 + t) * c.NE + q) * c.NE, c.NE);
}
// imagine group bits of episode b: gA = groupA | em0, gB = !groupA | em0 (entity_rnn_agent.py:97-101)
__device__ __forceinline__ void group_bits(const RCfg& c, const MlgEntityBatch& bt, const uint8_t* groupA, int b,
                                           uint32_t& gA, uint32_t& gB, uint32_t& em0) {
    em0 = em_bits(c, bt, b, 0);
    const uint32_t ga = mask_row_bits(groupA + (int64_t)b * c.NE, c.NE) & ((1u << c.NE) - 1u);
    gA = (ga | em0) & 0xFFFFu;
    gB = ((~ga) | em0) & 0xFFFFu;
}
// interact row q: pairs in the same group are masked (entity_rnn_agent.py:107-110); within = !interact
__device__ __forceinline__ uint32_t interact_row(uint32_t gA, uint32_t gB, int q) {
    const uint32_t a = ((gA >> q) & 1u) ? 0u : (~gA & 0xFFFFu);
    const uint32_t bb = ((gB >> q) & 1u) ? 0u : (~gB & 0xFFFFu);
    return a | bb;
}
__device__ __forceinline__ uint32_t active_row(uint32_t em0, int q) { return ((em0 >> q) & 1u) ? 0xFFFFu : em0; }
// dead agent rows of an item (bits < 8): entity-masked agents and padding slots >= NA
__device__ __forceinline__ uint32_t dead_bits(const RCfg& c, uint32_t em) {
    return ((em & ((1u << c.NA) - 1u)) | (~((1u << c.NA) - 1u))) & 0xFFu;
}

// ---- agent entity block forward (online: 3 copies; target: plain) ---------------------------------------
struct AgentPtrs {
    const float* P;
    float *x1, *qkv, *Pw, *o, *x2, *x3, *gi;
    const float* wsp;  // split-bf16 in_trans (hyper_split_kernel layout)
};

template <int S8>
__global__ void __launch_bounds__(64) ent_fwd_kernel(RCfg c_arg, MlgEntityBatch bt, const uint8_t* __restrict__ groupA,
                                                     RAgent L_arg, const float* __restrict__ ein, AgentPtrs on,
                                                     AgentPtrs tg, const float* __restrict__ msum) {
    const RCfg c = static_cfg<S8>(c_arg);
    const RAgent L = S8 ? make_ragent(S8Dims::D0, S8Dims::A) : L_arg;
    __shared__ float s_ein[NE * LDI];
    __shared__ float s_x1[NE * LDX];
    __shared__ float s_qkv[NE * LDQ];
    __shared__ float s_o[3][16 * LDX];
    __shared__ uint32_t s_m[3][2][16];
    __shared__ uint32_t s_dead[2];
    const int lane = threadIdx.x;
    const bool online = blockIdx.y == 0;
    const AgentPtrs& A = online ? on : tg;
    const int ncopy = online ? 3 : 1;
    const int R = online ? c.Ron : c.Rtg;
    const int i0 = blockIdx.x * 2;
    const int Te = t_eff(msum);
    // live items: t < max_t_filled and t <= the episode's live mixer items (the Q of step mix_len is the target of
    // the last live mixer item); the others only zero their GRU inputs (finite, deterministic recurrence there)
    auto live = [&](int i) { return i < c.I && i % c.T < Te && i % c.T <= mix_len(msum, i / c.T); };
    const bool v0 = live(i0), v1 = live(i0 + 1);
    if (!v0 && !v1) {
        for (int e = 0; e < 2; ++e) {
            const int i = i0 + e;
            if (i >= c.I || i % c.T >= Te) continue;
            const int b = i / c.T, t = i % c.T;
            for (int cc = 0; cc < ncopy; ++cc) {
                float* gi = A.gi + ((int64_t)t * R + ((int64_t)cc * c.B + b) * c.NA) * 3 * EMB;
                for (int q = lane; q < c.NA * 3 * EMB; q += 64) gi[q] = 0.f;
            }
        }
        return;
    }
    for (int k = lane; k < 3 * 16 * LDX; k += 64) (&s_o[0][0])[k] = 0.f;
    if (lane < 32) {
        const int e = lane >> 4, q = lane & 15, i = i0 + e;
        if (live(i)) {
            const int b = i / c.T, t = i % c.T;
            const uint32_t om = om_row(c, bt, b, t, q);
            s_m[0][e][q] = om;
            if (online) {
                uint32_t gA, gB, em0;
                group_bits(c, bt, groupA, b, gA, gB, em0);
                const uint32_t it = interact_row(gA, gB, q);
                s_m[1][e][q] = ((~it) & 0xFFFFu) | om;
                s_m[2][e][q] = it | om;
            }
            if (q == 0) s_dead[e] = dead_bits(c, em_bits(c, bt, b, t));
        } else {
            for (int cc = 0; cc < 3; ++cc) s_m[cc][e][q] = 0xFFFFu;
            if (q == 0) s_dead[e] = 0xFFu;
        }
    }
    wave_sync();
    for (int e = 0; e < 2; ++e) {
        const int i = i0 + e;
        if (!live(i)) continue;
        for (int k = lane; k < NE * c.K1; k += 64) s_ein[(k / c.K1) * LDI + k % c.K1] = ein[(int64_t)i * NE * c.K1 + k];
        wave_sync();
        dense_lds<true>(A.P + L.w1, L.K1, A.P + L.b1, EMB / 16, s_ein, LDI, L.K1 / 16, s_x1, LDX, lane);
        wave_sync();
#if defined(MLG_HYPER_F32)
        dense_lds<false>(A.P + L.win, EMB, nullptr, 3 * EMB / 16, s_x1, LDX, EMB / 16, s_qkv, LDQ, lane);
#else
        in_trans_lds_b16(A.wsp, s_x1, s_qkv, LDQ, lane);
#endif
        wave_sync();
        if (online) {
            for (int k = lane; k < NE * EMB; k += 64) A.x1[(int64_t)i * NE * EMB + k] = s_x1[(k / EMB) * LDX + k % EMB];
            for (int k = lane; k < NE * 3 * EMB; k += 64)
                A.qkv[(int64_t)i * NE * 3 * EMB + k] = s_qkv[(k / (3 * EMB)) * LDQ + k % (3 * EMB)];
        }
        for (int cc = 0; cc < ncopy; ++cc)
            attn_fwd(s_qkv, s_m[cc][e], c.NA, c.NE, s_o[cc] + e * NAS * LDX, LDX,
                     online ? A.Pw + ((int64_t)cc * c.I + i) * 1024 : nullptr, lane);
        wave_sync();
    }
    const int col = lane & 15, g = lane >> 4;
    const int e = col >> 3, n = col & 7, i = i0 + e;
    const bool valid = n < c.NA && live(i);
    // rows of a skipped item of the pair (t < max_t_filled, past the episode's live items): GRU inputs zeroed
    const bool zrow = !valid && n < c.NA && i < c.I && i % c.T < Te;
    const int b = (valid || zrow) ? i / c.T : 0, t = (valid || zrow) ? i % c.T : 0;
    const uint32_t dead = s_dead[0] | (s_dead[1] << 8);
    const bool rdead = (dead >> col) & 1u;
    for (int cc = 0; cc < ncopy; ++cc) {
        const int64_t r = ((int64_t)cc * c.B + b) * c.NA + n;
        const int64_t ro = ((int64_t)t * R + r);
        floatx4 x2[4], x3[4];
        bias_init<4>(x2, A.P + L.bout, 0, lane);
        mm_lds<4>(x2, A.P + L.wout, EMB, 0, s_o[cc], LDX, EMB / 16, lane);
        if (rdead) {
#pragma unroll
            for (int k = 0; k < 4; ++k) x2[k] = floatx4{0.f, 0.f, 0.f, 0.f};
        }
        bias_init<4>(x3, A.P + L.b2, 0, lane);
        mm_reg<4, 4>(x3, A.P + L.w2, EMB, 0, x2, lane);
#pragma unroll
        for (int k = 0; k < 4; ++k) x3[k] = relu4(x3[k]);
        if (valid && online) {
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                *reinterpret_cast<floatx4*>(A.o + ro * EMB + k * 16 + 4 * g) = ld4(s_o[cc] + col * LDX + k * 16 + 4 * g);
                *reinterpret_cast<floatx4*>(A.x2 + ro * EMB + k * 16 + 4 * g) = x2[k];
                *reinterpret_cast<floatx4*>(A.x3 + ro * EMB + k * 16 + 4 * g) = x3[k];
            }
        }
        // GI = [b_ir + b_hr + W_ir x | b_iz + b_hz + W_iz x | b_in + W_in x]
#pragma unroll
        for (int q = 0; q < 3; ++q) {
            floatx4 acc[4];
            bias_init<4>(acc, q < 2 ? A.P + L.brz + q * EMB : A.P + L.bih + 2 * EMB, 0, lane);
            mm_reg<4, 4>(acc, A.P + L.wih + (int64_t)q * EMB * EMB, EMB, 0, x3, lane);
            if (valid || zrow) {
#pragma unroll
                for (int k = 0; k < 4; ++k)
                    *reinterpret_cast<floatx4*>(A.gi + ro * 3 * EMB + q * EMB + k * 16 + 4 * g) =
                        valid ? acc[k] : floatx4{0.f, 0.f, 0.f, 0.f};
            }
        }
    }
}

// ---- GRU recurrence (online rows then target rows) ------------------------------------------------------
// grid (ntiles_on + ntiles_tg), 4 waves: wave w owns hidden chunk w, its W_hh rows in VGPRs.
__global__ void __launch_bounds__(256) rec_kernel(RCfg c, RAgent L, const float* __restrict__ Pon,
                                                  const float* __restrict__ Ptg, const float* __restrict__ gi_on,
                                                  const float* __restrict__ gi_tg, float* __restrict__ hs_on,
                                                  float* __restrict__ hs_tg, float* __restrict__ ws_gr,
                                                  float* __restrict__ ws_gz, float* __restrict__ ws_gn,
                                                  float* __restrict__ ws_ghn, const float* __restrict__ msum) {
    constexpr int H = EMB, HC = 4;
    const int Te = t_eff(msum);
    __shared__ __attribute__((aligned(16))) float hs[2][16 * LDX];
    const int nt_on = (c.Ron + 15) / 16;
    const bool online = (int)blockIdx.x < nt_on;
    const int tile = online ? blockIdx.x : blockIdx.x - nt_on;
    const int R = online ? c.Ron : c.Rtg;
    const float* P = online ? Pon : Ptg;
    const float* gi = online ? gi_on : gi_tg;
    float* hsg = online ? hs_on : hs_tg;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int col = lane & 15, g = lane >> 4;
    const int r = tile * 16 + col;
    const bool valid = r < R;
    const int f0 = w * 16 + 4 * g;
    floatx4 wr[3][HC];
#pragma unroll
    for (int q = 0; q < 3; ++q)
#pragma unroll
        for (int kc = 0; kc < HC; ++kc) wr[q][kc] = ld4(P + L.whh + (int64_t)(q * H + w * 16 + col) * H + kc * 16 + 4 * g);
    const floatx4 bhn = ld4(P + L.bhh + 2 * H + f0);
    const __amdgpu_buffer_rsrc_t rs_h = mlg_rsrc(hsg), rs_gr = mlg_rsrc(ws_gr), rs_gz = mlg_rsrc(ws_gz),
                                 rs_gn = mlg_rsrc(ws_gn), rs_ghn = mlg_rsrc(ws_ghn);
    for (int i = tid; i < 16 * LDX; i += blockDim.x) hs[0][i] = 0.f;
    if (valid) *reinterpret_cast<floatx4*>(hsg + (int64_t)r * H + f0) = floatx4{0.f, 0.f, 0.f, 0.f};
    const int rr = valid ? r : 0;
    auto gi_at = [&](int t, int q) { return ld4(gi + ((int64_t)t * R + rr) * 3 * H + q * H + f0); };
    floatx4 nr = gi_at(0, 0), nz = gi_at(0, 1), nn = gi_at(0, 2);
    __syncthreads();
    int cur = 0;
    for (int t = 0; t < Te; ++t) {
        floatx4 ar = nr, az = nz;
        const floatx4 gin = nn;
        if (t + 1 < Te) {
            nr = gi_at(t + 1, 0);
            nz = gi_at(t + 1, 1);
            nn = gi_at(t + 1, 2);
        }
        floatx4 ahn = bhn;
        const float* hrow = hs[cur] + col * LDX + 4 * g;
#pragma unroll
        for (int kc = 0; kc < HC; ++kc) {
            const floatx4 hin = ld4(hrow + kc * 16);
            ar = mfma_chunk(wr[0][kc], hin, ar);
            az = mfma_chunk(wr[1][kc], hin, az);
            ahn = mfma_chunk(wr[2][kc], hin, ahn);
        }
        const floatx4 hp = ld4(hs[cur] + col * LDX + f0);
        floatx4 rg, zg, ng, hn;
#pragma unroll
        for (int q = 0; q < 4; ++q) {  // gates on v_exp_f32 / v_rcp_f32 (as the QMIX learner's recurrence)
            rg[q] = fast_sigmoid(ar[q]);
            zg[q] = fast_sigmoid(az[q]);
            ng[q] = fast_tanh(gin[q] + rg[q] * ahn[q]);
            hn[q] = ng[q] + zg[q] * (hp[q] - ng[q]);
        }
        *reinterpret_cast<floatx4*>(hs[cur ^ 1] + col * LDX + f0) = hn;
        {  // branch-free stores (dropped rows: out-of-range buffer offsets), so the prefetch waits count them
            const int64_t o = ((int64_t)t * R + r) * H + f0;
            st4_if(rs_h, o + (int64_t)R * H, hn, valid);
            if (online) {
                st4_if(rs_gr, o, rg, valid);
                st4_if(rs_gz, o, zg, valid);
                st4_if(rs_gn, o, ng, valid);
                st4_if(rs_ghn, o, ahn, valid);
            }
        }
        __syncthreads();
        cur ^= 1;
    }
}

// The recurrences on 4-row tiles (gru4_device.h, shared with the QMIX learner): 4x the CUs of the 16-row tiles above
// on the sequential T loop. grid (ntiles4 online + ntiles4 target), 4 waves; online tiles store the gates.
__global__ void __launch_bounds__(256) rec4_kernel(RCfg c, RAgent L, const float* __restrict__ Pon,
                                                   const float* __restrict__ Ptg, const float* __restrict__ gi_on,
                                                   const float* __restrict__ gi_tg, float* __restrict__ hs_on,
                                                   float* __restrict__ hs_tg, float* __restrict__ ws_gr,
                                                   float* __restrict__ ws_gz, float* __restrict__ ws_gn,
                                                   float* __restrict__ ws_ghn, const float* __restrict__ msum) {
    const int nt_on = (c.Ron + 3) / 4;
    const bool online = (int)blockIdx.x < nt_on;
    const float* P = online ? Pon : Ptg;
    const mlg::Gru4Fwd a{online ? c.Ron : c.Rtg, P + L.whh, P + L.bhh, online ? gi_on : gi_tg, online ? hs_on : hs_tg,
                         ws_gr, ws_gz, ws_gn, ws_ghn, online};
    mlg::NoStamps st;
    mlg::gru4_fwd<EMB>(a, online ? blockIdx.x : blockIdx.x - nt_on, t_eff(msum), st);
}

// agent row r of a net -> (b, n); copy = r / (B * NA)
__device__ __forceinline__ void row_bn(const RCfg& c, int r, int& b, int& n) {
    n = r % c.NA;
    b = (r / c.NA) % c.B;
}

// fc3 for every (t, row): grid (ntiles_max, T, 2), Ap/16 waves (wave = action tile); masked agents -> 0
template <int S8>
__global__ void __launch_bounds__(128) q_kernel(RCfg c_arg, MlgEntityBatch bt, RAgent L_arg, const float* __restrict__ Pon,
                                                const float* __restrict__ Ptg, const float* __restrict__ hs_on,
                                                const float* __restrict__ hs_tg, float* __restrict__ mac,
                                                float* __restrict__ tmac, const float* __restrict__ msum) {
    const RCfg c = static_cfg<S8>(c_arg);
    const RAgent L = S8 ? make_ragent(S8Dims::D0, S8Dims::A) : L_arg;
    const bool online = blockIdx.z == 0;
    const int R = online ? c.Ron : c.Rtg;
    const int tile = blockIdx.x, t = blockIdx.y;
    if (tile * 16 >= R || t >= t_eff(msum)) return;
    const float* P = online ? Pon : Ptg;
    const float* hsg = (online ? hs_on : hs_tg) + (int64_t)(t + 1) * R * EMB;
    float* qout = online ? mac : tmac;
    const int lane = threadIdx.x & 63, at = threadIdx.x >> 6;
    const int col = lane & 15, g = lane >> 4;
    const int r = tile * 16 + col;
    const bool valid = r < R;
    int b = 0, n = 0;
    if (valid) row_bn(c, r, b, n);
    const bool dead = valid && bt.entity_mask[(eslot(bt, b) * bt.T1 + t) * c.NE + n] != 0;
    floatx4 q[1];
    bias_init<1>(q, P + L.b3, at, lane);
    mm_ptr<1>(q, P + L.w3, EMB, at, hsg + (int64_t)(valid ? r : 0) * EMB, EMB / 16, lane);
    if (valid) {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int a = at * 16 + 4 * g + k;
            if (a < c.A) qout[((int64_t)t * R + r) * c.A + a] = dead ? 0.f : q[0][k];
        }
    }
}

// ---- hypernet forward: grid (I, 8): y = k + 4 * net -------------------------------------------------------
struct HypPtrs {
    const float* Wsp[8];  // split in_trans of (k, net) at [k + 4 net]
    const float* Pon[4];
    const float* Ptg[4];
    float* x1m[4];
    float* qkvm[4];
    float* Pm[4];
    float* om[4];
    float* x2m[4];
    float* X[4];
    float* Xtg[4];
};

template <int S8>
__global__ void __launch_bounds__(64) hyper_fwd_kernel(RCfg c_arg, MlgEntityBatch bt, const uint8_t* __restrict__ groupA,
                                                       RHyper L_arg, const float* __restrict__ ein, HypPtrs hp,
                                                       const float* __restrict__ msum) {
    const RCfg c = static_cfg<S8>(c_arg);
    const RHyper L = S8 ? make_rhyper(S8Dims::D0) : L_arg;
    // s_ein and s_x1 live inside s_o (dead before the attention writes it): 21 KB of LDS per item instead of 29 KB,
    // seven workgroups per CU instead of five
    static_assert(NE * LDI + NE * LDX <= 32 * LDX, "s_ein + s_x1 alias s_o");
    __shared__ __attribute__((aligned(16))) float s_qkv[NE * LDQ];
    __shared__ __attribute__((aligned(16))) float s_o[32 * LDX];
    float* const s_ein = s_o;
    float* const s_x1 = s_o + NE * LDI;
    __shared__ uint32_t s_m[3][16];
    __shared__ uint32_t s_dead;
    const int lane = threadIdx.x;
    const int i = blockIdx.x, k = blockIdx.y & 3, net = blockIdx.y >> 2;
    const int b = i / c.T, t = i % c.T;
    // masked mixer item: nothing to compute, and nothing to write -- the wgrad jobs skip its rows (wgrad_device.h
    // bjob_items) and no other kernel reads its activations
    if (t >= t_eff(msum) - 1 || t >= mix_len(msum, b)) return;
    const int ts = net ? t + 1 : t;
    const int ie = b * c.T + ts;
    const float* P = net ? hp.Ptg[k] : hp.Pon[k];
    const int V = net ? 1 : nvar(k);
    if (lane < 16) {
        const int q = lane;
        const uint32_t em = em_bits(c, bt, b, ts);
        const uint32_t dead = dead_bits(c, em);
        // default AttentionHyperNet mask: agent q masked or entity j masked (flex_qmix.py:41-45)
        s_m[0][q] = (q < NAS && ((dead >> q) & 1u)) ? 0xFFFFu : (em & 0xFFFFu);
        if (V == 3) {
            uint32_t gA, gB, em0;
            group_bits(c, bt, groupA, b, gA, gB, em0);
            const uint32_t it = interact_row(gA, gB, q), ac = active_row(em0, q);
            s_m[1][q] = (((~it) & 0xFFFFu) | ac) & 0xFFFFu;  // W mask: within | active
            s_m[2][q] = (it | ac) & 0xFFFFu;                 // I mask: interact | active
        }
        if (q == 0) s_dead = dead;
    }
    for (int q = lane; q < NE * c.K1; q += 64) s_ein[(q / c.K1) * LDI + q % c.K1] = ein[(int64_t)ie * NE * c.K1 + q];
    wave_sync();
    dense_lds<true>(P + L.w1, L.K1, P + L.b1, EMB / 16, s_ein, LDI, L.K1 / 16, s_x1, LDX, lane);
    wave_sync();
#if defined(MLG_HYPER_F32)
    dense_lds<false>(P + L.win, EMB, nullptr, 3 * EMB / 16, s_x1, LDX, EMB / 16, s_qkv, LDQ, lane);
#else
    in_trans_lds_b16(hp.Wsp[k + 4 * net], s_x1, s_qkv, LDQ, lane);
#endif
    wave_sync();
    if (!net) {
        for (int q = lane; q < NE * EMB; q += 64) hp.x1m[k][(int64_t)i * NE * EMB + q] = s_x1[(q / EMB) * LDX + q % EMB];
        for (int q = lane; q < NE * 3 * EMB; q += 64)
            hp.qkvm[k][(int64_t)i * NE * 3 * EMB + q] = s_qkv[(q / (3 * EMB)) * LDQ + q % (3 * EMB)];
    }
    wave_sync();  // s_ein / s_x1 dead: s_o (same bytes) zeroed for the attention outputs
    for (int q = lane; q < 32 * LDX; q += 64) s_o[q] = 0.f;
    wave_sync();
    for (int v = 0; v < V; ++v)
        attn_fwd(s_qkv, s_m[v], c.NA, c.NE, s_o + v * NAS * LDX, LDX,
                 net ? nullptr : hp.Pm[k] + ((int64_t)v * c.I + i) * 1024, lane);
    wave_sync();
    const int col = lane & 15, g = lane >> 4;
    const uint32_t dead = s_dead;
    for (int tile = 0; tile * 16 < V * NAS; ++tile) {
        const int row = tile * 16 + col, v = row >> 3, n = row & 7;
        const bool rdead = (dead >> n) & 1u;
        floatx4 x2[4];
        bias_init<4>(x2, P + L.bout, 0, lane);
        mm_lds<4>(x2, P + L.wout, EMB, 0, s_o + tile * 16 * LDX, LDX, EMB / 16, lane);
        if (rdead) {
#pragma unroll
            for (int q = 0; q < 4; ++q) x2[q] = floatx4{0.f, 0.f, 0.f, 0.f};
        }
        floatx4 X[2];
        bias_init<2>(X, P + L.b2, 0, lane);
        mm_reg<2, 4>(X, P + L.w2, EMB, 0, x2, lane);
        if (rdead) X[0] = X[1] = floatx4{0.f, 0.f, 0.f, 0.f};
        if (v >= V) continue;  // rows n >= NA are written too (zeros): they are wgrad rows
        const int64_t ro = ((int64_t)v * c.I + i) * NAS + n;
        if (!net) {
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                *reinterpret_cast<floatx4*>(hp.om[k] + ro * EMB + q * 16 + 4 * g) = ld4(s_o + row * LDX + q * 16 + 4 * g);
                *reinterpret_cast<floatx4*>(hp.x2m[k] + ro * EMB + q * 16 + 4 * g) = x2[q];
            }
        }
        float* Xo = net ? hp.Xtg[k] + ((int64_t)i * NAS + n) * EM : hp.X[k] + ro * EM;
#pragma unroll
        for (int q = 0; q < 2; ++q) *reinterpret_cast<floatx4*>(Xo + q * 16 + 4 * g) = X[q];
    }
}

// ---- mixing, TD and the mixing backward: one wave per item ------------------------------------------------
struct MixIO {
    const float* X[4];
    const float* Xtg[4];
    float* dX[4];
    const float *mac, *tmac, *msum;
    float *dq, *d2, *part;
};

__device__ __forceinline__ float sum32(float v) {  // sum over lanes 0..31 (every lane of the half gets it)
#pragma unroll
    for (int m = 1; m < 32; m <<= 1) v += __shfl_xor(v, m);
    return v;
}
__device__ __forceinline__ float max32(float v) {
#pragma unroll
    for (int m = 1; m < 32; m <<= 1) v = fmaxf(v, __shfl_xor(v, m));
    return v;
}
__device__ __forceinline__ float sgnf(float x) { return x > 0.f ? 1.f : (x < 0.f ? -1.f : 0.f); }
__device__ __forceinline__ float elu_f(float x) { return x > 0.f ? x : expm1f(x); }
__device__ __forceinline__ float elu_d(float x) { return x > 0.f ? 1.f : expf(x); }

// mixing weight transform over the embed dim (lane = e): |x| or softmax (flex_qmix.py:96-99,103-106)
__device__ __forceinline__ float mw(float x, int softmax) {
    if (!softmax) return fabsf(x);
    const float m = max32(x);
    const float ex = expf(x - m);
    return ex / sum32(ex);
}
// backward of mw given the forward output y and input x
__device__ __forceinline__ float mw_bwd(float dy, float y, float x, int softmax) {
    if (!softmax) return dy * sgnf(x);
    return y * (dy - sum32(y * dy));
}

template <int S8>
__global__ void __launch_bounds__(64) mix_td_kernel(RCfg c_arg, MlgEntityBatch bt, MixIO io) {
    const RCfg c = static_cfg<S8>(c_arg);
    const int Te = (int)io.msum[1];
    const int lane = threadIdx.x;
    const int i = blockIdx.x;
    const int b = i / c.T, t = i % c.T;
    const int e = lane & 31;
    const int NA = c.NA;
    float* part = io.part + (int64_t)i * 8;
    if (t >= Te - 1 || t >= mix_len(io.msum, b)) {  // t = T - 1, past max_t_filled or the episode (mask 0): zero deltas
        if (lane < 8) part[lane] = 0.f;
        // dQ / d2 rows of the item's (copy, agent) rows: zeros (the item owns them; no memset pass)
        // dQ rows feed the reverse recurrence at every step; the d2 rows only the fc3 wgrad job, which skips them when
        // NA is a multiple of 8 (bjob_steps); dX rows only hyper_bwd and wgrad, which both skip the item
        const bool d2z = c.NA % 8 != 0;
        for (int q = lane; q < 3 * c.NA * (c.A + 1); q += 64) {
            const int cc = q / (c.NA * (c.A + 1)), rem = q % (c.NA * (c.A + 1)), n = rem / (c.A + 1), a2 = rem % (c.A + 1);
            const int64_t row = (int64_t)t * c.Ron + ((int64_t)cc * c.B + b) * c.NA + n;
            if (a2 == c.A) io.dq[row] = 0.f;
            else if (d2z) io.d2[row * c.A + a2] = 0.f;
        }
        return;
    }
    // Every global load of the item is issued before the first one is consumed: one wave per item, so the kernel
    // time is one item's chain of memory round trips (was ~100 dependent loads: per-agent / per-action loops with a
    // runtime trip count), not its arithmetic. Two round trips remain: the actions, then the chosen Q they index.
    const int64_t srow = eslot(bt, b) * bt.T1;
    const int hl = lane >> 5;  // half-wave: agent 2p + hl of pass p for the per-action rows (lane e = action)
    const int an = lane < NA ? (int)bt.actions[(srow + t) * NA + (lane < NA ? lane : 0)] : 0;
    const bool emv = lane < c.NE && bt.entity_mask[(srow + t) * c.NE + (lane < c.NE ? lane : 0)] != 0;
    const float r = bt.reward[srow + t];
    const float term = (float)bt.terminated[srow + t];
    const float m = emask_at(bt, b, t);
    int avv[NAS / 2];
    float tqv[NAS / 2], mqv[NAS / 2];
#pragma unroll
    for (int p = 0; p < NAS / 2; ++p) {
        const int n = 2 * p + hl, nn = n < NA ? n : 0, aa = e < c.A ? e : 0;
        avv[p] = bt.avail[((srow + t + 1) * NA + nn) * c.A + aa];
        tqv[p] = io.tmac[((int64_t)(t + 1) * c.Rtg + (int64_t)b * NA + nn) * c.A + aa];
        mqv[p] = c.double_q ? io.mac[((int64_t)(t + 1) * c.Ron + (int64_t)b * NA + nn) * c.A + aa] : 0.f;
    }
    // column e of every hypernet output row (rows n >= NA are allocated; their values are never used)
    const int64_t xo = (int64_t)i * NAS * EM + e, vstride = (int64_t)c.I * NAS * EM;
    float xt[4][NAS], xP[NAS], xW[NAS], xI[NAS], xwf[NAS], xb1[NAS], xV[NAS];
#pragma unroll
    for (int n = 0; n < NAS; ++n) {
#pragma unroll
        for (int k = 0; k < 4; ++k) xt[k][n] = io.Xtg[k][xo + n * EM];
        xP[n] = io.X[0][xo + n * EM];
        xW[n] = io.X[0][vstride + xo + n * EM];
        xI[n] = io.X[0][2 * vstride + xo + n * EM];
        xwf[n] = io.X[1][xo + n * EM];
        xb1[n] = io.X[2][xo + n * EM];
        xV[n] = io.X[3][xo + n * EM];
    }
    float caqv[3];  // lane n < NA: chosen Q of agent n in each copy
#pragma unroll
    for (int cc = 0; cc < 3; ++cc)
        caqv[cc] = lane < NA ? io.mac[((int64_t)t * c.Ron + ((int64_t)cc * c.B + b) * NA + (lane < NA ? lane : 0)) * c.A + an]
                             : 0.f;
    const uint32_t dead = dead_bits(c, (~((1u << c.NE) - 1u) & 0xFFFFu) | ((uint32_t)__ballot(emv) & 0xFFFFu));
    // ---- target max (double Q: the online argmax over the available actions picks the target Q) ----
    float tmax[NAS];
#pragma unroll
    for (int p = 0; p < NAS / 2; ++p) {
        const int n = 2 * p + hl;
        const bool ok = n < NA && e < c.A;
        const float tqm = avv[p] == 0 ? -9999999.f : tqv[p];
        float res;
        if (c.double_q) {  // argmax with the sequential scan's order (NaN first, ties -> lowest index): a total order
            float bv = ok ? (avv[p] == 0 ? -9999999.f : mqv[p]) : -INFINITY;
            int bi = ok ? e : 64 + e;
#pragma unroll
            for (int s2 = 1; s2 < 32; s2 <<= 1) {
                const float ov = __shfl_xor(bv, s2);
                const int oi = __shfl_xor(bi, s2);
                const bool take = amax_better(ov, oi, bv, bi);
                bv = take ? ov : bv;
                bi = take ? oi : bi;
            }
            res = __shfl(tqm, hl * 32 + (bi & 31));
        } else {  // fmaxf ignores NaN operands like the sequential fmaxf scan; NaN pads are neutral
            res = ok ? tqm : __builtin_nanf("");
#pragma unroll
            for (int s2 = 1; s2 < 32; s2 <<= 1) res = fmaxf(res, __shfl_xor(res, s2));
        }
        tmax[2 * p] = __shfl(res, 0);
        tmax[2 * p + 1] = __shfl(res, 32);
    }
    float caq[3][NAS];
    int act[NAS];
#pragma unroll
    for (int n = 0; n < NAS; ++n) {
        act[n] = __shfl(an, n);
#pragma unroll
        for (int cc = 0; cc < 3; ++cc) caq[cc][n] = __shfl(caqv[cc], n);
    }
    const float invN = 1.f / (float)NA, invNE = 1.f / ((float)NA * (float)EM);
    auto col_sum = [&](const float(&x)[NAS]) {  // column e over the agent rows, in row order
        float s = 0.f;
#pragma unroll
        for (int n = 0; n < NAS; ++n)
            if (n < NA) s += x[n];
        return s;
    };
    // ---- target mixer (flex_qmix on the t + 1 entities, target weights) ----
    float y_tg;
    {
        float pre = col_sum(xt[2]) * invN;  // b1
#pragma unroll
        for (int n = 0; n < NAS; ++n)
            if (n < NA) pre += tmax[n] * mw(xt[0][n], c.softmax);
        const float hid = elu_f(pre);
        const float wf = mw(col_sum(xt[1]) * invN, c.softmax);
        const float vsum = sum32(col_sum(xt[3]));
        y_tg = sum32(hid * wf) + vsum * invNE;
    }
    // ---- online mixer: plain and imagined ----
    const float b1 = col_sum(xb1) * invN;
    const float wfpre = col_sum(xwf) * invN;
    const float wf = mw(wfpre, c.softmax);
    const float vv = sum32(col_sum(xV)) * invNE;
    float w1P[NAS], w1W[NAS], w1I[NAS];
    float preP = b1, preI = b1;
#pragma unroll
    for (int n = 0; n < NAS; ++n) {
        w1P[n] = w1W[n] = w1I[n] = 0.f;
        if (n >= NA) continue;
        w1P[n] = mw(xP[n], c.softmax);
        w1W[n] = mw(xW[n], c.softmax);
        w1I[n] = mw(xI[n], c.softmax);
        preP += caq[0][n] * w1P[n];
    }
#pragma unroll
    for (int n = 0; n < NAS; ++n)
        if (n < NA) preI += caq[1][n] * w1W[n];
#pragma unroll
    for (int n = 0; n < NAS; ++n)
        if (n < NA) preI += caq[2][n] * w1I[n];
    const float hidP = elu_f(preP), hidI = elu_f(preI);
    const float yP = sum32(hidP * wf) + vv;
    const float yI = sum32(hidI * wf) + vv;
    const float target = r + c.gamma * (1.f - term) * y_tg;
    const float tdP = (yP - target) * m, tdI = (yI - target) * m;
    if (lane == 0) {
        part[0] = tdP * tdP;
        part[1] = tdI * tdI;
        part[2] = fabsf(tdP);
        part[3] = yP * m;
        part[4] = target * m;
        part[5] = m;
        part[6] = 0.f;
        part[7] = 0.f;
    }
    // ---- backward ----
    const float msum = io.msum[0];
    const float gP = 2.f * (1.f - c.lmbda) * tdP * m / msum;
    const float gI = 2.f * c.lmbda * tdI * m / msum;
    const float dwf = gP * hidP + gI * hidI;
    const float dv = gP + gI;
    const float dpP = gP * wf * elu_d(preP);
    const float dpI = gI * wf * elu_d(preI);
    const float db1 = dpP + dpI;
    const float dwfpre = mw_bwd(dwf, wf, wfpre, c.softmax);
    float* dXP = io.dX[0] + ((int64_t)0 * c.I + i) * NAS * EM;
    float* dXW = io.dX[0] + ((int64_t)1 * c.I + i) * NAS * EM;
    float* dXI = io.dX[0] + ((int64_t)2 * c.I + i) * NAS * EM;
    float* dXwf = io.dX[1] + (int64_t)i * NAS * EM;
    float* dXb1 = io.dX[2] + (int64_t)i * NAS * EM;
    float* dXV = io.dX[3] + (int64_t)i * NAS * EM;
    float dqP[NAS], dqW[NAS], dqI[NAS];
#pragma unroll
    for (int n = 0; n < NAS; ++n) {
        const bool live = n < NA && !((dead >> n) & 1u);
        float vP = 0.f, vW = 0.f, vI = 0.f, vwf = 0.f, vb1 = 0.f, vV = 0.f;
        if (n < NA) {
            vP = mw_bwd(caq[0][n] * dpP, w1P[n], xP[n], c.softmax);
            vW = mw_bwd(caq[1][n] * dpI, w1W[n], xW[n], c.softmax);
            vI = mw_bwd(caq[2][n] * dpI, w1I[n], xI[n], c.softmax);
            vwf = dwfpre * invN;
            vb1 = db1 * invN;
            vV = dv * invNE;
        }
        dqP[n] = sum32(w1P[n] * dpP);
        dqW[n] = sum32(w1W[n] * dpI);
        dqI[n] = sum32(w1I[n] * dpI);
        if (lane < 32) {
            dXP[n * EM + e] = live ? vP : 0.f;
            dXW[n * EM + e] = live ? vW : 0.f;
            dXI[n * EM + e] = live ? vI : 0.f;
            dXwf[n * EM + e] = live ? vwf : 0.f;
            dXb1[n * EM + e] = live ? vb1 : 0.f;
            dXV[n * EM + e] = live ? vV : 0.f;
        }
    }
    // dQ of the chosen actions (masked agents: q was masked_fill'ed -> 0) and whole d2 rows (no memset pass):
    // half-wave hl writes agent 2p + hl, lane e action e
#pragma unroll
    for (int p = 0; p < NAS / 2; ++p) {
        const int n = 2 * p + hl;
        if (2 * p >= NA) break;
        const bool live = n < NA && !((dead >> n) & 1u);
        const int actn = hl ? act[2 * p + 1] : act[2 * p];
        const float dd[3] = {hl ? dqP[2 * p + 1] : dqP[2 * p], hl ? dqW[2 * p + 1] : dqW[2 * p],
                             hl ? dqI[2 * p + 1] : dqI[2 * p]};
#pragma unroll
        for (int cc = 0; cc < 3; ++cc) {
            const int64_t row = (int64_t)t * c.Ron + ((int64_t)cc * c.B + b) * NA + n;
            const float v = live ? dd[cc] : 0.f;
            if (n < NA) {
                if (e < c.A) io.d2[row * c.A + e] = e == actn ? v : 0.f;
                if (e == 0) io.dq[row] = v;
            }
        }
    }
}

// One item's q | k | v rows (NE x 3 EMB, row-major in global) into LDS rows of stride LDQ: all of the lane's 24 loads
// issued before the first LDS write (a loop over them waited for each group of loads in turn, three round trips).
__device__ __forceinline__ void qkv_to_lds(const float* __restrict__ src, float* dst, int lane) {
    constexpr int NQ = NE * 3 * EMB / 64;
    static_assert(NE * 3 * EMB % 64 == 0, "qkv rows: whole 64-lane groups");
    float v[NQ];
#pragma unroll
    for (int u = 0; u < NQ; ++u) v[u] = src[lane + 64 * u];
#pragma unroll
    for (int u = 0; u < NQ; ++u) {
        const int q = lane + 64 * u;
        dst[(q / (3 * EMB)) * LDQ + q % (3 * EMB)] = v[u];
    }
}
// the relu mask row x[col][0 .. EMB) of a lane (4 quads at 16 q + 4 g)
__device__ __forceinline__ void load_relu_rows(const float* __restrict__ x, floatx4 (&xv)[4], int lane) {
#pragma unroll
    for (int q = 0; q < 4; ++q) xv[q] = ld4(x + q * 16 + 4 * (lane >> 4));
}

// ---- hypernet backward: grid (I, 4), one wave ---------------------------------------------------------------
struct HypBwd {
    const float* wspT[4];
    const float* Pon[4];
    const float* woutT[4];
    const float* w2T[4];
    const float* winT[4];
    const float* x1m[4];
    const float* qkvm[4];
    const float* Pm[4];
    const float* dX[4];
    float* doutm[4];
    float* dqkvm[4];
    float* dfc1m[4];
};

template <int S8>
__global__ void __launch_bounds__(64) hyper_bwd_kernel(RCfg c_arg, MlgEntityBatch bt, HypBwd hb,
                                                       const float* __restrict__ msum) {
    const RCfg c = static_cfg<S8>(c_arg);
    __shared__ float s_qkv[NE * LDQ];
    __shared__ float s_dqkv[NE * LDQ];
    __shared__ float s_do[32 * LDX];
    __shared__ float s_ds[NH * 16 * NE];
    const int lane = threadIdx.x;
    const int i = blockIdx.x, k = blockIdx.y;
    const int b = i / c.T, t = i % c.T;
    const int V = nvar(k);
    const int col = lane & 15, g = lane >> 4;
    // masked mixer item: its deltas are zero and only the wgrad jobs read them, which skip its rows
    if (t >= t_eff(msum) - 1 || t >= mix_len(msum, b)) return;
    const uint32_t dead = dead_bits(c, em_bits(c, bt, b, t));
    floatx4 x1v[4];  // fc1 activations for the final relu mask, requested now (used after the attention backward)
    load_relu_rows(hb.x1m[k] + ((int64_t)i * NE + col) * EMB, x1v, lane);
    qkv_to_lds(hb.qkvm[k] + (int64_t)i * NE * 3 * EMB, s_qkv, lane);
    for (int q = lane; q < 32 * LDX; q += 64) s_do[q] = 0.f;
    for (int tile = 0; tile * 16 < V * NAS; ++tile) {
        const int row = tile * 16 + col, v = row >> 3, n = row & 7;
        const bool valid = v < V && n < c.NA;
        const bool rdead = (dead >> n) & 1u;
        const int64_t ro = ((int64_t)(v < V ? v : 0) * c.I + i) * NAS + n;
        // dx2 = W2^T dX (dX rows of masked agents are zero already)
        floatx4 dx2[4];
        bias_init<4>(dx2, nullptr, 0, lane);
        mm_ptr<4>(dx2, hb.w2T[k], EM, 0, hb.dX[k] + ro * EM, EM / 16, lane);
        if (rdead || !valid) {
#pragma unroll
            for (int q = 0; q < 4; ++q) dx2[q] = floatx4{0.f, 0.f, 0.f, 0.f};
        }
        if (v < V) {  // padding rows (n >= NA) get zeros: they are wgrad rows
#pragma unroll
            for (int q = 0; q < 4; ++q) *reinterpret_cast<floatx4*>(hb.doutm[k] + ro * EMB + q * 16 + 4 * g) = dx2[q];
        }
        // dO = Wout^T dout
        floatx4 dO[4];
        bias_init<4>(dO, nullptr, 0, lane);
        mm_reg<4, 4>(dO, hb.woutT[k], EMB, 0, dx2, lane);
#pragma unroll
        for (int q = 0; q < 4; ++q) st_row(s_do + tile * 16 * LDX, LDX, q, dO[q], lane);
    }
    wave_sync();
    for (int v = 0; v < V; ++v) {
        const float* Pv = hb.Pm[k] + ((int64_t)v * c.I + i) * 1024;
        if (v == 0) attn_bwd<false>(s_qkv, Pv, c.NA, s_do + v * NAS * LDX, LDX, s_ds, s_dqkv, lane);
        else attn_bwd<true>(s_qkv, Pv, c.NA, s_do + v * NAS * LDX, LDX, s_ds, s_dqkv, lane);
        wave_sync();
    }
    for (int q = lane; q < NE * 3 * EMB; q += 64)
        hb.dqkvm[k][(int64_t)i * NE * 3 * EMB + q] = s_dqkv[(q / (3 * EMB)) * LDQ + q % (3 * EMB)];
    // dx1 = W_in^T dqkv * relu'(x1)
    floatx4 dx1[4];
    bias_init<4>(dx1, nullptr, 0, lane);
#if defined(MLG_HYPER_F32)
    mm_lds<4>(dx1, hb.winT[k], 3 * EMB, 0, s_dqkv, LDQ, 3 * EMB / 16, lane);
#else
    in_transT_lds_b16(dx1, hb.wspT[k], s_dqkv, lane);
#endif
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const floatx4 xv = x1v[q];
#pragma unroll
        for (int r = 0; r < 4; ++r) dx1[q][r] = xv[r] > 0.f ? dx1[q][r] : 0.f;
        *reinterpret_cast<floatx4*>(hb.dfc1m[k] + ((int64_t)i * NE + col) * EMB + q * 16 + 4 * g) = dx1[q];
    }
}

// ---- reverse-time GRU backward of the online rows ------------------------------------------------------------
__global__ void __launch_bounds__(256) rec_bwd_kernel(RCfg c, MlgEntityBatch bt, RAgent L, const float* __restrict__ P,
                                                      const float* __restrict__ ws_hs, const float* __restrict__ ws_gr,
                                                      const float* __restrict__ ws_gz, const float* __restrict__ ws_gn,
                                                      const float* __restrict__ ws_ghn, const float* __restrict__ dqv,
                                                      float* __restrict__ dgi, float* __restrict__ dgh,
                                                      const float* __restrict__ msum) {
    constexpr int H = EMB;
    constexpr int LDG = 3 * H + 4;
    constexpr int KC = 3 * H / 16;
    __shared__ __attribute__((aligned(16))) float sgh[2][16 * LDG];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int col = lane & 15, g = lane >> 4;
    const int r = blockIdx.x * 16 + col;
    const int R = c.Ron;
    const bool valid = r < R;
    int b = 0, n = 0;
    if (valid) row_bn(c, r, b, n);
    const int f0 = w * 16 + 4 * g;
    floatx4 wt[KC];
#pragma unroll
    for (int kc = 0; kc < KC; ++kc)
#pragma unroll
        for (int q = 0; q < 4; ++q) wt[kc][q] = P[L.whh + (int64_t)(kc * 16 + 4 * g + q) * H + w * 16 + col];
    const int rr = valid ? r : 0;
    const int64_t srow = eslot(bt, b) * bt.T1;
    struct Step {
        floatx4 rg, zg, ng, ghn, hp, w3;
        float dq;
    };
    auto load_step = [&](int t) {
        Step s;
        const int64_t o = ((int64_t)t * R + rr) * H + f0;
        s.rg = ld4(ws_gr + o);
        s.zg = ld4(ws_gz + o);
        s.ng = ld4(ws_gn + o);
        s.ghn = ld4(ws_ghn + o);
        s.hp = ld4(ws_hs + o);
        s.dq = 0.f;
        s.w3 = floatx4{0.f, 0.f, 0.f, 0.f};
        if (t < c.T - 1) {
            s.dq = dqv[(int64_t)t * R + rr];
            const int a = (int)bt.actions[(srow + t) * c.NA + n];
            s.w3 = ld4(P + L.w3 + (int64_t)a * H + f0);
        }
        return s;
    };
    const int Te = t_eff(msum);
    if (valid) {  // steps past max_t_filled: zero deltas (wgrad rows)
        for (int t = Te; t < c.T; ++t) {
            const int64_t o3 = ((int64_t)t * R + r) * 3 * H + f0;
#pragma unroll
            for (int q = 0; q < 3; ++q) {
                *reinterpret_cast<floatx4*>(dgi + o3 + q * H) = floatx4{0.f, 0.f, 0.f, 0.f};
                *reinterpret_cast<floatx4*>(dgh + o3 + q * H) = floatx4{0.f, 0.f, 0.f, 0.f};
            }
        }
    }
    floatx4 dh = {0.f, 0.f, 0.f, 0.f};
    const __amdgpu_buffer_rsrc_t rs_gi = mlg_rsrc(dgi), rs_gh = mlg_rsrc(dgh);
    Step nx = load_step(Te - 1);
    int cur = 0;
    for (int t = Te - 1; t >= 0; --t) {
        const Step s = nx;
        if (t > 0) nx = load_step(t - 1);
        if (valid && t < c.T - 1) dh += s.dq * s.w3;
        floatx4 drp, dzp, dnp, dghn, dhd;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const float dn = dh[q] * (1.f - s.zg[q]);
            const float dz = dh[q] * (s.hp[q] - s.ng[q]);
            dhd[q] = dh[q] * s.zg[q];
            dnp[q] = dn * (1.f - s.ng[q] * s.ng[q]);
            const float dr = dnp[q] * s.ghn[q];
            drp[q] = dr * s.rg[q] * (1.f - s.rg[q]);
            dzp[q] = dz * s.zg[q] * (1.f - s.zg[q]);
            dghn[q] = dnp[q] * s.rg[q];
        }
        float* gh = sgh[cur] + col * LDG;
        *reinterpret_cast<floatx4*>(gh + f0) = drp;
        *reinterpret_cast<floatx4*>(gh + H + f0) = dzp;
        *reinterpret_cast<floatx4*>(gh + 2 * H + f0) = dghn;
        {  // branch-free stores (dropped rows: out-of-range buffer offsets)
            const int64_t o3 = ((int64_t)t * R + r) * 3 * H + f0;
            st4_if(rs_gi, o3, drp, valid);
            st4_if(rs_gi, o3 + H, dzp, valid);
            st4_if(rs_gi, o3 + 2 * H, dnp, valid);
            st4_if(rs_gh, o3, drp, valid);
            st4_if(rs_gh, o3 + H, dzp, valid);
            st4_if(rs_gh, o3 + 2 * H, dghn, valid);
        }
        __syncthreads();
        const float* ghr = sgh[cur] + col * LDG + 4 * g;
        floatx4 dp[4] = {dhd, floatx4{0.f, 0.f, 0.f, 0.f}, floatx4{0.f, 0.f, 0.f, 0.f}, floatx4{0.f, 0.f, 0.f, 0.f}};
#pragma unroll
        for (int kc = 0; kc < KC; ++kc) dp[kc & 3] = mfma_chunk(wt[kc], ld4(ghr + kc * 16), dp[kc & 3]);
        dh = (dp[0] + dp[1]) + (dp[2] + dp[3]);  // four independent MFMA chains instead of one of 48
        cur ^= 1;
    }
}

// reverse-time GRU backward of the online rows on 4-row tiles (gru4_device.h); dh += dQ W3[a] (fc3 rows)
__global__ void __launch_bounds__(256) rec_bwd4_kernel(RCfg c, MlgEntityBatch bt, RAgent L, const float* __restrict__ P,
                                                       const float* __restrict__ ws_hs, const float* __restrict__ ws_gr,
                                                       const float* __restrict__ ws_gz, const float* __restrict__ ws_gn,
                                                       const float* __restrict__ ws_ghn, const float* __restrict__ dqv,
                                                       float* __restrict__ dgi, float* __restrict__ dgh,
                                                       const float* __restrict__ msum) {
    const int r = blockIdx.x * 4 + ((threadIdx.x & 63) & 3);
    int b = 0, n = 0;
    if (r < c.Ron) row_bn(c, r, b, n);
    const mlg::Gru4Bwd a{c.Ron, c.T, c.A, c.NA, P + L.whh, P + L.w3, ws_hs, ws_gr, ws_gz, ws_gn, ws_ghn, dqv,
                         bt.actions, dgi, dgh};
    mlg::NoStamps st;
    mlg::gru4_bwd<EMB>(a, blockIdx.x, t_eff(msum), eslot(bt, b) * bt.T1 * c.NA + n, st);
}

// ---- agent entity block backward: one wave per item pair --------------------------------------------------
struct EntBwd {
    const float *wihT, *w2T, *woutT, *winT;
    const float* wspT;
    const float *x1, *qkv, *Pw, *x3, *dgi;
    float *dfc2, *dout, *dqkv, *dfc1;
};

template <int S8>
__global__ void __launch_bounds__(64) ent_bwd_kernel(RCfg c_arg, MlgEntityBatch bt, EntBwd eb,
                                                     const float* __restrict__ msum) {
    const RCfg c = static_cfg<S8>(c_arg);
    __shared__ float s_do[3][16 * LDX];
    __shared__ float s_qkv[NE * LDQ];
    __shared__ float s_dqkv[NE * LDQ];
    __shared__ float s_ds[NH * 16 * NE];
    __shared__ uint32_t s_dead[2];
    const int lane = threadIdx.x;
    const int i0 = blockIdx.x * 2;
    const int col = lane & 15, g = lane >> 4;
    if (lane < 2) {
        const int i = i0 + lane;
        s_dead[lane] = i < c.I ? dead_bits(c, em_bits(c, bt, i / c.T, i % c.T)) : 0xFFu;
    }
    wave_sync();
    const int Te = t_eff(msum);
    // items with nonzero deltas: t < max_t_filled and t < the episode's live mixer items (every later item's dQ and
    // recurrent delta are exactly zero); the others write zero deltas, no math
    auto live = [&](int ii) { return ii < c.I && ii % c.T < Te && ii % c.T < mix_len(msum, ii / c.T); };
    const int e = col >> 3, n = col & 7, i = i0 + e;
    const bool row_ok = i < c.I && n < c.NA;
    const bool valid = row_ok && live(i);
    const int b = row_ok ? i / c.T : 0, t = row_ok ? i % c.T : 0;
    const uint32_t dead = s_dead[0] | (s_dead[1] << 8);
    const bool rdead = (dead >> col) & 1u;
    const bool any = live(i0) || live(i0 + 1);
    for (int cc = 0; cc < 3; ++cc) {
        const int64_t ro = (int64_t)t * c.Ron + ((int64_t)cc * c.B + b) * c.NA + n;
        if (!any) {
            if (row_ok && c.NA % 8 != 0) {  // t-major rows the wgrad jobs cannot skip (bjob_steps needs NA % 8 == 0)
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    *reinterpret_cast<floatx4*>(eb.dfc2 + ro * EMB + q * 16 + 4 * g) = floatx4{0.f, 0.f, 0.f, 0.f};
                    *reinterpret_cast<floatx4*>(eb.dout + ro * EMB + q * 16 + 4 * g) = floatx4{0.f, 0.f, 0.f, 0.f};
                }
            }
            continue;
        }
        // dx3 = W_ih^T dGI, relu' (the x3 rows requested with the product's operands)
        floatx4 x3v[4];
        load_relu_rows(eb.x3 + (valid ? ro : 0) * EMB, x3v, lane);
        floatx4 d3[4];
        bias_init<4>(d3, nullptr, 0, lane);
        mm_ptr<4>(d3, eb.wihT, 3 * EMB, 0, eb.dgi + (valid ? ro : 0) * 3 * EMB, 3 * EMB / 16, lane);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const floatx4 xv = x3v[q];
#pragma unroll
            for (int r = 0; r < 4; ++r) d3[q][r] = (valid && xv[r] > 0.f) ? d3[q][r] : 0.f;
            if (row_ok) *reinterpret_cast<floatx4*>(eb.dfc2 + ro * EMB + q * 16 + 4 * g) = d3[q];
        }
        // dx2 = W2^T dfc2, post mask -> dout
        floatx4 d2[4];
        bias_init<4>(d2, nullptr, 0, lane);
        mm_reg<4, 4>(d2, eb.w2T, EMB, 0, d3, lane);
        if (rdead || !valid) {
#pragma unroll
            for (int q = 0; q < 4; ++q) d2[q] = floatx4{0.f, 0.f, 0.f, 0.f};
        }
        if (row_ok) {
#pragma unroll
            for (int q = 0; q < 4; ++q) *reinterpret_cast<floatx4*>(eb.dout + ro * EMB + q * 16 + 4 * g) = d2[q];
        }
        floatx4 dO[4];
        bias_init<4>(dO, nullptr, 0, lane);
        mm_reg<4, 4>(dO, eb.woutT, EMB, 0, d2, lane);
#pragma unroll
        for (int q = 0; q < 4; ++q) st_row(s_do[cc], LDX, q, dO[q], lane);
    }
    wave_sync();
    for (int ee = 0; ee < 2; ++ee) {
        const int ii = i0 + ee;
        if (ii >= c.I) continue;
        if (!live(ii)) continue;  // past max_t_filled or the episode: zero deltas, skipped by the wgrad jobs
        floatx4 x1v[4];  // fc1 activations for the final relu mask, requested now
        load_relu_rows(eb.x1 + ((int64_t)ii * NE + col) * EMB, x1v, lane);
        qkv_to_lds(eb.qkv + (int64_t)ii * NE * 3 * EMB, s_qkv, lane);
        wave_sync();
        for (int cc = 0; cc < 3; ++cc) {
            const float* Pv = eb.Pw + ((int64_t)cc * c.I + ii) * 1024;
            if (cc == 0) attn_bwd<false>(s_qkv, Pv, c.NA, s_do[cc] + ee * NAS * LDX, LDX, s_ds, s_dqkv, lane);
            else attn_bwd<true>(s_qkv, Pv, c.NA, s_do[cc] + ee * NAS * LDX, LDX, s_ds, s_dqkv, lane);
            wave_sync();
        }
        for (int q = lane; q < NE * 3 * EMB; q += 64)
            eb.dqkv[(int64_t)ii * NE * 3 * EMB + q] = s_dqkv[(q / (3 * EMB)) * LDQ + q % (3 * EMB)];
        floatx4 dx1[4];
        bias_init<4>(dx1, nullptr, 0, lane);
#if defined(MLG_HYPER_F32)
        mm_lds<4>(dx1, eb.winT, 3 * EMB, 0, s_dqkv, LDQ, 3 * EMB / 16, lane);
#else
        in_transT_lds_b16(dx1, eb.wspT, s_dqkv, lane);
#endif
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const floatx4 xv = x1v[q];
#pragma unroll
            for (int r = 0; r < 4; ++r) dx1[q][r] = xv[r] > 0.f ? dx1[q][r] : 0.f;
            *reinterpret_cast<floatx4*>(eb.dfc1 + ((int64_t)ii * NE + col) * EMB + q * 16 + 4 * g) = dx1[q];
        }
        wave_sync();
    }
}

// ---- clip_grad_norm_ + RMSprop + stats -------------------------------------------------------------------
__global__ void __launch_bounds__(1024) refil_finish_kernel(const float* __restrict__ part, int n_items,
                                                      const float* __restrict__ msum_p, float* __restrict__ params,
                                                      float* __restrict__ grads, float* __restrict__ sq, int64_t n_params,
                                                      float lr, float alpha, float eps, float max_norm, int NA,
                                                      float lmbda, float* __restrict__ stats,
                                                      const float* __restrict__ nrm_part, int n_nrm,
                                                      double* __restrict__ trained, float* __restrict__ tsync) {
    __shared__ float red[1024];
    const int tid = threadIdx.x;
    // this thread's parameter, gradient and square average, requested before the norm reduction they wait for
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + tid;
    const bool has = i < n_params;
    const float g0 = has ? grads[i] : 0.f, sq0 = has ? sq[i] : 0.f, p0 = has ? params[i] : 0.f;
    float s = 0.f;
    for (int k = tid; k < n_nrm; k += blockDim.x) s += nrm_part[k];
    const float norm = sqrtf(mlg::block_sum_1024(s, red));
    const float coef = fminf(max_norm / (norm + 1e-6f), 1.f);
    if (has) {
        const float gi = g0 * coef;
        grads[i] = gi;
        const float a = alpha * sq0 + (1.f - alpha) * gi * gi;
        sq[i] = a;
        const float pn = p0 - lr * gi / (sqrtf(a) + eps);
        params[i] = pn;
        if (tsync) tsync[i] = pn;  // the target update due after this step (refil_learner.py:181-183), same launch
    }
    // the stat sums spread over blocks 0..3 (block 0: loss and im_loss, which combine; blocks 1..3 one each; same
    // order as one block doing all five: bit-identical)
    const float ms = msum_p[0];
    for (int q = blockIdx.x; q < 4; q += gridDim.x) {
        auto sum = [&](int k) {
            float v = 0.f;
            for (int j = tid; j < n_items; j += blockDim.x) v += part[(int64_t)j * 8 + k];
            return mlg::block_sum_1024(v, red);
        };
        if (q == 0) {
            const float s0 = sum(0), s1 = sum(1);
            if (tid == 0) {
                const float loss = s0 / ms, im = s1 / ms;
                stats[0] = (1.f - lmbda) * loss + lmbda * im;
                stats[1] = im;
            }
        } else {
            const float sk = sum(q + 1);
            if (tid == 0) stats[q + 2] = q == 1 ? sk / ms : sk / (ms * NA);
        }
    }
    if (blockIdx.x == 0 && tid == 0) {
        stats[2] = norm;
        stats[6] = ms;
        stats[7] = 0.f;
        if (trained) trained[0] += (double)ms;
    }
}

// ---- host ---------------------------------------------------------------------------------------------------
RJobs make_jobs(Plan& p, float* ws, float* grads, int64_t* slab_floats, int* n_tasks, int64_t* n_red) {
    const RCfg& c = p.c;
    auto at = [&](int64_t off) { return ws ? ws + off : (float*)nullptr; };
    auto gp = [&](int64_t off) { return grads ? grads + off : (float*)nullptr; };
    const RAgent& a = p.La;
    const int I16 = c.I * NE, TR = c.T * c.Ron;
    RJobs J;
    J.n = 0;
    // rows of items / steps past each episode's live mixer items carry exactly zero deltas (the backward kernels'
    // zero paths): every job skips them (mix_len at msum + 4, mask_sum_body)
    const float* ml = ws ? ws + p.w.msum + 4 : nullptr;
    // (not optional: the kernels above no longer write the skipped rows)
    auto items = [&](mlg::BJob j, int rpi) { return mlg::bjob_items(j, ml, rpi, c.I, c.T); };
    // t-major rows: 8-row groups share one episode only when NA is a multiple of 8 (refil_8); otherwise no skipping
    auto steps = [&](mlg::BJob j) { return c.NA % 8 == 0 ? mlg::bjob_steps(j, ml, c.Ron, c.NA, c.B) : j; };
    J.j[J.n++] = items(mlg::bjob(at(p.w.dfc1), EMB, at(p.w.ein), c.K1, gp(a.c_w1), gp(a.c_b1), EMB, c.D0, I16), NE);
    J.j[J.n++] = items(mlg::bjob(at(p.w.dqkv), 3 * EMB, at(p.w.x1), EMB, gp(a.c_win), nullptr, 3 * EMB, EMB, I16), NE);
    J.j[J.n++] = steps(mlg::bjob(at(p.w.dout), EMB, at(p.w.o), EMB, gp(a.c_wout), gp(a.c_bout), EMB, EMB, TR));
    J.j[J.n++] = steps(mlg::bjob(at(p.w.dfc2), EMB, at(p.w.x2), EMB, gp(a.c_w2), gp(a.c_b2), EMB, EMB, TR));
    J.j[J.n++] = steps(mlg::bjob(at(p.w.dgi), 3 * EMB, at(p.w.x3), EMB, gp(a.c_wih), gp(a.c_bih), 3 * EMB, EMB, TR));
    J.j[J.n++] = steps(mlg::bjob(at(p.w.dgh), 3 * EMB, at(p.w.hs_on), EMB, gp(a.c_whh), gp(a.c_bhh), 3 * EMB, EMB, TR));
    J.j[J.n++] = steps(mlg::bjob(at(p.w.d2), c.A, ws ? ws + p.w.hs_on + (int64_t)c.Ron * EMB : nullptr, EMB,
                                 gp(a.c_w3), gp(a.c_b3), c.A, EMB, TR));
    for (int k = 0; k < 4; ++k) {  // REFIL_HYPER_JOBS jobs, the table's last
        const RHyper& h = p.Lh;
        const int64_t G0 = p.n_agent + (int64_t)k * h.c_total;
        const int rows = nvar(k) * c.I * NAS;
        J.j[J.n++] = items(mlg::bjob(at(p.w.dfc1m[k]), EMB, at(p.w.ein), c.K1, gp(G0 + h.c_w1), gp(G0 + h.c_b1), EMB, c.D0,
                                     I16), NE);
        J.j[J.n++] = items(mlg::bjob(at(p.w.dqkvm[k]), 3 * EMB, at(p.w.x1m[k]), EMB, gp(G0 + h.c_win), nullptr, 3 * EMB,
                                     EMB, I16), NE);
        J.j[J.n++] = items(mlg::bjob(at(p.w.doutm[k]), EMB, at(p.w.om[k]), EMB, gp(G0 + h.c_wout), gp(G0 + h.c_bout), EMB,
                                     EMB, rows), NAS);
        J.j[J.n++] = items(mlg::bjob(at(p.w.dX[k]), EM, at(p.w.x2m[k]), EMB, gp(G0 + h.c_w2), gp(G0 + h.c_b2), EM, EMB,
                                     rows), NAS);
    }
    static_assert(REFIL_HYPER_JOBS == 4 * 4, "four jobs per hypernet");
    int64_t slab_part;
    *slab_floats = mlg::layout_bjobs(J, n_tasks, n_red, &slab_part);
    p.w.nrm = p.w.slab + slab_part;
    return J;
}

// The mixer's hypernetwork kernels run on a second stream beside the agent path: hyper_fwd needs only the
// prologue's outputs (beside ent_fwd -> rec4 -> q), hyper_bwd only mix_td's dX (beside rec_bwd4 -> ent_bwd); the
// sequential recurrences leave most CUs idle (mlg::side_stream, mlg_host.h).
int run_train(Plan& p, const MlgRefilLearnerCfg* cfg, const MlgRefilLearnerBufs* bufs, hipStream_t s) {
    const RCfg& c = p.c;
    const bool s8 = is_s8(c);  // the refil_8 shape: static instantiations of the per-item kernels
    float* ws = bufs->workspace;
    const WsR& w = p.w;
    MlgEntityBatch bt = bufs->batch;
    // host slot map: the prologue's argument, stored by it to the workspace for the later launches
    if (bufs->host_rows) bt.rows = reinterpret_cast<const int32_t*>(ws + w.rows);
    const float* params = bufs->params;
    const float* tparams = bufs->target_params;
    // ---- prologue, one launch: mask sum, parameter packs, in_trans splits, transposes, entity inputs ----
    Prologue P{};
    P.aj = agent_jobs(p.La);
    P.hj = hyper_jobs(p.Lh);
    MLG_REQUIRE(!P.aj.overflow && !P.hj.overflow, "refil learner: pack job table over capacity (%d)", CopyJobs::kCap);
    static_assert(2 * 4 <= CopyPairs::kCap && 2 * 4 + 2 <= HSplit::kCap, "prologue tables: one slot per block");
    P.ap.src[0] = params;
    P.ap.dst[0] = ws + w.pa_on;
    P.ap.src[1] = tparams;
    P.ap.dst[1] = ws + w.pa_tg;
    const RAgent& La = p.La;
    TrJobs& tj = P.tj;
    bool tr_bad = false;  // the transpose blocks cover jobs of <= 3 * EMB * EMB elements, TrJobs::kCap jobs
    auto tr = [&](const float* src, float* dst, int rows, int cols) {
        if (tj.n < TrJobs::kCap && (int64_t)rows * cols <= 3 * EMB * EMB) tj.j[tj.n++] = TrJob{src, dst, rows, cols};
        else tr_bad = true;
    };
    tr(params + La.c_win, ws + w.a_winT, 3 * EMB, EMB);
    tr(params + La.c_wout, ws + w.a_woutT, EMB, EMB);
    tr(params + La.c_w2, ws + w.a_w2T, EMB, EMB);
    tr(params + La.c_wih, ws + w.a_wihT, 3 * EMB, EMB);
    for (int k = 0; k < 4; ++k) {
        const int64_t G0 = p.n_agent + (int64_t)k * p.Lh.c_total;
        P.hp.src[2 * k] = params + G0;
        P.hp.dst[2 * k] = ws + w.ph_on[k];
        P.hp.src[2 * k + 1] = tparams + G0;
        P.hp.dst[2 * k + 1] = ws + w.ph_tg[k];
        tr(params + G0 + p.Lh.c_win, ws + w.h_winT[k], 3 * EMB, EMB);
        tr(params + G0 + p.Lh.c_wout, ws + w.h_woutT[k], EMB, EMB);
        tr(params + G0 + p.Lh.c_w2, ws + w.h_w2T[k], EM, EMB);
    }
    MLG_REQUIRE(!tr_bad, "refil learner: transpose job table over capacity or job larger than the grid");
    HSplit& hs = P.hs;
    for (int k = 0; k < 4; ++k) {
        const int64_t G0 = p.n_agent + (int64_t)k * p.Lh.c_total;
        hs.src[k] = params + G0 + p.Lh.c_win;
        hs.src[k + 4] = tparams + G0 + p.Lh.c_win;
        hs.dst[k] = ws + w.h_wsp[k];
        hs.dst[k + 4] = ws + w.h_wsp[k + 4];
    }
    hs.src[8] = params + La.c_win;
    hs.src[9] = tparams + La.c_win;
    hs.dst[8] = ws + w.h_wsp[8];
    hs.dst[9] = ws + w.h_wsp[9];
    for (int k = 0; k < 4; ++k) {
        P.hsT.src[k] = hs.src[k];
        P.hsT.dst[k] = ws + w.h_wspT[k];
    }
    P.hsT.src[4] = params + La.c_win;
    P.hsT.dst[4] = ws + w.h_wspT[4];
    P.c = c;
    P.bt = bt;
    if (bufs->host_rows) {
        P.n_rows_in = c.B;
        P.rows_dst = reinterpret_cast<int32_t*>(ws + w.rows);
        for (int b = 0; b < c.B; ++b) P.rows_in[b] = bufs->host_rows[b];
    }
    P.ein = ws + w.ein;
    P.msum = ws + w.msum;
    P.nb_a = (int)((P.aj.total + 255) / 256);
    P.nb_h = (int)((P.hj.total + 255) / 256);
    P.nb_s = (int)((REFIL_HSP + 255) / 256);
    P.nb_t = (3 * EMB * EMB + 255) / 256;
    P.nb_e = (int)(((int64_t)c.I * NE * c.K1 + 255) / 256);
    hipLaunchKernelGGL(prologue_kernel, dim3((unsigned)prologue_blocks(P)), dim3(256), 0, s, P);
    // read per call: a test can compare the one-stream and side-stream forms within one process
    const bool one_stream = getenv("MLG_REFIL_ONE_STREAM") != nullptr;
    mlg::SideStream* side = one_stream ? nullptr : mlg::side_stream(s);
    const hipStream_t sh = side ? side->s : s;  // the hypernet kernels' stream
    if (side) {
        MLG_REQUIRE(mlg::fork_join(side, 0, s, sh), "refil learner: side stream fork");
    }
    // ---- agent forward ----
    AgentPtrs on{ws + w.pa_on, ws + w.x1, ws + w.qkv, ws + w.P, ws + w.o, ws + w.x2, ws + w.x3, ws + w.gi_on,
                 ws + w.h_wsp[8]};
    AgentPtrs tg{ws + w.pa_tg, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, ws + w.gi_tg, ws + w.h_wsp[9]};
    hipLaunchKernelGGL(s8 ? ent_fwd_kernel<1> : ent_fwd_kernel<0>, dim3((unsigned)((c.I + 1) / 2), 2), dim3(64), 0, s, c,
                       bt, bufs->groupA, La,
                       ws + w.ein, on, tg, ws + w.msum);
    const int nt_on = (c.Ron + 15) / 16, nt_tg = (c.Rtg + 15) / 16;
    // the recurrences on 4-row tiles (default) or 16-row tiles (MLG_REFIL_REC16, A/B)
    static const bool rec16 = getenv("MLG_REFIL_REC16") != nullptr;
    if (rec16)
        hipLaunchKernelGGL(rec_kernel, dim3((unsigned)(nt_on + nt_tg)), dim3(256), 0, s, c, La, ws + w.pa_on,
                           ws + w.pa_tg, ws + w.gi_on, ws + w.gi_tg, ws + w.hs_on, ws + w.hs_tg, ws + w.gr, ws + w.gz,
                           ws + w.gn, ws + w.ghn, ws + w.msum);
    else
        hipLaunchKernelGGL(rec4_kernel, dim3((unsigned)((c.Ron + 3) / 4 + (c.Rtg + 3) / 4)), dim3(256), 0, s, c, La,
                           ws + w.pa_on, ws + w.pa_tg, ws + w.gi_on, ws + w.gi_tg, ws + w.hs_on, ws + w.hs_tg, ws + w.gr,
                           ws + w.gz, ws + w.gn, ws + w.ghn, ws + w.msum);
    hipLaunchKernelGGL(s8 ? q_kernel<1> : q_kernel<0>, dim3((unsigned)nt_on, (unsigned)c.T, 2), dim3(64 * (c.Ap / 16)), 0,
                       s, c, bt, La,
                       ws + w.pa_on, ws + w.pa_tg, ws + w.hs_on, ws + w.hs_tg, ws + w.mac, ws + w.tmac, ws + w.msum);
    // ---- mixer ----
    HypPtrs hp;
    for (int k = 0; k < 8; ++k) hp.Wsp[k] = ws + w.h_wsp[k];
    for (int k = 0; k < 4; ++k) {
        hp.Pon[k] = ws + w.ph_on[k];
        hp.Ptg[k] = ws + w.ph_tg[k];
        hp.x1m[k] = ws + w.x1m[k];
        hp.qkvm[k] = ws + w.qkvm[k];
        hp.Pm[k] = ws + w.Pm[k];
        hp.om[k] = ws + w.om[k];
        hp.x2m[k] = ws + w.x2m[k];
        hp.X[k] = ws + w.X[k];
        hp.Xtg[k] = ws + w.Xtg[k];
    }
    hipLaunchKernelGGL(s8 ? hyper_fwd_kernel<1> : hyper_fwd_kernel<0>, dim3((unsigned)c.I, 8), dim3(64), 0, sh, c, bt,
                       bufs->groupA, p.Lh, ws + w.ein, hp,
                       ws + w.msum);
    if (side) {
        MLG_REQUIRE(mlg::fork_join(side, 1, sh, s), "refil learner: side stream join");
    }
    MixIO io;
    for (int k = 0; k < 4; ++k) {
        io.X[k] = ws + w.X[k];
        io.Xtg[k] = ws + w.Xtg[k];
        io.dX[k] = ws + w.dX[k];
    }
    io.mac = ws + w.mac;
    io.tmac = ws + w.tmac;
    io.msum = ws + w.msum;
    io.dq = ws + w.dq;
    io.d2 = ws + w.d2;
    io.part = ws + w.part;
    hipLaunchKernelGGL(s8 ? mix_td_kernel<1> : mix_td_kernel<0>, dim3((unsigned)c.I), dim3(64), 0, s, c, bt, io);
    if (side) {
        MLG_REQUIRE(mlg::fork_join(side, 2, s, sh), "refil learner: side stream fork");
    }
    HypBwd hb;
    for (int k = 0; k < 4; ++k) {
        hb.Pon[k] = ws + w.ph_on[k];
        hb.woutT[k] = ws + w.h_woutT[k];
        hb.w2T[k] = ws + w.h_w2T[k];
        hb.winT[k] = ws + w.h_winT[k];
        hb.wspT[k] = ws + w.h_wspT[k];
        hb.x1m[k] = ws + w.x1m[k];
        hb.qkvm[k] = ws + w.qkvm[k];
        hb.Pm[k] = ws + w.Pm[k];
        hb.dX[k] = ws + w.dX[k];
        hb.doutm[k] = ws + w.doutm[k];
        hb.dqkvm[k] = ws + w.dqkvm[k];
        hb.dfc1m[k] = ws + w.dfc1m[k];
    }
    hipLaunchKernelGGL(s8 ? hyper_bwd_kernel<1> : hyper_bwd_kernel<0>, dim3((unsigned)c.I, 4), dim3(64), 0, sh, c, bt, hb,
                       ws + w.msum);
    // weight gradients: the hypernets' jobs (the table's last REFIL_HYPER_JOBS, final after hyper_bwd) run on the side
    // stream beside ent_bwd, the agent's after it; one reduce over the whole table (same chunk sums as one launch)
    int64_t slab_floats, n_red;
    int n_tasks;
    RJobs J = make_jobs(p, ws, bufs->grads, &slab_floats, &n_tasks, &n_red);
    int tH, tE;
    int64_t rH, rE;
    const RJobs JH = mlg::bjob_view(J, J.n - REFIL_HYPER_JOBS, J.n, &tH, &rH),
               JE = mlg::bjob_view(J, 0, J.n - REFIL_HYPER_JOBS, &tE, &rE);
    hipLaunchKernelGGL(mlg::wgrad_block_kernel<MJ>, dim3((unsigned)((tH + 3) / 4)), dim3(256), 0, sh, JH, ws + w.slab);
    if (side) MLG_REQUIRE(hipEventRecord(side->ev[3], sh) == hipSuccess, "refil learner: side stream record");
    // ---- agent backward ----
    if (rec16)
        hipLaunchKernelGGL(rec_bwd_kernel, dim3((unsigned)nt_on), dim3(256), 0, s, c, bt, La, ws + w.pa_on, ws + w.hs_on,
                           ws + w.gr, ws + w.gz, ws + w.gn, ws + w.ghn, ws + w.dq, ws + w.dgi, ws + w.dgh, ws + w.msum);
    else
        hipLaunchKernelGGL(rec_bwd4_kernel, dim3((unsigned)((c.Ron + 3) / 4)), dim3(256), 0, s, c, bt, La, ws + w.pa_on,
                           ws + w.hs_on, ws + w.gr, ws + w.gz, ws + w.gn, ws + w.ghn, ws + w.dq, ws + w.dgi, ws + w.dgh,
                           ws + w.msum);
    EntBwd eb{ws + w.a_wihT, ws + w.a_w2T, ws + w.a_woutT, ws + w.a_winT, ws + w.h_wspT[4], ws + w.x1, ws + w.qkv, ws + w.P, ws + w.x3,
              ws + w.dgi, ws + w.dfc2, ws + w.dout, ws + w.dqkv, ws + w.dfc1};
    hipLaunchKernelGGL(s8 ? ent_bwd_kernel<1> : ent_bwd_kernel<0>, dim3((unsigned)((c.I + 1) / 2)), dim3(64), 0, s, c, bt,
                       eb, ws + w.msum);
    // ---- weight gradients, clip, RMSprop ----
    hipLaunchKernelGGL(mlg::wgrad_block_kernel<MJ>, dim3((unsigned)((tE + 3) / 4)), dim3(256), 0, s, JE, ws + w.slab);
    if (side) MLG_REQUIRE(hipStreamWaitEvent(s, side->ev[3], 0) == hipSuccess, "refil learner: side stream join");
    const int n_red_blocks = (int)((n_red + 255) / 256);
    hipLaunchKernelGGL(mlg::wgrad_block_reduce_kernel<MJ>, dim3((unsigned)n_red_blocks), dim3(256), 0, s, J, ws + w.slab,
                       ws + p.w.nrm);
    const int64_t n_par = p.n_agent + p.n_mixer;
    hipLaunchKernelGGL(refil_finish_kernel, dim3((unsigned)((n_par + 1023) / 1024)), dim3(1024), 0, s, ws + w.part, c.I,
                       ws + w.msum, bufs->params, bufs->grads, bufs->square_avg, n_par, cfg->lr, cfg->optim_alpha,
                       cfg->optim_eps, cfg->grad_norm_clip, c.NA, c.lmbda, bufs->stats, ws + p.w.nrm, n_red_blocks,
                       bufs->trained_steps, bufs->target_sync);
    return mlg::check_launch("refil_train");
}

}  // namespace

extern "C" int64_t mlg_refil_param_counts(const MlgRefilLearnerCfg* c, int64_t* n_agent, int64_t* n_mixer) {
    if (check_cfg(c)) return -1;
    Plan p = make_plan(c, c->T);
    if (n_agent) *n_agent = p.n_agent;
    if (n_mixer) *n_mixer = p.n_mixer;
    return p.n_agent + p.n_mixer;
}

extern "C" int64_t mlg_refil_workspace_floats(const MlgRefilLearnerCfg* c) {
    if (check_cfg(c)) return -1;
    Plan p = make_plan(c, c->T);
    int64_t slab, n_red;
    int tasks;
    make_jobs(p, nullptr, nullptr, &slab, &tasks, &n_red);
    return p.w.total + slab;
}

namespace {
// ---- the imagine group draw (entity_rnn_agent.py:95-97) on the device: p_b ~ U(0, 1) per episode, then entity j of
// episode b in group A with probability p_b. Counter-based (mlg_rng: key = seed, counter = (draw, b, purpose 5,
// j + 1)); like the reference's th.rand / th.bernoulli it is a random draw, not a bit-reproduction of torch's stream.
__global__ void refil_groups_kernel(int B, int NE, uint64_t seed, uint32_t draw, uint8_t* __restrict__ groupA) {
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= B * NE) return;
    const int b = k / NE, j = k % NE;
    const float p = mlg_u01(mlg_rng(seed, mlg_ctr(draw, (uint32_t)b, 5u, 0u)));
    groupA[k] = (uint8_t)(mlg_u01(mlg_rng(seed, mlg_ctr(draw, (uint32_t)b, 5u, (uint32_t)j + 1u))) < p);
}
}  // namespace

extern "C" int mlg_refil_draw_groups(int32_t B, int32_t NE, uint64_t seed, uint32_t draw, uint8_t* groupA,
                                     void* stream) {
    // the counter keeps 16 bits of b and 12 of j + 1 (mlg_ctr): B <= 65536 and NE < 4096 keep every draw distinct
    MLG_REQUIRE(groupA && B >= 1 && B <= 65536 && NE >= 1 && NE < 4096, "refil_draw_groups: B=%d NE=%d", B, NE);
    hipLaunchKernelGGL(refil_groups_kernel, dim3((unsigned)((B * NE + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                       B, NE, seed, draw, groupA);
    return mlg::check_launch("refil_draw_groups");
}

extern "C" int mlg_refil_train(const MlgRefilLearnerCfg* c, const MlgRefilLearnerBufs* b, void* stream) {
    if (check_cfg(c)) return 1;
    MLG_REQUIRE(b && b->params && b->grads && b->square_avg && b->target_params && b->workspace && b->stats && b->groupA,
                "refil_train: null buffer");
    const MlgEntityBatch& bt = b->batch;
    MLG_REQUIRE(bt.entities && bt.obs_mask && bt.entity_mask && bt.actions && bt.avail && bt.reward && bt.terminated &&
                    bt.actions_onehot && bt.filled, "refil_train: batch has null tensors");
    MLG_REQUIRE(bt.B == c->B && bt.T1 >= c->T, "refil_train: batch B=%d T1=%d vs cfg B=%d T=%d", bt.B, bt.T1, c->B, c->T);
    MLG_REQUIRE(!b->host_rows || c->B <= MLG_INLINE_ROWS, "refil_train: host_rows needs B <= %d (got %d)",
                MLG_INLINE_ROWS, c->B);
    Plan p = make_plan(c, bt.T1);
    return run_train(p, c, b, (hipStream_t)stream);
}
